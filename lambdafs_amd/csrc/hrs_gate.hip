// Stream gates of the synchronous host-buffer calls' queued pipeline
// (hrs_hostpath.cpp, staged calls): a chunk's kernels are queued on its slot
// stream BEFORE the host has copied the chunk into the pinned staging, behind
// a one-wave gate that waits until the host publishes the chunk's tag in a
// coherent pinned flag word; after them a one-wave signal publishes the tag
// in the slot's done word, which the host polls before it copies the outputs
// out. The GPU then starts a chunk a few microseconds after its copy-in ends
// (a launch made at that point started 17 us later, profiles/r05/NOTES.md).
//
// Every gate has an exit every lane reaches: it gives up after `timeout`
// ticks of the constant-rate wall clock, records the miss in *fail and
// returns, so a queue never stays blocked (the host then discards the call's
// results and runs it again without gates). Flags are only ever written with
// vector stores.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hrs_internal.hpp"

namespace hrs {
namespace {

__global__ void __launch_bounds__(64) gate_kernel(const uint32_t* ready, uint32_t want, uint32_t* fail,
                                                  uint64_t timeout) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
  for (;;) {
    const uint32_t v = __hip_atomic_load(ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (static_cast<int32_t>(v - want) >= 0) return;  // tags are serial numbers (wrap-safe)
    if (static_cast<uint64_t>(wall_clock64()) - t0 > timeout) {
      __hip_atomic_store(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// The release makes the slot's outputs (written by the kernels before it on
// the stream) visible to the host before the tag.
__global__ void __launch_bounds__(64) signal_kernel(uint32_t* done, uint32_t tag) {
  if (threadIdx.x == 0) __hip_atomic_store(done, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

hipError_t launch_gate(const uint32_t* ready, uint32_t want, uint32_t* fail, uint64_t timeout, hipStream_t s) {
  hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, s, ready, want, fail, timeout);
  return hipGetLastError();
}

hipError_t launch_signal(uint32_t* done, uint32_t tag, hipStream_t s) {
  hipLaunchKernelGGL(signal_kernel, dim3(1), dim3(64), 0, s, done, tag);
  return hipGetLastError();
}

}  // namespace hrs
