// HBM ceiling probe (include/hrs_probe.h): the nontemporal 16-byte
// grid-stride copy of tools/copy_probe.hip, built into libhrs so bench.py
// measures its own copy ceiling beside the coding kernels in the same run.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/hrs_probe.h"
#include "hrs_device.hpp"
#include "hrs_launch.hpp"

namespace hrs {
namespace {

__global__ void __launch_bounds__(256) stream_copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                           uint64_t n) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
}

// Read-only stream: every 16-byte element loaded once (nontemporal); a lane
// stores its XOR only if it equals an impossible value, so the loads stay.
__global__ void __launch_bounds__(256) stream_read_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ sink,
                                                           uint64_t n) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    acc ^= __builtin_nontemporal_load(&src[i]);
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9E3779B9u && acc[0] == 0x7F4A7C15u) sink[threadIdx.x] = acc;
}

// Write-only stream: every 16-byte element stored once (nontemporal).
__global__ void __launch_bounds__(256) stream_write_kernel(u32x4* __restrict__ dst, uint64_t n) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t v = static_cast<uint32_t>(i);
    __builtin_nontemporal_store(u32x4{v, v ^ 0x5A5A5A5Au, ~v, v * 0x9E3779B9u}, &dst[i]);
  }
}

}  // namespace
}  // namespace hrs

extern "C" hrs_status hrs_probe_copy(const void* src, void* dst, size_t bytes, int blocks_per_cu, void* stream) {
  if (blocks_per_cu < 1 || blocks_per_cu > 32 || (bytes && (!src || !dst))) return HRS_EINVAL;
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | bytes) & 15u) return HRS_EALIGN;
  if (bytes == 0) return HRS_OK;
  const unsigned grid = static_cast<unsigned>(blocks_per_cu * hrs::device_cus());
  hrs::note_kernel("stream_copy_kernel");
  hipLaunchKernelGGL(hrs::stream_copy_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const hrs::u32x4*>(src), static_cast<hrs::u32x4*>(dst),
                     static_cast<uint64_t>(bytes / 16));
  return hipGetLastError() == hipSuccess ? HRS_OK : HRS_EDEVICE;
}

extern "C" hrs_status hrs_probe_read(const void* src, size_t bytes, int blocks_per_cu, void* sink, void* stream) {
  if (blocks_per_cu < 1 || blocks_per_cu > 32 || !sink || (bytes && !src)) return HRS_EINVAL;
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(sink) | bytes) & 15u) return HRS_EALIGN;
  if (bytes == 0) return HRS_OK;
  const unsigned grid = static_cast<unsigned>(blocks_per_cu * hrs::device_cus());
  hrs::note_kernel("stream_read_kernel");
  hipLaunchKernelGGL(hrs::stream_read_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const hrs::u32x4*>(src), static_cast<hrs::u32x4*>(sink),
                     static_cast<uint64_t>(bytes / 16));
  return hipGetLastError() == hipSuccess ? HRS_OK : HRS_EDEVICE;
}

extern "C" hrs_status hrs_probe_write(void* dst, size_t bytes, int blocks_per_cu, void* stream) {
  if (blocks_per_cu < 1 || blocks_per_cu > 32 || (bytes && !dst)) return HRS_EINVAL;
  if ((reinterpret_cast<uintptr_t>(dst) | bytes) & 15u) return HRS_EALIGN;
  if (bytes == 0) return HRS_OK;
  const unsigned grid = static_cast<unsigned>(blocks_per_cu * hrs::device_cus());
  hrs::note_kernel("stream_write_kernel");
  hipLaunchKernelGGL(hrs::stream_write_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<hrs::u32x4*>(dst), static_cast<uint64_t>(bytes / 16));
  return hipGetLastError() == hipSuccess ? HRS_OK : HRS_EDEVICE;
}
