// Host-side launch geometry shared by the kernel translation units
// (hrs_kernels.hip, hrs_runtime.hip, hrs_batch.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "hrs_internal.hpp"

namespace hrs {

// note_kernel with the template arguments spelled as rocprofv3 prints them:
// note_kernel_t("bitsliced_pipe_kernel", 1, 12) -> "bitsliced_pipe_kernel<1, 12>".
inline void kname_arg(std::string& s, int v) { s += std::to_string(v); }
inline void kname_arg(std::string& s, bool v) { s += v ? "true" : "false"; }
inline void kname_arg(std::string& s, const char* v) { s += v; }
template <typename... T>
inline void note_kernel_t(const char* base, T... v) {
  std::string s(base);
  if constexpr (sizeof...(T) > 0) {
    const char* sep = "<";
    ((s += sep, kname_arg(s, v), sep = ", "), ...);
    s += '>';
  }
  note_kernel(s.c_str());
}

// CU count per device, cached; handles on several host threads may race to
// fill it (same value), hence the relaxed atomics.
inline int device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  static std::atomic<int> cus_of[64];
  if (dev < 0 || dev >= 64) return 256;
  int cus = cus_of[dev].load(std::memory_order_relaxed);
  if (cus == 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cus_of[dev].store(cus, std::memory_order_relaxed);
  }
  return cus;
}

// Window -> wave order of a streaming kernel launch (hrs_device.hpp
// wave_tasks): C >= 1 = block-cyclic chunks of C windows per wave (1 = grid-
// stride), 0 = block range. Each kernel family passes its measured default;
// HRS_TASK_ORDER=<C> overrides every family (A/B runs), read per launch so
// one process can sweep it (tools/bench_order.py).
inline int task_order(int dflt) {
  const char* e = getenv("HRS_TASK_ORDER");
  if (e && *e) {
    const int c = atoi(e);
    if (c >= 0 && c <= 4096) return c;
  }
  return dflt;
}

// Defaults per family: grid-stride throughout (hrs_device.hpp wave_tasks,
// profiles/r04/q/order_sweep.jsonl, r/ and s/order_shapes.jsonl).
constexpr int kOrderStaticEncode = 1;  // encode_static / encode_cauchy / xor
constexpr int kOrderRuntime = 1;       // bitsliced (plain, pipelined, streaming) repairs
constexpr int kOrderBatch = 1;         // heterogeneous repair batches
constexpr int kOrderFusedEncode = 1;   // encode + CRC-32
constexpr int kOrderDecodeCrc = 1;     // repair + CRC-32
constexpr int kOrderCrc = 1;           // CRC-32 windows

template <class A>
inline A with_order(A a, int dflt) {
  a.order = task_order(dflt);
  return a;
}

// Streaming kernels: a fixed number of resident blocks per CU, grid-striding
// over the tasks. 2 x 256-thread blocks per CU (8 waves, each with a whole
// window's rows in flight) measured fastest for both the static and the
// runtime kernels (tools/kernel_lab.hip sweep, 256..1024 blocks); override
// with HRS_BLOCKS_PER_CU for experiments.
// VALU-bound shapes (the rolled bit loop: 3-4 erasure repairs, wide
// matrices) take 3 blocks per CU: the extra wave per SIMD hides more of the
// math (RS(10,4) 4-erasure decode +13%, profiles/r01/pipe/).
inline int blocks_per_cu(int dflt = 2) {
  static int v = [] {
    const char* e = getenv("HRS_BLOCKS_PER_CU");
    int x = e ? atoi(e) : 0;
    return (x >= 1 && x <= 32) ? x : 0;
  }();
  return v ? v : dflt;
}

// Zero-copy launches (kernels reading and writing pinned host memory across
// the host link, hrs_batch_api.cpp / hrs_hostpath.cpp) cap their grid: the
// link, not the CUs, bounds them, so a capped grid leaves the rest of the chip
// to other work. Set for the calling thread by a GridCap around the launch;
// every launcher sizes its grid through capped_grid (stream_grid, grid_for,
// and the fused / CRC launchers, whose 1,024- or 512-thread blocks take one
// CU each, so the cap in blocks is a cap in CUs there).
inline thread_local unsigned t_grid_cap = 0;

struct GridCap {
  unsigned prev;
  explicit GridCap(unsigned cap) : prev(t_grid_cap) { t_grid_cap = cap; }
  ~GridCap() { t_grid_cap = prev; }
};

inline unsigned capped_grid(uint64_t g) {
  if (t_grid_cap && g > t_grid_cap) g = t_grid_cap;
  return static_cast<unsigned>(g == 0 ? 1 : g);
}

inline unsigned stream_grid(uint64_t ntasks, int per_cu = 2) {
  const uint64_t want = static_cast<uint64_t>(blocks_per_cu(per_cu)) * device_cus();
  const uint64_t needed = (ntasks + kWavesPerBlock - 1) / kWavesPerBlock;
  uint64_t g = needed < want ? needed : want;
  return capped_grid(g);
}

template <typename Kernel>
inline unsigned grid_for(Kernel kernel, uint64_t work_items_per_block, uint64_t ntasks) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlockThreads, 0) != hipSuccess ||
      per_cu <= 0)
    per_cu = 2;
  const uint64_t resident = static_cast<uint64_t>(per_cu) * device_cus();
  const uint64_t needed = (ntasks + work_items_per_block - 1) / work_items_per_block;
  uint64_t g = needed < resident ? needed : resident;
  return capped_grid(g);
}

}  // namespace hrs
