// HBM ceiling probes (include/hrs_probe.h), built as their own library,
// libhrs_probe.so: bench.py and tools load it to measure this GPU's ceilings
// beside the coding kernels in the same run; the product library a DataNode
// JVM loads (libhrs.so) does not carry them.
//   - streams (copy / read-only / write-only) in the shape of round 1's
//     bandwidth lab (tools/bw_lab.hip, profiles/r01/lab8_bw_ceilings.txt): a
//     wave task is `chunk` KiB contiguous, one 16-byte access per lane per
//     KiB, all of the task's loads issued before any is consumed;
//   - the coding kernels' own access pattern with the math taken out
//     (hrs_probe_rows): 2 KiB column windows of `nread` rows of a stripe-major
//     [S][nrows][L] buffer read, `nwrite` rows written, nontemporal 16-byte
//     accesses, one wave task per window, as encode_static_kernel and the
//     pipelined repair kernel walk them (same window order, HRS_TASK_ORDER),
//     under a few load schedules.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/hrs_probe.h"
#include "hrs_device.hpp"
#include "hrs_launch.hpp"

namespace hrs {
namespace {

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}

template <bool NT>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Stream ops: 0 copy, 1 read-only (XOR kept alive by a data-dependent store
// to `sink`, practically never taken), 2 write-only; each over n 16-byte
// elements under one of three schedules (tools/copy_lab.hip measured them,
// profiles/r04/copy_lab/):
//   WAVE_TASKS  a wave task is D contiguous KiB (lane l moves the 16 bytes at
//               1024 j + 16 l of KiB j), wave tasks grid-striding;
//   GRID_STRIDE thread i moves elements i + j T (T = every thread of the
//               grid), D of them in flight before any is used;
//   BLOCK_RANGE block b owns the b-th of gridDim equal ranges and walks it
//               block-stride, D elements per thread in flight — each block
//               streams through one contiguous region (the fastest copy on
//               this pool: 5.75 TB/s against 5.36 for the grid-stride loop).
template <int OP, bool NT>
__device__ __forceinline__ void stream_op(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t i,
                                          u32x4& acc) {
  if constexpr (OP == 0) st16<NT>(&dst[i], ld16<NT>(&src[i]));
  else if constexpr (OP == 1) acc ^= ld16<NT>(&src[i]);
  else st16<NT>(&dst[i], u32x4{static_cast<uint32_t>(i), 0x5A5A5A5Au, ~static_cast<uint32_t>(i), 0u});
}

// D elements at base + j * step (j < D): all loads issued before any store.
template <int OP, int D, bool NT>
__device__ __forceinline__ void stream_group(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t base,
                                             uint64_t step, u32x4& acc) {
  if constexpr (OP == 2) {
#pragma unroll
    for (int j = 0; j < D; ++j) stream_op<2, NT>(src, dst, base + j * step, acc);
  } else {
    u32x4 v[D];
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = ld16<NT>(&src[base + j * step]);
#pragma unroll
    for (int j = 0; j < D; ++j) {
      if constexpr (OP == 0) st16<NT>(&dst[base + j * step], v[j]);
      else acc ^= v[j];
    }
  }
}

template <int OP, int SCHED, int D, bool NT>
__global__ void __launch_bounds__(1024) stream_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       uint64_t n) {
  u32x4 acc = {0u, 0u, 0u, 0u};
  const uint64_t T = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if constexpr (SCHED == HRS_PROBE_WAVE_TASKS) {
    const int lane = threadIdx.x & 63;
    const uint64_t ntasks = n / (64u * D);
    const uint64_t nw = T >> 6;
    for (uint64_t t = gid >> 6; t < ntasks; t += nw) stream_group<OP, D, NT>(src, dst, t * 64u * D + lane, 64u, acc);
    for (uint64_t i = ntasks * 64u * D + gid; i < n; i += T) stream_op<OP, false>(src, dst, i, acc);
  } else if constexpr (SCHED == HRS_PROBE_GRID_STRIDE) {
    uint64_t i = gid;
    for (; i + (D - 1) * T < n; i += D * T) stream_group<OP, D, NT>(src, dst, i, T, acc);
    for (; i < n; i += T) stream_op<OP, false>(src, dst, i, acc);
  } else {
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = per * blockIdx.x;
    const uint64_t hi = lo + per < n ? lo + per : n;
    const uint64_t B = blockDim.x;
    uint64_t i = lo + threadIdx.x;
    for (; i + (D - 1) * B < hi; i += D * B) stream_group<OP, D, NT>(src, dst, i, B, acc);
    for (; i < hi; i += B) stream_op<OP, false>(src, dst, i, acc);
  }
  if constexpr (OP == 1)
    if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9E3779B9u && acc[0] == 0x7F4A7C15u) dst[threadIdx.x & 255] = acc;
}

// The codec's access pattern without the GF math: task t = (stripe, 2 KiB
// window); read rows [nrows - R, nrows), write rows [0, W) with the XOR of the
// reads (+ the row index), every access nontemporal. D rows' loads in flight
// (row r + D issued before row r is used; sched_barriers stop the compiler
// hoisting more) and M dependent VALU steps per loaded dword stand in for the
// math: HBM serves a spaced-out request stream better than a burst, so the
// pattern's ceiling is the best of a few schedules, not the all-loads-first
// one (tools/pace_probe.hip, profiles/r03/ab/NOTES.md).
template <int M>
__device__ __forceinline__ u32x4 pace_work(u32x4 x) {
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = __builtin_amdgcn_alignbit(x[q], x[q], 7) ^ (0x9E3779B9u * (m + 1));
  return x;
}

template <int R, int W, int D, int M>
__global__ void __launch_bounds__(256) rows_kernel(uint8_t* __restrict__ base, uint64_t nstripes, int nrows,
                                                    uint64_t L, int order) {
  const int lane = threadIdx.x & 63;
  const uint64_t nwin = L / 2048u;
  const uint64_t ntasks = nstripes * nwin;
  const WaveTasks wt = wave_tasks(ntasks, order);  // the coding kernels' window order
  for (uint32_t j = 0; j < 0xFFFFFFFFu; ++j) {
    const uint64_t t = wt.at(j);
    if (t >= wt.end) break;
    const uint64_t s = t / nwin;
    uint8_t* sb = base + s * nrows * L + (t - s * nwin) * 2048u + lane * 16;
    u32x4 v[R][2];
    auto ld = [&](int r) {
      const u32x4* p = reinterpret_cast<const u32x4*>(sb + (nrows - R + r) * L);
      v[r][0] = __builtin_nontemporal_load(p);
      v[r][1] = __builtin_nontemporal_load(p + 64);
    };
#pragma unroll
    for (int r = 0; r < D && r < R; ++r) ld(r);
    u32x4 a = {0u, 0u, 0u, 0u}, b = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r + D < R) ld(r + D);
      __builtin_amdgcn_sched_barrier(0);
      a ^= pace_work<M>(v[r][0]);
      b ^= pace_work<M>(v[r][1]);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int o = 0; o < W; ++o) {
      u32x4* q = reinterpret_cast<u32x4*>(sb + o * L);
      __builtin_nontemporal_store(a + static_cast<uint32_t>(o), q);
      __builtin_nontemporal_store(b + static_cast<uint32_t>(o), q + 64);
    }
  }
}

template <int OP, int SCHED, int D>
hrs_status launch_stream_d(const void* src, void* dst, uint64_t n, bool nt, unsigned grid, unsigned block,
                           hipStream_t st) {
  auto k = nt ? stream_kernel<OP, SCHED, D, true> : stream_kernel<OP, SCHED, D, false>;
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, st, static_cast<const u32x4*>(src), static_cast<u32x4*>(dst), n);
  return hipGetLastError() == hipSuccess ? HRS_OK : HRS_EDEVICE;
}

template <int OP, int SCHED>
hrs_status launch_stream_s(const void* src, void* dst, uint64_t n, int depth, bool nt, unsigned grid, unsigned block,
                           hipStream_t st) {
  switch (depth) {
    case 1: return launch_stream_d<OP, SCHED, 1>(src, dst, n, nt, grid, block, st);
    case 2: return launch_stream_d<OP, SCHED, 2>(src, dst, n, nt, grid, block, st);
    case 4: return launch_stream_d<OP, SCHED, 4>(src, dst, n, nt, grid, block, st);
    default: return launch_stream_d<OP, SCHED, 8>(src, dst, n, nt, grid, block, st);
  }
}

template <int OP>
hrs_status launch_stream(const void* src, void* dst, size_t bytes, int schedule, int depth, int nt, int block,
                         int bpc, void* stream) {
  const unsigned grid = static_cast<unsigned>(bpc * device_cus());
  const uint64_t n = bytes / 16;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  switch (schedule) {
    case HRS_PROBE_WAVE_TASKS:
      return launch_stream_s<OP, HRS_PROBE_WAVE_TASKS>(src, dst, n, depth, nt != 0, grid, block, st);
    case HRS_PROBE_GRID_STRIDE:
      return launch_stream_s<OP, HRS_PROBE_GRID_STRIDE>(src, dst, n, depth, nt != 0, grid, block, st);
    default:
      return launch_stream_s<OP, HRS_PROBE_BLOCK_RANGE>(src, dst, n, depth, nt != 0, grid, block, st);
  }
}

// Schedules (rows in flight D, VALU steps per dword M): 0 = (R, 0) all loads
// first, no math; 1 = (3, 12); 2 = (5, 6); 3 = (1, 0).
template <int R, int W, int D, int M>
hrs_status launch_rows_dm(void* base, size_t nstripes, int nrows, size_t L, unsigned grid, hipStream_t st) {
  auto k = rows_kernel<R, W, D, M>;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, static_cast<uint8_t*>(base), static_cast<uint64_t>(nstripes),
                     nrows, static_cast<uint64_t>(L), task_order(kOrderStaticEncode));
  return hipGetLastError() == hipSuccess ? HRS_OK : HRS_EDEVICE;
}

template <int R, int W>
hrs_status launch_rows_rw(void* base, size_t nstripes, int nrows, size_t L, int schedule, unsigned grid,
                          hipStream_t st) {
  switch (schedule) {
    case 0: return launch_rows_dm<R, W, R, 0>(base, nstripes, nrows, L, grid, st);
    case 1: return launch_rows_dm<R, W, 3, 12>(base, nstripes, nrows, L, grid, st);
    case 2: return launch_rows_dm<R, W, 5, 6>(base, nstripes, nrows, L, grid, st);
    default: return launch_rows_dm<R, W, 1, 0>(base, nstripes, nrows, L, grid, st);
  }
}

bool stream_args_ok(int schedule, int depth, int block, int bpc) {
  return schedule >= HRS_PROBE_WAVE_TASKS && schedule <= HRS_PROBE_BLOCK_RANGE &&
         (depth == 1 || depth == 2 || depth == 4 || depth == 8) && (block == 256 || block == 512 || block == 1024) &&
         bpc >= 1 && bpc * block <= 8192;
}

}  // namespace
}  // namespace hrs

extern "C" hrs_status hrs_probe_stream(int op, const void* src, void* dst, size_t bytes, int schedule, int depth,
                                       int nontemporal, int block_threads, int blocks_per_cu, void* stream) {
  if (op < HRS_PROBE_COPY || op > HRS_PROBE_WRITE || !hrs::stream_args_ok(schedule, depth, block_threads, blocks_per_cu))
    return HRS_EINVAL;
  const bool need_src = op != HRS_PROBE_WRITE;
  if (bytes && ((need_src && !src) || !dst)) return HRS_EINVAL;
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | bytes) & 15u) return HRS_EALIGN;
  if (bytes == 0) return HRS_OK;
  switch (op) {
    case HRS_PROBE_COPY:
      return hrs::launch_stream<0>(src, dst, bytes, schedule, depth, nontemporal, block_threads, blocks_per_cu, stream);
    case HRS_PROBE_READ:
      return hrs::launch_stream<1>(src, dst, bytes, schedule, depth, nontemporal, block_threads, blocks_per_cu, stream);
    default:
      return hrs::launch_stream<2>(nullptr, dst, bytes, schedule, depth, nontemporal, block_threads, blocks_per_cu,
                                   stream);
  }
}

extern "C" hrs_status hrs_probe_rows(void* base, size_t nstripes, int nrows, size_t cell_bytes, int nread,
                                     int nwrite, int schedule, int blocks_per_cu, void* stream) {
  if (blocks_per_cu < 1 || blocks_per_cu > 32 || nrows < 1 || nread < 1 || nwrite < 0 || nread + nwrite > nrows ||
      schedule < 0 || schedule > 3)
    return HRS_EINVAL;
  if (nstripes && !base) return HRS_EINVAL;
  if ((reinterpret_cast<uintptr_t>(base) & 15u) || (cell_bytes % 2048u)) return HRS_EALIGN;
  if (nstripes == 0 || cell_bytes == 0) return HRS_OK;
  const unsigned grid = static_cast<unsigned>(blocks_per_cu * hrs::device_cus());
  const hipStream_t st = static_cast<hipStream_t>(stream);
  // The read / write counts of the shapes bench.py and the tests quote:
  // RS(10,4) encode and 1..4-erasure repairs, RS(6,3), RS(12,4), RS(3,2).
  switch (nread * 100 + nwrite) {
    case 1004: return hrs::launch_rows_rw<10, 4>(base, nstripes, nrows, cell_bytes, schedule, grid, st);
    case 1003: return hrs::launch_rows_rw<10, 3>(base, nstripes, nrows, cell_bytes, schedule, grid, st);
    case 1002: return hrs::launch_rows_rw<10, 2>(base, nstripes, nrows, cell_bytes, schedule, grid, st);
    case 1001: return hrs::launch_rows_rw<10, 1>(base, nstripes, nrows, cell_bytes, schedule, grid, st);
    case 1000: return hrs::launch_rows_rw<10, 0>(base, nstripes, nrows, cell_bytes, schedule, grid, st);
    case 603: return hrs::launch_rows_rw<6, 3>(base, nstripes, nrows, cell_bytes, schedule, grid, st);
    case 1204: return hrs::launch_rows_rw<12, 4>(base, nstripes, nrows, cell_bytes, schedule, grid, st);
    case 1202: return hrs::launch_rows_rw<12, 2>(base, nstripes, nrows, cell_bytes, schedule, grid, st);
    case 302: return hrs::launch_rows_rw<3, 2>(base, nstripes, nrows, cell_bytes, schedule, grid, st);
    default: return HRS_EINVAL;
  }
}
