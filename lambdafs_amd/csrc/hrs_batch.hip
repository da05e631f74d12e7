// gfx950 heterogeneous repair batches (hrs_decode_batch_dev): one erasure
// pattern per stripe, each task reading its stripe's plan; same arithmetic as
// the runtime kernels (hrs_runtime.hip).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "hrs_device.hpp"
#include "hrs_launch.hpp"

namespace hrs {
namespace {

__constant__ gf::Tables d_tables = gf::make_tables();

// ------------------------------- heterogeneous batches (one pattern per stripe)

// Plans and pattern indices are read through the constant address space so
// the per-task reads are scalar loads (s_load), not vector memory traffic.
typedef const __attribute__((address_space(4))) BatchPlan* ConstPlanPtr;
typedef const __attribute__((address_space(4))) int32_t* ConstIntPtr;

// Same arithmetic as bitsliced_kernel; the wave reads its stripe's plan
// (inputs, coefficients, output count) at the start of each task.
// PATV: lane l of the wave loads the pattern index of the wave's task
// k + l (k = 0, 64, ...) in one vector load; each task then takes its index
// with a readlane instead of a scalar load that waits on HBM before any of
// the task's row loads can issue (the stripes of consecutive tasks differ).
template <int NOUT, int NINB, bool PATV>
__global__ void __launch_bounds__(kBlockThreads) batch_bitsliced_kernel(const BatchArgs a) {
  const int lane = threadIdx.x & 63;
  const ConstPlanPtr plans = (ConstPlanPtr)a.plans;
  const ConstIntPtr pat = (ConstIntPtr)a.pat;
  int patv = 0;
  uint32_t k = 0;
  const WaveTasks wt = wave_tasks(a.ntasks, a.order);
  for (;; ++k) {
    const uint64_t t = wt.at(k);
    if (t >= wt.end) break;
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    int pidx;
    if constexpr (PATV) {
      if ((k & 63u) == 0) {
        const uint64_t tl = wt.at(k + static_cast<uint32_t>(lane));
        patv = tl < wt.end ? a.pat[tl / a.nwin] : 0;
      }
      pidx = __builtin_amdgcn_readlane(patv, static_cast<int>(k & 63u));
    } else {
      pidx = pat[stripe];
    }
    const ConstPlanPtr pl = plans + pidx;
    const int nin = pl->nin;
    const int nout = pl->nout;
    const uint8_t* sb = a.base + stripe * a.stripe_stride + off;
    uint32_t rows[NINB][8];
#pragma unroll
    for (int r = 0; r < NINB; ++r)
      if (r < nin) load_row(sb + static_cast<uint64_t>(pl->loc[r]) * a.row_stride, lane, rows[r]);
    uint32_t acc[NOUT][8];
#pragma unroll
    for (int o = 0; o < NOUT; ++o)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
#pragma unroll
    for (int r = 0; r < NINB; ++r) {
      if (r < nin) accumulate_row<NOUT, NINB>(acc, rows[r], pl->cw[r]);
    }
    uint8_t* ob = a.out + stripe * a.out_stripe_stride + off;
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      if (o < nout) {
        bitslice(acc[o]);
        store_row(ob + static_cast<uint64_t>(o) * a.out_row_stride, lane, acc[o]);
      }
    }
  }
}

// Streaming form for plans beyond the register-resident shapes (> 16 inputs,
// or > 8 with 6-8 outputs; wide codes): the stripe's inputs are walked in
// groups of D rows over two register sets, the next group loading while the
// current one is sliced and accumulated (as bitsliced_stream_kernel), each
// group's locations and coefficient words read from the plan by scalar loads.
template <int NOUT, int D>
__device__ __forceinline__ void batch_load_group(const ConstPlanPtr pl, int r0, int nin, const uint8_t* sb,
                                                 uint64_t row_stride, int lane, uint32_t (&rows)[D][8]) {
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (r0 + j < nin) load_row(sb + static_cast<uint64_t>(pl->loc[r0 + j]) * row_stride, lane, rows[j]);
}

template <int NOUT, int D>
__device__ __forceinline__ void batch_acc_group(const ConstPlanPtr pl, int r0, int nin, uint32_t (&acc)[NOUT][8],
                                                uint32_t (&rows)[D][8]) {
  constexpr int kNinb = NOUT >= 4 ? 16 : 8;  // BitLoop: rolled bit loop from 4 outputs
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (r0 + j < nin) accumulate_row<NOUT, kNinb>(acc, rows[j], pl->cw[r0 + j]);
}

template <int NOUT, int D>
__global__ void __launch_bounds__(kBlockThreads) batch_stream_kernel(const BatchArgs a) {
  const int lane = threadIdx.x & 63;
  const ConstPlanPtr plans = (ConstPlanPtr)a.plans;
  int patv = 0;
  uint32_t k = 0;
  const WaveTasks wt = wave_tasks(a.ntasks, a.order);
  for (;; ++k) {
    const uint64_t t = wt.at(k);
    if (t >= wt.end) break;
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    if ((k & 63u) == 0) {  // pattern indices of the next 64 tasks, one vector load
      const uint64_t tl = wt.at(k + static_cast<uint32_t>(lane));
      patv = tl < wt.end ? a.pat[tl / a.nwin] : 0;
    }
    const ConstPlanPtr pl = plans + __builtin_amdgcn_readlane(patv, static_cast<int>(k & 63u));
    int nin = pl->nin;
    asm volatile("" : "+s"(nin));
    const int nout = pl->nout;
    const uint8_t* sb = a.base + stripe * a.stripe_stride + off;
    uint32_t acc[NOUT][8];
#pragma unroll
    for (int o = 0; o < NOUT; ++o)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
    uint32_t ra[D][8], rb[D][8];
    batch_load_group<NOUT, D>(pl, 0, nin, sb, a.row_stride, lane, ra);
#pragma unroll 1
    for (int r0 = 0; r0 < nin; r0 += 2 * D) {
      if (r0 + D < nin) batch_load_group<NOUT, D>(pl, r0 + D, nin, sb, a.row_stride, lane, rb);
      batch_acc_group<NOUT, D>(pl, r0, nin, acc, ra);
      if (r0 + D >= nin) break;
      if (r0 + 2 * D < nin) batch_load_group<NOUT, D>(pl, r0 + 2 * D, nin, sb, a.row_stride, lane, ra);
      batch_acc_group<NOUT, D>(pl, r0 + D, nin, acc, rb);
    }
    uint8_t* ob = a.out + stripe * a.out_stripe_stride + off;
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      if (o < nout) {
        bitslice(acc[o]);
        store_row(ob + static_cast<uint64_t>(o) * a.out_row_stride, lane, acc[o]);
      }
    }
  }
}

// Byte columns [col0, len) of every stripe (tails, unaligned batches).
__global__ void __launch_bounds__(kBlockThreads) batch_bytewise_kernel(const BatchArgs a) {
  __shared__ uint8_t s_exp[512];
  __shared__ uint8_t s_log[256];
  for (int i = threadIdx.x; i < 512; i += blockDim.x) s_exp[i] = d_tables.exp[i];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_log[i] = d_tables.log[i];
  __syncthreads();
  const uint64_t ncol = a.len - a.col0;
  const uint64_t nthreads = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t idx = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; idx < a.ntasks;
       idx += nthreads) {
    const uint64_t stripe = idx / ncol;
    const uint64_t col = a.col0 + (idx - stripe * ncol);
    const BatchPlan& pl = a.plans[a.pat[stripe]];
    const uint8_t* sb = a.base + stripe * a.stripe_stride + col;
    uint8_t acc[kMaxOut] = {};
    for (int r = 0; r < pl.nin; ++r) {
      const uint8_t x = sb[static_cast<uint64_t>(pl.loc[r]) * a.row_stride];
      if (x == 0) continue;
      const int lx = s_log[x];
      const uint64_t w = pl.cw[r];
#pragma unroll
      for (int o = 0; o < kMaxOut; ++o) {
        const uint8_t c = static_cast<uint8_t>(w >> (8 * o));
        if (c != 0) acc[o] ^= s_exp[lx + s_log[c]];
      }
    }
    uint8_t* ob = a.out + stripe * a.out_stripe_stride + col;
    for (int o = 0; o < pl.nout; ++o) ob[static_cast<uint64_t>(o) * a.out_row_stride] = acc[o];
  }
}

// Batch kernel reads the pattern indices of its next 64 tasks with one
// vector load (PATV) instead of a dependent scalar load per task;
// HRS_BATCH_PATV=0 selects the per-task scalar read for A/B runs. (A
// software-pipelined batch kernel like bitsliced_pipe_kernel measured 3-4%
// slower, profiles/r01/pipe/batch_ab, and is not kept.)
bool use_pat_prefetch() {
  static bool v = [] {
    const char* e = getenv("HRS_BATCH_PATV");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <int NOUT, int NINB>
hipError_t launch_batch_n(const BatchArgs& a, hipStream_t s) {
  auto kern = use_pat_prefetch() ? batch_bitsliced_kernel<NOUT, NINB, true> : batch_bitsliced_kernel<NOUT, NINB, false>;
  note_kernel_t("batch_bitsliced_kernel", NOUT, NINB, use_pat_prefetch());
  const int per_cu = BitLoop<NOUT, NINB>::kRolled ? 3 : 2;
  hipLaunchKernelGGL(kern, dim3(stream_grid(a.ntasks, per_cu)), dim3(kBlockThreads), 0, s, with_order(a, kOrderBatch));
  return hipGetLastError();
}

template <int NOUT>
hipError_t launch_batch_stream_n(const BatchArgs& a, hipStream_t s) {
  auto kern = batch_stream_kernel<NOUT, 4>;
  note_kernel_t("batch_stream_kernel", NOUT, 4);
  const int per_cu = NOUT >= 4 ? 3 : 2;
  hipLaunchKernelGGL(kern, dim3(stream_grid(a.ntasks, per_cu)), dim3(kBlockThreads), 0, s, with_order(a, kOrderBatch));
  return hipGetLastError();
}

template <int NOUT>
hipError_t launch_batch_nout(const BatchArgs& a, int max_nin, hipStream_t s) {
  if (max_nin > kBatchMaxIn) return hipErrorInvalidValue;
  if (max_nin > 16 || (NOUT > 5 && max_nin > 8)) return launch_batch_stream_n<NOUT>(a, s);
  if (max_nin <= 4) return launch_batch_n<NOUT, 4>(a, s);
  if (max_nin <= 8) return launch_batch_n<NOUT, 8>(a, s);
  if constexpr (NOUT < 6) {
    if (max_nin <= 12) return launch_batch_n<NOUT, 12>(a, s);
    return launch_batch_n<NOUT, 16>(a, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_batch_bitsliced(const BatchArgs& a, int max_nout, int max_nin, hipStream_t s) {
  switch (max_nout) {
    case 1: return launch_batch_nout<1>(a, max_nin, s);
    case 2: return launch_batch_nout<2>(a, max_nin, s);
    case 3: return launch_batch_nout<3>(a, max_nin, s);
    case 4: return launch_batch_nout<4>(a, max_nin, s);
    case 5: return launch_batch_nout<5>(a, max_nin, s);
    case 6: return launch_batch_nout<6>(a, max_nin, s);
    case 7: return launch_batch_nout<7>(a, max_nin, s);
    case 8: return launch_batch_nout<8>(a, max_nin, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_batch_bytewise(const BatchArgs& a, hipStream_t s) {
  const unsigned g = grid_for(batch_bytewise_kernel, kBlockThreads, a.ntasks);
  note_kernel("batch_bytewise_kernel");
  hipLaunchKernelGGL(batch_bytewise_kernel, dim3(g), dim3(kBlockThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace hrs
