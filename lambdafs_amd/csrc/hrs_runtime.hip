// gfx950 runtime-matrix kernels: decode (and the encode of codes without a
// compile-time kernel) as out = M * in with the coefficients of M in the
// kernel arguments — bit-sliced rows, planes multiplied by alpha and
// accumulated under wave-uniform branches (see hrs_kernels.hip's header for
// the arithmetic; bitslice / xtime / accumulate_row in hrs_device.hpp).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "hrs_device.hpp"
#include "hrs_launch.hpp"

namespace hrs {
namespace {

template <int NOUT, int NINB>
__global__ void __launch_bounds__(kBlockThreads) bitsliced_kernel(const RowArgs a) {
  const int lane = threadIdx.x & 63;
  const WaveTasks wt = wave_tasks(a.ntasks, a.order);
  for (uint32_t j = 0; j < 0xFFFFFFFFu; ++j) {
    const uint64_t t = wt.at(j);
    if (t >= wt.end) break;
    int nin = a.nin;  // opaque per task: the r < nin predicates are not hoisted (they would spill)
    asm volatile("" : "+s"(nin));
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    const uint64_t in_base = stripe * a.in_stride + off;
    uint32_t rows[NINB][8];
#pragma unroll
    for (int r = 0; r < NINB; ++r)
      if (r < nin) load_row(a.in[r] + in_base, lane, rows[r]);
    uint32_t acc[NOUT][8];
    if (a.accumulate) {
#pragma unroll
      for (int o = 0; o < NOUT; ++o) {
        load_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
        bitslice(acc[o]);
      }
    } else {
#pragma unroll
      for (int o = 0; o < NOUT; ++o)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
    }
#pragma unroll
    for (int r = 0; r < NINB; ++r) {
      if (r < nin) accumulate_row<NOUT, NINB>(acc, rows[r], a.cw[r]);  // acc[o] ^= coef[o][r] * row
    }
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      bitslice(acc[o]);
      store_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
    }
  }
}

// Software-pipelined form of bitsliced_kernel for narrow outputs: two
// register sets of NINB rows, the next task's rows are loaded before the
// current task's math, so a wave keeps a window in flight while it computes
// (the plain kernel's loads sit idle during its ~1,000 VALU of slicing and
// multiplying). 2*NINB*8 + 8*NOUT VGPRs: NOUT <= 2, NINB <= 12 at 2 waves/SIMD.
template <int NOUT, int NINB>
__device__ __forceinline__ void load_task(const RowArgs& a, uint64_t t, int nin, int lane,
                                          uint32_t (&rows)[NINB][8]) {
  const uint64_t stripe = t / a.nwin;
  const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
  const uint64_t in_base = stripe * a.in_stride + off;
#pragma unroll
  for (int r = 0; r < NINB; ++r)
    if (r < nin) load_row(a.in[r] + in_base, lane, rows[r]);
}

template <int NOUT, int NINB>
__device__ __forceinline__ void apply_task(const RowArgs& a, uint64_t t, int nin, int lane,
                                           uint32_t (&rows)[NINB][8]) {
  const uint64_t stripe = t / a.nwin;
  const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
  uint32_t acc[NOUT][8];
  if (a.accumulate) {
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      load_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
      bitslice(acc[o]);
    }
  } else {
#pragma unroll
    for (int o = 0; o < NOUT; ++o)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
  }
#pragma unroll
  for (int r = 0; r < NINB; ++r) {
    if (r < nin) accumulate_row<NOUT, NINB>(acc, rows[r], a.cw[r]);
  }
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    bitslice(acc[o]);
    store_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
  }
}

template <int NOUT, int NINB>
__global__ void __launch_bounds__(kBlockThreads) bitsliced_pipe_kernel(const RowArgs a) {
  static_assert(!BitLoop<NOUT, NINB>::kRolled, "pipelined kernel takes the unrolled shapes only");
  const int lane = threadIdx.x & 63;
  int nin = a.nin;
  asm volatile("" : "+s"(nin));
  const WaveTasks wt = wave_tasks(a.ntasks, a.order);
  uint32_t j = 0;
  uint64_t t = wt.at(0);
  if (t >= wt.end) return;
  uint32_t ra[NINB][8], rb[NINB][8];
  load_task<NOUT, NINB>(a, t, nin, lane, ra);
  for (;;) {  // every wave leaves once its next task index passes its end
    const uint64_t t1 = wt.at(++j);
    if (t1 < wt.end) load_task<NOUT, NINB>(a, t1, nin, lane, rb);
    apply_task<NOUT, NINB>(a, t, nin, lane, ra);
    if (t1 >= wt.end) break;
    const uint64_t t2 = wt.at(++j);
    if (t2 < wt.end) load_task<NOUT, NINB>(a, t2, nin, lane, ra);
    apply_task<NOUT, NINB>(a, t1, nin, lane, rb);
    if (t2 >= wt.end) break;
    t = t2;
  }
}

// Streaming form for shapes the kernels above take in several launches (more
// inputs than they hold in registers: > 16 inputs, or > 8 with 6-8 outputs),
// whose later launches re-read and re-write every output (RS(20,8) encode moved
// 60 rows of HBM traffic per stripe instead of 28). Here a wave walks the
// window's inputs in groups of D rows with two register sets: group g + 1 is
// loaded while group g is bit-sliced and accumulated, so each input row is
// read once and each output written once for up to kMaxIn (32) inputs, and
// the wave still keeps D rows in flight. The coefficient words and row
// pointers of group g come from the kernel arguments by a wave-uniform index
// (scalar loads).
template <int NOUT, int D>
__device__ __forceinline__ void load_group(const RowArgs& a, int r0, int nin, uint64_t in_base, int lane,
                                           uint32_t (&rows)[D][8]) {
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (r0 + j < nin) load_row(a.in[r0 + j] + in_base, lane, rows[j]);
}

template <int NOUT, int D>
__device__ __forceinline__ void acc_group(const RowArgs& a, int r0, int nin, uint32_t (&acc)[NOUT][8],
                                          uint32_t (&rows)[D][8]) {
  constexpr int kNinb = NOUT >= 4 ? 16 : 8;  // BitLoop: rolled bit loop from 4 outputs
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (r0 + j < nin) accumulate_row<NOUT, kNinb>(acc, rows[j], a.cw[r0 + j]);
}

template <int NOUT, int D>
__global__ void __launch_bounds__(kBlockThreads) bitsliced_stream_kernel(const RowArgs a) {
  const int lane = threadIdx.x & 63;
  const WaveTasks wt = wave_tasks(a.ntasks, a.order);
  for (uint32_t j = 0; j < 0xFFFFFFFFu; ++j) {
    const uint64_t t = wt.at(j);
    if (t >= wt.end) break;
    int nin = a.nin;
    asm volatile("" : "+s"(nin));
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    const uint64_t in_base = stripe * a.in_stride + off;
    uint32_t acc[NOUT][8];
    if (a.accumulate) {
#pragma unroll
      for (int o = 0; o < NOUT; ++o) {
        load_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
        bitslice(acc[o]);
      }
    } else {
#pragma unroll
      for (int o = 0; o < NOUT; ++o)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
    }
    uint32_t ra[D][8], rb[D][8];
    load_group<NOUT, D>(a, 0, nin, in_base, lane, ra);
#pragma unroll 1
    for (int r0 = 0; r0 < nin; r0 += 2 * D) {
      if (r0 + D < nin) load_group<NOUT, D>(a, r0 + D, nin, in_base, lane, rb);
      acc_group<NOUT, D>(a, r0, nin, acc, ra);
      if (r0 + D >= nin) break;
      if (r0 + 2 * D < nin) load_group<NOUT, D>(a, r0 + 2 * D, nin, in_base, lane, ra);
      acc_group<NOUT, D>(a, r0 + D, nin, acc, rb);
    }
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      bitslice(acc[o]);
      store_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
    }
  }
}

// Rows per streamed group: 4 (8 rows of loads in flight per wave).
constexpr int kStreamGroup = 4;

// Software-pipelined runtime kernel for the unrolled shapes that fit (the 1-
// to 3-erasure repairs: RS(10,4) 1-erasure decode +3-10%, 2-3 erasures
// neutral); HRS_PIPE=0 selects the plain kernel for A/B runs. The same
// pipelining of the static encode (-1%) and of the heterogeneous batch
// kernel (-2%) measured slower and is not used (profiles/r01/pipe/ab2).
// Unrolled shapes whose two row sets + accumulators fit 2 waves/SIMD.
template <int NOUT, int NINB>
constexpr bool kPipeFits = !BitLoop<NOUT, NINB>::kRolled && 16 * NINB + 8 * NOUT <= 232;

bool use_pipe() {
  static bool v = [] {
    const char* e = getenv("HRS_PIPE");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <int NOUT, int NINB>
hipError_t launch_bits_n(const RowArgs& a, hipStream_t s) {
  auto kern = bitsliced_kernel<NOUT, NINB>;
  const char* name = "bitsliced_kernel";
  if constexpr (kPipeFits<NOUT, NINB>)
    if (use_pipe()) {
      kern = bitsliced_pipe_kernel<NOUT, NINB>;
      name = "bitsliced_pipe_kernel";
    }
  note_kernel_t(name, NOUT, NINB);
  const int per_cu = BitLoop<NOUT, NINB>::kRolled ? 3 : 2;
  hipLaunchKernelGGL(kern, dim3(stream_grid(a.ntasks, per_cu)), dim3(kBlockThreads), 0, s, with_order(a, kOrderRuntime));
  return hipGetLastError();
}

template <int NOUT>
hipError_t launch_bits(const RowArgs& a, hipStream_t s) {
  if (a.nin <= 4) return launch_bits_n<NOUT, 4>(a, s);
  if (a.nin <= 8) return launch_bits_n<NOUT, 8>(a, s);
  if constexpr (NOUT < 6) {  // wider outputs would spill: the host chunks them by 8 inputs
    if (a.nin <= 12) return launch_bits_n<NOUT, 12>(a, s);
    if (a.nin <= 16) return launch_bits_n<NOUT, 16>(a, s);
  }
  return hipErrorInvalidValue;
}

template <int NOUT>
hipError_t launch_stream_n(const RowArgs& a, hipStream_t s) {
  auto kern = bitsliced_stream_kernel<NOUT, kStreamGroup>;
  note_kernel_t("bitsliced_stream_kernel", NOUT, kStreamGroup);
  const int per_cu = NOUT >= 4 ? 3 : 2;
  hipLaunchKernelGGL(kern, dim3(stream_grid(a.ntasks, per_cu)), dim3(kBlockThreads), 0, s, with_order(a, kOrderRuntime));
  return hipGetLastError();
}

}  // namespace

hipError_t launch_bitsliced_stream(const RowArgs& a, hipStream_t s) {
  if (a.nin < 1 || a.nin > kMaxIn) return hipErrorInvalidValue;
  switch (a.nout) {
    case 1: return launch_stream_n<1>(a, s);
    case 2: return launch_stream_n<2>(a, s);
    case 3: return launch_stream_n<3>(a, s);
    case 4: return launch_stream_n<4>(a, s);
    case 5: return launch_stream_n<5>(a, s);
    case 6: return launch_stream_n<6>(a, s);
    case 7: return launch_stream_n<7>(a, s);
    case 8: return launch_stream_n<8>(a, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_bitsliced(const RowArgs& a, hipStream_t s) {
  switch (a.nout) {
    case 1: return launch_bits<1>(a, s);
    case 2: return launch_bits<2>(a, s);
    case 3: return launch_bits<3>(a, s);
    case 4: return launch_bits<4>(a, s);
    case 5: return launch_bits<5>(a, s);
    case 6: return launch_bits<6>(a, s);
    case 7: return launch_bits<7>(a, s);
    case 8: return launch_bits<8>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace hrs
