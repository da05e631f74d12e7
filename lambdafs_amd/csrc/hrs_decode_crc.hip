// gfx950 fused repair + CRC-32: the repaired cells of every stripe and the
// java.util.zip.CRC32 of each of them in ONE pass — what the Decoder does per
// lost block (decodeBulk, then the repaired block's CRC32 compared with the
// checksum the NameNode holds; Decoder.java:222-229, :645-655). Run as two
// passes (decode, then hrs_crc32_dev over the outputs) every repaired cell is
// written, then read back; fused, the CRC consumes the output words while they
// are still in registers.
//
// The decode half is bitsliced_pipe_kernel's (hrs_runtime.hip): one wave per
// (stripe, 2 KiB window), the next window's survivor rows loaded before the
// current window is sliced and multiplied. After a window's outputs are
// un-sliced and stored, lane l holds the 16-byte pieces at 16 l and
// 1024 + 16 l of each output: their raw CRCs (slicing-by-4), joined with
// Z_1024 and the Z_{16*2^t} lane tree, are the window's raw CRC, which lane 0
// writes to raw[stripe][output][window]; crc_fold_kernel then folds the
// windows of each (stripe, output) with Z_2048 and applies CRC32.update's
// chaining, exactly as it finishes the fused encode's windows.
//
// LDS: the window kernels' 156 KiB image (32 bank-private copies of the
// slicing tables, Z_1024, the lane tree). It admits one block per CU, so the
// block is 512 threads: the same 8 waves per CU (2 per SIMD) the plain repair
// kernel runs as two 256-thread blocks.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "hrs_device.hpp"
#include "hrs_launch.hpp"

namespace hrs {
namespace {

constexpr int kDecCrcThreads = 512;

template <int NOUT, int NINB>
__device__ __forceinline__ void dc_load_task(const RowArgs& a, uint64_t t, int nin, int lane,
                                             uint32_t (&rows)[NINB][8]) {
  const uint64_t stripe = t / a.nwin;
  const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
  const uint64_t in_base = stripe * a.in_stride + off;
#pragma unroll
  for (int r = 0; r < NINB; ++r)
    if (r < nin) load_row(a.in[r] + in_base, lane, rows[r]);
}

// The repair of task t: slice, multiply, un-slice and store its outputs;
// res receives the stored words for dc_crc_task. The accumulators are local
// and copied out at the end: accumulated in place through the reference, the
// 2- and 4-output forms compiled to thousands of v_mov_b64 shuffling them
// between register pairs at every coefficient branch (NOTES.md, decode_crc/).
template <int NOUT, int NINB>
__device__ __forceinline__ void dc_apply_task(const RowArgs& a, uint64_t t, int nin, int lane,
                                              uint32_t (&rows)[NINB][8], uint32_t (&res)[NOUT][8]) {
  const uint64_t stripe = t / a.nwin;
  const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
  uint32_t acc[NOUT][8];
#pragma unroll
  for (int o = 0; o < NOUT; ++o)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
#pragma unroll
  for (int r = 0; r < NINB; ++r) {
    if (r < nin) accumulate_row<NOUT, NINB>(acc, rows[r], a.cw[r]);  // acc[o] ^= coef[o][r] * row
  }
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    bitslice(acc[o]);
    store_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
#pragma unroll
    for (int q = 0; q < 8; ++q) res[o][q] = acc[o][q];
  }
}

// The raw CRC of task t's output windows: the lane's two pieces (slicing-by-4
// chains), joined with Z_1024, then the 6-level lane tree; lane 0 writes it.
// A chain of dependent LDS lookups and cross-lane shuffles (~1,500 cycles),
// so the kernel issues the NEXT task's loads before it (they would otherwise
// wait behind it and the wave would keep one window in flight instead of two).
template <int NOUT, bool DPP>
__device__ __forceinline__ void dc_crc_task(const DecodeCrcArgs& d, uint64_t t, int lane, const SliceTab& slices,
                                            const uint32_t* zchunk, const uint32_t* tree,
                                            const uint32_t (&acc)[NOUT][8]) {
  const uint64_t stripe = t / d.r.nwin;
  const uint64_t w = t - stripe * d.r.nwin;
  uint32_t c0[NOUT], c1[NOUT];
  rows_piece_crcs<NOUT>(slices, acc, c0, c1);
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    const uint32_t x = zmul_xor(zchunk, c0[o], c1[o]);
    const uint32_t c = DPP ? lane_tree_dpp(tree, x) : lane_tree(tree, x);
    if (lane == 0) d.raw[(stripe * NOUT + o) * d.r.nwin + w] = c;
  }
}

template <int NOUT, int NINB, bool DPP>
__global__ void __launch_bounds__(kDecCrcThreads) decode_crc_pipe_kernel(const DecodeCrcArgs d) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < kCrcLdsWordsA; i += kDecCrcThreads) lds[i] = d.tables[i];
  __syncthreads();
  const RowArgs& a = d.r;
  const int lane = threadIdx.x & 63;
  const SliceTab slices = slice_tab(lane);
  const uint32_t* zchunk = lds + kCrcSliceWords;
  const uint32_t* tree = zchunk + 1024;
  int nin = a.nin;
  asm volatile("" : "+s"(nin));
  const WaveTasks wt = wave_tasks(a.ntasks, a.order);
  uint32_t j = 0;
  uint64_t t = wt.at(0);
  if (t >= wt.end) return;
  uint32_t ra[NINB][8], rb[NINB][8];
  uint32_t acc[NOUT][8];
  dc_load_task<NOUT, NINB>(a, t, nin, lane, ra);
  uint64_t t1 = wt.at(++j);
  if (t1 < wt.end) dc_load_task<NOUT, NINB>(a, t1, nin, lane, rb);
  for (;;) {  // ra: task t, rb: task t1 in flight; every wave leaves once a task index passes its end
    dc_apply_task<NOUT, NINB>(a, t, nin, lane, ra, acc);
    const uint64_t t2 = wt.at(++j);
    if (t2 < wt.end) dc_load_task<NOUT, NINB>(a, t2, nin, lane, ra);
    dc_crc_task<NOUT, DPP>(d, t, lane, slices, zchunk, tree, acc);
    if (t1 >= wt.end) break;
    dc_apply_task<NOUT, NINB>(a, t1, nin, lane, rb, acc);
    const uint64_t t3 = wt.at(++j);
    if (t3 < wt.end) dc_load_task<NOUT, NINB>(a, t3, nin, lane, rb);
    dc_crc_task<NOUT, DPP>(d, t1, lane, slices, zchunk, tree, acc);
    if (t2 >= wt.end) break;
    t = t2;
    t1 = t3;
  }
}

// HRS_DCRC_TREE=0 (A/B runs): the lane tree's in-row levels by ds_bpermute
// (lane_tree) instead of DPP moves (lane_tree_dpp).
bool dcrc_dpp() {
  static const bool v = [] {
    const char* e = getenv("HRS_DCRC_TREE");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Plain (not pipelined) form for 2-4 outputs: the pipelined kernel's two row
// sets + outputs + CRC state exceed the register file there (<2,12>: 253
// VGPRs and 51 SGPRs spilled, 1.6x the plain repair; profiles/r03/ab/NOTES.md, decode_crc/).
// One row set; the other waves of the SIMD cover the CRC tail. THREADS = 768
// (3 waves/SIMD, <= 153 VGPRs) or 512 (2).
template <int NOUT, int NINB, int THREADS>
__global__ void __launch_bounds__(THREADS) decode_crc_kernel(const DecodeCrcArgs d) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < kCrcLdsWordsA; i += THREADS) lds[i] = d.tables[i];
  __syncthreads();
  const RowArgs& a = d.r;
  const int lane = threadIdx.x & 63;
  const SliceTab slices = slice_tab(lane);
  const uint32_t* zchunk = lds + kCrcSliceWords;
  const uint32_t* tree = zchunk + 1024;
  const WaveTasks wt = wave_tasks(a.ntasks, a.order);
  for (uint32_t j = 0; j < 0xFFFFFFFFu; ++j) {
    const uint64_t t = wt.at(j);
    if (t >= wt.end) break;
    int nin = a.nin;  // opaque per task: the r < nin predicates are not hoisted (they would spill)
    asm volatile("" : "+s"(nin));
    // written out, not through dc_load_task / dc_apply_task: with the helpers
    // the 2- and 4-output forms compile to thousands of v_mov_b64 shuffling the
    // accumulators between registers at every coefficient branch
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    const uint64_t in_base = stripe * a.in_stride + off;
    uint32_t rows[NINB][8];
#pragma unroll
    for (int r = 0; r < NINB; ++r)
      if (r < nin) load_row(a.in[r] + in_base, lane, rows[r]);
    uint32_t acc[NOUT][8];
#pragma unroll
    for (int o = 0; o < NOUT; ++o)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
#pragma unroll
    for (int r = 0; r < NINB; ++r)
      if (r < nin) accumulate_row<NOUT, NINB>(acc, rows[r], a.cw[r]);
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      bitslice(acc[o]);
      store_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
    }
    dc_crc_task<NOUT, true>(d, t, lane, slices, zchunk, tree, acc);
  }
}

// 768 threads (3 waves/SIMD) measured 3-10% faster than 512 for the 2- and
// 3-output repairs (profiles/r03/ab/decode_crc/v7_plain_inline_512_vs_768.jsonl); HRS_DCRC_THREADS=512
// for A/B runs.
int dcrc_threads() {
  static const int v = [] {
    const char* e = getenv("HRS_DCRC_THREADS");
    return (e && atoi(e) == 512) ? 512 : 768;
  }();
  return v;
}

template <int NOUT, int NINB>
hipError_t launch_dc(const DecodeCrcArgs& d, int cus, hipStream_t s) {
  DecodeCrcArgs dc = d;
  dc.r.order = task_order(kOrderDecodeCrc);
  if constexpr (NOUT >= 2) {
    const int threads = dcrc_threads();
    auto kern = threads == 768 ? decode_crc_kernel<NOUT, NINB, 768> : decode_crc_kernel<NOUT, NINB, 512>;
    const size_t shm = static_cast<size_t>(kCrcLdsWordsA) * 4;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(shm));
    if (e != hipSuccess) return e;
    note_kernel_t("decode_crc_kernel", NOUT, NINB, threads);
    const uint64_t per_block = threads / 64;
    uint64_t g = (d.r.ntasks + per_block - 1) / per_block;
    if (g > static_cast<uint64_t>(cus)) g = cus;
    g = capped_grid(g);  // zero-copy calls cap it (hrs::GridCap)
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(g)), dim3(threads), shm, s, dc);
    return hipGetLastError();
  } else {
    auto kern = dcrc_dpp() ? decode_crc_pipe_kernel<NOUT, NINB, true> : decode_crc_pipe_kernel<NOUT, NINB, false>;
    const size_t shm = static_cast<size_t>(kCrcLdsWordsA) * 4;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       static_cast<int>(shm));
    if (e != hipSuccess) return e;
    note_kernel_t("decode_crc_pipe_kernel", NOUT, NINB, dcrc_dpp());
    constexpr uint64_t per_block = kDecCrcThreads / 64;
    uint64_t g = (d.r.ntasks + per_block - 1) / per_block;
    if (g > static_cast<uint64_t>(cus)) g = cus;
    g = capped_grid(g);  // zero-copy calls cap it (hrs::GridCap)
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(g)), dim3(kDecCrcThreads), shm, s, dc);
    return hipGetLastError();
  }
}

template <int NOUT>
hipError_t launch_dc_n(const DecodeCrcArgs& d, int cus, hipStream_t s, bool* handled) {
  if (d.r.nin <= 4) return launch_dc<NOUT, 4>(d, cus, s);
  if (d.r.nin <= 8) return launch_dc<NOUT, 8>(d, cus, s);
  if constexpr (NOUT <= 3) {
    if (d.r.nin <= 12) return launch_dc<NOUT, 12>(d, cus, s);
  }
  *handled = false;
  return hipSuccess;
}

}  // namespace

hipError_t launch_decode_crc(const DecodeCrcArgs& d, int cus, hipStream_t s, bool* handled) {
  *handled = true;
  if (d.r.nin >= 1 && !d.r.accumulate) {
    switch (d.r.nout) {
      case 1: return launch_dc_n<1>(d, cus, s, handled);
      case 2: return launch_dc_n<2>(d, cus, s, handled);
      case 3: return launch_dc_n<3>(d, cus, s, handled);
      case 4: return launch_dc_n<4>(d, cus, s, handled);
      default: break;
    }
  }
  *handled = false;
  return hipSuccess;
}

}  // namespace hrs
