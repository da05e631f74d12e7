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

template <int NOUT, int NINB>
__device__ __forceinline__ void dc_apply_task(const DecodeCrcArgs& d, uint64_t t, int nin, int lane,
                                              const SliceTab& slices, const uint32_t* zchunk, const uint32_t* tree,
                                              uint32_t (&rows)[NINB][8]) {
  const RowArgs& a = d.r;
  const uint64_t stripe = t / a.nwin;
  const uint64_t w = t - stripe * a.nwin;
  const uint64_t off = w * kWindowBytes;
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
  }
  uint32_t c0[NOUT], c1[NOUT];
  rows_piece_crcs<NOUT>(slices, acc, c0, c1);
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    const uint32_t c = lane_tree(tree, zmul_xor(zchunk, c0[o], c1[o]));
    if (lane == 0) d.raw[(stripe * NOUT + o) * a.nwin + w] = c;
  }
}

template <int NOUT, int NINB>
__global__ void __launch_bounds__(kDecCrcThreads) decode_crc_pipe_kernel(const DecodeCrcArgs d) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < kCrcLdsWordsA; i += kDecCrcThreads) lds[i] = d.tables[i];
  __syncthreads();
  const RowArgs& a = d.r;
  const int lane = threadIdx.x & 63;
  const SliceTab slices = slice_tab(lane);
  const uint32_t* zchunk = lds + kCrcSliceWords;
  const uint32_t* tree = zchunk + 1024;
  const uint32_t nwaves = gridDim.x * (kDecCrcThreads / 64);
  int nin = a.nin;
  asm volatile("" : "+s"(nin));
  uint64_t t = wave_id_in_grid();
  if (t >= a.ntasks) return;
  uint32_t ra[NINB][8], rb[NINB][8];
  dc_load_task<NOUT, NINB>(a, t, nin, lane, ra);
  for (;;) {  // every wave leaves once its next task index passes ntasks
    const uint64_t t1 = t + nwaves;
    if (t1 < a.ntasks) dc_load_task<NOUT, NINB>(a, t1, nin, lane, rb);
    dc_apply_task<NOUT, NINB>(d, t, nin, lane, slices, zchunk, tree, ra);
    if (t1 >= a.ntasks) break;
    const uint64_t t2 = t1 + nwaves;
    if (t2 < a.ntasks) dc_load_task<NOUT, NINB>(a, t2, nin, lane, ra);
    dc_apply_task<NOUT, NINB>(d, t1, nin, lane, slices, zchunk, tree, rb);
    if (t2 >= a.ntasks) break;
    t = t2;
  }
}

template <int NOUT, int NINB>
hipError_t launch_dc(const DecodeCrcArgs& d, int cus, hipStream_t s) {
  auto kern = decode_crc_pipe_kernel<NOUT, NINB>;
  const size_t shm = static_cast<size_t>(kCrcLdsWordsA) * 4;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     static_cast<int>(shm));
  if (e != hipSuccess) return e;
  note_kernel_t("decode_crc_pipe_kernel", NOUT, NINB);
  constexpr uint64_t per_block = kDecCrcThreads / 64;
  uint64_t g = (d.r.ntasks + per_block - 1) / per_block;
  if (g > static_cast<uint64_t>(cus)) g = cus;
  if (g == 0) g = 1;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(g)), dim3(kDecCrcThreads), shm, s, d);
  return hipGetLastError();
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
