// gfx950 CRC-32 (java.util.zip.CRC32 / zlib) of device-resident cells, for the
// block checksums the hops drivers keep (Encoder.java:408-450,
// Decoder.java:222-229, :645-655). Two launches:
//
//  A. crc_window_kernel: one wave per 32 KiB window of one row of one stripe.
//     The window is 32 chunks of 1 KiB; lane l owns the 16-byte piece at
//     q * 1024 + 16 l of every chunk q, so each load instruction is one
//     contiguous 1 KiB wave access (a lane-contiguous layout capped the loads
//     at 3.8 TB/s, tools/crc_lab.hip). Each piece is 4 slicing-by-4 steps;
//     the lane joins its pieces in chunk order with Z_1024 (8 chunks in flight
//     at a time), and a 6-level lane tree joins the lanes with Z_{16*2^t}
//     (crc32.hpp). The slicing tables are replicated 32x in LDS so lane l
//     reads copy l % 32: ds_read_b32 banks are (address/4) mod 32 per 32-lane
//     group, so every data lookup is conflict-free (random byte indices into
//     one copy cost ~4-way conflicts: 3.5 -> 6.0 TB/s in the lab). The 156 KiB
//     image is shared by one 1024-thread block per CU. The row tail
//     (len mod 32 KiB) is a right-aligned window whose leading bytes are zero
//     (leading zeros do not change a raw CRC).
//  B. crc_fold_kernel: one wave per (stripe, row) folds its window CRCs
//     (G per lane with Z_window, then a lane tree with Z_{window*G*2^t}),
//     appends the tail window, and applies CRC32.update's affine chaining from
//     the running value crc_in.
// Both are HBM-read streams; algorithmic bytes = the rows' bytes, once.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "hrs_device.hpp"
#include "hrs_launch.hpp"

namespace hrs {
namespace {

// zmul / slice4 / lane_tree: hrs_device.hpp

template <bool ALIGNED>
__global__ void __launch_bounds__(kCrcBlockThreads) crc_window_kernel(const CrcWinArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < kCrcLdsWordsA; i += blockDim.x) lds[i] = a.tables[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const SliceTab slices = slice_tab(lane);
  const uint32_t* zchunk = lds + kCrcSliceWords;
  const uint32_t* tree = zchunk + 1024;
  const uint64_t wpr = a.nwin + (a.tail ? 1 : 0);
  const uint64_t ntasks = a.nstripes * a.nrows * wpr;
  const WaveTasks wt = wave_tasks(ntasks, a.order);
  for (uint32_t j = 0; j < 0xFFFFFFFFu; ++j) {
    const uint64_t t = wt.at(j);
    if (t >= wt.end) break;
    const uint64_t sr = t / wpr;
    const uint64_t w = t - sr * wpr;
    const uint64_t stripe = sr / a.nrows;
    const int row = static_cast<int>(sr - stripe * a.nrows);
    const uint8_t* base = a.rows[row] + stripe * a.stride[row];
    // the window covers [end - kCrcWindow, end); bytes below lo read as zero
    const bool full = w < a.nwin;
    const int64_t end = full ? static_cast<int64_t>((w + 1) * kCrcWindow) : static_cast<int64_t>(a.len);
    const int64_t lo = full ? static_cast<int64_t>(w * kCrcWindow) : static_cast<int64_t>(a.nwin * kCrcWindow);
    const int64_t start = end - kCrcWindow + lane * crc::kPieceBytes;
    uint32_t c = 0;
#pragma unroll 1
    for (int g = 0; g < crc::kPieces; g += kCrcGroup) {
      uint32_t words[kCrcGroup][4];
#pragma unroll
      for (int q = 0; q < kCrcGroup; ++q) {
        const int64_t pos0 = start + static_cast<int64_t>(g + q) * crc::kChunkBytes;
        if (ALIGNED && full) {
          const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + pos0));
          words[q][0] = v[0];
          words[q][1] = v[1];
          words[q][2] = v[2];
          words[q][3] = v[3];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint32_t x = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const int64_t pos = pos0 + 4 * j + b;
              if (pos >= lo) x |= static_cast<uint32_t>(base[pos]) << (8 * b);
            }
            words[q][j] = x;
          }
        }
      }
      uint32_t ch[kCrcGroup];
#pragma unroll
      for (int q = 0; q < kCrcGroup; ++q) ch[q] = 0u;
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int q = 0; q < kCrcGroup; ++q) ch[q] = slice4(slices, ch[q] ^ words[q][st]);
#pragma unroll
      for (int q = 0; q < kCrcGroup; ++q) c = (g + q == 0) ? ch[q] : (zmul(zchunk, c) ^ ch[q]);
    }
    c = lane_tree(tree, c);
    if (lane == 0) a.raw[(stripe * a.nrows_total + a.row0 + row) * wpr + w] = c;
  }
}

__global__ void __launch_bounds__(256) crc_fold_kernel(const CrcFoldArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < kCrcLdsWordsB; i += blockDim.x) lds[i] = a.tables[i];
  __syncthreads();
  const uint32_t* zw = lds;                    // Z_window
  const uint32_t* ztree = lds + 1024;          // Z_{window*G*2^t}, t = 0..5
  const uint32_t* ztail = lds + 7 * 1024;      // Z_tail
  const uint32_t* zlen = lds + 8 * 1024;       // Z_len
  const int lane = threadIdx.x & 63;
  const uint64_t wpr = a.nwin + (a.tail ? 1 : 0);
  const uint64_t pad = static_cast<uint64_t>(a.G) * 64 - a.nwin;
  const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
  for (uint64_t sr = wave_id_in_grid(); sr < a.nsr; sr += nwaves) {
    const uint32_t* raw = a.raw + sr * wpr;
    uint32_t c = 0;
    for (int g = 0; g < a.G; ++g) {
      const int64_t w = static_cast<int64_t>(lane) * a.G + g - static_cast<int64_t>(pad);
      if (w >= 0) c = zmul(zw, c) ^ raw[w];
    }
    c = lane_tree(ztree, c);
    if (lane == 0) {
      if (a.tail) c = zmul(ztail, c) ^ raw[a.nwin];
      const uint32_t state = (a.crc_in ? a.crc_in[sr] : 0u) ^ 0xFFFFFFFFu;
      a.crc_out[sr] = zmul(zlen, state) ^ c ^ 0xFFFFFFFFu;
    }
  }
}

unsigned fold_grid(uint64_t waves, int cus) {
  static const int per_cu = [] {
    const char* e = getenv("HRS_CRC_BLOCKS_PER_CU");
    const int x = e ? atoi(e) : 0;
    return (x >= 1 && x <= 16) ? x : kCrcFoldBlocksPerCU;
  }();
  uint64_t blocks = (waves + 3) / 4;
  const uint64_t cap = static_cast<uint64_t>(cus) * per_cu;
  if (blocks > cap) blocks = cap;
  return static_cast<unsigned>(blocks ? blocks : 1);
}

}  // namespace

hipError_t launch_crc_windows(const CrcWinArgs& a, bool aligned, int cus, hipStream_t s) {
  // one 1024-thread block per CU (the 156 KiB table image fills its LDS)
  const uint64_t waves = a.nstripes * a.nrows * (a.nwin + (a.tail ? 1 : 0));
  const uint64_t per_block = kCrcBlockThreads / 64;
  uint64_t g = (waves + per_block - 1) / per_block;
  if (g > static_cast<uint64_t>(cus)) g = cus;
  g = capped_grid(g);  // zero-copy calls cap it (hrs::GridCap)
  const size_t shm = static_cast<size_t>(kCrcLdsWordsA) * 4;
  auto k = aligned ? crc_window_kernel<true> : crc_window_kernel<false>;
  note_kernel(aligned ? "crc_window_kernel<true>" : "crc_window_kernel<false>");
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     static_cast<int>(shm));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3(static_cast<unsigned>(g)), dim3(kCrcBlockThreads), shm, s, with_order(a, kOrderCrc));
  return hipGetLastError();
}

hipError_t launch_crc_fold(const CrcFoldArgs& a, int cus, hipStream_t s) {
  const unsigned g = fold_grid(a.nsr, cus);
  const size_t shm = static_cast<size_t>(kCrcLdsWordsB) * 4;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(crc_fold_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(shm));
  if (e != hipSuccess) return e;
  note_kernel("crc_fold_kernel");
  hipLaunchKernelGGL(crc_fold_kernel, dim3(g), dim3(256), shm, s, a);
  return hipGetLastError();
}

}  // namespace hrs
