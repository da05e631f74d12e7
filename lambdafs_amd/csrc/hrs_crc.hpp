// Internal interface of the CRC-32 kernels (hrs_crc.hip, hrs_fused.hip) for hrs_dispatch.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "crc32.hpp"
#include "hrs_internal.hpp"

namespace hrs {

constexpr int kCrcWindow = static_cast<int>(crc::kWindowBytes);  // bytes per wave task (32 KiB)
constexpr int kCrcRep = 32;          // slicing tables replicated: lane l reads copy l % 32 (its own bank)
// slicing image word of (table j, entry e, copy c); layout: hrs_device.hpp slice4
constexpr int crc_slice_word(int j, int e, int c) { return (j >> 1) * 16384 + e * 64 + (j & 1) * 32 + c; }
constexpr int kCrcGroup = 8;         // chunks loaded and chained together (ILP)
constexpr int kCrcBlockThreads = 1024;  // 16 waves share one table image per CU
constexpr int kCrcMaxRows = 32;      // rows per window launch
constexpr int kCrcSliceWords = 4 * 256 * kCrcRep;           // 128 KiB
constexpr int kCrcLdsWordsA = kCrcSliceWords + 7 * 1024;    // + Z_1024, Z_{16*2^t} t = 0..5 (156 KiB)
constexpr int kCrcLdsWordsB = 9 * 1024;                     // Z_window, 6 tree levels, Z_tail, Z_len (36 KiB)
constexpr int kCrcFoldBlocksPerCU = 3;

// The LDS image of the window kernels (crc_window_kernel, the fused encode +
// CRC), built on the host and uploaded once per handle: the slicing-by-4
// tables (kCrcRep bank-private copies; table j = a byte followed by j more
// bytes of its word, i.e. the zlib slicing tables T8_0..T8_3), then Z_chunk
// (joins a lane's successive pieces, `chunk` bytes apart) and the lane tree
// Z_{piece * 2^t}, t = 0..5 (lane l + 2^t is piece * 2^t bytes later).
// tests/cpp/crc_tables dumps it for tests/test_crc_tables.py.
inline std::vector<uint32_t> crc_window_image(uint64_t piece, uint64_t chunk) {
  std::vector<uint32_t> h(kCrcLdsWordsA);
  const crc::Slice4 sl = crc::make_slice4();
  for (int j = 0; j < 4; ++j)
    for (int v = 0; v < 256; ++v)
      for (int r = 0; r < kCrcRep; ++r) h[crc_slice_word(j, v, r)] = sl.s[j].t[v];
  crc::to_tables(crc::zeros(chunk), &h[kCrcSliceWords]);
  for (int t = 0; t < 6; ++t) crc::to_tables(crc::zeros(piece << t), &h[kCrcSliceWords + (1 + t) * 1024]);
  return h;
}

struct CrcWinArgs {
  const uint8_t* rows[kCrcMaxRows];
  int nrows;        // rows in this launch
  int row0;         // index of rows[0] among all rows of the call
  int nrows_total;  // rows of the call (raw layout [stripe][row][window])
  int order;        // window -> wave order (task_order), set at launch
  uint64_t stride[kCrcMaxRows];  // bytes between stripes, per row
  uint64_t len;
  uint64_t nwin;    // full windows per row
  uint64_t tail;    // len - nwin * kCrcWindow
  uint64_t nstripes;
  uint32_t* raw;
  const uint32_t* tables;  // kCrcLdsWordsA words (device)
};

struct CrcFoldArgs {
  const uint32_t* raw;
  uint64_t nwin;
  uint64_t tail;
  uint64_t nsr;    // nstripes * nrows
  int G;           // full windows per lane: ceil(nwin / 64)
  int pad_;
  const uint32_t* tables;  // kCrcLdsWordsB words (device), built for this len
  const uint32_t* crc_in;  // nullable
  uint32_t* crc_out;
};

hipError_t launch_crc_windows(const CrcWinArgs& a, bool aligned, int cus, hipStream_t s);
hipError_t launch_crc_fold(const CrcFoldArgs& a, int cus, hipStream_t s);

// Fused encode + CRC-32 (hrs_fused.hip): one wave per (stripe, window of
// `subs` 2 KiB sub-windows: 32 KiB for large jobs, smaller when a job has too
// few 32 KiB windows to fill the chip) encodes the window's sub-windows and
// keeps the raw CRC of every data and parity row of the window, in the window
// kernel's decomposition (lane pieces joined with Z_1024, lanes with
// Z_{16*2^t}), so crc_fold_kernel finishes them with Z_window tables. Raw
// layout [stripe][row][window], rows = [data 0..k-1, parity 0..p-1].
constexpr int kFusedMaxK = 16;
constexpr int kFusedMaxP = 4;
struct EncodeCrcArgs {
  const uint8_t* in[kFusedMaxK];
  uint8_t* out[kFusedMaxP];
  uint64_t in_stride;
  uint64_t out_stride;
  uint64_t nwin;      // windows per row (len / (subs * 2 KiB), len a multiple)
  uint64_t nstripes;
  uint32_t subs;      // 2 KiB sub-windows per window: 1, 2, 4, 8 or 16
  uint32_t rep_mask;  // slicing-table copy of lane l = l & rep_mask (kCrcRep - 1; HRS_CRC_REP A/B)
  int order;          // window -> wave order (task_order), set at launch
  int pad_;
  uint32_t* raw;
  const uint32_t* tables;  // kCrcLdsWordsA words (device)
};

// family: kStaticRs / kStaticCauchy (hrs_internal.hpp). *handled = false when
// (family, k, p) has no fused kernel (the caller runs encode, then CRC).
hipError_t launch_encode_crc(int family, int k, int p, const EncodeCrcArgs& a, int cus, hipStream_t s,
                             bool* handled);

// Fused repair + CRC-32 (hrs_decode_crc.hip): the runtime-matrix apply of
// `r` (whole 2 KiB windows: r.nwin = len / 2 KiB, no accumulate) with the raw
// CRC of every output's window in raw[stripe][output][window]
// (crc_fold_kernel finishes them with 2 KiB windows). *handled = false for
// shapes without a fused kernel (> 4 outputs, > 12 inputs, > 8 at 4 outputs).
struct DecodeCrcArgs {
  RowArgs r;
  uint32_t* raw;
  const uint32_t* tables;  // kCrcLdsWordsA words (device)
};
hipError_t launch_decode_crc(const DecodeCrcArgs& d, int cus, hipStream_t s, bool* handled);

}  // namespace hrs
