// Internal interface of the CRC-32 kernels (hrs_crc.hip) for hrs_api.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hrs {

constexpr int kCrcWindow = 4096;     // bytes per wave task
constexpr int kCrcLaneBytes = 64;    // contiguous bytes per lane (16 words)
constexpr int kCrcRep = 4;           // slicing tables replicated across LDS banks
constexpr int kCrcChains = 4;        // independent 16-byte chains per lane (ILP)
constexpr int kCrcBlocksPerCU = 3;
constexpr int kCrcMaxRows = 32;      // rows per window launch
constexpr int kCrcSliceWords = 4 * 256 * kCrcRep;           // 16 KiB
constexpr int kCrcLdsWordsA = kCrcSliceWords + 7 * 1024;    // + Z_16, Z_{64*2^t} t = 0..5 (28 KiB)
constexpr int kCrcLdsWordsB = 9 * 1024;                     // Z_4096, 6 tree levels, Z_tail, Z_len (36 KiB)

struct CrcWinArgs {
  const uint8_t* rows[kCrcMaxRows];
  int nrows;        // rows in this launch
  int row0;         // index of rows[0] among all rows of the call
  int nrows_total;  // rows of the call (raw layout [stripe][row][window])
  int pad_;
  uint64_t stride;  // bytes between stripes
  uint64_t len;
  uint64_t nwin;    // full 4 KiB windows per row
  uint64_t tail;    // len - nwin * 4096
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

}  // namespace hrs
