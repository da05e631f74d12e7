// Internal interface between the C-ABI layer (hrs_api.cpp) and the gfx950
// kernels (hrs_kernels.hip).
#pragma once
#include <cstddef>
#include <cstdint>
#include <hip/hip_runtime.h>

namespace hrs {

// Rows one launch reads / writes. Larger problems are split by the host:
// inputs in chunks of kMaxIn (later chunks accumulate into the outputs),
// outputs in chunks of kMaxOut.
constexpr int kMaxIn = 32;         // RowArgs capacity (static kernels: k <= 32)
constexpr int kMaxInRuntime = 16;  // inputs per runtime-matrix launch (<= 5 outputs)
constexpr int kMaxInRuntimeWide = 8;  // inputs per launch with 6..8 outputs
inline int runtime_in_chunk(int nout) { return nout <= 5 ? kMaxInRuntime : kMaxInRuntimeWide; }
constexpr int kMaxOut = 8;

// One wave owns a 2 KiB column window of every row of one stripe: each lane
// moves 2 x 16 B per row (lane*16 and 1024 + lane*16), so both load
// instructions of a row are fully coalesced 1 KiB wave accesses.
constexpr int kWindowBytes = 2048;
constexpr int kBlockThreads = 256;
constexpr int kWavesPerBlock = kBlockThreads / 64;

struct RowArgs {
  const uint8_t* in[kMaxIn];
  uint8_t* out[kMaxOut];
  uint64_t cw[kMaxIn];            // runtime-matrix kernels: byte o of cw[i] = coefficient (output o, input i)
  uint64_t in_stride;             // bytes between stripes, all input rows
  uint64_t out_stride;            // bytes between stripes, all output rows
  uint64_t len;                   // bytes per row (cell size)
  uint64_t nwin;                  // ceil(len / kWindowBytes)
  uint64_t ntasks;                // nstripes * nwin
  int nin;
  int nout;
  int accumulate;                 // 1: XOR into existing outputs (input chunking)
  int pad_;
};

inline void set_coef(RowArgs& a, int o, int i, uint8_t v) {
  a.cw[i] = (a.cw[i] & ~(0xFFull << (8 * o))) | (static_cast<uint64_t>(v) << (8 * o));
}

enum class KernelKind : int {
  kStaticEncode = 0,   // compile-time encode matrix (3,2) (6,3) (10,4) (12,4)
  kBitsliced = 1,      // runtime matrix, bit-sliced
  kBytewise = 2,       // runtime matrix, one byte column per lane (any alignment)
};

// Launches; return hipSuccess or the launch error. `grid_cap` = 0 picks a
// chip-filling grid from the occupancy API.
// family: kStaticRs (hops generator-polynomial code) or kStaticCauchy (nrs).
enum { kStaticRs = 0, kStaticCauchy = 1 };
hipError_t launch_static_encode(int family, int k, int p, const RowArgs& a, hipStream_t s, bool* handled);
hipError_t launch_bitsliced(const RowArgs& a, hipStream_t s);
hipError_t launch_bytewise(const RowArgs& a, hipStream_t s);
hipError_t launch_xor(const RowArgs& a, hipStream_t s);
int device_cu_count();  // CUs of the current device (cached)  // out[0] = XOR of in[0..nin)

}  // namespace hrs
