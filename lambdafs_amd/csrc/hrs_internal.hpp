// Internal interface between the C-ABI host units (hrs_dispatch.cpp, hrs_batch_api.cpp) and the gfx950
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
  int order;                      // window -> wave order (hrs_launch.hpp task_order), set at launch
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
hipError_t launch_bitsliced_stream(const RowArgs& a, hipStream_t s);  // up to kMaxIn inputs, one pass
hipError_t launch_bytewise(const RowArgs& a, hipStream_t s);
hipError_t launch_xor(const RowArgs& a, hipStream_t s);
int device_cu_count();  // CUs of the current device (cached)

// The last kernel this thread launched, named as rocprofv3 demangles it
// (e.g. "encode_static_kernel<10, 4>"): the host units copy it onto the
// handle after a call's main launch (hrs_last_kernel), so a benchmark can
// look up the PMC traffic of the kernel the run actually used.
void note_kernel(const char* name);
const char* last_kernel();

// ---- heterogeneous batches: one erasure pattern per stripe (hrs_decode_batch_dev)

constexpr int kBatchMaxIn = 32;  // > 16 inputs (or > 8 with 6-8 outputs): batch_stream_kernel
constexpr int kHostBatchSlots = 3;  // chunk slots of the host-memory batch pipeline
constexpr int kAsyncSlots = 4;      // operations in flight per handle (hrs_*_submit / hrs_collect)
constexpr int kHostSlots = 8;       // chunk slots of a synchronous host-buffer call (at most; HRS_HOST_SLOTS)
struct BatchPlan {            // one erasure pattern, a device table entry
  int nin;                    // live survivor rows read
  int nout;                   // erased rows written
  int loc[kBatchMaxIn];       // hops location of input r
  uint64_t cw[kBatchMaxIn];   // byte o of cw[r] = coefficient (output o, input r)
};

struct BatchArgs {
  const uint8_t* base;        // location l of stripe s at base + s * stripe_stride + l * row_stride
  uint8_t* out;               // output t of stripe s at out + s * out_stripe_stride + t * out_row_stride
  uint64_t row_stride, stripe_stride, out_row_stride, out_stripe_stride;
  uint64_t len;               // bytes per row
  uint64_t col0;              // first byte column this launch covers (tails: nwin * 2048)
  uint64_t nwin;              // full 2 KiB windows per row (vector kernel)
  uint64_t ntasks;            // vector: nstripes * nwin; bytewise: nstripes * (len - col0)
  const BatchPlan* plans;     // device table
  const int32_t* pat;         // device: pattern index of each stripe
  int order;                  // window -> wave order (task_order), set at launch
  int pad_;
};

hipError_t launch_batch_bitsliced(const BatchArgs& a, int max_nout, int max_nin, hipStream_t s);

// ---- stream gates of the queued host pipeline (hrs_gate.hip)
// gate: waits until *ready (a coherent pinned word the host writes) reaches
// `want` (serial-number order), or `timeout` wall-clock ticks pass (then *fail
// = 1). signal: *done = tag with a system-scope release.
hipError_t launch_gate(const uint32_t* ready, uint32_t want, uint32_t* fail, uint64_t timeout, hipStream_t s);
hipError_t launch_signal(uint32_t* done, uint32_t tag, hipStream_t s);
hipError_t launch_batch_bytewise(const BatchArgs& a, hipStream_t s);

}  // namespace hrs
