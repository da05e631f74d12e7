// Internal interface shared by libhrs's host translation units (hrs_api.cpp,
// hrs_matrix.cpp, hrs_dispatch.cpp, hrs_hostpath.cpp, hrs_batch_api.cpp): the
// codec handle behind the C ABI's opaque hrs_codec, error reporting, and the
// functions one unit calls in another. Not part of the ABI (hidden symbols).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "../../include/hrs.h"
#include "crc32.hpp"
#include "hrs_internal.hpp"

namespace hrs {
class CopyPool;  // hrs_host.hpp
}

struct hrs_codec {
  int kind = HRS_CODE_RS;
  int k = 0;
  int p = 0;
  int n = 0;
  int device = 0;
  int kernel_mode = 0;
  std::vector<uint8_t> g;  // p x k
  // SimpleRegeneratingCode: s SRC parities (after init's adjustment), r RS
  // parities, group degree d, and each location's group neighbours
  int src_s = 0, src_r = 0, src_d = 0;
  std::vector<std::vector<int>> groups;
  hipStream_t stream = nullptr;
  std::map<std::vector<int>, std::vector<uint8_t>> decode_cache;
  // CRC-32 state (hrs_crc32_dev): fixed window tables, per-length fold tables, scratch
  uint32_t* crc_tables_a = nullptr;
  // fold tables per (row length, window), LRU: an entry is freed only once the
  // event recorded after its latest fold launch has completed
  struct FoldTables {
    uint32_t* dev = nullptr;
    // the latest fold that read the tables on each stream that has used them
    // (slot streams, caller streams): the tables may be freed once every one
    // of these events has completed
    struct Use {
      hipStream_t stream;
      hipEvent_t ev;
    };
    std::vector<Use> uses;
    uint64_t tick = 0;
  };
  std::map<uint64_t, FoldTables> crc_fold_tables;
  uint64_t crc_fold_tick = 0;
  uint32_t* crc_raw = nullptr;
  size_t crc_raw_bytes = 0;
  hipEvent_t crc_raw_done = nullptr;  // recorded after the latest use (crc_scratch)
  bool crc_raw_used = false;
  std::map<uint64_t, hrs::crc::Mat> crc_zmats;  // host-side Z_len, chaining chunk CRCs
  // hrs_decode_batch_dev: two slots (plans + per-stripe pattern index), each
  // a device buffer and its pinned staging; a slot is reused once the event
  // recorded after its launches has completed.
  struct BatchSlot {
    uint8_t* dev = nullptr;
    uint8_t* host = nullptr;
    size_t bytes = 0;
    hipEvent_t done = nullptr;
    bool pending = false;
  } batch[2];
  int batch_next = 0;
  // host-buffer calls: chunk slots (8 by default, HRS_HOST_SLOTS 2-8),
  // each pinned staging + device rows + its own stream; a slot is reused once
  // its D2H event has completed
  struct HostSlot {
    uint8_t* pin = nullptr;
    uint8_t* pin_dev = nullptr;  // device address of `pin` (zero-copy kernels)
    uint8_t* dev = nullptr;
    size_t bytes = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
  } host[hrs::kHostSlots];
  // gated staged pipeline (hrs_hostpath.cpp staged_run): coherent pinned
  // ready / done / miss words, the next chunk tag, the gates' timeout in
  // wall-clock ticks, and the chunk shapes (CRC mode, length) run before
  uint32_t* qflags = nullptr;
  uint32_t qtag = 0;
  uint64_t gate_timeout = 0;
  std::set<uint64_t> staged_shapes;
  std::map<uint64_t, std::vector<uint32_t>> crc_ztabs;  // Z_n as 4 x 256 tables, by n (host folds)
  // host-memory batches (hrs_*_batch_host): a ring of chunk slots, each a
  // device image + output block, pinned staging (pageable callers only) and
  // its own compute stream; every slot's H2D goes on one copy-in stream and
  // every D2H on one copy-out stream, so the two directions of the link run
  // at once (the link is full duplex: profiles/r04/duplex/). Per slot:
  // in_done after its H2D, comp_done after its kernels, done after its D2H.
  struct HostBatchSlot {
    uint8_t* dev = nullptr;
    size_t dev_bytes = 0;
    uint8_t* pin = nullptr;
    uint8_t* pin_dev = nullptr;  // device address of `pin` (zero-copy kernels)
    size_t pin_bytes = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    hipEvent_t in_done = nullptr;
    hipEvent_t comp_done = nullptr;
  } hbatch[hrs::kHostBatchSlots];
  hipStream_t hbatch_in = nullptr;   // H2D of every host-batch slot
  hipStream_t hbatch_out = nullptr;  // D2H of every host-batch slot
  // asynchronous host-buffer calls (hrs_*_submit / hrs_collect): a ring of
  // operation slots, each pinned staging + device rows + its own stream; an
  // operation occupies its slot from submit until it is collected
  struct AsyncSlot {
    uint8_t* pin = nullptr;
    uint8_t* pin_dev = nullptr;  // device address of `pin` (zero-copy kernels)
    uint8_t* dev = nullptr;
    size_t bytes = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    hipEvent_t t_start = nullptr;  // timing events (hrs_set_timing)
    hipEvent_t t_end = nullptr;
    bool timed = false;   // this operation recorded t_start / t_end
    bool busy = false;
    bool queued = false;  // GPU work was queued (len > 0)
    uint64_t ticket = 0;
    int nout = 0, nlive = 0, ncrc = 0;
    size_t len = 0, pitch = 0, crc_off = 0;
  } async[hrs::kAsyncSlots];
  uint64_t async_tickets = 0;
  bool timing = false;  // hrs_set_timing: asynchronous operations record timing events
  std::string err;
  std::string last_kernel;  // main kernel of the latest coding call (hrs_last_kernel)
  const char* last_host_path = "";  // hrs_last_host_path: "pinned" | "staged" | "copy_engine"
  int numa_node = -2;               // NUMA node of the device's PCI function (-1 unknown, -2 not read yet)
};


#pragma GCC visibility push(hidden)
namespace hrs::api {

// ---- errors (hrs_api.cpp): record the message on the handle (or, for
// create errors, per thread) and return st
hrs_status fail(hrs_codec* c, hrs_status st, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
hrs_status hip_fail(hrs_codec* c, hipError_t e, const char* what);

// Keeps the caller's current device across a call on codec->device.
struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (dev < 0) {  // host-only handle
      ok = false;
      return;
    }
    if (hipGetDevice(&prev) != hipSuccess) {
      ok = false;
      return;
    }
    if (prev != dev && hipSetDevice(dev) != hipSuccess) ok = false;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// ---- zero copy (hrs_batch_api.cpp): kernels read and write pinned host
// memory across the host link directly instead of H2D -> kernel -> D2H — the
// link then carries both directions at once with no copy-engine calls
// (profiles/r04/NOTES.md). HRS_ZEROCOPY=0 turns it off (A/B runs; read per
// call); HRS_ZC_BLOCKS caps the grid of such launches (hrs::GridCap).
bool zero_copy_on();
unsigned zero_copy_blocks();
// Host memory the runtime allocated pinned (hipHostMalloc, torch
// pin_memory), [p, p + len) inside one allocation. Caller-registered
// (hipHostRegister) pageable memory is not: its pages can move.
bool runtime_pinned(const void* p, size_t len);
// Device address of runtime-pinned host memory [p, p + len) when it equals
// the host address, or false (pageable or registered memory: staged).
bool host_device_ptr(const void* p, size_t len, uint8_t** dp);
// The host copy pool (hrs_host.hpp), its workers placed for this handle's
// GPU: on the GPU's NUMA node, where its pinned staging lives, unless
// HRS_HOST_HOME=caller (hrs_hostpath.cpp).
hrs::CopyPool& copy_pool(hrs_codec* c);
// How copy-ins store into pinned staging (hrs::kStore*; HRS_HOST_NT).
uint8_t host_store_mode();

// The compile-time encode kernels hold the hops RS generator (rs) or the
// ISA-L Cauchy rows (nrs) of a (k, p) shape; only those families' G may take
// them. SRC's G (XOR groups over RS(k, r)) and XOR's all-ones row may not.
inline bool static_encode_family(const hrs_codec* c) { return c->kind == HRS_CODE_RS || c->kind == HRS_CODE_NRS; }

bool decode_locations_ok(const hrs_codec* c, const int* erased, int ne, const int* to_read, int nr, const int* ntr,
                         int nn);

// ---- matrices (hrs_matrix.cpp)
bool gf_invert(std::vector<uint8_t>& a, int m);
void rs_decode_rows(int n, const int* erased, int ne, const int* ntr, int nn, int zero_ntr, std::vector<uint8_t>& d);
hrs_status build_decode_matrix(hrs_codec* c, const int* erased, int ne, const int* ntr, int nn, int zero_ntr,
                               std::vector<uint8_t>& d);
hrs_status build_nrs_decode_matrix(hrs_codec* c, int ne, const int* ntr, int nn, std::vector<uint8_t>& d);
const std::vector<uint8_t>* cached_decode_matrix(hrs_codec* c, const int* erased, int ne, const int* ntr, int nn,
                                                 int zero_ntr, hrs_status* st);
std::vector<int> src_neighbors(const hrs_codec* c, int loc);
void src_params(int k, int p, int s_in, int* s, int* r, int* d);
hrs_status src_locations(hrs_codec* c, const int* erased, int ne, std::vector<int>& out);
hrs_status decode5_matrix(hrs_codec* c, const int* erased, int ne, const int* ntr, int nn,
                          const uint8_t* const* rows, std::vector<uint8_t>& tmp, const uint8_t** out,
                          const int* to_read = nullptr, int nr = -1);
void init_encode_matrix(hrs_codec* c);

// ---- device dispatch + CRC (hrs_dispatch.cpp)
hrs_status run_apply(hrs_codec* c, const uint8_t* m, int nout, int nin, const uint8_t* const* in_rows,
                     size_t in_stride, uint8_t* const* out_rows, size_t out_stride, size_t len, size_t nstripes,
                     hipStream_t s, bool static_kp);
size_t crc_raw_bytes_for(size_t len, size_t nstripes, int nrows);
hrs_status run_crc(hrs_codec* c, const uint8_t* const* rows, const size_t* strides, int nrows, size_t len,
                   size_t nstripes, const uint32_t* crc_in, uint32_t* crc_out, hipStream_t s, uint32_t* raw);
// host_fold_win != NULL: when the fused one-pass kernel runs, no fold is
// launched; the raw window CRCs stay in `raw` (layout [stripe][row][window])
// and *host_fold_win receives the window size for the caller's host fold
// (0: the two-pass path ran and wrote crc_out itself).
hrs_status encode_crc_impl(hrs_codec* c, const uint8_t* const* in_rows, size_t in_stride, uint8_t* const* out_rows,
                           size_t out_stride, size_t len, size_t nstripes, const uint32_t* crc_in, uint32_t* crc_out,
                           hipStream_t s, uint32_t* raw, uint64_t* host_fold_win = nullptr);
hrs_status apply_crc_impl(hrs_codec* c, const uint8_t* m, int nout, int nin, const uint8_t* const* in_rows,
                          size_t in_stride, uint8_t* const* out_rows, size_t out_stride, size_t len, size_t nstripes,
                          const uint32_t* crc_in, uint32_t* crc_out, hipStream_t s, uint32_t* raw,
                          uint64_t* host_fold_win = nullptr);
// Whether encode_crc_impl / apply_crc_impl (nlive live inputs) take their
// one-pass kernel for a job of this shape, rows 16-byte aligned: the
// zero-copy host calls checksum through host memory only then (a two-pass CRC
// would read the cells across the link a second time).
bool encode_crc_one_pass(const hrs_codec* c, size_t len, size_t nstripes);
bool apply_crc_one_pass(const hrs_codec* c, int nout, int nlive, size_t len);

}  // namespace hrs::api
#pragma GCC visibility pop
