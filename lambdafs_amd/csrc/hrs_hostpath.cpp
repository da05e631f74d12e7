// Host-buffer calls, the JNI path: synchronous encodeBulk / decodeBulk over
// pageable rows through two pinned staging slots (with optional block
// CRC-32s chained on the host), and the asynchronous submit / wait / collect
// rounds over a ring of operation slots.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hrs.h"
#include "hrs_codec.hpp"
#include "crc32.hpp"
#include "hrs_host.hpp"
#include "hrs_internal.hpp"
#include "hrs_launch.hpp"

namespace hrs::api {

// Device scratch for the host-buffer calls: `rows` rows of `pitch` bytes.
size_t pitch_for(size_t len) { return (len + 255) & ~static_cast<size_t>(255); }

hrs_status host_slot(hrs_codec* c, int i, size_t bytes) {
  hrs_codec::HostSlot& h = c->host[i];
  if (!h.stream) {
    hipError_t e = hipStreamCreateWithFlags(&h.stream, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail(c, e, "hipStreamCreate");
    e = hipEventCreateWithFlags(&h.done, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventCreate");
  }
  if (h.bytes >= bytes) return HRS_OK;
  (void)hipStreamSynchronize(h.stream);
  if (h.dev) (void)hipFree(h.dev);
  if (h.pin) (void)hipHostFree(h.pin);
  h.dev = nullptr;
  h.pin = nullptr;
  h.pin_dev = nullptr;
  h.bytes = 0;
  hipError_t e = hipMalloc(&h.dev, bytes);
  if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
  e = hipHostMalloc(&h.pin, bytes, hipHostMallocDefault);
  if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
  if (!host_device_ptr(h.pin, bytes, &h.pin_dev)) h.pin_dev = nullptr;  // then the calls take the copy engine
  h.bytes = bytes;
  return HRS_OK;
}


// Block checksums carried through a host-buffer call (Encoder.java:408-450,
// Decoder.java:222-229 / :645-655): kCrcEncode = CRC-32 of the k inputs then
// the p outputs (the encode matrix is c->g), kCrcOutputs = of the nout outputs.
// Each chunk's CRCs come back with its outputs and are chained on the host,
// crc = Z_len(crc) ^ crc_chunk (zlib crc32_combine), starting from `in`
// (NULL = fresh CRC32 objects).
enum HostCrcMode { kCrcNone = 0, kCrcEncode = 1, kCrcOutputs = 2 };
struct HostCrc {
  int mode = kCrcNone;
  const uint32_t* in = nullptr;
  uint32_t* out = nullptr;
};

const hrs::crc::Mat& crc_zmat(hrs_codec* c, uint64_t len) {
  auto it = c->crc_zmats.find(len);
  if (it == c->crc_zmats.end()) it = c->crc_zmats.emplace(len, hrs::crc::zeros(len)).first;
  return it->second;
}

// Z_len as 4 byte-indexed tables (crc32.hpp to_tables), for host folds.
const uint32_t* crc_ztab(hrs_codec* c, uint64_t len) {
  auto it = c->crc_ztabs.find(len);
  if (it == c->crc_ztabs.end()) {
    std::vector<uint32_t> t(4 * 256);
    hrs::crc::to_tables(crc_zmat(c, len), t.data());
    it = c->crc_ztabs.emplace(len, std::move(t)).first;
  }
  return it->second.data();
}

inline uint32_t ztab_apply(const uint32_t* t, uint32_t v) {
  return t[v & 0xFFu] ^ t[256 + ((v >> 8) & 0xFFu)] ^ t[512 + ((v >> 16) & 0xFFu)] ^ t[768 + (v >> 24)];
}

// Checksummed staged chunks fold their raw window CRCs on the host
// (HRS_HOST_FOLD=0: a fold kernel per chunk, the round-5 form; read per call).
bool host_fold_on() {
  const char* e = getenv("HRS_HOST_FOLD");
  return !(e && e[0] == '0');
}

// Rows the caller holds in memory the runtime allocated pinned (hipHostMalloc,
// torch pin_memory) are visible to the GPU at their own addresses and never
// move: the zero-copy kernel runs over them in place, one launch, no staging
// copies ("pinned"). Taken when zero copy is on, every live input and output
// row lies wholly inside such an allocation and is 16-byte aligned, and a
// checksummed call's kernel is one-pass (a two-pass CRC would read the cells
// across the link twice); otherwise false and nothing done.
// Pageable memory the caller registered with hipHostRegister is NOT taken
// here: registration maps the pages for the GPU without pinning them, and in
// round 5 GPU writes into registered pages were lost when a page moved during
// a kernel ("Platform constraint"). Such rows are staged.
bool host_apply_pinned(hrs_codec* c, const uint8_t* m, int nout, int nin, const uint8_t* const* din,
                       uint8_t* const* out_rows, size_t len, bool static_kp, const HostCrc& crc, int ncrc,
                       hrs_status* st) {
  if (!zero_copy_on()) return false;
  int nlive = 0;
  for (int i = 0; i < nin; ++i) {
    if (!din[i]) continue;
    uint8_t* d = nullptr;
    if (!aligned16(din[i]) || !host_device_ptr(din[i], len, &d) || d != din[i]) return false;
    ++nlive;
  }
  for (int o = 0; o < nout; ++o) {
    uint8_t* d = nullptr;
    if (!aligned16(out_rows[o]) || !host_device_ptr(out_rows[o], len, &d) || d != out_rows[o]) return false;
  }
  if (crc.mode == kCrcEncode && !encode_crc_one_pass(c, len, 1)) return false;
  if (crc.mode == kCrcOutputs && !apply_crc_one_pass(c, nout, nlive, len)) return false;
  // the chunk CRC words in slot 0's pinned staging, the raw window CRCs in its device buffer
  const size_t words = static_cast<size_t>(std::max(ncrc, 1)) * sizeof(uint32_t);
  const size_t raw_off = (words + 255) & ~static_cast<size_t>(255);
  hrs_status s0 = host_slot(c, 0, ncrc > 0 ? raw_off + crc_raw_bytes_for(len, 1, ncrc) : words);
  if (s0 == HRS_OK && !c->host[0].pin_dev) return false;
  if (s0 != HRS_OK) {
    *st = s0;
    return true;
  }
  hrs_codec::HostSlot& h = c->host[0];
  c->last_host_path = "pinned";
  uint32_t* cw = reinterpret_cast<uint32_t*>(h.pin_dev);
  uint32_t* raw = reinterpret_cast<uint32_t*>(h.dev + raw_off);
  hrs_status rs = HRS_OK;
  {
    hrs::GridCap cap(zero_copy_blocks());
    if (crc.mode == kCrcEncode)
      rs = encode_crc_impl(c, din, 0, out_rows, 0, len, 1, nullptr, cw, h.stream, raw);
    else if (crc.mode == kCrcOutputs)
      rs = apply_crc_impl(c, m, nout, nin, din, 0, out_rows, 0, len, 1, nullptr, cw, h.stream, raw);
    else
      rs = run_apply(c, m, nout, nin, din, 0, out_rows, 0, len, 1, h.stream, static_kp);
  }
  const hipError_t e = hipStreamSynchronize(h.stream);
  if (rs == HRS_OK && e != hipSuccess) rs = hip_fail(c, e, "hipStreamSynchronize");
  if (rs == HRS_OK && ncrc > 0) {  // CRC32.update chaining from the running values
    const uint32_t* part = reinterpret_cast<const uint32_t*>(h.pin);
    const hrs::crc::Mat& z = crc_zmat(c, len);
    for (int r = 0; r < ncrc; ++r) crc.out[r] = hrs::crc::apply(z, crc.out[r]) ^ part[r];
  }
  *st = rs;
  return true;
}

// ---- the staged pipeline (pageable rows) ----
// The caller's rows are cut into column chunks (the first HRS_HOST_FIRST
// bytes, then HRS_HOST_CHUNK each) that rotate through a ring of S slots
// (HRS_HOST_SLOTS), each with its own pinned staging and stream. Per chunk:
// the copy pool moves its live input columns into the slot's staging, the
// zero-copy kernel works on the staging across the link (or, HRS_ZEROCOPY=0
// and for chunks no one-pass kernel takes, H2D -> kernel -> D2H), and the
// pool moves its output columns out. Chunks are copied out in order as soon
// as they are done (not only when their slot is needed again), so only the
// last chunk's copy-out follows the link time; each chunk's CRC words are
// kept and chained in order at the end.
// Gated (HRS_HOST_GATE=1): every chunk's kernels are queued S chunks ahead,
// each behind a gate kernel that waits for the chunk's tag in a pinned flag
// word (hrs_gate.hip) and followed by a signal kernel the host polls; the host
// publishes the tag as soon as the copy-in ends, so no launch sits between a
// chunk's copy-in and its kernel. Measured slower (each gate / signal
// dispatch costs the slot stream more than the launch latency it hides:
// profiles/r06/NOTES.md), so it is an A/B knob; by default a chunk is
// launched after its copy-in and its completion is an event.
static size_t env_window_bytes(const char* name, size_t dflt) {
  const char* e = getenv(name);
  const long x = e ? atol(e) : 0;
  if (x < static_cast<long>(hrs::kWindowBytes)) return dflt;
  return static_cast<size_t>(x) / hrs::kWindowBytes * hrs::kWindowBytes;
}

// Defaults measured with tools/host_pipeline_sweep (profiles/r06/NOTES.md):
// 128 KiB x 8 slots, once the copy pool's batches stopped ending in a
// condition-variable sleep (r06q / r06r, same box, 3 copy workers; RS(10,4)
// 1 MiB calls, encode / decode / encode + CRC / decode + CRC): 0.267 / 0.245 /
// 0.283 / 0.244 ms against 0.281 / 0.248 / 0.293 / 0.255 at 256 KiB x 4 (the
// round-6 default before) and 0.314 / 0.271 / 0.348 / 0.271 at 512 KiB x 2
// (round 5); in-place floor on pinned rows 0.224 / 0.213 / 0.238 / 0.221.
size_t host_chunk_bytes(bool) { return env_window_bytes("HRS_HOST_CHUNK", 128 << 10); }
size_t host_first_bytes(size_t chunk) { return std::min(chunk, env_window_bytes("HRS_HOST_FIRST", chunk)); }

int host_slots(bool) {
  const char* e = getenv("HRS_HOST_SLOTS");
  const int x = e ? atoi(e) : 0;
  return (x >= 2 && x <= hrs::kHostSlots) ? x : 8;
}

// Stores of the copy-ins into the pinned staging (HRS_HOST_NT, read per
// call). The GPU reads the staging next, across the link, and the staging
// lives on the GPU's NUMA node: lines a CPU of the other socket left dirty in
// its caches make every such read a cross-socket snoop. Default ("1"):
// nontemporal stores, so the lines are in memory (RS(10,4) 1 MiB staged
// encode from the other socket 0.33-0.36 ms with cached stores, 0.28 with
// nontemporal; from the GPU's node 0.255-0.262 vs 0.264-0.269: never worse;
// profiles/r06/NOTES.md §4, r06x / r06y). "auto": nontemporal only from CPUs
// off the GPU's node; "0": cached.
uint8_t host_store_mode() {
  const char* e = getenv("HRS_HOST_NT");
  if (!e) return hrs::kStoreStream;
  if (strcmp(e, "auto") == 0) return hrs::kStoreRemote;
  return e[0] == '0' ? hrs::kStorePlain : hrs::kStoreStream;
}

// NUMA node of the handle's device: its PCI function's, from sysfs (cached).
static int device_numa_node(hrs_codec* c) {
  if (c->numa_node != -2) return c->numa_node;
  int node = -1;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, c->device) == hipSuccess) {
    for (char* q = bus; *q; ++q) *q = static_cast<char>(tolower(*q));
    char path[160];
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    if (FILE* f = fopen(path, "r")) {
      if (fscanf(f, "%d", &node) != 1) node = -1;
      fclose(f);
    }
  } else {
    (void)hipGetLastError();
  }
  c->numa_node = node;
  return node;
}

hrs::CopyPool& copy_pool(hrs_codec* c) {
  hrs::CopyPool::set_home_node(device_numa_node(c), c->device);
  return hrs::CopyPool::instance();
}

bool host_gate_on() {
  const char* e = getenv("HRS_HOST_GATE");
  return e && e[0] == '1';
}

// Coherent pinned flag words of the gated pipeline, one 128-byte line each:
// ready[kHostSlots], done[kHostSlots], then the gates' miss word.
constexpr int kFlagWords = 32;
inline uint32_t* flag_ready(hrs_codec* c, int sl) { return c->qflags + sl * kFlagWords; }
inline uint32_t* flag_done(hrs_codec* c, int sl) { return c->qflags + (hrs::kHostSlots + sl) * kFlagWords; }
inline uint32_t* flag_fail(hrs_codec* c) { return c->qflags + 2 * hrs::kHostSlots * kFlagWords; }

bool gate_flags(hrs_codec* c) {
  if (c->qflags) return true;
  void* p = nullptr;
  const size_t bytes = (2 * hrs::kHostSlots + 1) * kFlagWords * sizeof(uint32_t);
  if (hipHostMalloc(&p, bytes, hipHostMallocCoherent) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  uint8_t* d = nullptr;
  if (!host_device_ptr(p, bytes, &d)) {  // the gates read the flags at their host address
    (void)hipHostFree(p);
    return false;
  }
  std::memset(p, 0, bytes);
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0) khz = 100000;
  c->gate_timeout = static_cast<uint64_t>(khz) * 1000u * 10u;  // 10 s of wall-clock ticks
  c->qflags = static_cast<uint32_t*>(p);
  return true;
}

inline uint32_t flag_load(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline bool tag_reached(uint32_t v, uint32_t want) { return static_cast<int32_t>(v - want) >= 0; }

hrs_status staged_run(hrs_codec* c, const uint8_t* m, int nout, int nin, const uint8_t* const* in_rows,
                      uint8_t* const* out_rows, size_t len, bool static_kp, const HostCrc& crc, int ncrc,
                      const std::vector<int>& slot_of, int nlive, bool gate, bool* missed) {
  *missed = false;
  struct Span {
    size_t off, len;
  };
  const size_t chunk = std::min(len, host_chunk_bytes(crc.mode != kCrcNone));
  const size_t first = host_first_bytes(chunk);
  std::vector<Span> ch;
  for (size_t off = 0; off < len;) {
    const size_t l = std::min(ch.empty() ? first : chunk, len - off);
    ch.push_back({off, l});
    off += l;
  }
  const size_t C = ch.size();
  const int S = static_cast<int>(std::min<size_t>(host_slots(crc.mode != kCrcNone), C));
  const size_t pitch = pitch_for(chunk);
  // slot layout: nlive + nout rows of `pitch`, then (CRC only) the chunk's
  // ncrc CRC words, then the raw window-CRC scratch (device side only)
  const size_t crc_off = pitch * static_cast<size_t>(nlive + nout);
  const size_t raw_off = crc_off + ((ncrc * sizeof(uint32_t) + 255) & ~static_cast<size_t>(255));
  // raw window CRCs: in the device buffer for a fold kernel; for a host fold
  // (zero-copy chunks) in the pinned staging at the same offset
  const size_t need = ncrc ? raw_off + crc_raw_bytes_for(chunk, 1, ncrc) : crc_off;
  for (int i = 0; i < S; ++i) {
    hrs_status st = host_slot(c, i, need);
    if (st != HRS_OK) return st;
  }
  // zero copy: the kernel reads the chunk from the slot's pinned staging and
  // writes its outputs (and the chunk CRCs) there, across the host link — no
  // H2D / D2H. A checksummed chunk goes this way only when its one-pass
  // kernel takes it (a two-pass CRC would read the cells across the link a
  // second time); other chunks take the copy engine. The raw window CRCs stay
  // in device memory.
  bool zc_ok = zero_copy_on();
  for (int i = 0; i < S; ++i) zc_ok &= c->host[i].pin_dev != nullptr;
  auto zc_chunk = [&](size_t lj) {
    if (!zc_ok) return false;
    if (crc.mode == kCrcEncode) return encode_crc_one_pass(c, lj, 1);
    if (crc.mode == kCrcOutputs) return apply_crc_one_pass(c, nout, nlive, lj);
    return true;
  };
  // Gates only for chunk shapes this handle has run before: a first run may
  // upload CRC tables (a synchronous copy, and an LRU eviction's hipFree
  // waits for the device) while its own gates hold the slot streams.
  auto shape = [&](size_t lj) { return static_cast<uint64_t>(crc.mode) << 56 | static_cast<uint64_t>(lj); };
  bool all_zc = true, seen = true;
  for (const Span& sp : ch) {
    all_zc &= zc_chunk(sp.len);
    seen &= c->staged_shapes.count(shape(sp.len)) > 0;
  }
  gate = gate && all_zc && seen && gate_flags(c);
  c->last_host_path = all_zc ? "staged" : "copy_engine";
  hrs::CopyPool& pool = copy_pool(c);
  std::vector<hrs::CopyJob> jobs;
  std::vector<uint32_t> parts(static_cast<size_t>(ncrc) * C);
  std::vector<const uint8_t*> din(nin);
  std::vector<uint8_t*> dout(nout);
  hrs::CopyPool::Hold hold;  // the pool's workers stay awake for this call
  // Copies go to the pool as one batch per step: the outputs of every chunk
  // that is done (copy_out) and the next chunk's inputs (copy_in). A chunk's
  // input rows and output rows are disjoint regions of its slot, so a chunk's
  // copy-out and its slot's next copy-in may share a batch.
  const uint8_t nt = host_store_mode();
  auto copy_in = [&](size_t j) {
    const hrs_codec::HostSlot& h = c->host[j % S];
    for (int i = 0; i < nin; ++i)
      if (slot_of[i] >= 0) jobs.push_back({h.pin + pitch * slot_of[i], in_rows[i] + ch[j].off, ch[j].len, nt});
  };
  std::vector<uint64_t> fold_win(C, 0);  // window of a chunk whose raw CRCs the host folds (0: GPU-folded)
  auto copy_out = [&](size_t j) {
    const hrs_codec::HostSlot& h = c->host[j % S];
    for (int o = 0; o < nout; ++o) jobs.push_back({out_rows[o] + ch[j].off, h.pin + pitch * (nlive + o), ch[j].len});
    if (!ncrc) return;
    if (!fold_win[j]) {
      std::memcpy(&parts[j * ncrc], h.pin + crc_off, ncrc * sizeof(uint32_t));
      return;
    }
    // CRC-32 of the chunk's cell of row r from its raw window CRCs
    // (crc32.hpp: raw(A || B) = Z_|B|(raw(A)) ^ raw(B); crc = Z_len(~0) ^ raw ^ ~0)
    const size_t nw = ch[j].len / fold_win[j];
    const uint32_t* zw = crc_ztab(c, fold_win[j]);
    const uint32_t* zl = crc_ztab(c, ch[j].len);
    const uint32_t* raw = reinterpret_cast<const uint32_t*>(h.pin + raw_off);
    // up to 16 rows' chains advance in lockstep, so their table lookups
    // overlap (a 14-row chunk of 64 windows: 1.4-1.7 us instead of 3.7-3.9
    // row by row, on the build host)
    const uint32_t zinit = ztab_apply(zl, ~0u);
    for (int r0 = 0; r0 < ncrc; r0 += 16) {
      const int m = std::min(16, ncrc - r0);
      uint32_t x[16] = {0};
      for (size_t w = 0; w < nw; ++w)
        for (int r = 0; r < m; ++r) x[r] = ztab_apply(zw, x[r]) ^ raw[(r0 + r) * nw + w];
      for (int r = 0; r < m; ++r) parts[j * ncrc + r0 + r] = zinit ^ x[r] ^ ~0u;
    }
  };
  auto flush = [&] {
    if (!jobs.empty()) pool.run(jobs);
    jobs.clear();
  };
  // the chunk's kernels (and, off the zero-copy path, its H2D and D2H) on its slot's stream
  auto launch = [&](size_t j) -> hrs_status {
    hrs_codec::HostSlot& h = c->host[j % S];
    const size_t lj = ch[j].len;
    const bool zc = zc_chunk(lj);
    // only zero-copy chunks cap their grid (the link bounds them); a chunk
    // sent back to the copy engine runs on device memory with the full grid
    hrs::GridCap cap(zc ? zero_copy_blocks() : 0u);
    if (nlive > 0 && !zc) {
      hipError_t e = hipMemcpyAsync(h.dev, h.pin, pitch * (nlive - 1) + lj, hipMemcpyHostToDevice, h.stream);
      if (e != hipSuccess) return hip_fail(c, e, "hipMemcpyAsync H2D");
    }
    uint8_t* img = zc ? h.pin_dev : h.dev;
    for (int i = 0; i < nin; ++i) din[i] = slot_of[i] >= 0 ? img + pitch * slot_of[i] : nullptr;
    for (int o = 0; o < nout; ++o) dout[o] = img + pitch * (nlive + o);
    uint32_t* dcrc = reinterpret_cast<uint32_t*>(img + crc_off);
    // zero-copy chunks leave their raw window CRCs in the pinned staging and
    // the host folds them at copy-out (no fold launch per chunk)
    const bool hf = zc && host_fold_on();
    uint32_t* draw = reinterpret_cast<uint32_t*>(hf ? h.pin_dev + raw_off : h.dev + raw_off);
    uint64_t* fw = hf ? &fold_win[j] : nullptr;
    hrs_status st;
    if (crc.mode == kCrcEncode)
      st = encode_crc_impl(c, din.data(), 0, dout.data(), 0, lj, 1, nullptr, dcrc, h.stream, draw, fw);
    else if (crc.mode == kCrcOutputs)  // repair + CRC of the repaired cells (fused where the shape allows)
      st = apply_crc_impl(c, m, nout, nin, din.data(), 0, dout.data(), 0, lj, 1, nullptr, dcrc, h.stream, draw, fw);
    else
      st = run_apply(c, m, nout, nin, din.data(), 0, dout.data(), 0, lj, 1, h.stream, static_kp);
    if (st != HRS_OK) return st;
    if (!zc) {  // outputs (and the chunk CRCs right behind them) back to the staging
      const size_t back = ncrc ? crc_off + ncrc * sizeof(uint32_t) - pitch * nlive : pitch * (nout - 1) + lj;
      hipError_t e = hipMemcpyAsync(h.pin + pitch * nlive, h.dev + pitch * nlive, back, hipMemcpyDeviceToHost,
                                    h.stream);
      if (e != hipSuccess) return hip_fail(c, e, "hipMemcpyAsync D2H");
    }
    return HRS_OK;
  };
  size_t out_next = 0;  // chunks [0, out_next) are copied out
  hrs_status st = HRS_OK;
  if (gate) {
    const uint32_t tag0 = c->qtag;
    c->qtag += static_cast<uint32_t>(C);
    auto tag = [&](size_t j) { return tag0 + static_cast<uint32_t>(j) + 1u; };
    // test hooks (tests/test_host_path.py): a short gate timeout and a host
    // stall before chunk 1 is published exercise the miss -> re-run path
    const char* te = getenv("HRS_GATE_TIMEOUT_US");
    const uint64_t timeout = te && atol(te) > 0 ? c->gate_timeout / 10000000u * static_cast<uint64_t>(atol(te))
                                                : c->gate_timeout;
    const char* de = getenv("HRS_GATE_DELAY_US");
    const long delay_us = de ? atol(de) : 0;
    auto enqueue = [&](size_t j) -> hrs_status {
      const int sl = static_cast<int>(j % S);
      const hipStream_t hs = c->host[sl].stream;
      hipError_t e = hrs::launch_gate(flag_ready(c, sl), tag(j), flag_fail(c), timeout, hs);
      if (e != hipSuccess) return hip_fail(c, e, "gate launch");
      hrs_status s2 = launch(j);
      if (s2 != HRS_OK) return s2;
      e = hrs::launch_signal(flag_done(c, sl), tag(j), hs);
      return e == hipSuccess ? HRS_OK : hip_fail(c, e, "signal launch");
    };
    auto done = [&](size_t j) { return tag_reached(flag_load(flag_done(c, static_cast<int>(j % S))), tag(j)); };
    auto wait_done = [&](size_t j) -> hrs_status {
      for (uint32_t spin = 1; !done(j); ++spin) {
        if ((spin & 4095u) == 0) {  // a failed stream never signals: surface its error
          const hipError_t e = hipStreamQuery(c->host[j % S].stream);
          if (e != hipSuccess && e != hipErrorNotReady) return hip_fail(c, e, "staged chunk");
        }
        __builtin_ia32_pause();
      }
      return HRS_OK;
    };
    for (size_t j = 0; j < static_cast<size_t>(S) && st == HRS_OK; ++j) st = enqueue(j);
    for (size_t j = 0; j < C && st == HRS_OK; ++j) {
      while (st == HRS_OK && out_next + S <= j) {  // the slot's previous chunk must be out
        st = wait_done(out_next);
        if (st == HRS_OK) copy_out(out_next++);
      }
      if (st != HRS_OK) break;
      while (out_next < j && done(out_next)) copy_out(out_next++);
      copy_in(j);
      flush();
      if (j == 1 && delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
      __atomic_store_n(flag_ready(c, static_cast<int>(j % S)), tag(j), __ATOMIC_RELEASE);
      if (j + S < C) st = enqueue(j + S);
    }
    while (st == HRS_OK && out_next < C) {
      st = wait_done(out_next);
      if (st == HRS_OK) copy_out(out_next++);
      while (out_next < C && done(out_next)) copy_out(out_next++);
      flush();
    }
    jobs.clear();
    if (st != HRS_OK) {  // open every gate of this call so its queued work drains
      for (int sl = 0; sl < S; ++sl) __atomic_store_n(flag_ready(c, sl), tag0 + static_cast<uint32_t>(C), __ATOMIC_RELEASE);
      return st;
    }
    if (__atomic_load_n(flag_fail(c), __ATOMIC_ACQUIRE)) {
      __atomic_store_n(flag_fail(c), 0u, __ATOMIC_RELEASE);
      *missed = true;
      return HRS_OK;
    }
  } else {
    auto ev = [&](size_t j) { return c->host[j % S].done; };
    for (size_t j = 0; j < C; ++j) {
      while (out_next + S <= j) {  // the slot's previous chunk must be out
        hipError_t e = hipEventSynchronize(ev(out_next));
        if (e != hipSuccess) return hip_fail(c, e, "hipEventSynchronize");
        copy_out(out_next++);
      }
      while (out_next < j && hipEventQuery(ev(out_next)) == hipSuccess) copy_out(out_next++);
      copy_in(j);
      flush();
      st = launch(j);
      if (st != HRS_OK) return st;
      hipError_t e = hipEventRecord(ev(j), c->host[j % S].stream);
      if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
    }
    while (out_next < C) {
      hipError_t e = hipEventSynchronize(ev(out_next));
      if (e != hipSuccess) return hip_fail(c, e, "hipEventSynchronize");
      copy_out(out_next++);
      while (out_next < C && hipEventQuery(ev(out_next)) == hipSuccess) copy_out(out_next++);
      flush();
    }
  }
  if (c->staged_shapes.size() > 256) c->staged_shapes.clear();
  for (const Span& sp : ch) c->staged_shapes.insert(shape(sp.len));
  for (size_t j = 0; j < C && ncrc; ++j) {  // CRC32.update chaining over the chunks in column order
    const hrs::crc::Mat& z = crc_zmat(c, ch[j].len);
    for (int r = 0; r < ncrc; ++r) crc.out[r] = hrs::crc::apply(z, crc.out[r]) ^ parts[j * ncrc + r];
  }
  return HRS_OK;
}

hrs_status host_apply_impl(hrs_codec* c, const uint8_t* m, int nout, int nin, const uint8_t* const* in_rows,
                           uint8_t* const* out_rows, size_t len, bool static_kp, const HostCrc& crc) {
  const int ncrc = crc.mode == kCrcEncode ? nin + nout : crc.mode == kCrcOutputs ? nout : 0;
  if (ncrc > 0) {  // the running values; an empty call leaves them as they are
    for (int r = 0; r < ncrc; ++r) crc.out[r] = crc.in ? crc.in[r] : 0u;
  }
  if (len == 0 || nout == 0) return HRS_OK;
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
  std::vector<int> slot_of(nin, -1);  // staging row of each live input
  int nlive = 0;
  for (int i = 0; i < nin; ++i) {
    bool any = crc.mode == kCrcEncode;  // every source is checksummed
    for (int o = 0; o < nout; ++o) any |= m[o * nin + i] != 0;
    if (!any) continue;
    if (!in_rows[i]) return fail(c, HRS_EINVAL, "input row %d is NULL", i);
    slot_of[i] = nlive++;
  }
  for (int o = 0; o < nout; ++o)
    if (!out_rows[o]) return fail(c, HRS_EINVAL, "output row %d is NULL", o);
  {
    std::vector<const uint8_t*> live_rows(nin);
    for (int i = 0; i < nin; ++i) live_rows[i] = slot_of[i] >= 0 ? in_rows[i] : nullptr;
    hrs_status st = HRS_OK;
    if (host_apply_pinned(c, m, nout, nin, live_rows.data(), out_rows, len, static_kp, crc, ncrc, &st)) return st;
  }
  std::vector<uint32_t> start(crc.out, crc.out + ncrc);  // crc.out may alias crc.in: kept for a re-run
  bool missed = false;
  hrs_status st = staged_run(c, m, nout, nin, in_rows, out_rows, len, static_kp, crc, ncrc, slot_of, nlive,
                             host_gate_on(), &missed);
  if (st == HRS_OK && missed) {  // a gate gave up waiting: discard everything and run it without gates
    std::copy(start.begin(), start.end(), crc.out);
    st = staged_run(c, m, nout, nin, in_rows, out_rows, len, static_kp, crc, ncrc, slot_of, nlive, false, &missed);
  }
  return st;
}

// A call that fails part-way may leave a slot's H2D / kernel / D2H in
// flight; the next call would then memcpy into staging the DMA engine is
// still reading or writing. So a failed call drains both slot streams before
// it returns (a successful one has already waited for every slot it used).
hrs_status host_apply(hrs_codec* c, const uint8_t* m, int nout, int nin, const uint8_t* const* in_rows,
                      uint8_t* const* out_rows, size_t len, bool static_kp, const HostCrc& crc = HostCrc()) {
  const hrs_status st = host_apply_impl(c, m, nout, nin, in_rows, out_rows, len, static_kp, crc);
  if (st != HRS_OK)
    for (auto& h : c->host)
      if (h.stream) (void)hipStreamSynchronize(h.stream);
  return st;
}

// ---------------------------------------- asynchronous host-buffer calls
// An Encoder / Decoder round split in two: submit copies the caller's rows
// into a free slot's pinned staging (the rows may be reused as soon as it
// returns: Java heap arrays are pinned only for the call) and queues H2D ->
// kernel -> D2H on the slot's stream; collect waits for that operation and
// copies its output rows (and chained CRCs) out. While round r runs on the
// GPU the caller reads round r + 1 and submits it, so successive rounds
// overlap (Encoder.java:421-453 runs them back to back).

hrs_status async_slot(hrs_codec* c, hrs_codec::AsyncSlot& a, size_t bytes) {
  if (!a.stream) {
    hipError_t e = hipStreamCreateWithFlags(&a.stream, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail(c, e, "hipStreamCreate");
    e = hipEventCreateWithFlags(&a.done, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventCreate");
  }
  if (a.bytes >= bytes) return HRS_OK;
  (void)hipStreamSynchronize(a.stream);
  if (a.dev) (void)hipFree(a.dev);
  if (a.pin) (void)hipHostFree(a.pin);
  a.dev = nullptr;
  a.pin = nullptr;
  a.pin_dev = nullptr;
  a.bytes = 0;
  hipError_t e = hipMalloc(&a.dev, bytes);
  if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
  e = hipHostMalloc(&a.pin, bytes, hipHostMallocDefault);
  if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
  if (!host_device_ptr(a.pin, bytes, &a.pin_dev)) a.pin_dev = nullptr;
  a.bytes = bytes;
  return HRS_OK;
}

hrs_status async_submit_impl(hrs_codec* c, hrs_codec::AsyncSlot& a, const uint8_t* m, int nout, int nin,
                             const uint8_t* const* in_rows, size_t len, bool static_kp, int crc_mode) {
  const int ncrc = crc_mode == kCrcEncode ? nin + nout : crc_mode == kCrcOutputs ? nout : 0;
  std::vector<int> slot_of(nin, -1);
  int nlive = 0;
  for (int i = 0; i < nin; ++i) {
    bool any = crc_mode == kCrcEncode;
    for (int o = 0; o < nout; ++o) any |= m[o * nin + i] != 0;
    if (!any) continue;
    if (!in_rows[i]) return fail(c, HRS_EINVAL, "input row %d is NULL", i);
    slot_of[i] = nlive++;
  }
  const size_t pitch = pitch_for(len);
  const size_t crc_off = pitch * static_cast<size_t>(nlive + nout);
  const size_t raw_off = crc_off + ((ncrc * sizeof(uint32_t) + 255) & ~static_cast<size_t>(255));
  const size_t need = ncrc ? raw_off + crc_raw_bytes_for(len, 1, ncrc) : crc_off;
  hrs_status st = async_slot(c, a, need);
  if (st != HRS_OK) return st;
  std::vector<hrs::CopyJob> jobs;
  for (int i = 0; i < nin; ++i)
    if (slot_of[i] >= 0) jobs.push_back({a.pin + pitch * slot_of[i], in_rows[i], len, host_store_mode()});
  copy_pool(c).run(jobs);
  uint8_t* const zpin = a.pin_dev;  // zero copy, as host_apply_impl
  const bool zc = zero_copy_on() && zpin &&
                  (crc_mode == kCrcEncode  ? encode_crc_one_pass(c, len, 1)
                   : crc_mode == kCrcOutputs ? apply_crc_one_pass(c, nout, nlive, len)
                                             : true);
  hrs::GridCap cap(zc ? zero_copy_blocks() : 0u);
  a.timed = false;
  if (c->timing) {
    for (hipEvent_t* ev : {&a.t_start, &a.t_end})
      if (!*ev) {
        hipError_t e = hipEventCreate(ev);
        if (e != hipSuccess) return hip_fail(c, e, "hipEventCreate");
      }
    hipError_t e = hipEventRecord(a.t_start, a.stream);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
    a.timed = true;
  }
  if (nlive > 0 && !zc) {
    hipError_t e = hipMemcpyAsync(a.dev, a.pin, pitch * (nlive - 1) + len, hipMemcpyHostToDevice, a.stream);
    if (e != hipSuccess) return hip_fail(c, e, "hipMemcpyAsync H2D");
  }
  std::vector<const uint8_t*> din(nin);
  std::vector<uint8_t*> dout(nout);
  uint8_t* img = zc ? zpin : a.dev;
  for (int i = 0; i < nin; ++i) din[i] = slot_of[i] >= 0 ? img + pitch * slot_of[i] : nullptr;
  for (int o = 0; o < nout; ++o) dout[o] = img + pitch * (nlive + o);
  uint32_t* dcrc = reinterpret_cast<uint32_t*>(img + crc_off);
  uint32_t* draw = reinterpret_cast<uint32_t*>(a.dev + raw_off);
  if (crc_mode == kCrcEncode)
    st = encode_crc_impl(c, din.data(), 0, dout.data(), 0, len, 1, nullptr, dcrc, a.stream, draw);
  else if (crc_mode == kCrcOutputs)
    st = apply_crc_impl(c, m, nout, nin, din.data(), 0, dout.data(), 0, len, 1, nullptr, dcrc, a.stream, draw);
  else
    st = run_apply(c, m, nout, nin, din.data(), 0, dout.data(), 0, len, 1, a.stream, static_kp);
  if (st != HRS_OK) return st;
  const size_t back = ncrc ? crc_off + ncrc * sizeof(uint32_t) - pitch * nlive : pitch * (nout - 1) + len;
  hipError_t e = hipSuccess;
  if (!zc) {
    e = hipMemcpyAsync(a.pin + pitch * nlive, a.dev + pitch * nlive, back, hipMemcpyDeviceToHost, a.stream);
    if (e != hipSuccess) return hip_fail(c, e, "hipMemcpyAsync D2H");
  }
  if (a.timed && (e = hipEventRecord(a.t_end, a.stream)) != hipSuccess) return hip_fail(c, e, "hipEventRecord");
  e = hipEventRecord(a.done, a.stream);
  if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
  a.nout = nout;
  a.nlive = nlive;
  a.ncrc = ncrc;
  a.len = len;
  a.pitch = pitch;
  a.crc_off = crc_off;
  a.queued = true;
  return HRS_OK;
}

hrs_status async_submit(hrs_codec* c, const uint8_t* m, int nout, int nin, const uint8_t* const* in_rows, size_t len,
                        bool static_kp, int crc_mode, uint64_t* ticket) {
  if (!ticket) return fail(c, HRS_EINVAL, "ticket is NULL");
  *ticket = 0;
  int free_slot = -1;
  for (int i = 0; i < hrs::kAsyncSlots && free_slot < 0; ++i)
    if (!c->async[i].busy) free_slot = i;
  if (free_slot < 0)
    return fail(c, HRS_EINVAL, "all %d asynchronous slots hold uncollected operations: collect one first",
                hrs::kAsyncSlots);
  hrs_codec::AsyncSlot& a = c->async[free_slot];
  const int ncrc = crc_mode == kCrcEncode ? nin + nout : crc_mode == kCrcOutputs ? nout : 0;
  a.queued = false;
  a.timed = false;
  a.nout = nout;
  a.ncrc = ncrc;
  a.len = len;
  if (len > 0 && nout > 0) {
    DeviceGuard g(c->device);
    if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
    const hrs_status st = async_submit_impl(c, a, m, nout, nin, in_rows, len, static_kp, crc_mode);
    if (st != HRS_OK) {  // leave nothing in flight in a slot marked free
      if (a.stream) (void)hipStreamSynchronize(a.stream);
      a.queued = false;
      return st;
    }
  }
  a.busy = true;
  a.ticket = ++c->async_tickets;
  *ticket = a.ticket;
  return HRS_OK;
}

}  // namespace hrs::api

using namespace hrs::api;

extern "C" {

hrs_status hrs_encode(hrs_codec* c, const uint8_t* const* inputs, uint8_t* const* outputs, size_t len) {
  if (!c) return HRS_EINVAL;
  if (!inputs || !outputs) return fail(c, HRS_EINVAL, "inputs/outputs is NULL");
  return host_apply(c, c->g.data(), c->p, c->k, inputs, outputs, len, static_encode_family(c));
}

hrs_status hrs_encode_crc(hrs_codec* c, const uint8_t* const* inputs, uint8_t* const* outputs, size_t len,
                          const uint32_t* crc_in, uint32_t* crc_out) {
  if (!c) return HRS_EINVAL;
  if (!inputs || !outputs || !crc_out) return fail(c, HRS_EINVAL, "inputs/outputs/crc_out is NULL");
  HostCrc crc;
  crc.mode = kCrcEncode;
  crc.in = crc_in;
  crc.out = crc_out;
  return host_apply(c, c->g.data(), c->p, c->k, inputs, outputs, len, static_encode_family(c), crc);
}

hrs_status hrs_decode_crc(hrs_codec* c, const uint8_t* const* read_bufs, uint8_t* const* write_bufs,
                          const int* erased, int ne, const int* to_read, int nr, const int* ntr, int nn, size_t len,
                          const uint32_t* crc_in, uint32_t* crc_out) {
  if (!c) return HRS_EINVAL;
  (void)to_read;
  if (!read_bufs || (ne > 0 && (!write_bufs || !erased || !crc_out)) || ne < 0 || nn < 0 || nr < 0 ||
      (nn > 0 && !ntr))
    return fail(c, HRS_EINVAL, "bad decode arguments");
  if (!decode_locations_ok(c, erased, ne, to_read, nr, ntr, nn))
    return fail(c, HRS_EINVAL, "location out of range [0,%d)", c->n);
  if (ne == 0) return HRS_OK;
  std::vector<uint8_t> tmp;
  const uint8_t* d = nullptr;
  hrs_status st = decode5_matrix(c, erased, ne, ntr, nn, read_bufs, tmp, &d, to_read, to_read ? nr : -1);
  if (st != HRS_OK) return st;
  HostCrc crc;
  crc.mode = kCrcOutputs;
  crc.in = crc_in;
  crc.out = crc_out;
  return host_apply(c, d, ne, c->n, read_bufs, write_bufs, len, false, crc);
}

hrs_status hrs_decode(hrs_codec* c, const uint8_t* const* read_bufs, uint8_t* const* write_bufs, const int* erased,
                      int ne, const int* to_read, int nr, const int* ntr, int nn, size_t len) {
  if (!c) return HRS_EINVAL;
  (void)to_read;
  if (!read_bufs || (ne > 0 && (!write_bufs || !erased)) || ne < 0 || nn < 0 || nr < 0 || (nn > 0 && !ntr))
    return fail(c, HRS_EINVAL, "bad decode arguments");
  if (!decode_locations_ok(c, erased, ne, to_read, nr, ntr, nn))
    return fail(c, HRS_EINVAL, "location out of range [0,%d)", c->n);
  if (ne == 0 && c->kind == HRS_CODE_RS) return HRS_OK;
  std::vector<uint8_t> tmp;
  const uint8_t* d = nullptr;
  hrs_status st = decode5_matrix(c, erased, ne, ntr, nn, read_bufs, tmp, &d, to_read, to_read ? nr : -1);
  if (st != HRS_OK) return st;
  return host_apply(c, d, ne, c->n, read_bufs, write_bufs, len, false);
}

hrs_status hrs_decode3(hrs_codec* c, const uint8_t* const* read_bufs, uint8_t* const* write_bufs, const int* erased,
                       int ne, size_t len) {
  if (!c) return HRS_EINVAL;
  if (ne < 0 || (ne > 0 && (!read_bufs || !write_bufs || !erased))) return fail(c, HRS_EINVAL, "bad decode3 arguments");
  if (c->kind == HRS_CODE_XOR) {  // XORCode.decodeBulk 3-arg == 5-arg (XORCode.java:140-145)
    std::vector<uint8_t> tmp;
    const uint8_t* d = nullptr;
    hrs_status st = decode5_matrix(c, erased, ne, nullptr, 0, read_bufs, tmp, &d);
    if (st != HRS_OK) return st;
    return host_apply(c, d, ne, c->n, read_bufs, write_bufs, len, false);
  }
  if (c->kind == HRS_CODE_NRS || c->kind == HRS_CODE_SRC)  // only ReedSolomonCode / XORCode have it
    return fail(c, HRS_EINVAL, "decodeBulk(readBufs, writeBufs, erasedLocations) is not supported by this code");
  if (ne == 0) return HRS_OK;  // ReedSolomonCode.java:170-172
  if (ne > c->p) return fail(c, HRS_EINVAL, "%d erasures > parity size %d", ne, c->p);  // errSignature[p]
  hrs_status st;
  const std::vector<uint8_t>* d = cached_decode_matrix(c, erased, ne, erased, ne, 0, &st);
  if (!d) return st;
  return host_apply(c, d->data(), ne, c->n, read_bufs, write_bufs, len, false);
}

hrs_status hrs_encode_submit(hrs_codec* c, const uint8_t* const* inputs, size_t len, int checksums, uint64_t* ticket) {
  if (!c) return HRS_EINVAL;
  if (!inputs) return fail(c, HRS_EINVAL, "inputs is NULL");
  return async_submit(c, c->g.data(), c->p, c->k, inputs, len, static_encode_family(c),
                      checksums ? kCrcEncode : kCrcNone, ticket);
}

hrs_status hrs_decode_submit(hrs_codec* c, const uint8_t* const* read_bufs, const int* erased, int ne,
                             const int* to_read, int nr, const int* ntr, int nn, size_t len, int checksums,
                             uint64_t* ticket) {
  if (!c) return HRS_EINVAL;
  if (!read_bufs || ne < 0 || nn < 0 || nr < 0 || (ne > 0 && !erased) || (nn > 0 && !ntr))
    return fail(c, HRS_EINVAL, "bad decode arguments");
  if (!decode_locations_ok(c, erased, ne, to_read, nr, ntr, nn))
    return fail(c, HRS_EINVAL, "location out of range [0,%d)", c->n);
  std::vector<uint8_t> tmp;
  const uint8_t* d = nullptr;
  if (ne > 0) {
    hrs_status st = decode5_matrix(c, erased, ne, ntr, nn, read_bufs, tmp, &d, to_read, to_read ? nr : -1);
    if (st != HRS_OK) return st;
  }
  return async_submit(c, d, ne, c->n, read_bufs, ne > 0 ? len : 0, false, checksums ? kCrcOutputs : kCrcNone, ticket);
}

hrs_status hrs_collect(hrs_codec* c, uint64_t ticket, uint8_t* const* outputs, uint32_t* crc_io) {
  if (!c) return HRS_EINVAL;
  hrs_codec::AsyncSlot* a = nullptr;
  for (auto& s : c->async)
    if (s.busy && s.ticket == ticket) a = &s;
  if (!a) return fail(c, HRS_EINVAL, "no uncollected operation with ticket %llu", static_cast<unsigned long long>(ticket));
  if (a->nout > 0 && a->len > 0 && !outputs) return fail(c, HRS_EINVAL, "outputs is NULL");
  if (a->ncrc > 0 && !crc_io) return fail(c, HRS_EINVAL, "crc_io is NULL for a checksummed operation");
  for (int o = 0; o < a->nout && a->len > 0; ++o)
    if (!outputs[o]) return fail(c, HRS_EINVAL, "output row %d is NULL", o);
  hrs_status st = HRS_OK;
  if (a->queued) {
    hipError_t e = hipEventSynchronize(a->done);
    if (e != hipSuccess) {
      // the slot's H2D / kernel / D2H may still be in flight: drain its stream
      // before the slot is marked free, so the next submit cannot refill
      // staging the DMA engine is still using
      st = hip_fail(c, e, "hipEventSynchronize");
      DeviceGuard g(c->device);
      (void)hipStreamSynchronize(a->stream);
    }
  }
  if (st == HRS_OK && a->queued) {
    std::vector<hrs::CopyJob> jobs;
    for (int o = 0; o < a->nout; ++o) jobs.push_back({outputs[o], a->pin + a->pitch * (a->nlive + o), a->len});
    copy_pool(c).run(jobs);
  }
  if (st == HRS_OK && a->ncrc > 0 && a->queued) {  // CRC32.update chaining: crc = Z_len(crc) ^ crc(cell)
    const uint32_t* part = reinterpret_cast<const uint32_t*>(a->pin + a->crc_off);
    const hrs::crc::Mat& z = crc_zmat(c, a->len);
    for (int r = 0; r < a->ncrc; ++r) crc_io[r] = hrs::crc::apply(z, crc_io[r]) ^ part[r];
  }
  a->busy = false;
  a->queued = false;
  return st;
}

hrs_status hrs_wait(hrs_codec* c, uint64_t ticket) {
  if (!c) return HRS_EINVAL;
  for (auto& s : c->async)
    if (s.busy && s.ticket == ticket) {
      if (!s.queued) return HRS_OK;
      hipError_t e = hipEventSynchronize(s.done);
      return e == hipSuccess ? HRS_OK : hip_fail(c, e, "hipEventSynchronize");
    }
  return fail(c, HRS_EINVAL, "no uncollected operation with ticket %llu", static_cast<unsigned long long>(ticket));
}

hrs_status hrs_release(hrs_codec* c, uint64_t ticket) {
  if (!c) return HRS_EINVAL;
  for (auto& s : c->async)
    if (s.busy && s.ticket == ticket) {
      hrs_status st = HRS_OK;
      if (s.queued) {  // nothing of this round may still read or write the slot's staging
        DeviceGuard g(c->device);
        const hipError_t e = hipStreamSynchronize(s.stream);
        if (e != hipSuccess) st = hip_fail(c, e, "hipStreamSynchronize");
      }
      s.busy = false;
      s.queued = false;
      return st;
    }
  return fail(c, HRS_EINVAL, "no uncollected operation with ticket %llu", static_cast<unsigned long long>(ticket));
}

hrs_status hrs_ticket_shape(const hrs_codec* c, uint64_t ticket, int* num_outputs, size_t* len, int* num_crcs) {
  if (!c) return HRS_EINVAL;
  for (const auto& s : c->async)
    if (s.busy && s.ticket == ticket) {
      if (num_outputs) *num_outputs = s.nout;
      if (len) *len = s.len;
      if (num_crcs) *num_crcs = s.ncrc;
      return HRS_OK;
    }
  return HRS_EINVAL;
}

hrs_status hrs_set_timing(hrs_codec* c, int on) {
  if (!c) return HRS_EINVAL;
  c->timing = on != 0;
  return HRS_OK;
}

hrs_status hrs_ticket_gpu_ms(const hrs_codec* cc, uint64_t ticket, float* ms) {
  auto* c = const_cast<hrs_codec*>(cc);
  if (!c || !ms) return HRS_EINVAL;
  for (auto& s : c->async)
    if (s.busy && s.ticket == ticket) {
      if (!s.queued || !s.timed) return fail(c, HRS_EINVAL, "operation %llu was submitted without timing",
                                             static_cast<unsigned long long>(ticket));
      DeviceGuard g(c->device);
      const hipError_t e = hipEventElapsedTime(ms, s.t_start, s.t_end);
      return e == hipSuccess ? HRS_OK : hip_fail(c, e, "hipEventElapsedTime");
    }
  return fail(c, HRS_EINVAL, "no uncollected operation with ticket %llu", static_cast<unsigned long long>(ticket));
}

int hrs_pending(const hrs_codec* c) {
  if (!c) return -1;
  int n = 0;
  for (const auto& s : c->async) n += s.busy;
  return n;
}

}  // extern "C"
