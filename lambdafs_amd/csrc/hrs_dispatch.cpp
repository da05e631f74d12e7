// Device-resident dispatch: the matrix-apply planner that picks a gfx950
// kernel per shape (static encode, XOR, resident / pipelined / streaming
// runtime kernels, byte-granular tails), the CRC-32 machinery (LDS table
// images, fold tables, raw-CRC scratch, fused encode + CRC), and the hrs_*_dev
// entry points.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/hrs.h"
#include "hrs_codec.hpp"
#include "crc32.hpp"
#include "hrs_crc.hpp"
#include "hrs_internal.hpp"

namespace hrs::api {

using hrs::RowArgs;

// out_o = XOR_i m[o][i] * in_i for every stripe. `static_kp` allows the
// compile-time encode kernels when m is this codec's G and inputs are the k
// data rows in order.
hrs_status run_apply(hrs_codec* c, const uint8_t* m, int nout, int nin, const uint8_t* const* in_rows,
                     size_t in_stride, uint8_t* const* out_rows, size_t out_stride, size_t len,
                     size_t nstripes, hipStream_t s, bool static_kp) {
  if (nout < 0 || nin < 0 || nout > 255 || nin > 255) return fail(c, HRS_EINVAL, "bad matrix shape %dx%d", nout, nin);
  if (nout == 0 || len == 0 || nstripes == 0) return HRS_OK;
  for (int o = 0; o < nout; ++o)
    if (!out_rows[o]) return fail(c, HRS_EINVAL, "output row %d is NULL", o);
  // Inputs whose coefficients are zero for every output contribute nothing:
  // skip them (saves their HBM reads; exact, since 0 * x = 0).
  std::vector<int> live;
  for (int i = 0; i < nin; ++i) {
    bool any = false;
    for (int o = 0; o < nout; ++o) any |= m[o * nin + i] != 0;
    if (any) {
      if (!in_rows[i]) return fail(c, HRS_EINVAL, "input row %d is NULL but has nonzero coefficients", i);
      live.push_back(i);
    }
  }
  if (static_cast<int>(live.size()) != nin || !static_encode_family(c) || m != c->g.data()) static_kp = false;
  bool vec_ok = (in_stride % 16 == 0) && (out_stride % 16 == 0);
  for (int i : live) vec_ok &= aligned16(in_rows[i]);
  for (int o = 0; o < nout; ++o) vec_ok &= aligned16(out_rows[o]);
  const int mode = c->kernel_mode;
  if (mode == 2) vec_ok = false;
  if (mode == 1 || mode == 2) static_kp = false;

  const uint64_t nwin = vec_ok ? len / hrs::kWindowBytes : 0;
  const uint64_t tail_off = nwin * hrs::kWindowBytes;
  const uint64_t tail = len - tail_off;

  if (live.empty()) {  // all-zero matrix: outputs are zero
    for (int o = 0; o < nout; ++o)
      for (size_t st = 0; st < nstripes; ++st) {
        hipError_t e = hipMemsetAsync(out_rows[o] + st * out_stride, 0, len, s);
        if (e != hipSuccess) return hip_fail(c, e, "hipMemsetAsync");
      }
    return HRS_OK;
  }

  if (static_kp && nwin > 0) {
    RowArgs a{};
    for (int i = 0; i < nin; ++i) a.in[i] = in_rows[i];
    for (int o = 0; o < nout; ++o) a.out[o] = out_rows[o];
    a.in_stride = in_stride;
    a.out_stride = out_stride;
    a.len = len;
    a.nwin = nwin;
    a.ntasks = nwin * nstripes;
    a.nin = nin;
    a.nout = nout;
    bool handled = false;
    const int family = c->kind == HRS_CODE_NRS ? hrs::kStaticCauchy : hrs::kStaticRs;
    hipError_t e = hrs::launch_static_encode(family, c->k, c->p, a, s, &handled);
    if (e != hipSuccess) return hip_fail(c, e, "static encode launch");
    if (handled) {
      c->last_kernel = hrs::last_kernel();
      if (tail == 0) return HRS_OK;
      std::vector<const uint8_t*> tin(nin);
      std::vector<uint8_t*> tout(nout);
      for (int i = 0; i < nin; ++i) tin[i] = in_rows[i] + tail_off;
      for (int o = 0; o < nout; ++o) tout[o] = out_rows[o] + tail_off;
      // tail < one window: run_apply sends it to the byte-granular kernel
      return run_apply(c, m, nout, nin, tin.data(), in_stride, tout.data(), out_stride, tail, nstripes, s, false);
    }
  }

  const int nlive = static_cast<int>(live.size());
  // A single output whose live coefficients are all 1 is a plain XOR of rows
  // (the XOR code, XORCode.java:99-145): no bit-slicing needed.
  bool all_ones = (nout == 1) && nwin > 0 && mode == 0;
  for (int i : live) all_ones &= m[i] == 1;
  if (all_ones) {
    for (int i0 = 0; i0 < nlive; i0 += hrs::kMaxInRuntime) {
      const int ni = std::min(hrs::kMaxInRuntime, nlive - i0);
      RowArgs a{};
      for (int i = 0; i < ni; ++i) a.in[i] = in_rows[live[i0 + i]];
      a.out[0] = out_rows[0];
      a.in_stride = in_stride;
      a.out_stride = out_stride;
      a.len = len;
      a.nwin = nwin;
      a.ntasks = nwin * nstripes;
      a.nin = ni;
      a.nout = 1;
      a.accumulate = i0 > 0;
      hipError_t e = hrs::launch_xor(a, s);
      if (e != hipSuccess) return hip_fail(c, e, "xor launch");
      c->last_kernel = hrs::last_kernel();
      if (tail > 0) {
        RowArgs b = a;
        for (int i = 0; i < ni; ++i) {
          b.in[i] = a.in[i] + tail_off;
          hrs::set_coef(b, 0, i, 1);
        }
        b.out[0] = a.out[0] + tail_off;
        b.len = tail;
        b.nwin = 0;
        b.ntasks = tail * nstripes;
        e = hrs::launch_bytewise(b, s);
        if (e != hipSuccess) return hip_fail(c, e, "bytewise launch");
      }
    }
    return HRS_OK;
  }
  // Shapes the register-resident kernels would take in several launches go to
  // the streaming kernel (each input read once, each output written once, up
  // to kMaxIn inputs per launch), and so do 13-16 inputs with 3+ outputs, where
  // holding all 16 rows costs the resident kernel its occupancy (RS(16,4)
  // encode 4.50 -> 3.03 ms; 1-2 outputs and <= 12 inputs stay resident, where
  // streaming measured equal or slower: profiles/r02/stream). HRS_STREAM=0
  // keeps the chunked launches, 2 streams every runtime-matrix launch.
  static const int stream_mode = [] {
    const char* e = getenv("HRS_STREAM");
    return e ? atoi(e) : 1;
  }();
  const bool stream_ok = stream_mode != 0;
  for (int o0 = 0; o0 < nout; o0 += hrs::kMaxOut) {
    const int no = std::min(hrs::kMaxOut, nout - o0);
    const int resident = hrs::runtime_in_chunk(no);
    const bool stream = stream_ok && mode == 0 && nwin > 0 &&
                        (nlive > resident || (nlive > 12 && no >= 3) || stream_mode == 2);
    const int chunk = stream ? hrs::kMaxIn : resident;
    for (int i0 = 0; i0 < nlive; i0 += chunk) {
      const int ni = std::min(chunk, nlive - i0);
      RowArgs a{};
      for (int i = 0; i < ni; ++i) a.in[i] = in_rows[live[i0 + i]];
      for (int o = 0; o < no; ++o) {
        a.out[o] = out_rows[o0 + o];
        for (int i = 0; i < ni; ++i) hrs::set_coef(a, o, i, m[(o0 + o) * nin + live[i0 + i]]);
      }
      a.in_stride = in_stride;
      a.out_stride = out_stride;
      a.nin = ni;
      a.nout = no;
      a.accumulate = i0 > 0;
      if (nwin > 0) {
        a.len = len;
        a.nwin = nwin;
        a.ntasks = nwin * nstripes;
        hipError_t e = stream ? hrs::launch_bitsliced_stream(a, s) : hrs::launch_bitsliced(a, s);
        if (e != hipSuccess) return hip_fail(c, e, "bitsliced launch");
        c->last_kernel = hrs::last_kernel();
      }
      if (tail > 0) {
        RowArgs b = a;
        for (int i = 0; i < ni; ++i) b.in[i] = a.in[i] + tail_off;
        for (int o = 0; o < no; ++o) b.out[o] = a.out[o] + tail_off;
        b.len = tail;
        b.nwin = 0;
        b.ntasks = tail * nstripes;
        hipError_t e = hrs::launch_bytewise(b, s);
        if (e != hipSuccess) return hip_fail(c, e, "bytewise launch");
      }
    }
  }
  return HRS_OK;
}

// ------------------------------------------------------------------ CRC-32

hrs_status upload(hrs_codec* c, const std::vector<uint32_t>& h, uint32_t** out) {
  hipError_t e = hipMalloc(out, h.size() * 4);
  if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipMalloc: %s", hipGetErrorString(e));
  e = hipMemcpy(*out, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(c, e, "hipMemcpy tables");
  return HRS_OK;
}

// The window kernels' LDS image (hrs_crc.hpp crc_window_image), uploaded once.
hrs_status crc_image(hrs_codec* c, uint64_t piece, uint64_t chunk, uint32_t** out) {
  if (*out) return HRS_OK;
  return upload(c, hrs::crc_window_image(piece, chunk), out);
}

hrs_status crc_window_tables(hrs_codec* c) {
  return crc_image(c, hrs::crc::kPieceBytes, hrs::crc::kChunkBytes, &c->crc_tables_a);
}

// Fold tables for rows of `len` bytes cut in windows of `win` bytes (32 KiB,
// or a smaller fused window), keyed by (len, win). At most kFoldCacheMax
// entries; a new key evicts the least recently used one once the latest fold
// that read it on EVERY stream that used it has completed (FoldTables::uses:
// one event per stream, re-recorded by each fold on that stream). A table is
// shared by the handle's slot streams and callers' streams, and no fold waits
// on another stream's (a cross-stream wait on every fold cost the host-buffer
// calls up to 2x, profiles/r04/NOTES.md). The host waits only for those
// events (hipFree itself may still synchronize the device).
constexpr size_t kFoldCacheMax = 64;

hrs_status crc_fold_tables(hrs_codec* c, uint64_t len, uint64_t win, hrs_codec::FoldTables** out) {
  const uint64_t key = len << 5 | static_cast<uint64_t>(__builtin_ctzll(win));
  auto it = c->crc_fold_tables.find(key);
  if (it != c->crc_fold_tables.end()) {
    it->second.tick = ++c->crc_fold_tick;
    *out = &it->second;
    return HRS_OK;
  }
  namespace cr = hrs::crc;
  const uint64_t nwin = len / win, tail = len % win;
  const uint64_t G = (nwin + 63) / 64;
  std::vector<uint32_t> h(hrs::kCrcLdsWordsB);
  cr::to_tables(cr::zeros(win), &h[0]);
  for (int t = 0; t < 6; ++t) cr::to_tables(cr::zeros(win * G << t), &h[(1 + t) * 1024]);
  cr::to_tables(cr::zeros(tail), &h[7 * 1024]);
  cr::to_tables(cr::zeros(len), &h[8 * 1024]);
  if (c->crc_fold_tables.size() >= kFoldCacheMax) {
    auto lru = c->crc_fold_tables.begin();
    for (auto i = c->crc_fold_tables.begin(); i != c->crc_fold_tables.end(); ++i)
      if (i->second.tick < lru->second.tick) lru = i;
    hrs_codec::FoldTables& v = lru->second;
    for (auto& u : v.uses) {
      hipError_t e = hipEventSynchronize(u.ev);
      if (e != hipSuccess) return hip_fail(c, e, "hipEventSynchronize");
    }
    for (auto& u : v.uses) (void)hipEventDestroy(u.ev);
    (void)hipFree(v.dev);
    c->crc_fold_tables.erase(lru);
  }
  hrs_codec::FoldTables v;
  hrs_status st = upload(c, h, &v.dev);
  if (st != HRS_OK) {
    if (v.dev) (void)hipFree(v.dev);
    return st;
  }
  v.tick = ++c->crc_fold_tick;
  *out = &(c->crc_fold_tables[key] = v);
  return HRS_OK;
}

// Records that a fold on stream s read the tables (after its launch). At most
// kFoldUsesMax streams are tracked per table; a further one first waits for
// the oldest tracked use and takes over its event.
constexpr size_t kFoldUsesMax = 32;

hrs_status fold_tables_used(hrs_codec* c, hrs_codec::FoldTables* ft, hipStream_t s) {
  hrs_codec::FoldTables::Use* u = nullptr;
  for (auto& x : ft->uses)
    if (x.stream == s) u = &x;
  if (!u && ft->uses.size() >= kFoldUsesMax) {  // many caller streams: retire the oldest use
    hrs_codec::FoldTables::Use old = ft->uses.front();
    ft->uses.erase(ft->uses.begin());
    const hipError_t e = hipEventSynchronize(old.ev);
    if (e != hipSuccess) {
      (void)hipEventDestroy(old.ev);
      return hip_fail(c, e, "hipEventSynchronize");
    }
    ft->uses.push_back({s, old.ev});
    u = &ft->uses.back();
  }
  if (!u) {
    hrs_codec::FoldTables::Use nu{s, nullptr};
    const hipError_t e = hipEventCreateWithFlags(&nu.ev, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventCreate");
    ft->uses.push_back(nu);
    u = &ft->uses.back();
  }
  const hipError_t e = hipEventRecord(u->ev, s);
  return e == hipSuccess ? HRS_OK : hip_fail(c, e, "hipEventRecord");
}

// Raw-CRC scratch of at least `bytes` (the fold reads it after the window
// pass), shared by every device CRC call on this handle whatever its stream.
// Uses are chained: a call on stream s first waits (on the GPU) for the event
// recorded after the previous use, and records it again when its own
// launches are queued (crc_scratch_release). So the last event covers every
// earlier use, and growing the buffer waits for that event before hipFree.
hrs_status crc_scratch(hrs_codec* c, size_t bytes, hipStream_t s) {
  bytes = std::max<size_t>(4, bytes);
  if (!c->crc_raw_done) {
    hipError_t e = hipEventCreateWithFlags(&c->crc_raw_done, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventCreate");
  }
  if (c->crc_raw_bytes < bytes) {
    if (c->crc_raw) {
      if (c->crc_raw_used) {
        hipError_t e = hipEventSynchronize(c->crc_raw_done);
        if (e != hipSuccess) return hip_fail(c, e, "hipEventSynchronize");
      }
      (void)hipFree(c->crc_raw);
      c->crc_raw = nullptr;
      c->crc_raw_bytes = 0;
      c->crc_raw_used = false;
    }
    hipError_t e = hipMalloc(&c->crc_raw, bytes);
    if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    c->crc_raw_bytes = bytes;
  }
  if (c->crc_raw_used) {
    hipError_t e = hipStreamWaitEvent(s, c->crc_raw_done, 0);
    if (e != hipSuccess) return hip_fail(c, e, "hipStreamWaitEvent");
  }
  return HRS_OK;
}

hrs_status crc_scratch_release(hrs_codec* c, hipStream_t s, hrs_status st) {
  hipError_t e = hipEventRecord(c->crc_raw_done, s);
  if (e != hipSuccess) return st != HRS_OK ? st : hip_fail(c, e, "hipEventRecord");
  c->crc_raw_used = true;
  return st;
}

// Folds the raw window CRCs (windows of `win` bytes) of nsr (stripe, row)
// pairs into CRC32 values.
hrs_status crc_fold(hrs_codec* c, size_t len, uint64_t nsr, const uint32_t* crc_in, uint32_t* crc_out, hipStream_t s,
                    uint32_t* raw, uint64_t win = hrs::kCrcWindow) {
  hrs_codec::FoldTables* ft = nullptr;
  hrs_status st = crc_fold_tables(c, len, win, &ft);
  if (st != HRS_OK) return st;
  const uint32_t* fold = ft->dev;
  hrs::CrcFoldArgs f{};
  f.raw = raw;
  f.nwin = len / win;
  f.tail = len % win;
  f.nsr = nsr;
  f.G = static_cast<int>((f.nwin + 63) / 64);
  f.tables = fold;
  f.crc_in = crc_in;
  f.crc_out = crc_out;
  hipError_t e = hrs::launch_crc_fold(f, hrs::device_cu_count(), s);
  if (e != hipSuccess) return hip_fail(c, e, "crc fold launch");
  return fold_tables_used(c, ft, s);  // the tables may be freed once this fold has run
}

// Sub-windows (2 KiB) per fused window: 16 (32 KiB) when the job has
// kFusedWavesPerCU waves per CU at that size, else the largest smaller power
// of two that does (down to 1: a job with fewer 2 KiB sub-windows than that
// takes one wave per sub-window). 0: len is not a multiple of 2 KiB.
constexpr uint64_t kFusedWavesPerCU = 8;

uint32_t fused_subs(size_t len, size_t nstripes) {
  if (len == 0 || len % hrs::kWindowBytes) return 0;
  const uint64_t want = kFusedWavesPerCU * static_cast<uint64_t>(hrs::device_cu_count());
  uint32_t subs = 16;
  while (subs > 1 && (len % (subs * hrs::kWindowBytes) || nstripes * (len / (subs * hrs::kWindowBytes)) < want))
    subs >>= 1;
  return subs;
}

// Bytes of raw window-CRC scratch a CRC pass over nrows rows of nstripes
// stripes needs: one word per window, the tail window included, at the
// smallest window any pass may use (a fused 2 KiB window), so the size holds
// for any shorter row or smaller job sized by it.
size_t crc_raw_bytes_for(size_t len, size_t nstripes, int nrows) {
  const uint64_t wpr = (len + hrs::kWindowBytes - 1) / hrs::kWindowBytes;
  return std::max<size_t>(4, nstripes * static_cast<size_t>(nrows) * wpr * 4);
}

// CRC-32 of nrows rows per stripe, row r at rows[r] + stripe * strides[r]:
// window pass + fold, raw window CRCs in `raw` (crc_raw_bytes_for bytes).
// crc_out[s * nrows + r].
hrs_status run_crc(hrs_codec* c, const uint8_t* const* rows, const size_t* strides, int nrows, size_t len,
                   size_t nstripes, const uint32_t* crc_in, uint32_t* crc_out, hipStream_t s, uint32_t* raw) {
  hrs_status st = crc_window_tables(c);
  if (st != HRS_OK) return st;
  const uint64_t nwin = len / hrs::kCrcWindow, tail = len % hrs::kCrcWindow;
  const uint64_t wpr = nwin + (tail ? 1 : 0);
  const int cus = hrs::device_cu_count();
  bool aligned = true;
  for (int r = 0; r < nrows; ++r) aligned &= aligned16(rows[r]) && strides[r] % 16 == 0;
  if (wpr > 0) {
    for (int r0 = 0; r0 < nrows; r0 += hrs::kCrcMaxRows) {
      hrs::CrcWinArgs a{};
      a.nrows = std::min(hrs::kCrcMaxRows, nrows - r0);
      for (int r = 0; r < a.nrows; ++r) {
        a.rows[r] = rows[r0 + r];
        a.stride[r] = strides[r0 + r];
      }
      a.row0 = r0;
      a.nrows_total = nrows;
      a.len = len;
      a.nwin = nwin;
      a.tail = tail;
      a.nstripes = nstripes;
      a.raw = raw;
      a.tables = c->crc_tables_a;
      hipError_t e = hrs::launch_crc_windows(a, aligned, cus, s);
      if (e != hipSuccess) return hip_fail(c, e, "crc window launch");
    }
  }
  return crc_fold(c, len, nstripes * nrows, crc_in, crc_out, s, raw);
}

// Slicing-table copies the fused kernel's lanes spread over: 32 (each lane of
// a 32-lane group on its own LDS bank); HRS_CRC_REP = 16 | 8 | 4 | 2 | 1 reads
// fewer copies (A/B of the replication factor, profiles/r03/ab/NOTES.md; read per call).
uint32_t crc_rep_mask() {
  const char* e = getenv("HRS_CRC_REP");
  const int r = e ? atoi(e) : hrs::kCrcRep;
  return (r >= 1 && r <= hrs::kCrcRep && (r & (r - 1)) == 0) ? static_cast<uint32_t>(r - 1) : hrs::kCrcRep - 1;
}

// Encode + CRC-32 of the k sources and p parities (hrs_encode_crc_dev's
// semantics) with raw window CRCs in `raw` (crc_raw_bytes_for(len, nstripes, n)).
bool encode_crc_one_pass(const hrs_codec* c, size_t len, size_t nstripes) {
  if (!(c->kind == HRS_CODE_RS || c->kind == HRS_CODE_NRS) || !(c->kernel_mode == 0 || c->kernel_mode == 3) ||
      fused_subs(len, nstripes) == 0)
    return false;
  const int k = c->k, p = c->p;  // the shapes hrs_fused.hip instantiates (launch_encode_crc)
  if (c->kind == HRS_CODE_NRS) return (k == 10 && p == 4) || (k == 6 && p == 3);
  return (k == 10 && p == 4) || (k == 6 && p == 3) || (k == 3 && p == 2) || (k == 12 && p == 4);
}

bool apply_crc_one_pass(const hrs_codec* c, int nout, int nlive, size_t len) {
  return (c->kernel_mode == 0 || c->kernel_mode == 3) && len > 0 && len % hrs::kWindowBytes == 0 && nlive >= 1 &&
         nout >= 1 && nout <= 4 && nlive <= (nout == 4 ? 8 : 12);
}

hrs_status encode_crc_impl(hrs_codec* c, const uint8_t* const* in_rows, size_t in_stride, uint8_t* const* out_rows,
                           size_t out_stride, size_t len, size_t nstripes, const uint32_t* crc_in, uint32_t* crc_out,
                           hipStream_t s, uint32_t* raw, uint64_t* host_fold_win) {
  if (host_fold_win) *host_fold_win = 0;
  const int k = c->k, p = c->p, n = c->n;
  // one pass: a static (k, p) of rs / nrs, whole 2 KiB sub-windows, 16-byte aligned rows.
  // A wave walks its window's sub-windows serially over k + p rows (~20 us
  // per 2 KiB sub-window at RS(10,4)), so jobs with few 32 KiB windows take
  // smaller windows (fused_subs) instead of leaving CUs idle.
  const uint32_t subs = fused_subs(len, nstripes);
  bool fused = (c->kind == HRS_CODE_RS || c->kind == HRS_CODE_NRS) && (c->kernel_mode == 0 || c->kernel_mode == 3) &&
               subs > 0 && k <= hrs::kFusedMaxK && p <= hrs::kFusedMaxP && in_stride % 16 == 0 &&
               out_stride % 16 == 0;
  for (int i = 0; i < k && fused; ++i) fused &= aligned16(in_rows[i]);
  for (int o = 0; o < p && fused; ++o) fused &= aligned16(out_rows[o]);
  if (fused) {
    hrs_status st = crc_window_tables(c);
    if (st != HRS_OK) return st;
    hrs::EncodeCrcArgs a{};
    for (int i = 0; i < k; ++i) a.in[i] = in_rows[i];
    for (int o = 0; o < p; ++o) a.out[o] = out_rows[o];
    a.in_stride = in_stride;
    a.out_stride = out_stride;
    a.subs = subs;
    a.rep_mask = crc_rep_mask();
    a.nwin = len / (subs * hrs::kWindowBytes);
    a.nstripes = nstripes;
    a.raw = raw;
    a.tables = c->crc_tables_a;
    bool handled = false;
    const int family = c->kind == HRS_CODE_NRS ? hrs::kStaticCauchy : hrs::kStaticRs;
    hipError_t e = hrs::launch_encode_crc(family, k, p, a, hrs::device_cu_count(), s, &handled);
    if (e != hipSuccess) return hip_fail(c, e, "fused encode+crc launch");
    if (handled) c->last_kernel = hrs::last_kernel();
    if (handled && host_fold_win) {  // the caller folds the raw window CRCs on the host
      *host_fold_win = subs * hrs::kWindowBytes;
      return HRS_OK;
    }
    if (handled) return crc_fold(c, len, nstripes * n, crc_in, crc_out, s, raw, subs * hrs::kWindowBytes);
  }
  // two passes: encode, then the CRC of the k sources and p parities
  hrs_status st = run_apply(c, c->g.data(), p, k, in_rows, in_stride, out_rows, out_stride, len, nstripes, s,
                            static_encode_family(c));
  if (st != HRS_OK) return st;
  std::vector<const uint8_t*> rows(n);
  std::vector<size_t> strides(n);
  for (int i = 0; i < k; ++i) {
    rows[i] = in_rows[i];
    strides[i] = in_stride;
  }
  for (int o = 0; o < p; ++o) {
    rows[k + o] = out_rows[o];
    strides[k + o] = out_stride;
  }
  return run_crc(c, rows.data(), strides.data(), n, len, nstripes, crc_in, crc_out, s, raw);
}

// out_o = XOR_i m[o][i] * in_i for every stripe, plus the CRC-32 of every
// output row (crc_out[s * nout + o], continuing crc_in): the Decoder's repair
// and the checksum of the repaired cells, with raw window CRCs in `raw`
// (crc_raw_bytes_for(len, nstripes, nout)). Fused (hrs_decode_crc.hip) for
// the pipelined repair shapes on whole 2 KiB windows and aligned rows; else
// the apply, then the CRC pass over its outputs.
hrs_status apply_crc_impl(hrs_codec* c, const uint8_t* m, int nout, int nin, const uint8_t* const* in_rows,
                          size_t in_stride, uint8_t* const* out_rows, size_t out_stride, size_t len, size_t nstripes,
                          const uint32_t* crc_in, uint32_t* crc_out, hipStream_t s, uint32_t* raw,
                          uint64_t* host_fold_win) {
  if (host_fold_win) *host_fold_win = 0;
  if (nout < 0 || nin < 0 || nout > 255 || nin > 255) return fail(c, HRS_EINVAL, "bad matrix shape %dx%d", nout, nin);
  if (nout == 0 || nstripes == 0) return HRS_OK;
  for (int o = 0; o < nout; ++o)
    if (!out_rows[o]) return fail(c, HRS_EINVAL, "output row %d is NULL", o);
  std::vector<int> live;
  for (int i = 0; i < nin; ++i) {
    bool any = false;
    for (int o = 0; o < nout; ++o) any |= m[o * nin + i] != 0;
    if (any) live.push_back(i);
  }
  const int nlive = static_cast<int>(live.size());
  bool fused = (c->kernel_mode == 0 || c->kernel_mode == 3) && len > 0 && len % hrs::kWindowBytes == 0 &&
               nlive >= 1 && nout <= 4 && nlive <= (nout == 4 ? 8 : 12) && in_stride % 16 == 0 &&
               out_stride % 16 == 0;
  for (int i : live) fused &= in_rows[i] != nullptr && aligned16(in_rows[i]);
  for (int o = 0; o < nout && fused; ++o) fused &= aligned16(out_rows[o]);
  if (fused) {
    hrs_status st = crc_window_tables(c);
    if (st != HRS_OK) return st;
    hrs::DecodeCrcArgs d{};
    for (int j = 0; j < nlive; ++j) d.r.in[j] = in_rows[live[j]];
    for (int o = 0; o < nout; ++o) {
      d.r.out[o] = out_rows[o];
      for (int j = 0; j < nlive; ++j) hrs::set_coef(d.r, o, j, m[o * nin + live[j]]);
    }
    d.r.in_stride = in_stride;
    d.r.out_stride = out_stride;
    d.r.len = len;
    d.r.nwin = len / hrs::kWindowBytes;
    d.r.ntasks = d.r.nwin * nstripes;
    d.r.nin = nlive;
    d.r.nout = nout;
    d.raw = raw;
    d.tables = c->crc_tables_a;
    bool handled = false;
    hipError_t e = hrs::launch_decode_crc(d, hrs::device_cu_count(), s, &handled);
    if (e != hipSuccess) return hip_fail(c, e, "fused decode+crc launch");
    if (handled) {
      c->last_kernel = hrs::last_kernel();
      if (host_fold_win) {  // the caller folds the raw window CRCs on the host
        *host_fold_win = hrs::kWindowBytes;
        return HRS_OK;
      }
      return crc_fold(c, len, nstripes * nout, crc_in, crc_out, s, raw, hrs::kWindowBytes);
    }
  }
  hrs_status st = run_apply(c, m, nout, nin, in_rows, in_stride, out_rows, out_stride, len, nstripes, s, false);
  if (st != HRS_OK) return st;
  std::vector<size_t> strides(nout, out_stride);
  return run_crc(c, out_rows, strides.data(), nout, len, nstripes, crc_in, crc_out, s, raw);
}

}  // namespace hrs::api

using namespace hrs::api;

extern "C" {

hrs_status hrs_crc32_dev(hrs_codec* c, const uint8_t* const* rows, int nrows, size_t stride, size_t len,
                         size_t nstripes, const uint32_t* crc_in, uint32_t* crc_out, void* stream) {
  if (!c) return HRS_EINVAL;
  if (!rows || !crc_out || nrows < 1 || nrows > 255) return fail(c, HRS_EINVAL, "bad crc32 arguments");
  for (int r = 0; r < nrows; ++r)
    if (!rows[r] && len) return fail(c, HRS_EINVAL, "row %d is NULL", r);
  if (nstripes == 0) return HRS_OK;
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
  std::vector<size_t> strides(nrows, stride);
  hipStream_t s = static_cast<hipStream_t>(stream);
  hrs_status st = crc_scratch(c, crc_raw_bytes_for(len, nstripes, nrows), s);
  if (st != HRS_OK) return st;
  return crc_scratch_release(c, s, run_crc(c, rows, strides.data(), nrows, len, nstripes, crc_in, crc_out, s,
                                           c->crc_raw));
}

hrs_status hrs_encode_crc_dev(hrs_codec* c, const uint8_t* const* in_rows, size_t in_stride, uint8_t* const* out_rows,
                              size_t out_stride, size_t len, size_t nstripes, const uint32_t* crc_in,
                              uint32_t* crc_out, void* stream) {
  if (!c) return HRS_EINVAL;
  if (!in_rows || !out_rows || !crc_out) return fail(c, HRS_EINVAL, "row or crc arrays are NULL");
  for (int i = 0; i < c->k; ++i)
    if (!in_rows[i] && len) return fail(c, HRS_EINVAL, "input row %d is NULL", i);
  for (int o = 0; o < c->p; ++o)
    if (!out_rows[o] && len) return fail(c, HRS_EINVAL, "output row %d is NULL", o);
  if (nstripes == 0) return HRS_OK;
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  hrs_status st = crc_scratch(c, crc_raw_bytes_for(len, nstripes, c->n), s);
  if (st != HRS_OK) return st;
  return crc_scratch_release(
      c, s, encode_crc_impl(c, in_rows, in_stride, out_rows, out_stride, len, nstripes, crc_in, crc_out, s, c->crc_raw));
}

hrs_status hrs_encode_dev(hrs_codec* c, const uint8_t* const* in_rows, size_t in_stride, uint8_t* const* out_rows,
                          size_t out_stride, size_t len, size_t nstripes, void* stream) {
  if (!c) return HRS_EINVAL;
  if (!in_rows || !out_rows) return fail(c, HRS_EINVAL, "row arrays are NULL");
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
  return run_apply(c, c->g.data(), c->p, c->k, in_rows, in_stride, out_rows, out_stride, len, nstripes,
                   static_cast<hipStream_t>(stream), static_encode_family(c));
}

hrs_status hrs_decode_dev(hrs_codec* c, const uint8_t* const* rows, size_t in_stride, uint8_t* const* out_rows,
                          size_t out_stride, const int* erased, int ne, const int* ntr, int nn, size_t len,
                          size_t nstripes, void* stream) {
  if (!c) return HRS_EINVAL;
  if (!rows || ne < 0 || nn < 0 || (ne > 0 && (!out_rows || !erased)) || (nn > 0 && !ntr))
    return fail(c, HRS_EINVAL, "bad decode arguments");
  if (ne == 0 && c->kind == HRS_CODE_RS) return HRS_OK;
  std::vector<uint8_t> tmp;
  const uint8_t* d = nullptr;
  hrs_status st = decode5_matrix(c, erased, ne, ntr, nn, rows, tmp, &d);
  if (st != HRS_OK) return st;
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
  return run_apply(c, d, ne, c->n, rows, in_stride, out_rows, out_stride, len, nstripes,
                   static_cast<hipStream_t>(stream), false);
}

hrs_status hrs_decode_crc_dev(hrs_codec* c, const uint8_t* const* rows, size_t in_stride, uint8_t* const* out_rows,
                              size_t out_stride, const int* erased, int ne, const int* ntr, int nn, size_t len,
                              size_t nstripes, const uint32_t* crc_in, uint32_t* crc_out, void* stream) {
  if (!c) return HRS_EINVAL;
  if (!rows || ne < 0 || nn < 0 || (ne > 0 && (!out_rows || !erased || !crc_out)) || (nn > 0 && !ntr))
    return fail(c, HRS_EINVAL, "bad decode arguments");
  if (ne == 0 || nstripes == 0) return HRS_OK;
  std::vector<uint8_t> tmp;
  const uint8_t* d = nullptr;
  hrs_status st = decode5_matrix(c, erased, ne, ntr, nn, rows, tmp, &d);
  if (st != HRS_OK) return st;
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  st = crc_scratch(c, crc_raw_bytes_for(len, nstripes, ne), s);
  if (st != HRS_OK) return st;
  return crc_scratch_release(c, s, apply_crc_impl(c, d, ne, c->n, rows, in_stride, out_rows, out_stride, len, nstripes,
                                                  crc_in, crc_out, s, c->crc_raw));
}

hrs_status hrs_apply_dev(hrs_codec* c, const uint8_t* m, int nout, int nin, const uint8_t* const* in_rows,
                         size_t in_stride, uint8_t* const* out_rows, size_t out_stride, size_t len, size_t nstripes,
                         void* stream) {
  if (!c) return HRS_EINVAL;
  if (!m || !in_rows || !out_rows || nout < 1 || nin < 1 || nout > 255 || nin > 255)
    return fail(c, HRS_EINVAL, "bad apply arguments");
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
  return run_apply(c, m, nout, nin, in_rows, in_stride, out_rows, out_stride, len, nstripes,
                   static_cast<hipStream_t>(stream), false);
}

}  // extern "C"
