// Batches: heterogeneous repair batches on the device (one erasure pattern
// per stripe, plans uploaded through pinned slots, one batch launch) and the
// host-memory batch pipelines (hrs_decode_batch_host / hrs_encode_batch_host:
// chunks of stripes through a ring of device slots, H2D of exactly the rows
// read, D2H of exactly the rows written).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hrs.h"
#include "hrs_codec.hpp"
#include "hrs_host.hpp"
#include "hrs_internal.hpp"
#include "hrs_launch.hpp"

namespace hrs::api {

// The plans of a heterogeneous repair batch: one per distinct erasure
// pattern (its live survivor locations and packed coefficients), the pattern
// index of every stripe, and each pattern's full ne x n matrix (for the
// per-stripe fallback when a pattern exceeds the batch kernel's shape).
struct BatchPlanSet {
  std::vector<hrs::BatchPlan> plans;
  std::vector<int32_t> pat;
  std::vector<std::vector<uint8_t>> mats;
  bool fused = true;  // every pattern fits one batch_bitsliced launch
  int max_nout = 0, max_nin = 0;
};

hrs_status build_batch_plans(hrs_codec* c, const int* erased, int max_erased, size_t nstripes, BatchPlanSet& ps) {
  std::map<std::vector<int>, int> ids;
  ps.pat.assign(nstripes, 0);
  std::vector<int> key, to_read(c->n), ntr;
  for (size_t s = 0; s < nstripes; ++s) {
    key.clear();
    for (int t = 0; t < max_erased && erased[s * max_erased + t] >= 0; ++t) key.push_back(erased[s * max_erased + t]);
    auto it = ids.find(key);
    if (it != ids.end()) {
      ps.pat[s] = it->second;
      continue;
    }
    const int ne = static_cast<int>(key.size());
    for (int e : key)
      if (e >= c->n) return fail(c, HRS_EINVAL, "stripe %zu: erased location %d out of range", s, e);
    hrs::BatchPlan pl{};
    std::vector<uint8_t> m(static_cast<size_t>(ne) * c->n, 0);
    if (ne > 0) {
      int nr = 0;
      hrs_status st = hrs_locations_to_read_list(c, key.data(), ne, to_read.data(), &nr);
      if (st != HRS_OK) return st;
      ntr.clear();  // Decoder.java:303-338: everything not read, erased included
      for (int l = 0; l < c->n; ++l)
        if (std::find(to_read.begin(), to_read.begin() + nr, l) == to_read.begin() + nr ||
            std::find(key.begin(), key.end(), l) != key.end())
          ntr.push_back(l);
      std::vector<int> tr_sorted(to_read.begin(), to_read.begin() + nr);
      std::sort(tr_sorted.begin(), tr_sorted.end());
      std::vector<uint8_t> tmp;
      const uint8_t* d = nullptr;
      st = decode5_matrix(c, key.data(), ne, ntr.data(), static_cast<int>(ntr.size()), nullptr, tmp, &d,
                          tr_sorted.data(), nr);
      if (st != HRS_OK) return st;
      std::memcpy(m.data(), d, m.size());
      for (int l = 0; l < c->n; ++l) {  // live inputs, ascending location
        bool live = false;
        for (int o = 0; o < ne; ++o) live |= m[static_cast<size_t>(o) * c->n + l] != 0;
        if (!live) continue;
        if (pl.nin < hrs::kBatchMaxIn) {
          pl.loc[pl.nin] = l;
          for (int o = 0; o < ne; ++o)
            pl.cw[pl.nin] |= static_cast<uint64_t>(m[static_cast<size_t>(o) * c->n + l]) << (8 * o);
        }
        ++pl.nin;
      }
    }
    pl.nout = ne;
    if (pl.nin > hrs::kBatchMaxIn) ps.fused = false;
    ps.max_nout = std::max(ps.max_nout, ne);
    ps.max_nin = std::max(ps.max_nin, pl.nin);
    const int id = static_cast<int>(ps.plans.size());
    ids.emplace(key, id);
    ps.plans.push_back(pl);
    ps.mats.push_back(std::move(m));
    ps.pat[s] = id;
  }
  // one launch covers every pattern at (max_nout, max_nin); shapes beyond the
  // register-resident batch kernel take its streaming form (hrs_batch.hip)
  return HRS_OK;
}

// Repairs stripes [s0, s0 + ns) of a batch whose plans live at dplans / dpat
// (device; dpat indexed by the absolute stripe number) on stream hs. `stripes`
// and `out` point at stripe s0. ps.fused == false: one run_apply per stripe.
hrs_status launch_batch(hrs_codec* c, const BatchPlanSet& ps, const hrs::BatchPlan* dplans, const int32_t* dpat,
                        const uint8_t* stripes, size_t row_stride, size_t stripe_stride, uint8_t* out,
                        size_t out_row_stride, size_t out_stripe_stride, size_t len, size_t s0, size_t ns,
                        hipStream_t hs) {
  if (!ps.fused) {
    std::vector<const uint8_t*> rows(c->n);
    std::vector<uint8_t*> outs(hrs::kMaxOut);
    for (size_t i = 0; i < ns; ++i) {
      const int id = ps.pat[s0 + i];
      const hrs::BatchPlan& pl = ps.plans[id];
      if (pl.nout == 0) continue;
      for (int l = 0; l < c->n; ++l) rows[l] = stripes + i * stripe_stride + l * row_stride;
      for (int o = 0; o < pl.nout; ++o) outs[o] = out + i * out_stripe_stride + o * out_row_stride;
      hrs_status st = run_apply(c, ps.mats[id].data(), pl.nout, c->n, rows.data(), 0, outs.data(), 0, len, 1, hs, false);
      if (st != HRS_OK) return st;
    }
    return HRS_OK;
  }
  hrs::BatchArgs a{};
  a.base = stripes;
  a.out = out;
  a.row_stride = row_stride;
  a.stripe_stride = stripe_stride;
  a.out_row_stride = out_row_stride;
  a.out_stripe_stride = out_stripe_stride;
  a.len = len;
  a.plans = dplans;
  a.pat = dpat + s0;
  const bool vec = c->kernel_mode != 2 && aligned16(stripes) && aligned16(out) && row_stride % 16 == 0 &&
                   stripe_stride % 16 == 0 && out_row_stride % 16 == 0 && out_stripe_stride % 16 == 0;
  a.nwin = vec ? len / hrs::kWindowBytes : 0;
  if (a.nwin > 0) {
    a.ntasks = a.nwin * ns;
    hipError_t e = hrs::launch_batch_bitsliced(a, ps.max_nout, ps.max_nin, hs);
    if (e != hipSuccess) return hip_fail(c, e, "batch launch");
    c->last_kernel = hrs::last_kernel();
  }
  a.col0 = a.nwin * hrs::kWindowBytes;
  if (a.col0 < len) {
    a.ntasks = (len - a.col0) * ns;
    hipError_t e = hrs::launch_batch_bytewise(a, hs);
    if (e != hipSuccess) return hip_fail(c, e, "batch bytewise launch");
  }
  return HRS_OK;
}

// Uploads plans + pattern indices through the next of the handle's two
// batch slots (pinned staging + device buffer; a slot is reused once the
// event recorded after its last launch has completed). Returns the device
// copies in *dplans / *dpat; the caller records sl.done after its launches.
hrs_status upload_batch_plans(hrs_codec* c, const BatchPlanSet& ps, hipStream_t hs, hrs_codec::BatchSlot** slot,
                              const hrs::BatchPlan** dplans, const int32_t** dpat) {
  const size_t plan_bytes = ps.plans.size() * sizeof(hrs::BatchPlan);
  const size_t need = plan_bytes + ps.pat.size() * sizeof(int32_t);
  hrs_codec::BatchSlot& sl = c->batch[c->batch_next];
  c->batch_next ^= 1;
  if (sl.pending) {
    hipError_t e = hipEventSynchronize(sl.done);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventSynchronize");
    sl.pending = false;
  }
  if (!sl.done) {
    hipError_t e = hipEventCreateWithFlags(&sl.done, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventCreate");
  }
  if (sl.bytes < need) {
    if (sl.dev) (void)hipFree(sl.dev);
    if (sl.host) (void)hipHostFree(sl.host);
    sl.dev = nullptr;
    sl.host = nullptr;
    sl.bytes = 0;
    const size_t bytes = std::max<size_t>(need, 64 << 10);
    hipError_t e = hipMalloc(&sl.dev, bytes);
    if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    e = hipHostMalloc(&sl.host, bytes, hipHostMallocDefault);
    if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
    sl.bytes = bytes;
  }
  std::memcpy(sl.host, ps.plans.data(), plan_bytes);
  std::memcpy(sl.host + plan_bytes, ps.pat.data(), ps.pat.size() * sizeof(int32_t));
  hipError_t e = hipMemcpyAsync(sl.dev, sl.host, need, hipMemcpyHostToDevice, hs);
  if (e != hipSuccess) return hip_fail(c, e, "hipMemcpyAsync plans");
  *slot = &sl;
  *dplans = reinterpret_cast<const hrs::BatchPlan*>(sl.dev);
  *dpat = reinterpret_cast<const int32_t*>(sl.dev + plan_bytes);
  return HRS_OK;
}

// ------------------------------------------------ host-memory batches
// (hrs_decode_batch_host / hrs_encode_batch_host). Stripes start and end in
// host memory (DataNode sockets, local block files). Chunks of stripes flow
// through a ring of device slots: H2D of exactly the rows the chunk's codes
// read (on the copy-in stream) -> kernel (on the slot's stream) -> D2H of
// exactly the rows they write (on the copy-out stream), chained by events,
// so one chunk's D2H overlaps the next chunks' H2D on the full-duplex link.
// Pinned caller buffers are DMA'd directly and the whole job is queued before
// the host waits once; pageable ones go through each slot's pinned staging
// (copy pool), the host then waits for a slot before refilling it.

// Host memory the runtime allocated pinned, [p, p + len) inside one
// allocation: hipHostMalloc'd (torch pin_memory included) is an HSA pool
// allocation whose pages the driver holds for the allocation's lifetime.
// The GPU reads and writes only such memory in place (zero copy, or DMA by
// the copy engines). Pageable memory the caller registered with
// hipHostRegister reports HSA_EXT_POINTER_TYPE_LOCKED: the registration maps
// its pages for the GPU without pinning them, and a page that moves while a
// kernel writes it loses the writes into the freed old page (round 5: 5 of 11
// long fuzz runs; DESIGN.md §7 "Platform constraint"). It is staged like any
// pageable memory. So is device memory (HSA type too, but not host memory).
bool runtime_pinned(const void* p, size_t len) {
  if (!p) return false;
  hipPointerAttribute_t attr{};
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory is reported as an error: clear it
    return false;
  }
  if (attr.type != hipMemoryTypeHost) return false;
  hsa_amd_pointer_info_t info{};
  info.size = sizeof info;
  if (hsa_amd_pointer_info(p, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return false;
  if (info.type != HSA_EXT_POINTER_TYPE_HSA || !info.hostBaseAddress) return false;
  const uintptr_t b = reinterpret_cast<uintptr_t>(info.hostBaseAddress), a = reinterpret_cast<uintptr_t>(p);
  return a >= b && len <= info.sizeInBytes && a - b <= info.sizeInBytes - len;
}

bool zero_copy_on() {
  const char* e = getenv("HRS_ZEROCOPY");
  return !(e && e[0] == '0');
}

// 64 blocks (256 waves) keep the host link as busy as a full grid does:
// config 5's repair 28.99 ms at 64 vs 29.66 uncapped, its encode 28.55 vs
// 29.57 (tools/bench_hbatch.py, profiles/r04/d/) — and leave 3/4 of the chip
// free for other work. HRS_ZC_BLOCKS=0 lifts the cap.
unsigned zero_copy_blocks() {
  const char* e = getenv("HRS_ZC_BLOCKS");
  const long x = e ? atol(e) : 64;
  return x > 0 ? static_cast<unsigned>(x) : 0u;
}

// Zero copy is taken only where the device address IS the host address
// (HIP's unified addressing on these systems): then any pointer into a pinned
// allocation, base or interior, is valid in a kernel as it stands, with no
// question of how an interior pointer's offset maps. Anything else (pageable
// or caller-registered memory, another mapping) is staged.
bool host_device_ptr(const void* p, size_t len, uint8_t** dp) {
  if (!p || !runtime_pinned(p, len)) return false;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void*>(p), 0) != hipSuccess || !d) {
    (void)hipGetLastError();
    return false;
  }
  if (d != p) return false;
  *dp = static_cast<uint8_t*>(d);
  return true;
}

// Bytes a strided batch spans from its base: the last stripe's last row end.
size_t batch_span(size_t nstripes, size_t stripe_stride, int rows, size_t row_stride, size_t len) {
  return (nstripes - 1) * stripe_stride + static_cast<size_t>(rows - 1) * row_stride + len;
}

size_t hbatch_target_bytes() {  // read per call (A/B runs in one process)
  const char* e = getenv("HRS_HBATCH_BYTES");
  const long x = e ? atol(e) : 0;
  return static_cast<size_t>(x > 0 ? x : 48l << 20);  // device image per chunk
}

// A staged batch's copy-out of a finished slot goes to the copy pool in one
// batch with the slot's next copy-in (HRS_HBATCH_MERGE=0: two batches, the
// round-5 form; read per call, A/B runs).
bool hbatch_merge() {
  const char* e = getenv("HRS_HBATCH_MERGE");
  return !(e && e[0] == '0');
}

// H2D and D2H on their own streams (one per direction, shared by the slots),
// or on each slot's stream behind and ahead of its kernels (HRS_HBATCH_DUPLEX=0:
// the round-3 pipeline, kept for A/B runs; read per call so one process can
// interleave both: tools/bench_hbatch.py).
bool hbatch_duplex() {
  const char* e = getenv("HRS_HBATCH_DUPLEX");
  return e && e[0] == '1';
}

hrs_status hbatch_slot(hrs_codec* c, int i, size_t dev_bytes, size_t pin_bytes) {
  hrs_codec::HostBatchSlot& h = c->hbatch[i];
  if (!h.stream) {
    hipError_t e = hipStreamCreateWithFlags(&h.stream, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail(c, e, "hipStreamCreate");
    for (hipEvent_t* ev : {&h.done, &h.in_done, &h.comp_done}) {
      e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
      if (e != hipSuccess) return hip_fail(c, e, "hipEventCreate");
    }
  }
  for (hipStream_t* s : {&c->hbatch_in, &c->hbatch_out})
    if (!*s) {
      hipError_t e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
      if (e != hipSuccess) return hip_fail(c, e, "hipStreamCreate");
    }
  if (h.dev_bytes < dev_bytes) {
    (void)hipStreamSynchronize(c->hbatch_in);
    (void)hipStreamSynchronize(c->hbatch_out);
    (void)hipStreamSynchronize(h.stream);
    if (h.dev) (void)hipFree(h.dev);
    h.dev = nullptr;
    h.dev_bytes = 0;
    hipError_t e = hipMalloc(&h.dev, dev_bytes);
    if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipMalloc(%zu): %s", dev_bytes, hipGetErrorString(e));
    h.dev_bytes = dev_bytes;
  }
  if (h.pin_bytes < pin_bytes) {
    (void)hipStreamSynchronize(c->hbatch_in);
    (void)hipStreamSynchronize(c->hbatch_out);
    (void)hipStreamSynchronize(h.stream);
    if (h.pin) (void)hipHostFree(h.pin);
    h.pin = nullptr;
    h.pin_dev = nullptr;
    h.pin_bytes = 0;
    hipError_t e = hipHostMalloc(&h.pin, pin_bytes, hipHostMallocDefault);
    if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipHostMalloc(%zu): %s", pin_bytes, hipGetErrorString(e));
    if (!host_device_ptr(h.pin, pin_bytes, &h.pin_dev)) h.pin_dev = nullptr;
    h.pin_bytes = pin_bytes;
  }
  return HRS_OK;
}

// Rows moved for one stripe: runs of consecutive locations [l0, l0 + cnt).
struct RowRun {
  int l0, cnt;
};

// H2D of `runs` of stripe i of the chunk: host rows at hsrc + l * hrow (host
// stripe base), device rows at ddst + l * dpitch.
hrs_status h2d_runs(hrs_codec* c, const std::vector<RowRun>& runs, uint8_t* ddst, size_t dpitch, const uint8_t* hsrc,
                    size_t hrow, size_t len, hipStream_t s) {
  for (const RowRun& r : runs) {
    hipError_t e;
    if (r.cnt == 1 || (hrow == len && dpitch == len))
      e = hipMemcpyAsync(ddst + r.l0 * dpitch, hsrc + r.l0 * hrow, (r.cnt - 1) * dpitch + len, hipMemcpyHostToDevice, s);
    else
      e = hipMemcpy2DAsync(ddst + r.l0 * dpitch, dpitch, hsrc + r.l0 * hrow, hrow, len, r.cnt, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return hip_fail(c, e, "H2D");
  }
  return HRS_OK;
}

hrs_status d2h_rows(hrs_codec* c, uint8_t* hdst, size_t hrow, const uint8_t* dsrc, size_t dpitch, size_t len, int cnt,
                    hipStream_t s) {
  if (cnt <= 0) return HRS_OK;
  hipError_t e;
  if (cnt == 1 || (hrow == len && dpitch == len))
    e = hipMemcpyAsync(hdst, dsrc, (cnt - 1) * dpitch + len, hipMemcpyDeviceToHost, s);
  else
    e = hipMemcpy2DAsync(hdst, hrow, dsrc, dpitch, len, cnt, hipMemcpyDeviceToHost, s);
  return e == hipSuccess ? HRS_OK : hip_fail(c, e, "D2H");
}

std::vector<RowRun> runs_of(const int* locs, int nlocs) {  // locs ascending
  std::vector<RowRun> v;
  for (int i = 0; i < nlocs; ++i) {
    if (!v.empty() && v.back().l0 + v.back().cnt == locs[i])
      ++v.back().cnt;
    else
      v.push_back({locs[i], 1});
  }
  return v;
}

// The whole-job driver. Per chunk [s0, s0 + ns): `reads(i)` lists the row
// runs stripe s0 + i needs on the device, `compute(slot, s0, ns, dimg,
// dout)` queues the kernels on the slot's stream, `writes(i)` = how many
// output rows stripe s0 + i has (rows 0.. of its output block). Host
// stripe s: rows at hin + s * in_stripe + l * in_row; outputs at
// hout + s * out_stripe + t * out_row.
template <typename Reads, typename Compute, typename Writes>
hrs_status host_batch(hrs_codec* c, const uint8_t* hin, size_t in_row, size_t in_stripe, int img_rows, uint8_t* hout,
                      size_t out_row, size_t out_stripe, int out_rows_max, size_t len, size_t nstripes, Reads reads,
                      Compute compute, Writes writes) {
  const size_t dpitch = (len + 255) & ~static_cast<size_t>(255);
  const size_t img_stripe = dpitch * static_cast<size_t>(img_rows);
  const size_t out_stripe_dev = dpitch * static_cast<size_t>(out_rows_max);
  size_t chunk = std::max<size_t>(1, hbatch_target_bytes() / std::max<size_t>(1, img_stripe));
  chunk = std::min(chunk, nstripes);
  const bool pinned = runtime_pinned(hin, batch_span(nstripes, in_stripe, img_rows, in_row, len)) &&
                      runtime_pinned(hout, batch_span(nstripes, out_stripe, out_rows_max, out_row, len));
  const size_t dev_bytes = chunk * (img_stripe + out_stripe_dev);
  const size_t pin_bytes = pinned ? 0 : dev_bytes;  // staging mirrors the device image
  // pageable callers, zero copy: the kernels read each chunk's image from the
  // slot's pinned staging and write its outputs there (no device image, no
  // H2D / D2H); the host copies in and out of staging as before
  bool zc = !pinned && zero_copy_on();
  for (int i = 0; i < hrs::kHostBatchSlots; ++i) {
    hrs_status st = hbatch_slot(c, i, zc ? 0 : dev_bytes, pin_bytes);
    if (st != HRS_OK) return st;
  }
  uint8_t* zc_img[hrs::kHostBatchSlots] = {};
  for (int i = 0; i < hrs::kHostBatchSlots && zc; ++i) zc &= (zc_img[i] = c->hbatch[i].pin_dev) != nullptr;
  for (int i = 0; i < hrs::kHostBatchSlots && !zc && !pinned; ++i) {  // staging not device-mapped: copy engine
    hrs_status st = hbatch_slot(c, i, dev_bytes, pin_bytes);
    if (st != HRS_OK) return st;
  }
  hrs::GridCap cap(zc ? zero_copy_blocks() : 0u);
  hrs::CopyPool& pool = copy_pool(c);
  const uint8_t nt = host_store_mode();
  std::vector<hrs::CopyJob> jobs;
  const bool duplex = hbatch_duplex();
  const bool merge = hbatch_merge();
  struct Pending {
    bool busy = false;
    bool used = false;  // the slot's events have been recorded by this call
    size_t s0 = 0, ns = 0;
  } pend[hrs::kHostBatchSlots];
  // wait for a slot; pageable: queue the copies of its outputs out of
  // staging in `jobs` (the caller runs them, merged with the slot's next
  // copy-in: the output block and the input image are disjoint)
  auto finish = [&](int sl) -> hrs_status {
    if (!pend[sl].busy) return HRS_OK;
    hrs_codec::HostBatchSlot& h = c->hbatch[sl];
    hipError_t e = hipEventSynchronize(h.done);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventSynchronize");
    if (!pinned) {
      const uint8_t* pout = h.pin + chunk * img_stripe;
      for (size_t i = 0; i < pend[sl].ns; ++i) {
        const size_t s = pend[sl].s0 + i;
        for (int t = 0; t < writes(s); ++t)
          jobs.push_back({hout + s * out_stripe + t * out_row, pout + i * out_stripe_dev + t * dpitch, len});
      }
    }
    pend[sl].busy = false;
    return HRS_OK;
  };
  size_t j = 0;
  for (size_t s0 = 0; s0 < nstripes; s0 += chunk, ++j) {
    const int sl = static_cast<int>(j % hrs::kHostBatchSlots);
    hrs_codec::HostBatchSlot& h = c->hbatch[sl];
    const size_t ns = std::min(chunk, nstripes - s0);
    if (!pinned) {
      jobs.clear();
      hrs_status st = finish(sl);
      if (st != HRS_OK) return st;
      if (!merge && !jobs.empty()) {
        pool.run(jobs);
        jobs.clear();
      }
      for (size_t i = 0; i < ns; ++i)
        for (const RowRun& r : reads(s0 + i))
          for (int q = 0; q < r.cnt; ++q) {
            const int l = r.l0 + q;
            jobs.push_back({h.pin + i * img_stripe + l * dpitch, hin + (s0 + i) * in_stripe + l * in_row, len, nt});
          }
      pool.run(jobs);
    }
    // stream of each stage; in duplex mode the H2D waits until the slot's
    // previous kernels have read its image, the kernels until the previous
    // D2H has read its output block, the D2H until this chunk's kernels
    hipError_t e = hipSuccess;
    if (zc) {  // the kernels work on the staging itself
      uint8_t* zimg = zc_img[sl];
      hrs_status st = compute(h.stream, s0, ns, zimg, img_stripe, dpitch, zimg + chunk * img_stripe, out_stripe_dev);
      if (st != HRS_OK) return st;
      if ((e = hipEventRecord(h.done, h.stream)) != hipSuccess) return hip_fail(c, e, "hipEventRecord");
      pend[sl].busy = pend[sl].used = true;
      pend[sl].s0 = s0;
      pend[sl].ns = ns;
      continue;
    }
    const hipStream_t s_in = duplex ? c->hbatch_in : h.stream;
    const hipStream_t s_out = duplex ? c->hbatch_out : h.stream;
    if (duplex && pend[sl].used && (e = hipStreamWaitEvent(s_in, h.comp_done, 0)) != hipSuccess)
      return hip_fail(c, e, "hipStreamWaitEvent");
    uint8_t* dimg = h.dev;
    uint8_t* dout = h.dev + chunk * img_stripe;
    for (size_t i = 0; i < ns; ++i) {
      const uint8_t* src = pinned ? hin + (s0 + i) * in_stripe : h.pin + i * img_stripe;
      hrs_status st = h2d_runs(c, reads(s0 + i), dimg + i * img_stripe, dpitch, src, pinned ? in_row : dpitch, len,
                               s_in);
      if (st != HRS_OK) return st;
    }
    if (duplex) {
      if ((e = hipEventRecord(h.in_done, s_in)) != hipSuccess) return hip_fail(c, e, "hipEventRecord");
      if ((e = hipStreamWaitEvent(h.stream, h.in_done, 0)) != hipSuccess) return hip_fail(c, e, "hipStreamWaitEvent");
      if (pend[sl].used && (e = hipStreamWaitEvent(h.stream, h.done, 0)) != hipSuccess)
        return hip_fail(c, e, "hipStreamWaitEvent");
    }
    hrs_status st = compute(h.stream, s0, ns, dimg, img_stripe, dpitch, dout, out_stripe_dev);
    if (st != HRS_OK) return st;
    if (duplex) {
      if ((e = hipEventRecord(h.comp_done, h.stream)) != hipSuccess) return hip_fail(c, e, "hipEventRecord");
      if ((e = hipStreamWaitEvent(s_out, h.comp_done, 0)) != hipSuccess) return hip_fail(c, e, "hipStreamWaitEvent");
    }
    for (size_t i = 0; i < ns; ++i) {
      const size_t s = s0 + i;
      st = pinned ? d2h_rows(c, hout + s * out_stripe, out_row, dout + i * out_stripe_dev, dpitch, len, writes(s), s_out)
                  : d2h_rows(c, h.pin + chunk * img_stripe + i * out_stripe_dev, dpitch, dout + i * out_stripe_dev,
                             dpitch, len, writes(s), s_out);
      if (st != HRS_OK) return st;
    }
    if ((e = hipEventRecord(h.done, s_out)) != hipSuccess) return hip_fail(c, e, "hipEventRecord");
    pend[sl].busy = true;
    pend[sl].used = true;
    pend[sl].s0 = s0;
    pend[sl].ns = ns;
  }
  for (int k = 1; k <= hrs::kHostBatchSlots; ++k) {  // in chunk order
    jobs.clear();
    hrs_status st = finish(static_cast<int>((j + k - 1) % hrs::kHostBatchSlots));
    if (st != HRS_OK) return st;
    if (!jobs.empty()) pool.run(jobs);
  }
  return HRS_OK;
}

// A failed host batch may leave slot work in flight: drain every slot stream.
hrs_status drain_hbatch(hrs_codec* c, hrs_status st) {
  if (st != HRS_OK) {
    for (hipStream_t s : {c->hbatch_in, c->hbatch_out})
      if (s) (void)hipStreamSynchronize(s);
    for (auto& h : c->hbatch)
      if (h.stream) (void)hipStreamSynchronize(h.stream);
  }
  return st;
}

// hrs_decode_batch_host with pinned stripes and outputs: one batch launch
// whose kernels read the survivors and write the repaired cells across the
// host link directly (zero copy). The plans go up first on slot 0's stream;
// the call returns once the launch has completed.
hrs_status zero_copy_batch(hrs_codec* c, const BatchPlanSet& ps, const uint8_t* ds, size_t row_stride,
                           size_t stripe_stride, uint8_t* dout, size_t out_row_stride, size_t out_stripe_stride,
                           size_t len, size_t nstripes) {
  hrs_status st = hbatch_slot(c, 0, 0, 0);
  if (st != HRS_OK) return st;
  const hipStream_t hs = c->hbatch[0].stream;
  hrs_codec::BatchSlot* bsl = nullptr;
  const hrs::BatchPlan* dplans = nullptr;
  const int32_t* dpat = nullptr;
  if (ps.fused) {
    st = upload_batch_plans(c, ps, hs, &bsl, &dplans, &dpat);
    if (st != HRS_OK) return st;
  }
  {
    hrs::GridCap cap(zero_copy_blocks());
    st = launch_batch(c, ps, dplans, dpat, ds, row_stride, stripe_stride, dout, out_row_stride, out_stripe_stride,
                      len, 0, nstripes, hs);
  }
  if (st != HRS_OK) return st;
  if (bsl) {
    const hipError_t e = hipEventRecord(bsl->done, hs);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
    bsl->pending = true;
  }
  const hipError_t e = hipStreamSynchronize(hs);
  return e == hipSuccess ? HRS_OK : hip_fail(c, e, "hipStreamSynchronize");
}

// ---------------------------------------------- device sets (hrs_*_multi)
// contiguous stripe ranges, one host thread per device, no data
// exchange. Each range is an ordinary single-handle host batch; the handles
// are independent (their own slots, streams and staging), so the ranges run
// concurrently with no shared state beyond the process-wide copy pool, which
// takes batches from every open call in turn.

hrs_status check_device_set(hrs_codec* const* cs, int nc) {
  if (!cs || nc < 1) return fail(nullptr, HRS_EINVAL, "device set: need at least one codec");
  for (int i = 0; i < nc; ++i)
    if (!cs[i]) return fail(cs[0] ? cs[0] : nullptr, HRS_EINVAL, "device set: codecs[%d] is NULL", i);
  hrs_codec* c0 = cs[0];
  if (nc > 1024) return fail(c0, HRS_EINVAL, "device set: %d codecs (at most 1024)", nc);
  for (int i = 0; i < nc; ++i) {
    const hrs_codec* c = cs[i];
    if (c->kind != c0->kind || c->k != c0->k || c->p != c0->p || c->src_s != c0->src_s)
      return fail(c0, HRS_EINVAL, "device set: codecs[%d] is another code than codecs[0]", i);
    for (int j = 0; j < i; ++j)
      if (cs[j] == c) return fail(c0, HRS_EINVAL, "device set: codecs[%d] and codecs[%d] are one handle", j, i);
  }
  for (int i = 0; i < nc; ++i)
    if (cs[i]->device < 0) return fail(c0, HRS_EDEVICE, "device set: codecs[%d] is a host-only handle", i);
  return HRS_OK;
}

// Runs f(codec, first stripe, stripe count) for each member's range on its
// own thread (member 0 on the caller's); returns the first failing member's
// status with its message moved to codecs[0].
template <typename F>
hrs_status run_device_set(hrs_codec* const* cs, int nc, size_t nstripes, F f) {
  std::vector<hrs_status> st(nc, HRS_OK);
  auto lo = [&](int i) { return static_cast<size_t>((static_cast<unsigned __int128>(nstripes) * i) / nc); };
  auto member = [&](int i) {
    const size_t a = lo(i), b = lo(i + 1);
    if (b > a) st[i] = f(cs[i], a, b - a);
  };
  std::vector<std::thread> th;
  th.reserve(nc);
  int inline_from = nc;  // members a thread could not be started for run here
  for (int i = 1; i < nc; ++i) {
    try {
      th.emplace_back(member, i);
    } catch (const std::exception&) {
      inline_from = i;
      break;
    }
  }
  member(0);
  for (int i = inline_from; i < nc; ++i) member(i);
  for (auto& t : th) t.join();
  for (int i = 0; i < nc; ++i)
    if (st[i] != HRS_OK) {
      if (i > 0) {
        const std::string msg = cs[i]->err;
        fail(cs[0], st[i], "device set member %d (device %d), stripes [%zu, %zu): %s", i, cs[i]->device, lo(i),
             lo(i + 1), msg.c_str());
      }
      return st[i];
    }
  return HRS_OK;
}

}  // namespace hrs::api

using namespace hrs::api;

namespace {

// hrs_last_host_path of a host batch: "pinned" when the stripes (and a
// decode's outputs) lie in runtime-pinned memory and zero copy is on.
const char* batch_path(bool pinned) {
  if (!zero_copy_on()) return "copy_engine";
  return pinned ? "pinned" : "staged";
}

hrs_status decode_batch_host_impl(hrs_codec* c, const uint8_t* stripes, size_t row_stride, size_t stripe_stride,
                                  const int* erased, int max_erased, uint8_t* out, size_t out_row_stride,
                                  size_t out_stripe_stride, size_t len, size_t nstripes) {
  if (!c) return HRS_EINVAL;
  if (!stripes || !out || max_erased < 0 || max_erased > hrs::kMaxOut || (max_erased > 0 && !erased))
    return fail(c, HRS_EINVAL, "bad batch decode arguments (max_erased must be in [0, %d])", hrs::kMaxOut);
  if (nstripes == 0 || len == 0 || max_erased == 0) return HRS_OK;
  if (nstripes > 0x7fffffffu) return fail(c, HRS_EINVAL, "too many stripes");
  BatchPlanSet ps;
  hrs_status st = build_batch_plans(c, erased, max_erased, nstripes, ps);
  if (st != HRS_OK) return st;
  if (ps.max_nout == 0) return HRS_OK;
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
  uint8_t *zs = nullptr, *zo = nullptr;
  if (zero_copy_on() && host_device_ptr(stripes, batch_span(nstripes, stripe_stride, c->n, row_stride, len), &zs) &&
      host_device_ptr(out, batch_span(nstripes, out_stripe_stride, max_erased, out_row_stride, len), &zo))
    return drain_hbatch(c, zero_copy_batch(c, ps, zs, row_stride, stripe_stride, zo, out_row_stride,
                                           out_stripe_stride, len, nstripes));
  // rows each pattern reads: its live locations (every location for the
  // per-stripe fallback of wide patterns, which reads what its matrix needs)
  std::vector<std::vector<RowRun>> pruns(ps.plans.size());
  for (size_t id = 0; id < ps.plans.size(); ++id) {
    const hrs::BatchPlan& pl = ps.plans[id];
    if (pl.nin <= hrs::kBatchMaxIn) {
      pruns[id] = runs_of(pl.loc, pl.nin);
    } else {
      std::vector<int> live;
      for (int l = 0; l < c->n; ++l)
        for (int o = 0; o < pl.nout; ++o)
          if (ps.mats[id][static_cast<size_t>(o) * c->n + l]) {
            live.push_back(l);
            break;
          }
      pruns[id] = runs_of(live.data(), static_cast<int>(live.size()));
    }
  }
  // plans + pattern indices: one upload for the whole job, on slot 0's
  // stream; the other slot streams wait for it
  hrs_codec::BatchSlot* bsl = nullptr;
  const hrs::BatchPlan* dplans = nullptr;
  const int32_t* dpat = nullptr;
  st = hbatch_slot(c, 0, 0, 0);
  if (st != HRS_OK) return st;
  if (ps.fused) {
    st = upload_batch_plans(c, ps, c->hbatch[0].stream, &bsl, &dplans, &dpat);
    if (st != HRS_OK) return st;
    hipError_t e = hipEventRecord(bsl->done, c->hbatch[0].stream);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
    bsl->pending = true;
    for (int i = 1; i < hrs::kHostBatchSlots; ++i) {
      st = hbatch_slot(c, i, 0, 0);
      if (st != HRS_OK) return st;
      e = hipStreamWaitEvent(c->hbatch[i].stream, bsl->done, 0);
      if (e != hipSuccess) return hip_fail(c, e, "hipStreamWaitEvent");
    }
  }
  auto reads = [&](size_t s) -> const std::vector<RowRun>& { return pruns[ps.pat[s]]; };
  auto writes = [&](size_t s) -> int { return ps.plans[ps.pat[s]].nout; };
  auto compute = [&](hipStream_t hs, size_t s0, size_t ns, uint8_t* dimg, size_t img_stripe, size_t dpitch,
                     uint8_t* dout, size_t out_stripe_dev) -> hrs_status {
    return launch_batch(c, ps, dplans, dpat, dimg, dpitch, img_stripe, dout, dpitch, out_stripe_dev, len, s0, ns, hs);
  };
  st = host_batch(c, stripes, row_stride, stripe_stride, c->n, out, out_row_stride, out_stripe_stride, ps.max_nout,
                  len, nstripes, reads, compute, writes);
  if (st == HRS_OK && bsl) {  // the plan slot is reused only after this job's kernels
    hipError_t e = hipEventRecord(bsl->done, c->hbatch[0].stream);
    if (e != hipSuccess) st = hip_fail(c, e, "hipEventRecord");
  }
  return drain_hbatch(c, st);
}

hrs_status encode_batch_host_impl(hrs_codec* c, uint8_t* stripes, size_t row_stride, size_t stripe_stride, size_t len,
                                  size_t nstripes) {
  if (!c) return HRS_EINVAL;
  if (!stripes) return fail(c, HRS_EINVAL, "stripes is NULL");
  if (nstripes == 0 || len == 0) return HRS_OK;
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
  const int k = c->k, p = c->p;
  uint8_t* zs = nullptr;
  if (zero_copy_on() && host_device_ptr(stripes, batch_span(nstripes, stripe_stride, c->n, row_stride, len), &zs)) {
    // runtime-pinned: the kernel works on the caller's stripes in place
    hrs_status st = hbatch_slot(c, 0, 0, 0);
    if (st != HRS_OK) return st;
    const hipStream_t hs = c->hbatch[0].stream;
    std::vector<const uint8_t*> in(k);
    std::vector<uint8_t*> outp(p);
    for (int i = 0; i < k; ++i) in[i] = zs + static_cast<size_t>(p + i) * row_stride;
    for (int r = 0; r < p; ++r) outp[r] = zs + static_cast<size_t>(r) * row_stride;
    {
      hrs::GridCap cap(zero_copy_blocks());
      st = run_apply(c, c->g.data(), p, k, in.data(), stripe_stride, outp.data(), stripe_stride, len, nstripes, hs,
                     static_encode_family(c));
    }
    if (st == HRS_OK) {
      const hipError_t e = hipStreamSynchronize(hs);
      if (e != hipSuccess) st = hip_fail(c, e, "hipStreamSynchronize");
    }
    return drain_hbatch(c, st);
  }
  const std::vector<RowRun> data_rows{{p, k}};  // hops locations p..n-1: one run
  auto reads = [&](size_t) -> const std::vector<RowRun>& { return data_rows; };
  auto writes = [&](size_t) -> int { return p; };
  std::vector<const uint8_t*> in(k);
  std::vector<uint8_t*> outp(p);
  auto compute = [&](hipStream_t hs, size_t, size_t ns, uint8_t* dimg, size_t img_stripe, size_t dpitch,
                     uint8_t* dout, size_t out_stripe_dev) -> hrs_status {
    for (int i = 0; i < k; ++i) in[i] = dimg + static_cast<size_t>(p + i) * dpitch;
    for (int r = 0; r < p; ++r) outp[r] = dout + static_cast<size_t>(r) * dpitch;
    return run_apply(c, c->g.data(), p, k, in.data(), img_stripe, outp.data(), out_stripe_dev, len, ns, hs,
                     static_encode_family(c));
  };
  // parity rows 0..p-1 of each stripe are written in place
  return drain_hbatch(c, host_batch(c, stripes, row_stride, stripe_stride, c->n, stripes, row_stride, stripe_stride,
                                    p, len, nstripes, reads, compute, writes));
}

}  // namespace

extern "C" {

hrs_status hrs_decode_batch_dev(hrs_codec* c, const uint8_t* stripes, size_t row_stride, size_t stripe_stride,
                                const int* erased, int max_erased, uint8_t* out, size_t out_row_stride,
                                size_t out_stripe_stride, size_t len, size_t nstripes, void* stream) {
  if (!c) return HRS_EINVAL;
  if (!stripes || !out || max_erased < 0 || max_erased > hrs::kMaxOut || (max_erased > 0 && !erased))
    return fail(c, HRS_EINVAL, "bad batch decode arguments (max_erased must be in [0, %d])", hrs::kMaxOut);
  if (nstripes == 0 || len == 0 || max_erased == 0) return HRS_OK;
  if (nstripes > 0x7fffffffu) return fail(c, HRS_EINVAL, "too many stripes");
  BatchPlanSet ps;
  hrs_status st = build_batch_plans(c, erased, max_erased, nstripes, ps);
  if (st != HRS_OK) return st;
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
  hipStream_t hs = static_cast<hipStream_t>(stream);
  if (ps.max_nout == 0) return HRS_OK;
  if (!ps.fused)  // shapes beyond the batch kernel (wide codes): one launch per stripe
    return launch_batch(c, ps, nullptr, nullptr, stripes, row_stride, stripe_stride, out, out_row_stride,
                        out_stripe_stride, len, 0, nstripes, hs);
  hrs_codec::BatchSlot* sl = nullptr;
  const hrs::BatchPlan* dplans = nullptr;
  const int32_t* dpat = nullptr;
  st = upload_batch_plans(c, ps, hs, &sl, &dplans, &dpat);
  if (st != HRS_OK) return st;
  st = launch_batch(c, ps, dplans, dpat, stripes, row_stride, stripe_stride, out, out_row_stride, out_stripe_stride,
                    len, 0, nstripes, hs);
  if (st != HRS_OK) return st;
  hipError_t e = hipEventRecord(sl->done, hs);
  if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
  sl->pending = true;
  return HRS_OK;
}

hrs_status hrs_decode_batch_host(hrs_codec* c, const uint8_t* stripes, size_t row_stride, size_t stripe_stride,
                                 const int* erased, int max_erased, uint8_t* out, size_t out_row_stride,
                                 size_t out_stripe_stride, size_t len, size_t nstripes) {
  if (!c) return HRS_EINVAL;
  if (!stripes || !out || max_erased < 0 || max_erased > hrs::kMaxOut || (max_erased > 0 && !erased))
    return fail(c, HRS_EINVAL, "bad batch decode arguments (max_erased must be in [0, %d])", hrs::kMaxOut);
  if (nstripes == 0 || len == 0 || max_erased == 0) return HRS_OK;
  if (nstripes > 0x7fffffffu) return fail(c, HRS_EINVAL, "too many stripes");
  const hrs_status st = decode_batch_host_impl(c, stripes, row_stride, stripe_stride, erased, max_erased, out,
                                               out_row_stride, out_stripe_stride, len, nstripes);
  if (st == HRS_OK) {
    DeviceGuard g(c->device);
    c->last_host_path =
        batch_path(g.ok && runtime_pinned(stripes, batch_span(nstripes, stripe_stride, c->n, row_stride, len)) &&
                   runtime_pinned(out, batch_span(nstripes, out_stripe_stride, max_erased, out_row_stride, len)));
  }
  return st;
}

hrs_status hrs_encode_batch_host(hrs_codec* c, uint8_t* stripes, size_t row_stride, size_t stripe_stride, size_t len,
                                 size_t nstripes) {
  if (!c) return HRS_EINVAL;
  if (!stripes) return fail(c, HRS_EINVAL, "stripes is NULL");
  if (nstripes == 0 || len == 0) return HRS_OK;
  const hrs_status st = encode_batch_host_impl(c, stripes, row_stride, stripe_stride, len, nstripes);
  if (st == HRS_OK) {
    DeviceGuard g(c->device);
    c->last_host_path =
        batch_path(g.ok && runtime_pinned(stripes, batch_span(nstripes, stripe_stride, c->n, row_stride, len)));
  }
  return st;
}

hrs_status hrs_decode_batch_host_multi(hrs_codec* const* codecs, int ncodecs, const uint8_t* stripes,
                                       size_t row_stride, size_t stripe_stride, const int* erased, int max_erased,
                                       uint8_t* out, size_t out_row_stride, size_t out_stripe_stride, size_t len,
                                       size_t nstripes) {
  hrs_status st = check_device_set(codecs, ncodecs);
  if (st != HRS_OK) return st;
  if (!stripes || !out || max_erased < 0 || max_erased > hrs::kMaxOut || (max_erased > 0 && !erased))
    return fail(codecs[0], HRS_EINVAL, "bad batch decode arguments (max_erased must be in [0, %d])", hrs::kMaxOut);
  if (nstripes == 0 || len == 0 || max_erased == 0) return HRS_OK;
  return run_device_set(codecs, ncodecs, nstripes, [&](hrs_codec* c, size_t s0, size_t ns) {
    return hrs_decode_batch_host(c, stripes + s0 * stripe_stride, row_stride, stripe_stride,
                                 erased + s0 * static_cast<size_t>(max_erased), max_erased,
                                 out + s0 * out_stripe_stride, out_row_stride, out_stripe_stride, len, ns);
  });
}

hrs_status hrs_encode_batch_host_multi(hrs_codec* const* codecs, int ncodecs, uint8_t* stripes, size_t row_stride,
                                       size_t stripe_stride, size_t len, size_t nstripes) {
  hrs_status st = check_device_set(codecs, ncodecs);
  if (st != HRS_OK) return st;
  if (!stripes) return fail(codecs[0], HRS_EINVAL, "stripes is NULL");
  if (nstripes == 0 || len == 0) return HRS_OK;
  return run_device_set(codecs, ncodecs, nstripes, [&](hrs_codec* c, size_t s0, size_t ns) {
    return hrs_encode_batch_host(c, stripes + s0 * stripe_stride, row_stride, stripe_stride, len, ns);
  });
}

}  // extern "C"
