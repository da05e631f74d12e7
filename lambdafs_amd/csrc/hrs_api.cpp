// C ABI of libhrs (include/hrs.h): codec lifecycle, coding matrices, the
// decode-matrix cache, and dispatch of the gfx950 kernels.
//
// Mirrors the Java codec plugin surface io.hops.erasure_coding.ErasureCode
// (hadoop-hdfs/.../io/hops/erasure_coding/ErasureCode.java:25-182) as
// implemented by ReedSolomonCode (hops-erasure-coding/.../ReedSolomonCode.java).
// Matrices are derived in closed form here; the CPU restatement of the
// reference's per-byte loops lives only in oracle/ (test infrastructure).
// Lifecycle, queries and matrices; the coding calls live in hrs_dispatch.cpp
// (device batches), hrs_hostpath.cpp (host buffers) and hrs_batch_api.cpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/hrs.h"
#include "hrs_codec.hpp"
#include <cstdarg>

#include "gf256.hpp"

namespace hrs::api {

namespace gf = hrs::gf;

thread_local std::string g_create_error;

hrs_status fail(hrs_codec* c, hrs_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c)
    c->err = buf;
  else
    g_create_error = buf;
  return st;
}

hrs_status hip_fail(hrs_codec* c, hipError_t e, const char* what) {
  return fail(c, HRS_EDEVICE, "%s: %s", what, hipGetErrorString(e));
}

static bool in_range(const int* v, int nv, int n) {
  for (int i = 0; i < nv; ++i)
    if (v[i] < 0 || v[i] >= n) return false;
  return true;
}

// Location lists of a 5-arg decode, as the reference indexes them: not-to-read
// locations always (primitivePower / data), erased ones except in
// ReedSolomonCode (it only compares them, ReedSolomonCode.java:158-165), and
// locationsToRead only in SimpleRegeneratingCode (RS, nrs and XOR ignore it).
// Repeats are allowed: the Java accepts them (hrs_matrix.cpp rs_decode_rows).
bool decode_locations_ok(const hrs_codec* c, const int* erased, int ne, const int* to_read, int nr, const int* ntr,
                         int nn) {
  if (!in_range(ntr, nn, c->n)) return false;
  if (c->kind != HRS_CODE_RS && !in_range(erased, ne, c->n)) return false;
  if (c->kind == HRS_CODE_SRC && to_read && !in_range(to_read, nr, c->n)) return false;
  return true;
}


void init_code(hrs_codec* c, int code, int k, int p, int src_s) {
  c->k = k;
  c->p = p;
  c->n = k + p;
  c->kind = code;
  if (code == HRS_CODE_SRC) {
    src_params(k, p, src_s, &c->src_s, &c->src_r, &c->src_d);
    c->groups.resize(c->n);
    for (int l = 0; l < c->n; ++l) c->groups[l] = src_neighbors(c, l);
  }
  init_encode_matrix(c);
}

hrs_status create_impl(int code, int stripe_size, int parity_size, int src_s, const hrs_opts* opts, hrs_codec** out) {
  if (!out) return fail(nullptr, HRS_EINVAL, "out is NULL");
  *out = nullptr;
  if (code != HRS_CODE_RS && code != HRS_CODE_XOR && code != HRS_CODE_NRS && code != HRS_CODE_SRC)
    return fail(nullptr, HRS_EINVAL, "unknown code family %d", code);
  if (code == HRS_CODE_SRC && (src_s < 0 || src_s > parity_size))
    return fail(nullptr, HRS_EINVAL, "SRC parities %d outside [0, parity size %d]", src_s, parity_size);
  if (code == HRS_CODE_XOR && parity_size != 1)
    return fail(nullptr, HRS_EINVAL, "XOR code needs parity size 1 (XORCode.java:47), got %d", parity_size);
  if (stripe_size < 1 || parity_size < 1 || stripe_size + parity_size >= gf::kFieldSize ||
      parity_size > gf::kMaxParity)
    return fail(nullptr, HRS_EINVAL, "unsupported RS(%d,%d): need k>=1, 1<=p<=%d, k+p<256", stripe_size,
                parity_size, gf::kMaxParity);
  if (opts)
    for (int r : opts->reserved)
      if (r != 0) return fail(nullptr, HRS_EINVAL, "hrs_opts.reserved must be zero");
  int dev = opts ? opts->device : -1;
  if (dev < -1 && dev != HRS_DEVICE_NONE)
    return fail(nullptr, HRS_EDEVICE, "no HIP device %d (ordinals are >= 0; -1 = current device)", dev);
  if (dev == HRS_DEVICE_NONE) {  // host-only handle: matrices and locations, no coding
    auto* c = new hrs_codec();
    c->device = HRS_DEVICE_NONE;
    init_code(c, code, stripe_size, parity_size, src_s);
    *out = c;
    return HRS_OK;
  }
  if (dev < 0) {
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return fail(nullptr, HRS_EDEVICE, "hipGetDevice: %s", hipGetErrorString(e));
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess) return fail(nullptr, HRS_EDEVICE, "no HIP device %d (%s)", dev, hipGetErrorString(e));
  if (dev >= ndev) return fail(nullptr, HRS_EDEVICE, "no HIP device %d (%d visible)", dev, ndev);
  auto* c = new hrs_codec();
  c->device = dev;
  init_code(c, code, stripe_size, parity_size, src_s);
  {
    DeviceGuard g(dev);
    e = g.ok ? hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) : hipErrorInvalidDevice;
  }
  if (e != hipSuccess) {
    delete c;
    return fail(nullptr, HRS_EDEVICE, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  *out = c;
  return HRS_OK;
}


}  // namespace hrs::api

using namespace hrs::api;

extern "C" {

const char* hrs_version(void) { return "hrs 0.1.0 (gfx950)"; }

hrs_status hrs_create(int stripe_size, int parity_size, const hrs_opts* opts, hrs_codec** out) {
  return hrs_create_code(HRS_CODE_RS, stripe_size, parity_size, opts, out);
}

int hrs_code_kind(const hrs_codec* c) { return c ? c->kind : -1; }

hrs_status hrs_create_code(int code, int stripe_size, int parity_size, const hrs_opts* opts, hrs_codec** out) {
  // HRS_CODE_SRC here = the Java's deprecated (stripeSize, paritySize)
  // constructor: no SRC parities (SimpleRegeneratingCode.java:44-47)
  return create_impl(code, stripe_size, parity_size, 0, opts, out);
}

hrs_status hrs_create_src(int stripe_size, int parity_size, int src_parity_size, const hrs_opts* opts,
                          hrs_codec** out) {
  return create_impl(HRS_CODE_SRC, stripe_size, parity_size, src_parity_size, opts, out);
}

hrs_status hrs_src_layout(const hrs_codec* c, int* src_parities, int* rs_parities, int* group_degree) {
  if (!c || c->kind != HRS_CODE_SRC) return HRS_EINVAL;
  if (src_parities) *src_parities = c->src_s;
  if (rs_parities) *rs_parities = c->src_r;
  if (group_degree) *group_degree = c->src_d;
  return HRS_OK;
}

void hrs_destroy(hrs_codec* c) {
  if (!c) return;
  if (c->device == HRS_DEVICE_NONE) {
    delete c;
    return;
  }
  DeviceGuard g(c->device);
  if (c->stream) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamDestroy(c->stream);
  }
  if (c->crc_tables_a) (void)hipFree(c->crc_tables_a);
  for (auto& kv : c->crc_fold_tables) {
    for (auto& u : kv.second.uses) {
      (void)hipEventSynchronize(u.ev);
      (void)hipEventDestroy(u.ev);
    }
    (void)hipFree(kv.second.dev);
  }
  if (c->crc_raw_done) {
    (void)hipEventSynchronize(c->crc_raw_done);
    (void)hipEventDestroy(c->crc_raw_done);
  }
  if (c->crc_raw) (void)hipFree(c->crc_raw);
  for (auto& h : c->host) {
    if (h.stream) {
      (void)hipStreamSynchronize(h.stream);
      (void)hipStreamDestroy(h.stream);
    }
    if (h.done) (void)hipEventDestroy(h.done);
    if (h.dev) (void)hipFree(h.dev);
    if (h.pin) (void)hipHostFree(h.pin);
  }
  if (c->qflags) (void)hipHostFree(c->qflags);  // every slot stream has drained above
  for (auto& a : c->async) {
    if (a.stream) {
      (void)hipStreamSynchronize(a.stream);
      (void)hipStreamDestroy(a.stream);
    }
    for (hipEvent_t e : {a.done, a.t_start, a.t_end})
      if (e) (void)hipEventDestroy(e);
    if (a.dev) (void)hipFree(a.dev);
    if (a.pin) (void)hipHostFree(a.pin);
  }
  for (hipStream_t s : {c->hbatch_in, c->hbatch_out})
    if (s) (void)hipStreamSynchronize(s);
  for (auto& h : c->hbatch) {
    if (h.stream) {
      (void)hipStreamSynchronize(h.stream);
      (void)hipStreamDestroy(h.stream);
    }
    for (hipEvent_t e : {h.done, h.in_done, h.comp_done})
      if (e) (void)hipEventDestroy(e);
    if (h.dev) (void)hipFree(h.dev);
    if (h.pin) (void)hipHostFree(h.pin);
  }
  for (hipStream_t s : {c->hbatch_in, c->hbatch_out})
    if (s) (void)hipStreamDestroy(s);
  for (auto& b : c->batch) {
    if (b.done) {
      (void)hipEventSynchronize(b.done);
      (void)hipEventDestroy(b.done);
    }
    if (b.dev) (void)hipFree(b.dev);
    if (b.host) (void)hipHostFree(b.host);
  }
  delete c;
}

const char* hrs_last_error(const hrs_codec* c) { return c ? c->err.c_str() : g_create_error.c_str(); }

const char* hrs_last_kernel(const hrs_codec* c) { return c ? c->last_kernel.c_str() : ""; }

const char* hrs_last_host_path(const hrs_codec* c) { return c ? c->last_host_path : ""; }

int hrs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int hrs_codec_device(const hrs_codec* c) { return c ? c->device : -1; }

int hrs_stripe_size(const hrs_codec* c) { return c ? c->k : -1; }
int hrs_parity_size(const hrs_codec* c) { return c ? c->p : -1; }
int hrs_symbol_size(const hrs_codec* c) { return c ? 8 : -1; }  // log2(256), ReedSolomonCode.java:223-226

hrs_status hrs_set_kernel_mode(hrs_codec* c, int mode) {
  if (!c || mode < 0 || mode > 3) return HRS_EINVAL;
  c->kernel_mode = mode;
  return HRS_OK;
}

hrs_status hrs_locations_to_read_list(const hrs_codec* cc, const int* erased, int num_erased, int* to_read,
                                      int* num_to_read) {
  auto* c = const_cast<hrs_codec*>(cc);
  if (!c || !to_read || !num_to_read || num_erased < 0 || (num_erased > 0 && !erased)) return HRS_EINVAL;
  *num_to_read = 0;
  if (c->kind == HRS_CODE_SRC) {
    std::vector<int> v;
    hrs_status st = src_locations(c, erased, num_erased, v);
    if (st != HRS_OK) return st;
    std::copy(v.begin(), v.end(), to_read);
    *num_to_read = static_cast<int>(v.size());
    return HRS_OK;
  }
  // ErasureCode.java:89-113: scan locations from the top, keep the first k good ones.
  int got = 0;
  for (int loc = c->n - 1; loc >= 0 && got < c->k; --loc) {
    bool bad = false;
    for (int i = 0; i < num_erased; ++i) bad |= erased[i] == loc;
    if (!bad) to_read[got++] = loc;
  }
  if (got != c->k) {
    std::string s = "Locations ";
    for (int i = 0; i < num_erased; ++i) s += " " + std::to_string(erased[i]);
    return fail(c, HRS_ETOOMANY, "%s", s.c_str());
  }
  *num_to_read = got;
  return HRS_OK;
}

hrs_status hrs_locations_to_read(const hrs_codec* cc, const int* erased, int num_erased, int* to_read) {
  auto* c = const_cast<hrs_codec*>(cc);
  if (!c || !to_read || num_erased < 0 || (num_erased > 0 && !erased)) return HRS_EINVAL;
  std::vector<int> v(c->n);
  int m = 0;
  hrs_status st = hrs_locations_to_read_list(c, erased, num_erased, v.data(), &m);
  if (st != HRS_OK) return st;
  if (m != c->k)
    return fail(c, HRS_EINVAL, "%d locations to read (not stripe_size): use hrs_locations_to_read_list", m);
  std::copy(v.begin(), v.begin() + m, to_read);
  return HRS_OK;
}

hrs_status hrs_encode_matrix(const hrs_codec* c, uint8_t* g) {
  if (!c || !g) return HRS_EINVAL;
  std::memcpy(g, c->g.data(), c->g.size());
  return HRS_OK;
}

hrs_status hrs_decode_matrix(const hrs_codec* cc, const int* erased, int ne, const int* ntr, int nn, int zero_ntr,
                             uint8_t* d) {
  auto* c = const_cast<hrs_codec*>(cc);
  if (!c || !d || ne < 0 || nn < 0 || (ne && !erased) || (nn && !ntr)) return HRS_EINVAL;
  std::vector<uint8_t> m;
  hrs_status st;
  if (c->kind == HRS_CODE_XOR) {
    const uint8_t* x = nullptr;
    st = decode5_matrix(c, erased, ne, ntr, nn, nullptr, m, &x);
  } else if (c->kind == HRS_CODE_SRC) {
    const uint8_t* x = nullptr;
    st = decode5_matrix(c, erased, ne, ntr, nn, nullptr, m, &x);
    if (st == HRS_OK && ne > 0) m.assign(x, x + static_cast<size_t>(ne) * c->n);
  } else if (c->kind == HRS_CODE_NRS) {
    for (int t = 0; t < ne; ++t)
      if (erased[t] < 0 || erased[t] >= c->n) return fail(c, HRS_EINVAL, "erased location %d out of range", erased[t]);
    st = build_nrs_decode_matrix(c, ne, ntr, nn, m);
  } else {
    st = build_decode_matrix(c, erased, ne, ntr, nn, zero_ntr, m);
  }
  if (st == HRS_OK && !m.empty()) std::memcpy(d, m.data(), m.size());
  return st;
}

}  // extern "C"
