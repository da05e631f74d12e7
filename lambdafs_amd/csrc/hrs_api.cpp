// C ABI of libhrs (include/hrs.h): codec lifecycle, coding matrices, the
// decode-matrix cache, and dispatch of the gfx950 kernels.
//
// Mirrors the Java codec plugin surface io.hops.erasure_coding.ErasureCode
// (hadoop-hdfs/.../io/hops/erasure_coding/ErasureCode.java:25-182) as
// implemented by ReedSolomonCode (hops-erasure-coding/.../ReedSolomonCode.java).
// Matrices are derived in closed form here; the CPU restatement of the
// reference's per-byte loops lives only in oracle/ (test infrastructure).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hrs.h"
#include "crc32.hpp"
#include "gf256.hpp"
#include "hrs_crc.hpp"
#include "hrs_host.hpp"
#include "hrs_internal.hpp"

using hrs::RowArgs;
namespace gf = hrs::gf;

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
  std::map<uint64_t, uint32_t*> crc_fold_tables;
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
  // host-buffer calls: two chunk slots, each pinned staging + device rows +
  // its own stream; a slot is reused once its D2H event has completed
  struct HostSlot {
    uint8_t* pin = nullptr;
    uint8_t* dev = nullptr;
    size_t bytes = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
  } host[2];
  // host-memory batches (hrs_*_batch_host): a ring of chunk slots, each a
  // device image + output block, pinned staging (pageable callers only) and
  // its own stream
  struct HostBatchSlot {
    uint8_t* dev = nullptr;
    size_t dev_bytes = 0;
    uint8_t* pin = nullptr;
    size_t pin_bytes = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
  } hbatch[hrs::kHostBatchSlots];
  // asynchronous host-buffer calls (hrs_*_submit / hrs_collect): a ring of
  // operation slots, each pinned staging + device rows + its own stream; an
  // operation occupies its slot from submit until it is collected
  struct AsyncSlot {
    uint8_t* pin = nullptr;
    uint8_t* dev = nullptr;
    size_t bytes = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    bool busy = false;
    bool queued = false;  // GPU work was queued (len > 0)
    uint64_t ticket = 0;
    int nout = 0, nlive = 0, ncrc = 0;
    size_t len = 0, pitch = 0, crc_off = 0;
  } async[hrs::kAsyncSlots];
  uint64_t async_tickets = 0;
  std::string err;
};

namespace {

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

// ---------------------------------------------------------- GF linear algebra

// In-place Gauss-Jordan inverse of an m x m matrix over GF(2^8). False if singular.
bool gf_invert(std::vector<uint8_t>& a, int m) {
  std::vector<uint8_t> inv(static_cast<size_t>(m) * m, 0);
  for (int i = 0; i < m; ++i) inv[i * m + i] = 1;
  for (int col = 0; col < m; ++col) {
    int piv = -1;
    for (int r = col; r < m; ++r)
      if (a[r * m + col]) {
        piv = r;
        break;
      }
    if (piv < 0) return false;
    if (piv != col)
      for (int j = 0; j < m; ++j) {
        std::swap(a[piv * m + j], a[col * m + j]);
        std::swap(inv[piv * m + j], inv[col * m + j]);
      }
    const uint8_t s = gf::inv(a[col * m + col]);
    for (int j = 0; j < m; ++j) {
      a[col * m + j] = gf::mul(a[col * m + j], s);
      inv[col * m + j] = gf::mul(inv[col * m + j], s);
    }
    for (int r = 0; r < m; ++r) {
      if (r == col || a[r * m + col] == 0) continue;
      const uint8_t f = a[r * m + col];
      for (int j = 0; j < m; ++j) {
        a[r * m + j] ^= gf::mul(f, a[col * m + j]);
        inv[r * m + j] ^= gf::mul(f, inv[col * m + j]);
      }
    }
  }
  a.swap(inv);
  return true;
}

// Decode rows in closed form over an RS stripe of n locations (see hrs.h).
// With x_j = alpha^ntr[j] and syndromes S_i = sum_l A[i][l] d_l,
// A[i][l] = alpha^(i*l) (0 where zeroed), the reference solves V z = S with
// V[i][j] = x_j^i (GaloisField.java:232-246; ReedSolomonCode.java:127-142),
// so z = V^-1 A d. Locations are validated by the caller.
bool rs_decode_rows(int n, const int* erased, int ne, const int* ntr, int nn, int zero_ntr, std::vector<uint8_t>& d) {
  d.assign(static_cast<size_t>(ne) * n, 0);
  if (ne == 0 || nn == 0) return true;
  std::vector<char> in_ntr(n, 0);
  for (int j = 0; j < nn; ++j) in_ntr[ntr[j]] = 1;
  const int m = nn;
  std::vector<uint8_t> v(static_cast<size_t>(m) * m);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < m; ++j) v[i * m + j] = gf::alpha_pow(static_cast<long>(ntr[j]) * i);
  if (!gf_invert(v, m)) return false;
  for (int t = 0; t < ne; ++t) {
    int j = -1;
    for (int q = 0; q < nn; ++q)
      if (ntr[q] == erased[t]) {
        j = q;
        break;
      }
    if (j < 0) continue;  // not in not_to_read: stays 0 (ReedSolomonCode.java:158-165)
    for (int l = 0; l < n; ++l) {
      if (zero_ntr && in_ntr[l]) continue;
      uint8_t acc = 0;
      for (int i = 0; i < m; ++i) acc ^= gf::mul(v[j * m + i], gf::alpha_pow(static_cast<long>(i) * l));
      d[static_cast<size_t>(t) * n + l] = acc;
    }
  }
  return true;
}

hrs_status build_decode_matrix(hrs_codec* c, const int* erased, int ne, const int* ntr, int nn,
                               int zero_ntr, std::vector<uint8_t>& d) {
  const int n = c->n;
  std::vector<char> in_ntr(n, 0);
  for (int j = 0; j < nn; ++j) {
    if (ntr[j] < 0 || ntr[j] >= n) return fail(c, HRS_EINVAL, "location %d out of range [0,%d)", ntr[j], n);
    if (in_ntr[ntr[j]]) return fail(c, HRS_EINVAL, "duplicate location %d", ntr[j]);
    in_ntr[ntr[j]] = 1;
  }
  for (int t = 0; t < ne; ++t)
    if (erased[t] < 0 || erased[t] >= n) return fail(c, HRS_EINVAL, "erased location %d out of range", erased[t]);
  if (!rs_decode_rows(n, erased, ne, ntr, nn, zero_ntr, d)) return fail(c, HRS_EINVAL, "singular Vandermonde system");
  return HRS_OK;
}

hrs_status build_nrs_decode_matrix(hrs_codec* c, int ne, const int* ntr, int nn, std::vector<uint8_t>& d);

const std::vector<uint8_t>* cached_decode_matrix(hrs_codec* c, const int* erased, int ne, const int* ntr, int nn,
                                                 int zero_ntr, hrs_status* st) {
  std::vector<int> key;
  key.reserve(ne + nn + 3);
  key.push_back(zero_ntr);
  key.push_back(ne);
  key.insert(key.end(), erased, erased + ne);
  key.push_back(nn);
  key.insert(key.end(), ntr, ntr + nn);
  auto it = c->decode_cache.find(key);
  if (it != c->decode_cache.end()) {
    *st = HRS_OK;
    return &it->second;
  }
  std::vector<uint8_t> d;
  *st = c->kind == HRS_CODE_NRS ? build_nrs_decode_matrix(c, ne, ntr, nn, d)
                                : build_decode_matrix(c, erased, ne, ntr, nn, zero_ntr, d);
  if (*st != HRS_OK) return nullptr;
  if (c->decode_cache.size() > 4096) c->decode_cache.clear();
  return &(c->decode_cache[key] = std::move(d));
}

// nrs (NativeReedSolomonCode.java:90-152 over erasure_coder.c:102-230): hops
// location l maps to Apache index a(l) = l + k for parity (l < p), l - p for
// data. Every not-to-read location is treated as erased; the decoder takes the
// first k remaining Apache indices as survivors (processErasures), inverts
// their rows of [I; Cauchy] and emits one row per not-to-read location in
// ascending Apache order: data rows of the inverse, parity rows = E[e] * inv.
// The Java copies output i into writeBufs[i] for i < writeBufs.length, so
// output t decodes the t-th smallest Apache not-to-read index, whichever
// location erased[t] names (reproduced here, bug-compatibly). Returned as an
// ne x n matrix over hops locations.
hrs_status build_nrs_decode_matrix(hrs_codec* c, int ne, const int* ntr, int nn, std::vector<uint8_t>& d) {
  const int k = c->k, p = c->p, n = c->n;
  if (nn > p) return fail(c, HRS_EINVAL, "%d not-to-read locations leave fewer than %d survivors", nn, k);
  if (ne > nn)  // bwriteBufs has |notToRead| entries (NativeReedSolomonCode.java:96,145-149)
    return fail(c, HRS_EINVAL, "%d erased locations > %d not-to-read locations", ne, nn);
  std::vector<char> gone(n, 0);
  std::vector<int> mod(nn);
  for (int j = 0; j < nn; ++j) {
    if (ntr[j] < 0 || ntr[j] >= n) return fail(c, HRS_EINVAL, "location %d out of range [0,%d)", ntr[j], n);
    const int a = ntr[j] < p ? ntr[j] + k : ntr[j] - p;
    if (gone[a]) return fail(c, HRS_EINVAL, "duplicate location %d", ntr[j]);
    gone[a] = 1;
    mod[j] = a;
  }
  std::sort(mod.begin(), mod.end());
  auto erow = [&](int a, int j) -> uint8_t {  // [I; Cauchy] (ISA-L gf_gen_cauchy1_matrix)
    return a < k ? static_cast<uint8_t>(a == j) : gf::inv(static_cast<uint8_t>(a ^ j));
  };
  std::vector<int> idx;
  for (int a = 0; a < n && static_cast<int>(idx.size()) < k; ++a)
    if (!gone[a]) idx.push_back(a);
  std::vector<uint8_t> b(static_cast<size_t>(k) * k);
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < k; ++j) b[i * k + j] = erow(idx[i], j);
  if (!gf_invert(b, k)) return fail(c, HRS_EINVAL, "singular survivor matrix");
  d.assign(static_cast<size_t>(ne) * n, 0);
  for (int t = 0; t < ne; ++t) {
    const int e = mod[t];
    for (int i = 0; i < k; ++i) {
      uint8_t s = 0;
      if (e < k) {
        s = b[e * k + i];
      } else {
        for (int j = 0; j < k; ++j) s ^= gf::mul(b[j * k + i], erow(e, j));
      }
      const int a = idx[i];
      const int hops = a < k ? a + p : a - k;
      d[static_cast<size_t>(t) * n + hops] = s;
    }
  }
  return HRS_OK;
}

// ------------------------------------------------ SimpleRegeneratingCode
// (SimpleRegeneratingCode.java). Locations: [SRC parities 0..s-1, RS
// parities s..p-1, data p..n-1]; the RS stripe is locations s..n-1 (RS
// parities first). Group g < s = SRC parity g + RS-stripe positions
// [g*d, (g+1)*d); the last ("implied") group = the remaining RS-stripe
// positions + every SRC parity.

int src_group(const hrs_codec* c, int loc) {  // getSRCGroup, :415-426
  if (0 <= loc && loc < c->src_s) return loc;
  if (c->src_s <= loc && loc < c->n) return (loc - c->src_s) / c->src_d;
  return -1;
}

std::vector<int> src_neighbors(const hrs_codec* c, int loc) {  // getSRCGroupNeighbors, :371-409
  std::vector<int> v;
  const int g = src_group(c, loc), s = c->src_s, d = c->src_d;
  if (g < s) {
    if (g != loc) v.push_back(g);
    for (int i = s + g * d; i < s + (g + 1) * d; ++i)
      if (i != loc) v.push_back(i);
  } else {
    for (int i = 0; i < s; ++i) v.push_back(i);
    for (int i = s + g * d; i < c->n; ++i)
      if (i != loc) v.push_back(i);
  }
  return v;
}

// init's adjustment (:70-90): fewer SRC parities until the groups fit
void src_params(int k, int p, int s_in, int* s, int* r, int* d) {
  int ss = s_in, rr = p - s_in;
  int dd = (k + rr + ss) / (ss + 1);  // ceil((k + r) / (s + 1))
  while (dd * ss >= k + rr) {
    --ss;
    ++rr;
    dd = (k + rr + ss) / (ss + 1);
  }
  *s = ss;
  *r = rr;
  *d = dd;
}

bool src_conflict(const hrs_codec* c, const int* locs, int n) {  // groupConflict, :432-453
  std::vector<int> count(c->src_s + 1, 0);
  for (int i = 0; i < n; ++i)
    if (locs[i] < c->src_s) {
      count[c->src_s] = 1;
      break;
    }
  for (int i = 0; i < n; ++i)
    if (count[src_group(c, locs[i])]++ > 0) return true;
  return false;
}

// locationsToReadForDecode, :300-366 (an ordered list of variable length)
hrs_status src_locations(hrs_codec* c, const int* erased, int ne, std::vector<int>& out) {
  out.clear();
  for (int i = 0; i < ne; ++i)
    if (erased[i] < 0 || erased[i] >= c->n) return fail(c, HRS_EINVAL, "erased location %d out of range", erased[i]);
  if (ne == 1) {
    out = c->groups[erased[0]];
    return HRS_OK;
  }
  if (!src_conflict(c, erased, ne)) {
    for (int i = 0; i < ne; ++i)
      for (int loc : c->groups[erased[i]])
        if (std::find(out.begin(), out.end(), loc) == out.end()) out.push_back(loc);
    return HRS_OK;
  }
  for (int loc = c->src_s; loc < c->n && static_cast<int>(out.size()) < c->k; ++loc)
    if (std::find(erased, erased + ne, loc) == erased + ne) out.push_back(loc);
  if (static_cast<int>(out.size()) != c->k) {
    std::string s = "Locations ";
    for (int i = 0; i < ne; ++i) s += " " + std::to_string(erased[i]);
    return fail(c, HRS_ETOOMANY, "%s", s.c_str());
  }
  return HRS_OK;
}

// p x k: RS parities = the hops generator over r roots (same construction as
// ReedSolomonCode); SRC parity i = XOR of RS-stripe positions [d*i, d*(i+1))
// (encode, :116-157).
void src_encode_matrix(hrs_codec* c) {
  const int k = c->k, s = c->src_s, r = c->src_r, d = c->src_d;
  std::vector<uint8_t> grs(static_cast<size_t>(r) * k);
  gf::encode_matrix(k, r, grs.data());
  std::fill(c->g.begin(), c->g.end(), 0);
  for (int i = 0; i < r; ++i)
    for (int j = 0; j < k; ++j) c->g[static_cast<size_t>(s + i) * k + j] = grs[static_cast<size_t>(i) * k + j];
  for (int i = 0; i < s; ++i)
    for (int j = d * i; j < d * (i + 1); ++j) {
      if (j < r)
        for (int q = 0; q < k; ++q) c->g[static_cast<size_t>(i) * k + q] ^= grs[static_cast<size_t>(j) * k + q];
      else
        c->g[static_cast<size_t>(i) * k + (j - r)] ^= 1;
    }
}

// decode 5-arg, :194-277, as an ne x n matrix over the read values:
//  one erasure      -> XOR of locationsToRead;
//  no group clash   -> XOR of each erased location's group;
//  otherwise        -> RS decode of the RS stripe at its not-to-read
//                      positions (decodeReedSolomon, :162-182), then each
//                      erased SRC parity = XOR of its (repaired) group.
hrs_status build_src_decode_matrix(hrs_codec* c, const int* erased, int ne, const int* to_read, int nr, const int* ntr,
                                   int nn, std::vector<uint8_t>& d) {
  const int n = c->n, s = c->src_s, r = c->src_r, nrs = c->n - c->src_s;
  for (int t = 0; t < ne; ++t)
    if (erased[t] < 0 || erased[t] >= n) return fail(c, HRS_EINVAL, "erased location %d out of range", erased[t]);
  for (int j = 0; j < nr; ++j)
    if (to_read[j] < 0 || to_read[j] >= n) return fail(c, HRS_EINVAL, "location %d out of range", to_read[j]);
  for (int j = 0; j < nn; ++j)
    if (ntr[j] < 0 || ntr[j] >= n) return fail(c, HRS_EINVAL, "location %d out of range", ntr[j]);
  d.assign(static_cast<size_t>(ne) * n, 0);
  if (ne == 1) {
    for (int j = 0; j < nr; ++j) d[to_read[j]] ^= 1;
    return HRS_OK;
  }
  if (!src_conflict(c, erased, ne)) {
    for (int t = 0; t < ne; ++t)
      for (int loc : c->groups[erased[t]]) d[static_cast<size_t>(t) * n + loc] ^= 1;
    return HRS_OK;
  }
  std::vector<int> ers;
  for (int j = 0; j < nn; ++j)
    if (ntr[j] >= s) ers.push_back(ntr[j] - s);
  const int m = static_cast<int>(ers.size());
  if (m > r) return fail(c, HRS_EINVAL, "%d not-to-read RS locations > %d RS parities", m, r);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < i; ++j)
      if (ers[i] == ers[j]) return fail(c, HRS_EINVAL, "duplicate location %d", ers[i] + s);
  std::vector<uint8_t> drs;
  if (!rs_decode_rows(nrs, ers.data(), m, ers.data(), m, 1, drs)) return fail(c, HRS_EINVAL, "singular Vandermonde system");
  // row of location l after the RS repair, over the read values
  auto fixed = [&](int l, uint8_t* row) {
    if (l >= s) {
      for (int q = 0; q < m; ++q)
        if (ers[q] == l - s) {
          for (int col = 0; col < nrs; ++col) row[s + col] ^= drs[static_cast<size_t>(q) * nrs + col];
          return;
        }
    }
    row[l] ^= 1;
  };
  for (int t = 0; t < ne; ++t) {
    uint8_t* row = &d[static_cast<size_t>(t) * n];
    if (erased[t] < s)
      for (int loc : c->groups[erased[t]]) fixed(loc, row);
    else
      fixed(erased[t], row);
  }
  return HRS_OK;
}

// ---------------------------------------------------------------- dispatch

// The matrix a 5-arg decodeBulk applies (ne x n), per code family.
//  RS : cached closed-form matrix; more than p not-to-read locations throw in
//       the Java (errSignature is sized p, ReedSolomonCode.java:60).
//  NRS: see build_nrs_decode_matrix.
//  XOR: exactly one erased location; the output is the XOR of every other row
//       (XORCode.java:115-145 ignores toRead/notToRead). Rows the caller passes
//       as NULL are the zeros the reference reads there (StripeReader.java:111-120).
hrs_status decode5_matrix(hrs_codec* c, const int* erased, int ne, const int* ntr, int nn,
                          const uint8_t* const* rows, std::vector<uint8_t>& tmp, const uint8_t** out,
                          const int* to_read = nullptr, int nr = -1) {
  for (int t = 0; t < ne; ++t)
    if (erased[t] < 0 || erased[t] >= c->n) return fail(c, HRS_EINVAL, "erased location %d out of range", erased[t]);
  if (c->kind == HRS_CODE_XOR) {
    if (ne != 1) return fail(c, HRS_EINVAL, "XOR code decodes exactly one erased location (got %d)", ne);
    tmp.assign(c->n, 1);
    tmp[erased[0]] = 0;
    if (rows)
      for (int l = 0; l < c->n; ++l)
        if (!rows[l]) tmp[l] = 0;
    *out = tmp.data();
    return HRS_OK;
  }
  if (c->kind == HRS_CODE_SRC) {
    // without an explicit locationsToRead (device calls), it is every
    // location outside not_to_read, as Decoder.java:303-338 builds them
    std::vector<int> tr;
    if (!to_read || nr < 0) {
      for (int l = 0; l < c->n; ++l)
        if (std::find(ntr, ntr + nn, l) == ntr + nn) tr.push_back(l);
    } else {
      tr.assign(to_read, to_read + nr);
    }
    std::vector<int> key{3, ne};
    key.insert(key.end(), erased, erased + ne);
    key.push_back(static_cast<int>(tr.size()));
    key.insert(key.end(), tr.begin(), tr.end());
    key.push_back(nn);
    key.insert(key.end(), ntr, ntr + nn);
    auto it = c->decode_cache.find(key);
    if (it == c->decode_cache.end()) {
      std::vector<uint8_t> d;
      hrs_status st = build_src_decode_matrix(c, erased, ne, tr.data(), static_cast<int>(tr.size()), ntr, nn, d);
      if (st != HRS_OK) return st;
      if (c->decode_cache.size() > 4096) c->decode_cache.clear();
      it = c->decode_cache.emplace(key, std::move(d)).first;
    }
    *out = it->second.data();
    return HRS_OK;
  }
  if (c->kind == HRS_CODE_RS && nn > c->p)
    return fail(c, HRS_EINVAL, "%d not-to-read locations > parity size %d", nn, c->p);
  hrs_status st;
  const std::vector<uint8_t>* d = cached_decode_matrix(c, erased, ne, ntr, nn, 1, &st);
  if (!d) return st;
  *out = d->data();
  return HRS_OK;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// The compile-time encode kernels hold the hops RS generator (rs) or the
// ISA-L Cauchy rows (nrs) of a (k, p) shape; only those families' G may take
// them. SRC's G (XOR groups over RS(k, r)) and XOR's all-ones row may not.
bool static_encode_family(const hrs_codec* c) { return c->kind == HRS_CODE_RS || c->kind == HRS_CODE_NRS; }

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

// Device scratch for the host-buffer calls: `rows` rows of `pitch` bytes.
size_t pitch_for(size_t len) { return (len + 255) & ~static_cast<size_t>(255); }

// Host rows -> device, apply m, device -> host rows; synchronous. The rows
// (pageable: a JNI-pinned Java array) go through pinned staging in column
// chunks over two slots: while the copy pool moves chunk j into one slot's
// staging (and chunk j-2's outputs out of it), the GPU runs chunk j-1's H2D,
// kernel and D2H on the other slot's stream.
size_t host_chunk_bytes() {
  static const size_t v = [] {
    const char* e = getenv("HRS_HOST_CHUNK");
    long x = e ? atol(e) : 0;
    if (x < static_cast<long>(hrs::kWindowBytes)) x = 512 << 10;  // measured best (tools/host_sweep.sh)
    return static_cast<size_t>(x) / hrs::kWindowBytes * hrs::kWindowBytes;
  }();
  return v;
}

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
  h.bytes = 0;
  hipError_t e = hipMalloc(&h.dev, bytes);
  if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
  e = hipHostMalloc(&h.pin, bytes, hipHostMallocDefault);
  if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
  h.bytes = bytes;
  return HRS_OK;
}

size_t crc_raw_bytes_for(size_t len, size_t nstripes, int nrows);
hrs_status run_crc(hrs_codec* c, const uint8_t* const* rows, const size_t* strides, int nrows, size_t len,
                   size_t nstripes, const uint32_t* crc_in, uint32_t* crc_out, hipStream_t s, uint32_t* raw);
hrs_status encode_crc_impl(hrs_codec* c, const uint8_t* const* in_rows, size_t in_stride, uint8_t* const* out_rows,
                           size_t out_stride, size_t len, size_t nstripes, const uint32_t* crc_in, uint32_t* crc_out,
                           hipStream_t s, uint32_t* raw);

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
  const size_t chunk = std::min(len, host_chunk_bytes());
  const size_t pitch = pitch_for(chunk);
  const size_t nchunks = (len + chunk - 1) / chunk;
  // slot layout: nlive + nout rows of `pitch`, then (CRC only) the chunk's
  // ncrc CRC words, then the raw window-CRC scratch (device side only)
  const size_t crc_off = pitch * static_cast<size_t>(nlive + nout);
  const size_t raw_off = crc_off + ((ncrc * sizeof(uint32_t) + 255) & ~static_cast<size_t>(255));
  const size_t need = ncrc ? raw_off + crc_raw_bytes_for(chunk, 1, ncrc) : crc_off;
  for (int i = 0; i < 2; ++i) {
    hrs_status st = host_slot(c, i, need);
    if (st != HRS_OK) return st;
  }
  hrs::CopyPool& pool = hrs::CopyPool::instance();
  std::vector<hrs::CopyJob> jobs;
  size_t pend_off[2] = {0, 0}, pend_len[2] = {0, 0};
  bool pending[2] = {false, false};
  auto finish = [&](int sl) -> hrs_status {  // wait for a slot, copy its outputs out
    if (!pending[sl]) return HRS_OK;
    hipError_t e = hipEventSynchronize(c->host[sl].done);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventSynchronize");
    jobs.clear();
    for (int o = 0; o < nout; ++o)
      jobs.push_back({out_rows[o] + pend_off[sl], c->host[sl].pin + pitch * (nlive + o), pend_len[sl]});
    pool.run(jobs);
    if (ncrc) {  // chunks finish in order: chain this one onto the running values
      const uint32_t* part = reinterpret_cast<const uint32_t*>(c->host[sl].pin + crc_off);
      const hrs::crc::Mat& z = crc_zmat(c, pend_len[sl]);
      for (int r = 0; r < ncrc; ++r) crc.out[r] = hrs::crc::apply(z, crc.out[r]) ^ part[r];
    }
    pending[sl] = false;
    return HRS_OK;
  };
  std::vector<const uint8_t*> din(nin);
  std::vector<uint8_t*> dout(nout);
  for (size_t j = 0; j < nchunks; ++j) {
    const int sl = static_cast<int>(j & 1);
    hrs_codec::HostSlot& h = c->host[sl];
    hrs_status st = finish(sl);
    if (st != HRS_OK) return st;
    const size_t off = j * chunk, lj = std::min(chunk, len - off);
    jobs.clear();
    for (int i = 0; i < nin; ++i)
      if (slot_of[i] >= 0) jobs.push_back({h.pin + pitch * slot_of[i], in_rows[i] + off, lj});
    pool.run(jobs);
    if (nlive > 0) {
      hipError_t e = hipMemcpyAsync(h.dev, h.pin, pitch * (nlive - 1) + lj, hipMemcpyHostToDevice, h.stream);
      if (e != hipSuccess) return hip_fail(c, e, "hipMemcpyAsync H2D");
    }
    for (int i = 0; i < nin; ++i) din[i] = slot_of[i] >= 0 ? h.dev + pitch * slot_of[i] : nullptr;
    for (int o = 0; o < nout; ++o) dout[o] = h.dev + pitch * (nlive + o);
    uint32_t* dcrc = reinterpret_cast<uint32_t*>(h.dev + crc_off);
    uint32_t* draw = reinterpret_cast<uint32_t*>(h.dev + raw_off);
    if (crc.mode == kCrcEncode)
      st = encode_crc_impl(c, din.data(), 0, dout.data(), 0, lj, 1, nullptr, dcrc, h.stream, draw);
    else
      st = run_apply(c, m, nout, nin, din.data(), 0, dout.data(), 0, lj, 1, h.stream, static_kp);
    if (st != HRS_OK) return st;
    if (crc.mode == kCrcOutputs) {
      std::vector<size_t> strides(nout, 0);
      st = run_crc(c, dout.data(), strides.data(), nout, lj, 1, nullptr, dcrc, h.stream, draw);
      if (st != HRS_OK) return st;
    }
    // outputs (and the chunk CRCs right behind them) back to the staging
    const size_t back = ncrc ? crc_off + ncrc * sizeof(uint32_t) - pitch * nlive : pitch * (nout - 1) + lj;
    hipError_t e = hipMemcpyAsync(h.pin + pitch * nlive, h.dev + pitch * nlive, back, hipMemcpyDeviceToHost, h.stream);
    if (e != hipSuccess) return hip_fail(c, e, "hipMemcpyAsync D2H");
    e = hipEventRecord(h.done, h.stream);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
    pending[sl] = true;
    pend_off[sl] = off;
    pend_len[sl] = lj;
  }
  for (size_t j = nchunks > 2 ? nchunks - 2 : 0; j < nchunks; ++j) {
    hrs_status st = finish(static_cast<int>(j & 1));
    if (st != HRS_OK) return st;
  }
  return HRS_OK;
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
  a.bytes = 0;
  hipError_t e = hipMalloc(&a.dev, bytes);
  if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
  e = hipHostMalloc(&a.pin, bytes, hipHostMallocDefault);
  if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
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
    if (slot_of[i] >= 0) jobs.push_back({a.pin + pitch * slot_of[i], in_rows[i], len});
  hrs::CopyPool::instance().run(jobs);
  if (nlive > 0) {
    hipError_t e = hipMemcpyAsync(a.dev, a.pin, pitch * (nlive - 1) + len, hipMemcpyHostToDevice, a.stream);
    if (e != hipSuccess) return hip_fail(c, e, "hipMemcpyAsync H2D");
  }
  std::vector<const uint8_t*> din(nin);
  std::vector<uint8_t*> dout(nout);
  for (int i = 0; i < nin; ++i) din[i] = slot_of[i] >= 0 ? a.dev + pitch * slot_of[i] : nullptr;
  for (int o = 0; o < nout; ++o) dout[o] = a.dev + pitch * (nlive + o);
  uint32_t* dcrc = reinterpret_cast<uint32_t*>(a.dev + crc_off);
  uint32_t* draw = reinterpret_cast<uint32_t*>(a.dev + raw_off);
  if (crc_mode == kCrcEncode)
    st = encode_crc_impl(c, din.data(), 0, dout.data(), 0, len, 1, nullptr, dcrc, a.stream, draw);
  else
    st = run_apply(c, m, nout, nin, din.data(), 0, dout.data(), 0, len, 1, a.stream, static_kp);
  if (st != HRS_OK) return st;
  if (crc_mode == kCrcOutputs) {
    std::vector<size_t> strides(nout, 0);
    st = run_crc(c, dout.data(), strides.data(), nout, len, 1, nullptr, dcrc, a.stream, draw);
    if (st != HRS_OK) return st;
  }
  const size_t back = ncrc ? crc_off + ncrc * sizeof(uint32_t) - pitch * nlive : pitch * (nout - 1) + len;
  hipError_t e = hipMemcpyAsync(a.pin + pitch * nlive, a.dev + pitch * nlive, back, hipMemcpyDeviceToHost, a.stream);
  if (e != hipSuccess) return hip_fail(c, e, "hipMemcpyAsync D2H");
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

void init_encode_matrix(hrs_codec* c) {
  c->g.resize(static_cast<size_t>(c->p) * c->k);
  if (c->kind == HRS_CODE_XOR) {
    std::fill(c->g.begin(), c->g.end(), 1);  // XORCode.encodeBulk, XORCode.java:99-113
  } else if (c->kind == HRS_CODE_SRC) {
    src_encode_matrix(c);
  } else if (c->kind == HRS_CODE_NRS) {
    // Cauchy rows of ISA-L gf_gen_cauchy1_matrix (erasure_coder.c:47-60):
    // parity r = Apache row k + r, G[r][c] = 1 / ((k + r) ^ c)
    for (int r = 0; r < c->p; ++r)
      for (int j = 0; j < c->k; ++j) c->g[r * c->k + j] = gf::inv(static_cast<uint8_t>((c->k + r) ^ j));
  } else
    gf::encode_matrix(c->k, c->p, c->g.data());
}

bool sorted_unique_ok(const int* v, int nv, int n) {
  for (int i = 0; i < nv; ++i)
    if (v[i] < 0 || v[i] >= n) return false;
  return true;
}

// ------------------------------------------------------------------ CRC-32

hrs_status upload(hrs_codec* c, const std::vector<uint32_t>& h, uint32_t** out) {
  hipError_t e = hipMalloc(out, h.size() * 4);
  if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipMalloc: %s", hipGetErrorString(e));
  e = hipMemcpy(*out, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(c, e, "hipMemcpy tables");
  return HRS_OK;
}

// The LDS image of the window kernels (crc_window_kernel, the fused encode +
// CRC): slicing tables (32 bank-private copies), then Z_chunk (joins a lane's
// successive pieces, `chunk` bytes apart) and the lane tree Z_{piece * 2^t}
// (lane l + 2^t is piece * 2^t bytes later).
hrs_status crc_image(hrs_codec* c, uint64_t piece, uint64_t chunk, uint32_t** out) {
  if (*out) return HRS_OK;
  namespace cr = hrs::crc;
  std::vector<uint32_t> h(hrs::kCrcLdsWordsA);
  const cr::Slice4 sl = cr::make_slice4();
  for (int j = 0; j < 4; ++j)
    for (int v = 0; v < 256; ++v)
      for (int r = 0; r < hrs::kCrcRep; ++r) h[hrs::crc_slice_word(j, v, r)] = sl.s[j].t[v];
  cr::to_tables(cr::zeros(chunk), &h[hrs::kCrcSliceWords]);
  for (int t = 0; t < 6; ++t) cr::to_tables(cr::zeros(piece << t), &h[hrs::kCrcSliceWords + (1 + t) * 1024]);
  return upload(c, h, out);
}

hrs_status crc_window_tables(hrs_codec* c) {
  return crc_image(c, hrs::crc::kPieceBytes, hrs::crc::kChunkBytes, &c->crc_tables_a);
}

// Fold tables for rows of `len` bytes cut in windows of `win` bytes (32 KiB,
// or a smaller fused window), keyed by (len, win).
hrs_status crc_fold_tables(hrs_codec* c, uint64_t len, uint64_t win, const uint32_t** out) {
  const uint64_t key = len << 5 | static_cast<uint64_t>(__builtin_ctzll(win));
  auto it = c->crc_fold_tables.find(key);
  if (it != c->crc_fold_tables.end()) {
    *out = it->second;
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
  if (c->crc_fold_tables.size() >= 16) {
    (void)hipDeviceSynchronize();
    for (auto& kv : c->crc_fold_tables) (void)hipFree(kv.second);
    c->crc_fold_tables.clear();
  }
  uint32_t* d = nullptr;
  hrs_status st = upload(c, h, &d);
  if (st != HRS_OK) return st;
  c->crc_fold_tables[key] = d;
  *out = d;
  return HRS_OK;
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
  const uint32_t* fold = nullptr;
  hrs_status st = crc_fold_tables(c, len, win, &fold);
  if (st != HRS_OK) return st;
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
  return HRS_OK;
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

// Encode + CRC-32 of the k sources and p parities (hrs_encode_crc_dev's
// semantics) with raw window CRCs in `raw` (crc_raw_bytes_for(len, nstripes, n)).
hrs_status encode_crc_impl(hrs_codec* c, const uint8_t* const* in_rows, size_t in_stride, uint8_t* const* out_rows,
                           size_t out_stride, size_t len, size_t nstripes, const uint32_t* crc_in, uint32_t* crc_out,
                           hipStream_t s, uint32_t* raw) {
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
    a.nwin = len / (subs * hrs::kWindowBytes);
    a.nstripes = nstripes;
    a.raw = raw;
    a.tables = c->crc_tables_a;
    bool handled = false;
    const int family = c->kind == HRS_CODE_NRS ? hrs::kStaticCauchy : hrs::kStaticRs;
    hipError_t e = hrs::launch_encode_crc(family, k, p, a, hrs::device_cu_count(), s, &handled);
    if (e != hipSuccess) return hip_fail(c, e, "fused encode+crc launch");
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

}  // namespace

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

const char* hrs_version(void) { return "hrs 0.1.0 (gfx950)"; }

hrs_status hrs_create(int stripe_size, int parity_size, const hrs_opts* opts, hrs_codec** out) {
  return hrs_create_code(HRS_CODE_RS, stripe_size, parity_size, opts, out);
}

int hrs_code_kind(const hrs_codec* c) { return c ? c->kind : -1; }

}  // extern "C"

namespace {

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
  if (e != hipSuccess || dev >= ndev)
    return fail(nullptr, HRS_EDEVICE, "no HIP device %d (%s)", dev, hipGetErrorString(e));
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

}  // namespace

extern "C" {

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
  for (auto& kv : c->crc_fold_tables) (void)hipFree(kv.second);
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
  for (auto& a : c->async) {
    if (a.stream) {
      (void)hipStreamSynchronize(a.stream);
      (void)hipStreamDestroy(a.stream);
    }
    if (a.done) (void)hipEventDestroy(a.done);
    if (a.dev) (void)hipFree(a.dev);
    if (a.pin) (void)hipHostFree(a.pin);
  }
  for (auto& h : c->hbatch) {
    if (h.stream) {
      (void)hipStreamSynchronize(h.stream);
      (void)hipStreamDestroy(h.stream);
    }
    if (h.done) (void)hipEventDestroy(h.done);
    if (h.dev) (void)hipFree(h.dev);
    if (h.pin) (void)hipHostFree(h.pin);
  }
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
  if (!sorted_unique_ok(erased, ne, c->n) || !sorted_unique_ok(ntr, nn, c->n) ||
      (to_read && !sorted_unique_ok(to_read, nr, c->n)))
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
  if (!sorted_unique_ok(erased, ne, c->n) || !sorted_unique_ok(ntr, nn, c->n) || (to_read && !sorted_unique_ok(to_read, nr, c->n)))
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

}  // extern "C"

namespace {

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
// through a ring of device slots, one stream each: H2D of exactly the rows
// the chunk's codes read -> kernel -> D2H of exactly the rows they write.
// Pinned caller buffers are DMA'd directly and the whole job is queued before
// the host waits once; pageable ones go through each slot's pinned staging
// (copy pool), the host then waits for a slot before refilling it.

bool is_pinned(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t attr{};
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory is reported as an error: clear it
    return false;
  }
  return attr.type == hipMemoryTypeHost;
}

size_t hbatch_target_bytes() {
  static const size_t v = [] {
    const char* e = getenv("HRS_HBATCH_BYTES");
    long x = e ? atol(e) : 0;
    return static_cast<size_t>(x > 0 ? x : 48l << 20);  // device image per chunk
  }();
  return v;
}

hrs_status hbatch_slot(hrs_codec* c, int i, size_t dev_bytes, size_t pin_bytes) {
  hrs_codec::HostBatchSlot& h = c->hbatch[i];
  if (!h.stream) {
    hipError_t e = hipStreamCreateWithFlags(&h.stream, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail(c, e, "hipStreamCreate");
    e = hipEventCreateWithFlags(&h.done, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventCreate");
  }
  if (h.dev_bytes < dev_bytes) {
    (void)hipStreamSynchronize(h.stream);
    if (h.dev) (void)hipFree(h.dev);
    h.dev = nullptr;
    h.dev_bytes = 0;
    hipError_t e = hipMalloc(&h.dev, dev_bytes);
    if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipMalloc(%zu): %s", dev_bytes, hipGetErrorString(e));
    h.dev_bytes = dev_bytes;
  }
  if (h.pin_bytes < pin_bytes) {
    (void)hipStreamSynchronize(h.stream);
    if (h.pin) (void)hipHostFree(h.pin);
    h.pin = nullptr;
    h.pin_bytes = 0;
    hipError_t e = hipHostMalloc(&h.pin, pin_bytes, hipHostMallocDefault);
    if (e != hipSuccess) return fail(c, HRS_ENOMEM, "hipHostMalloc(%zu): %s", pin_bytes, hipGetErrorString(e));
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
  const bool pinned = is_pinned(hin) && is_pinned(hout);
  const size_t dev_bytes = chunk * (img_stripe + out_stripe_dev);
  const size_t pin_bytes = pinned ? 0 : dev_bytes;  // staging mirrors the device image
  for (int i = 0; i < hrs::kHostBatchSlots; ++i) {
    hrs_status st = hbatch_slot(c, i, dev_bytes, pin_bytes);
    if (st != HRS_OK) return st;
  }
  hrs::CopyPool& pool = hrs::CopyPool::instance();
  std::vector<hrs::CopyJob> jobs;
  struct Pending {
    bool busy = false;
    size_t s0 = 0, ns = 0;
  } pend[hrs::kHostBatchSlots];
  // pageable: wait for a slot, then copy its outputs out of staging
  auto finish = [&](int sl) -> hrs_status {
    if (!pend[sl].busy) return HRS_OK;
    hrs_codec::HostBatchSlot& h = c->hbatch[sl];
    hipError_t e = hipEventSynchronize(h.done);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventSynchronize");
    if (!pinned) {
      jobs.clear();
      const uint8_t* pout = h.pin + chunk * img_stripe;
      for (size_t i = 0; i < pend[sl].ns; ++i) {
        const size_t s = pend[sl].s0 + i;
        for (int t = 0; t < writes(s); ++t)
          jobs.push_back({hout + s * out_stripe + t * out_row, pout + i * out_stripe_dev + t * dpitch, len});
      }
      pool.run(jobs);
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
      hrs_status st = finish(sl);
      if (st != HRS_OK) return st;
      jobs.clear();
      for (size_t i = 0; i < ns; ++i)
        for (const RowRun& r : reads(s0 + i))
          for (int q = 0; q < r.cnt; ++q) {
            const int l = r.l0 + q;
            jobs.push_back({h.pin + i * img_stripe + l * dpitch, hin + (s0 + i) * in_stripe + l * in_row, len});
          }
      pool.run(jobs);
    }
    uint8_t* dimg = h.dev;
    uint8_t* dout = h.dev + chunk * img_stripe;
    for (size_t i = 0; i < ns; ++i) {
      const uint8_t* src = pinned ? hin + (s0 + i) * in_stripe : h.pin + i * img_stripe;
      hrs_status st = h2d_runs(c, reads(s0 + i), dimg + i * img_stripe, dpitch, src, pinned ? in_row : dpitch, len,
                               h.stream);
      if (st != HRS_OK) return st;
    }
    hrs_status st = compute(h.stream, s0, ns, dimg, img_stripe, dpitch, dout, out_stripe_dev);
    if (st != HRS_OK) return st;
    for (size_t i = 0; i < ns; ++i) {
      const size_t s = s0 + i;
      st = pinned ? d2h_rows(c, hout + s * out_stripe, out_row, dout + i * out_stripe_dev, dpitch, len, writes(s), h.stream)
                  : d2h_rows(c, h.pin + chunk * img_stripe + i * out_stripe_dev, dpitch, dout + i * out_stripe_dev,
                             dpitch, len, writes(s), h.stream);
      if (st != HRS_OK) return st;
    }
    hipError_t e = hipEventRecord(h.done, h.stream);
    if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
    pend[sl].busy = true;
    pend[sl].s0 = s0;
    pend[sl].ns = ns;
  }
  for (int sl = 0; sl < hrs::kHostBatchSlots; ++sl) {
    hrs_status st = finish(sl);
    if (st != HRS_OK) return st;
  }
  return HRS_OK;
}

// A failed host batch may leave slot work in flight: drain every slot stream.
hrs_status drain_hbatch(hrs_codec* c, hrs_status st) {
  if (st != HRS_OK)
    for (auto& h : c->hbatch)
      if (h.stream) (void)hipStreamSynchronize(h.stream);
  return st;
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
  BatchPlanSet ps;
  hrs_status st = build_batch_plans(c, erased, max_erased, nstripes, ps);
  if (st != HRS_OK) return st;
  if (ps.max_nout == 0) return HRS_OK;
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
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

hrs_status hrs_encode_batch_host(hrs_codec* c, uint8_t* stripes, size_t row_stride, size_t stripe_stride, size_t len,
                                 size_t nstripes) {
  if (!c) return HRS_EINVAL;
  if (!stripes) return fail(c, HRS_EINVAL, "stripes is NULL");
  if (nstripes == 0 || len == 0) return HRS_OK;
  DeviceGuard g(c->device);
  if (!g.ok) return fail(c, HRS_EDEVICE, "cannot select HIP device %d", c->device);
  const int k = c->k, p = c->p;
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
  if (!sorted_unique_ok(erased, ne, c->n) || !sorted_unique_ok(ntr, nn, c->n) ||
      (to_read && !sorted_unique_ok(to_read, nr, c->n)))
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
    if (e != hipSuccess) st = hip_fail(c, e, "hipEventSynchronize");
  }
  if (st == HRS_OK && a->queued) {
    std::vector<hrs::CopyJob> jobs;
    for (int o = 0; o < a->nout; ++o) jobs.push_back({outputs[o], a->pin + a->pitch * (a->nlive + o), a->len});
    hrs::CopyPool::instance().run(jobs);
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

int hrs_pending(const hrs_codec* c) {
  if (!c) return -1;
  int n = 0;
  for (const auto& s : c->async) n += s.busy;
  return n;
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
