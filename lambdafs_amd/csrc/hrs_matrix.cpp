// Coding matrices of every code family behind the C ABI, in closed form:
// the RS decode rows (syndromes + Vandermonde solve of ReedSolomonCode.java as
// one GF(2^8) matrix), ISA-L's Cauchy decode for `nrs`, SimpleRegeneratingCode's
// local groups and decode cases, the per-handle decode-matrix cache, and the
// encode matrix of each family. Host code only (no kernels here).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/hrs.h"
#include "hrs_codec.hpp"
#include "gf256.hpp"

namespace hrs::api {

namespace gf = hrs::gf;

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

// GaloisField.divide through the reference's table (GaloisField.java:107-118):
// divTable[a][0] is never written, so a division by zero yields 0. It happens
// when a location list repeats an entry (x_j ^ x_{j-i-1} == 0 in the solve).
constexpr uint8_t java_div(uint8_t a, uint8_t b) { return b == 0 ? 0 : gf::div(a, b); }

// ReedSolomonCode.decode 3-arg (ReedSolomonCode.java:127-142) on one column
// of symbols: zero the locations (zero_locs; the bulk 3-arg decodeBulk,
// :168-185, substitutes the rows as they are), syndromes S_i = data(alpha^i)
// (GaloisField.substitute, :375-383), then GaloisField.solveVandermondeSystem
// (:232-246) in place. values[nl].
void rs_decode_column(int n, uint8_t* data, const int* loc, int nl, bool zero_locs, uint8_t* values) {
  if (nl == 0) return;
  if (zero_locs)
    for (int i = 0; i < nl; ++i) data[loc[i]] = 0;
  std::vector<uint8_t> x(nl);
  for (int i = 0; i < nl; ++i) {
    x[i] = gf::alpha_pow(loc[i]);
    const uint8_t a = gf::alpha_pow(i);
    uint8_t r = 0, y = 1;
    for (int l = 0; l < n; ++l) {
      r ^= gf::mul(data[l], y);
      y = gf::mul(a, y);
    }
    values[i] = r;
  }
  for (int i = 0; i < nl - 1; ++i)
    for (int j = nl - 1; j > i; --j) values[j] ^= gf::mul(x[i], values[j - 1]);
  for (int i = nl - 1; i >= 0; --i) {
    for (int j = i + 1; j < nl; ++j) values[j] = java_div(values[j], x[j] ^ x[j - i - 1]);
    for (int j = i; j < nl - 1; ++j) values[j] ^= values[j + 1];
  }
}

// The decode rows over an RS stripe of n locations (see hrs.h), built as
// SURVEY §0.3 prescribes: the reference decode runs on every unit vector e_l
// and its outputs form column l. The decode is GF(2^8)-linear in the data
// (every division is by a value of the locations alone), so D * stripe
// reproduces the Java byte for byte on every input it accepts, repeated
// locations and erased locations outside not_to_read included.
//  zero_ntr = 1, decodeBulk 5-arg (:144-166, :191-211): decode over ntr with
//    ntr zeroed; output t copies the FIRST ntr entry equal to erased[t], and
//    stays 0 when there is none (an erased value of any range).
//  zero_ntr = 0, decodeBulk 3-arg (ntr is the erased list): nothing zeroed,
//    output t is solution t.
// Locations in ntr are validated by the caller.
void rs_decode_rows(int n, const int* erased, int ne, const int* ntr, int nn, int zero_ntr, std::vector<uint8_t>& d) {
  d.assign(static_cast<size_t>(ne) * n, 0);
  if (ne == 0 || nn == 0) return;
  std::vector<int> pick(ne, -1);  // solution index feeding output t
  for (int t = 0; t < ne; ++t) {
    if (!zero_ntr && t < nn && ntr[t] == erased[t]) {
      pick[t] = t;
      continue;
    }
    for (int j = 0; j < nn; ++j)
      if (ntr[j] == erased[t]) {
        pick[t] = j;
        break;
      }
  }
  std::vector<uint8_t> col(n), y(nn);
  for (int l = 0; l < n; ++l) {
    std::fill(col.begin(), col.end(), 0);
    col[l] = 1;
    rs_decode_column(n, col.data(), ntr, nn, zero_ntr != 0, y.data());
    for (int t = 0; t < ne; ++t)
      if (pick[t] >= 0) d[static_cast<size_t>(t) * n + l] = y[pick[t]];
  }
}

// RS decode rows with the reference's argument limits: a not-to-read
// location outside [0, n) indexes primitivePower / data out of bounds in the
// Java (an exception); more than p of them overflow errSignature
// (ReedSolomonCode.java:60), checked by the callers that know the form.
hrs_status build_decode_matrix(hrs_codec* c, const int* erased, int ne, const int* ntr, int nn,
                               int zero_ntr, std::vector<uint8_t>& d) {
  const int n = c->n;
  for (int j = 0; j < nn; ++j)
    if (ntr[j] < 0 || ntr[j] >= n) return fail(c, HRS_EINVAL, "location %d out of range [0,%d)", ntr[j], n);
  if (!zero_ntr)  // the 3-arg form indexes primitivePower with every erased location
    for (int t = 0; t < ne; ++t)
      if (erased[t] < 0 || erased[t] >= n) return fail(c, HRS_EINVAL, "erased location %d out of range", erased[t]);
  rs_decode_rows(n, erased, ne, ntr, nn, zero_ntr, d);
  return HRS_OK;
}

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
  rs_decode_rows(nrs, ers.data(), m, ers.data(), m, 1, drs);
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
//  RS : cached matrix of the reference decode (rs_decode_rows); more than p
//       not-to-read locations throw in the Java (errSignature is sized p,
//       ReedSolomonCode.java:60).
//  NRS: see build_nrs_decode_matrix.
//  XOR: exactly one erased location; the output is the XOR of every other row
//       (XORCode.java:115-145 ignores toRead/notToRead). Rows the caller passes
//       as NULL are the zeros the reference reads there (StripeReader.java:111-120).
hrs_status decode5_matrix(hrs_codec* c, const int* erased, int ne, const int* ntr, int nn,
                          const uint8_t* const* rows, std::vector<uint8_t>& tmp, const uint8_t** out,
                          const int* to_read, int nr) {
  // ReedSolomonCode's 5-arg decode only compares erased locations with
  // not-to-read ones (ReedSolomonCode.java:158-165): any value is accepted
  // and one that matches none decodes to 0. The other families index with them.
  if (c->kind != HRS_CODE_RS)
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

}  // namespace hrs::api
