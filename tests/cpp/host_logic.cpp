// Host-only logic of libhrs under the sanitizers (make asan): every code
// family's matrices and survivor lists through HRS_DEVICE_NONE handles,
// checked against the oracle on unit vectors / non-codeword columns; the
// decode-matrix cache driven past its eviction bound; batch-plan building for
// heterogeneous and wide patterns; argument errors. Device calls on a
// host-only handle must fail cleanly (HRS_EDEVICE) after their host-side work.
// Also runs the oracle's bulk loops at small sizes, so ASan/UBSan cover them.
//
// Prints one JSON line; exit status 0 iff every check passed.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "hrs.h"
#include "rs_oracle.h"

namespace {

int checks = 0, failures = 0;
std::string first;

void expect(bool ok, const std::string& what) {
  ++checks;
  if (!ok && failures++ == 0) first = what;
}

uint64_t rng_state = 0x5EED;
uint8_t rnd8() {
  rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
  return static_cast<uint8_t>(rng_state >> 56);
}

hrs_codec* host_handle(int code, int k, int p, int s = 0) {
  hrs_opts o{};
  o.device = HRS_DEVICE_NONE;
  hrs_codec* c = nullptr;
  const hrs_status st = code == HRS_CODE_SRC ? hrs_create_src(k, p, s, &o, &c) : hrs_create_code(code, k, p, &o, &c);
  expect(st == HRS_OK && c, "create host-only handle");
  return c;
}

// Decoder.java:303-338 arrays from an erased list and the code's survivors.
bool decoder_sets(hrs_codec* c, int n, const std::vector<int>& erased, std::vector<int>& tr, std::vector<int>& ntr) {
  std::vector<int> buf(n);
  int m = 0;
  if (hrs_locations_to_read_list(c, erased.data(), static_cast<int>(erased.size()), buf.data(), &m) != HRS_OK)
    return false;
  tr.clear();
  ntr.clear();
  for (int l = 0; l < n; ++l) {
    bool rd = false, er = false;
    for (int i = 0; i < m; ++i) rd |= buf[i] == l;
    for (int e : erased) er |= e == l;
    if (rd) tr.push_back(l);
    if (!rd || er) ntr.push_back(l);
  }
  return true;
}

uint8_t gmul(uint8_t a, uint8_t b) { return static_cast<uint8_t>(orc_gf_mul(a, b)); }

// D (ne x n) applied to columns cols[n][C]
std::vector<std::vector<uint8_t>> apply(const std::vector<uint8_t>& d, int ne, int n,
                                        const std::vector<std::vector<uint8_t>>& cols) {
  const size_t C = cols[0].size();
  std::vector<std::vector<uint8_t>> out(ne, std::vector<uint8_t>(C, 0));
  for (int t = 0; t < ne; ++t)
    for (int l = 0; l < n; ++l)
      if (d[static_cast<size_t>(t) * n + l])
        for (size_t j = 0; j < C; ++j) out[t][j] ^= gmul(d[static_cast<size_t>(t) * n + l], cols[l][j]);
  return out;
}

void rs_checks(int k, int p) {
  const int n = k + p;
  hrs_codec* c = host_handle(HRS_CODE_RS, k, p);
  std::vector<uint8_t> g(static_cast<size_t>(k) * p);
  expect(hrs_encode_matrix(c, g.data()) == HRS_OK, "rs encode matrix");
  std::vector<int> msg(k), par(p);
  for (int col = 0; col < k; ++col) {
    for (int j = 0; j < k; ++j) msg[j] = j == col;
    orc_rs_encode(k, p, msg.data(), par.data());
    for (int r = 0; r < p; ++r) expect(g[r * k + col] == par[r], "rs G vs oracle");
  }
  // every 1- and 2-erasure pattern: D vs the oracle's per-byte decodeBulk on
  // non-codeword columns
  const size_t C = 8;
  std::vector<std::vector<uint8_t>> cols(n, std::vector<uint8_t>(C));
  for (auto& r : cols)
    for (auto& b : r) b = rnd8();
  for (int a = 0; a < n; ++a)
    for (int b = a; b < n; ++b) {
      std::vector<int> er = {a};
      if (b != a) er.push_back(b);
      std::vector<int> tr, ntr;
      if (!decoder_sets(c, n, er, tr, ntr)) {
        expect(false, "rs locations");
        continue;
      }
      const int ne = static_cast<int>(er.size());
      std::vector<uint8_t> d(static_cast<size_t>(ne) * n);
      expect(hrs_decode_matrix(c, er.data(), ne, ntr.data(), static_cast<int>(ntr.size()), 1, d.data()) == HRS_OK,
             "rs decode matrix");
      std::vector<std::vector<uint8_t>> in = cols;
      for (int l : ntr) std::fill(in[l].begin(), in[l].end(), 0);
      std::vector<uint8_t*> rp(n), wp(ne);
      std::vector<std::vector<uint8_t>> want(ne, std::vector<uint8_t>(C));
      for (int l = 0; l < n; ++l) rp[l] = in[l].data();
      for (int t = 0; t < ne; ++t) wp[t] = want[t].data();
      orc_rs_decode_bulk5(k, p, rp.data(), wp.data(), er.data(), ne, tr.data(), static_cast<int>(tr.size()),
                          ntr.data(), static_cast<int>(ntr.size()), C);
      expect(apply(d, ne, n, in) == want, "rs D vs oracle decodeBulk");
      // 3-arg decode matrix vs the oracle's bulk 3-arg
      std::vector<uint8_t> d3(static_cast<size_t>(ne) * n);
      expect(hrs_decode_matrix(c, er.data(), ne, er.data(), ne, 0, d3.data()) == HRS_OK, "rs decode3 matrix");
      std::vector<std::vector<uint8_t>> w3(ne, std::vector<uint8_t>(C));
      std::vector<std::vector<uint8_t>> in3 = cols;
      std::vector<uint8_t*> rp3(n), wp3(ne);
      for (int l = 0; l < n; ++l) rp3[l] = in3[l].data();
      for (int t = 0; t < ne; ++t) wp3[t] = w3[t].data();
      orc_rs_decode_bulk3(k, p, rp3.data(), wp3.data(), er.data(), ne, C);
      expect(apply(d3, ne, n, cols) == w3, "rs D3 vs oracle decodeBulk3");
    }
  // the device entry points on a host-only handle: host work, then EDEVICE
  std::vector<const uint8_t*> rows(n, nullptr);
  std::vector<uint8_t*> outs(p, nullptr);
  std::vector<uint8_t> buf(64);
  for (auto& r : rows) r = buf.data();
  for (auto& o : outs) o = buf.data();
  expect(hrs_encode(c, rows.data(), outs.data(), 64) == HRS_EDEVICE, "host-only encode -> EDEVICE");
  // asynchronous rounds: no slot is taken by a failed submit
  uint64_t t = 7;
  expect(hrs_encode_submit(c, rows.data(), 64, 1, &t) == HRS_EDEVICE && t == 0, "host-only submit -> EDEVICE");
  expect(hrs_encode_submit(c, rows.data(), 64, 0, nullptr) == HRS_EINVAL, "submit without a ticket");
  expect(hrs_pending(c) == 0, "failed submits hold no slot");
  // zero-length rounds need no device: a ticket that collects to nothing
  uint64_t z[5] = {0, 0, 0, 0, 0};
  int taken = 0;
  for (auto& zt : z) taken += hrs_encode_submit(c, rows.data(), 0, 1, &zt) == HRS_OK;
  expect(taken == 4 && hrs_pending(c) == 4 && z[4] == 0, "4 slots, the 5th submit refused");
  int nout = -1, ncrc = -1;
  size_t ln = 1;
  expect(hrs_ticket_shape(c, z[2], &nout, &ln, &ncrc) == HRS_OK && nout == p && ln == 0 && ncrc == n,
         "ticket shape");
  std::vector<uint32_t> crc(n, 0x1234u);
  expect(hrs_collect(c, z[2], outs.data(), nullptr) == HRS_EINVAL, "checksummed collect needs crc_io");
  expect(hrs_collect(c, z[2], outs.data(), crc.data()) == HRS_OK && crc[0] == 0x1234u && hrs_pending(c) == 3,
         "empty round leaves the running CRCs");
  expect(hrs_collect(c, z[2], outs.data(), crc.data()) == HRS_EINVAL, "a ticket collects once");
  for (int i : {0, 1, 3}) expect(hrs_collect(c, z[i], outs.data(), crc.data()) == HRS_OK, "collect the rest");
  expect(hrs_pending(c) == 0 && hrs_ticket_shape(c, z[0], nullptr, nullptr, nullptr) == HRS_EINVAL, "all collected");
  // hrs_release drops an uncollected operation and frees its slot
  for (auto& zt : z) zt = 0;
  taken = 0;
  for (int i = 0; i < 4; ++i) taken += hrs_encode_submit(c, rows.data(), 0, 0, &z[i]) == HRS_OK;
  expect(taken == 4 && hrs_release(c, z[1]) == HRS_OK && hrs_pending(c) == 3, "release frees a slot");
  expect(hrs_release(c, z[1]) == HRS_EINVAL && hrs_collect(c, z[1], outs.data(), nullptr) == HRS_EINVAL,
         "a released ticket is gone");
  expect(hrs_encode_submit(c, rows.data(), 0, 0, &z[4]) == HRS_OK && hrs_pending(c) == 4, "its slot is reusable");
  for (int i : {0, 2, 3, 4}) expect(hrs_release(c, z[i]) == HRS_OK, "release the rest");
  expect(hrs_pending(c) == 0 && hrs_release(nullptr, 1) == HRS_EINVAL, "all released");
  hrs_destroy(c);
}

void cache_and_batch_checks() {
  // RS(20,8): > 4096 distinct (erased, not-to-read) patterns through hrs_decode
  // (the cached path), crossing the cache's eviction bound
  const int k = 20, p = 8, n = 28;
  hrs_codec* c = host_handle(HRS_CODE_RS, k, p);
  std::vector<uint8_t> row(32, 1);
  std::vector<const uint8_t*> rp(n, row.data());
  std::vector<uint8_t> o0(32), o1(32);
  uint8_t* wp[2] = {o0.data(), o1.data()};
  int patterns = 0, edevice = 0;
  for (int a = 0; a < n && patterns < 5000; ++a)
    for (int b = a + 1; b < n && patterns < 5000; ++b)
      for (int x = 0; x < n && patterns < 5000; ++x) {
        if (x == a || x == b) continue;
        int er[2] = {a, b};
        int ntr[3] = {a, b, x};
        if (ntr[2] < ntr[1]) std::swap(ntr[2], ntr[1]);
        if (ntr[1] < ntr[0]) std::swap(ntr[1], ntr[0]);
        if (ntr[2] < ntr[1]) std::swap(ntr[2], ntr[1]);
        ++patterns;
        edevice += hrs_decode(c, rp.data(), wp, er, 2, nullptr, 0, ntr, 3, 32) == HRS_EDEVICE;
      }
  expect(patterns == 5000 && edevice == 5000, "5000 cached patterns -> EDEVICE after matrix build");
  // batch plans: mixed pattern widths, including ones beyond the batch kernel
  const size_t S = 64;
  std::vector<int> er(S * 8, -1);
  for (size_t s = 0; s < S; ++s) {
    const int ne = static_cast<int>(s % 9);  // 0..8 lost
    for (int t = 0; t < ne; ++t) er[s * 8 + t] = (static_cast<int>(s) * 3 + t * 5) % n;
    // keep each list ascending and distinct
    std::vector<int> v(er.begin() + s * 8, er.begin() + s * 8 + ne);
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    for (int t = 0; t < 8; ++t) er[s * 8 + t] = t < static_cast<int>(v.size()) ? v[t] : -1;
  }
  std::vector<uint8_t> img(static_cast<size_t>(n) * 64), out(8 * 64);
  expect(hrs_decode_batch_dev(c, img.data(), 64, 0, er.data(), 8, out.data(), 64, 0, 64, S, nullptr) == HRS_EDEVICE,
         "batch dev plans -> EDEVICE");
  expect(hrs_decode_batch_host(c, img.data(), 64, 0, er.data(), 8, out.data(), 64, 0, 64, S) == HRS_EDEVICE,
         "batch host plans -> EDEVICE");
  std::vector<int> bad(S, -1);
  bad[3] = 40;
  expect(hrs_decode_batch_host(c, img.data(), 64, 0, bad.data(), 1, out.data(), 64, 0, 64, S) == HRS_EINVAL,
         "batch out-of-range location -> EINVAL");
  hrs_destroy(c);
}

void other_codes() {
  // nrs: every not-to-read set of 1..4 of RS(10,4), D vs the oracle
  {
    const int k = 10, p = 4, n = 14;
    hrs_codec* c = host_handle(HRS_CODE_NRS, k, p);
    const size_t C = 6;
    std::vector<std::vector<uint8_t>> cols(n, std::vector<uint8_t>(C));
    for (auto& r : cols)
      for (auto& b : r) b = rnd8();
    for (int mask = 1; mask < (1 << n); ++mask) {
      if (__builtin_popcount(mask) > p) continue;
      std::vector<int> ntr;
      for (int l = 0; l < n; ++l)
        if (mask >> l & 1) ntr.push_back(l);
      const int nn = static_cast<int>(ntr.size());
      std::vector<uint8_t> d(static_cast<size_t>(nn) * n);
      expect(hrs_decode_matrix(c, ntr.data(), nn, ntr.data(), nn, 1, d.data()) == HRS_OK, "nrs matrix");
      std::vector<std::vector<uint8_t>> in = cols;
      for (int l : ntr) std::fill(in[l].begin(), in[l].end(), 0);
      std::vector<uint8_t*> rp(n), wp(nn);
      std::vector<std::vector<uint8_t>> want(nn, std::vector<uint8_t>(C));
      for (int l = 0; l < n; ++l) rp[l] = in[l].data();
      for (int t = 0; t < nn; ++t) wp[t] = want[t].data();
      expect(orc_nrs_decode_bulk(k, p, rp.data(), wp.data(), ntr.data(), nn, ntr.data(), nn, C) == 0, "nrs oracle");
      expect(apply(d, nn, n, in) == want, "nrs D vs oracle");
    }
    hrs_destroy(c);
  }
  // src(10,6,2): every 1..3-erasure pattern the code repairs
  {
    const int k = 10, p = 6, s = 2, n = 16;
    hrs_codec* c = host_handle(HRS_CODE_SRC, k, p, s);
    const size_t C = 6;
    std::vector<std::vector<uint8_t>> cols(n, std::vector<uint8_t>(C));
    for (auto& r : cols)
      for (auto& b : r) b = rnd8();
    int repaired = 0;
    for (int mask = 1; mask < (1 << n); ++mask) {
      if (__builtin_popcount(mask) > 3) continue;
      std::vector<int> er;
      for (int l = 0; l < n; ++l)
        if (mask >> l & 1) er.push_back(l);
      std::vector<int> tr, ntr;
      if (!decoder_sets(c, n, er, tr, ntr)) continue;  // TooManyErasedLocations
      const int ne = static_cast<int>(er.size());
      std::vector<uint8_t> d(static_cast<size_t>(ne) * n);
      expect(hrs_decode_matrix(c, er.data(), ne, ntr.data(), static_cast<int>(ntr.size()), 1, d.data()) == HRS_OK,
             "src matrix");
      std::vector<std::vector<uint8_t>> in = cols;
      for (int l : ntr) std::fill(in[l].begin(), in[l].end(), 0);
      std::vector<uint8_t*> rp(n), wp(ne);
      std::vector<std::vector<uint8_t>> want(ne, std::vector<uint8_t>(C));
      for (int l = 0; l < n; ++l) rp[l] = in[l].data();
      for (int t = 0; t < ne; ++t) wp[t] = want[t].data();
      expect(orc_src_decode_bulk(k, p, s, rp.data(), wp.data(), er.data(), ne, tr.data(), static_cast<int>(tr.size()),
                                 ntr.data(), static_cast<int>(ntr.size()), C) == 0,
             "src oracle");
      expect(apply(d, ne, n, in) == want, "src D vs oracle");
      ++repaired;
    }
    expect(repaired > 500, "src patterns");
    hrs_destroy(c);
  }
  // xor
  {
    hrs_codec* c = host_handle(HRS_CODE_XOR, 10, 1);
    std::vector<uint8_t> d(11);
    int er = 4;
    expect(hrs_decode_matrix(c, &er, 1, nullptr, 0, 1, d.data()) == HRS_OK && d[4] == 0 && d[0] == 1, "xor matrix");
    hrs_destroy(c);
  }
}

void argument_errors() {
  hrs_codec* c = host_handle(HRS_CODE_RS, 10, 4);
  int to_read[14];
  int five[5] = {0, 1, 2, 3, 4};
  expect(hrs_locations_to_read(c, five, 5, to_read) == HRS_ETOOMANY, "too many erased");
  int dup[2] = {3, 3};
  std::vector<uint8_t> d(28);
  // a repeated not-to-read location is accepted, as by the Java (its solve
  // divides by zero: divTable[y][0] = 0); the row equals the oracle's decode
  expect(hrs_decode_matrix(c, dup, 1, dup, 2, 1, d.data()) == HRS_OK, "repeated location");
  for (int l = 0; l < 14; ++l) {
    int col[14] = {0}, val[1] = {0};
    col[l] = 1;
    orc_rs_decode5(10, 4, col, dup, 1, val, nullptr, 0, dup, 2);
    expect(d[l] == val[0], "repeated location row vs oracle");
  }
  int far[1] = {99};
  expect(hrs_decode_matrix(c, far, 1, far, 1, 1, d.data()) == HRS_EINVAL, "location out of range");
  expect(hrs_decode_matrix(c, nullptr, 1, far, 1, 1, d.data()) == HRS_EINVAL, "NULL erased");
  hrs_codec* bad = nullptr;
  expect(hrs_create(0, 4, nullptr, &bad) == HRS_EINVAL && !bad, "RS(0,4)");
  expect(hrs_create(200, 60, nullptr, &bad) == HRS_EINVAL, "k + p >= 256");
  hrs_opts o{};
  o.device = HRS_DEVICE_NONE;
  o.reserved[3] = 1;
  expect(hrs_create(10, 4, &o, &bad) == HRS_EINVAL, "reserved opts");
  expect(std::strlen(hrs_last_error(nullptr)) > 0, "create error message");
  expect(hrs_set_kernel_mode(c, 7) == HRS_EINVAL, "kernel mode range");
  hrs_destroy(c);
  hrs_destroy(nullptr);
}

void oracle_bulk() {
  // the oracle's bulk loops at odd sizes (ASan: no row overrun)
  for (int len : {1, 7, 33, 257}) {
    const int k = 6, p = 3, n = 9;
    std::vector<std::vector<uint8_t>> rows(n, std::vector<uint8_t>(len));
    for (auto& r : rows)
      for (auto& b : r) b = rnd8();
    std::vector<uint8_t*> in(k), out(p);
    for (int i = 0; i < k; ++i) in[i] = rows[p + i].data();
    for (int r = 0; r < p; ++r) out[r] = rows[r].data();
    std::vector<std::vector<uint8_t>> keep(rows.begin() + p, rows.end());
    orc_rs_encode_bulk(k, p, in.data(), out.data(), len);  // zeroes in
    for (int i = 0; i < k; ++i) rows[p + i] = keep[i];
    int er[2] = {1, 5}, tr[6], ntr[3];
    const int m = orc_locations_to_read(k, p, er, 2, tr);
    expect(m == k, "oracle locations");
    int nn = 0;
    for (int l = 0; l < n; ++l) {
      bool rd = false;
      for (int i = 0; i < m; ++i) rd |= tr[i] == l;
      if (!rd) ntr[nn++] = l;
    }
    std::vector<uint8_t> w0(len), w1(len);
    uint8_t* wp[2] = {w0.data(), w1.data()};
    std::vector<uint8_t*> rp(n);
    std::vector<std::vector<uint8_t>> z = rows;
    for (int j = 0; j < nn; ++j) std::fill(z[ntr[j]].begin(), z[ntr[j]].end(), 0);
    for (int l = 0; l < n; ++l) rp[l] = z[l].data();
    orc_rs_decode_bulk5(k, p, rp.data(), wp, er, 2, tr, m, ntr, nn, len);
    expect(w0 == rows[1] && w1 == rows[5], "oracle round trip");
    std::vector<uint8_t> x(len);
    orc_xor_encode_bulk(k, in.data(), x.data(), len);
    std::vector<std::vector<uint8_t>> nro(p, std::vector<uint8_t>(len));
    std::vector<uint8_t*> np(p);
    for (int r = 0; r < p; ++r) np[r] = nro[r].data();
    orc_nrs_encode_bulk(k, p, in.data(), np.data(), len);
    orc_src_encode_bulk(k, p, 1, in.data(), np.data(), len);
  }
}

}  // namespace

int main() {
  for (auto kp : {std::pair<int, int>{10, 4}, {12, 4}, {6, 3}, {3, 2}}) rs_checks(kp.first, kp.second);
  cache_and_batch_checks();
  other_codes();
  argument_errors();
  oracle_bulk();
  const bool ok = failures == 0;
  printf("{\"mode\": \"host-logic\", \"ok\": %s, \"checks\": %d, \"failures\": %d, \"first_failure\": \"%s\"}\n",
         ok ? "true" : "false", checks, failures, first.c_str());
  return ok ? 0 : 1;
}
