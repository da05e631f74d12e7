// A/B sweep of the staged synchronous host-buffer pipeline's knobs
// (hrs_hostpath.cpp staged_run: HRS_HOST_CHUNK, HRS_HOST_SLOTS,
// HRS_HOST_FIRST, HRS_HOST_GATE, HRS_HOST_NT, HRS_HOST_FOLD, all read per call), interleaved
// round by
// round in one process over the four calls the JNI shim makes per Encoder /
// Decoder round: hrs_encode / hrs_decode / hrs_encode_crc / hrs_decode_crc on
// one RS(k,p) stripe of L-byte pageable rows (default RS(10,4), 1 MiB).
// Every variant's parity, CRCs and repaired row must equal the first
// variant's (and the repaired row the lost one), or the tool fails.
// ROWS=pinned in a variant's environment runs it on a hipHostMalloc'd copy of
// the rows (the in-place path).
// Usage: host_pipeline_sweep [calls] [rounds] [L] [name:chunk:slots:first:gate[:nt[:fold[:K=V+K=V]]],...]
//   (one JSON line per variant, medians)
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../include/hrs.h"

struct Variant {
  std::string name, chunk, slots, first, gate, nt = "0", fold = "1";
  std::string extra;  // more environment for this variant: KEY=VAL+KEY=VAL (unset for the others)
};

// Default variants; argv[4] may list others as name:chunk:slots:first:gate,...
static std::vector<Variant> default_variants() {
  return {{"c512_s2", "524288", "2", "0", "0"},      {"c256_s4", "262144", "4", "0", "0"},
          {"c128_s4", "131072", "4", "0", "0"},      {"c128_s8", "131072", "8", "0", "0"},
          {"c512_s2_gate", "524288", "2", "0", "1"}, {"c256_s2_gate", "262144", "2", "0", "1"},
          {"c256_s4_gate", "262144", "4", "0", "1"}, {"c128_s4_gate", "131072", "4", "0", "1"}};
}

static std::vector<Variant> parse_variants(const char* spec) {
  std::vector<Variant> v;
  std::string s(spec);
  size_t pos = 0;
  while (pos < s.size()) {
    size_t end = s.find(',', pos);
    if (end == std::string::npos) end = s.size();
    std::string item = s.substr(pos, end - pos), f[8] = {"", "", "", "", "", "0", "1", ""};
    size_t q = 0;
    for (int i = 0; i < 8 && q < item.size(); ++i) {
      size_t c = item.find(':', q);
      f[i] = item.substr(q, c == std::string::npos ? std::string::npos : c - q);
      q = c == std::string::npos ? item.size() : c + 1;
    }
    v.push_back({f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7]});
    pos = end + 1;
  }
  return v;
}

static std::vector<std::pair<std::string, std::string>> split_env(const std::string& s) {
  std::vector<std::pair<std::string, std::string>> kv;
  size_t pos = 0;
  while (pos < s.size()) {
    size_t end = s.find('+', pos);
    if (end == std::string::npos) end = s.size();
    const std::string item = s.substr(pos, end - pos);
    const size_t eq = item.find('=');
    if (eq != std::string::npos) kv.emplace_back(item.substr(0, eq), item.substr(eq + 1));
    pos = end + 1;
  }
  return kv;
}

int main(int argc, char** argv) {
  const int calls = argc > 1 ? atoi(argv[1]) : 100;
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  const size_t L = argc > 3 ? static_cast<size_t>(atol(argv[3])) : static_cast<size_t>(1) << 20;
  const int k = 10, p = 4, n = k + p;
  hrs_opts o{};
  o.device = 0;
  hrs_codec* c = nullptr;
  if (hrs_create(k, p, &o, &c) != HRS_OK) {
    fprintf(stderr, "hrs_create failed\n");
    return 1;
  }
  std::vector<std::vector<uint8_t>> rows(n, std::vector<uint8_t>(L));
  uint64_t z = 0x9E3779B97F4A7C15ull;
  for (int r = p; r < n; ++r)
    for (size_t i = 0; i + 8 <= L; i += 8) {
      z ^= z << 13, z ^= z >> 7, z ^= z << 17;
      memcpy(&rows[r][i], &z, 8);
    }
  std::vector<uint8_t> lost(L);
  // Row sets: the pageable rows above, and (variants with ROWS=pinned) a
  // copy in hipHostMalloc'd memory, the in-place "pinned" path's floor.
  struct RowSet {
    std::vector<uint8_t*> row;
    uint8_t* lost;
  };
  RowSet pageable{{}, lost.data()}, pinned{{}, nullptr};
  for (int r = 0; r < n; ++r) pageable.row.push_back(rows[r].data());
  const int erased[1] = {p};
  int to_read[16];
  if (hrs_locations_to_read(c, erased, 1, to_read) != HRS_OK) return 1;
  const int nr = k;
  std::sort(to_read, to_read + nr);
  std::vector<int> ntr;
  for (int l = 0; l < n; ++l)
    if (!std::binary_search(to_read, to_read + nr, l)) ntr.push_back(l);
  std::vector<const uint8_t*> reads(n, nullptr);
  // the parity rows are read after the first encode has filled them
  std::vector<uint32_t> crc(n), dcrc(1);
  const std::vector<Variant> kVariants = argc > 4 ? parse_variants(argv[4]) : default_variants();
  const int nv = static_cast<int>(kVariants.size());
  std::vector<std::vector<double>> t(nv * 4);
  std::vector<std::string> paths(nv);
  std::vector<uint8_t> ref_par;
  std::vector<uint32_t> ref_crc;
  uint32_t ref_dcrc = 0;
  bool ok = true;
  auto time_it = [&](auto&& fn) {
    for (int i = 0; i < 3; ++i) fn();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < calls; ++i) fn();
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / calls;
  };
  for (int rd = 0; rd < rounds; ++rd)
    for (int v = 0; v < nv; ++v) {
      const Variant& V = kVariants[v];
      bool use_pinned = false;
      for (const auto& kv : split_env(V.extra)) use_pinned |= kv.first == "ROWS" && kv.second == "pinned";
      if (use_pinned && pinned.row.empty()) {
        void* m = nullptr;
        if (hipHostMalloc(&m, (n + 1) * L, hipHostMallocDefault) != hipSuccess) {
          fprintf(stderr, "hipHostMalloc failed\n");
          return 1;
        }
        for (int r = 0; r < n; ++r) {
          pinned.row.push_back(static_cast<uint8_t*>(m) + r * L);
          memcpy(pinned.row[r], rows[r].data(), L);
        }
        pinned.lost = static_cast<uint8_t*>(m) + n * L;
      }
      const RowSet& rs = use_pinned ? pinned : pageable;
      std::vector<const uint8_t*> in(k);
      std::vector<uint8_t*> par(p);
      for (int i = 0; i < k; ++i) in[i] = rs.row[p + i];
      for (int r = 0; r < p; ++r) par[r] = rs.row[r];
      uint8_t* lostp = rs.lost;
      setenv("HRS_HOST_CHUNK", V.chunk.c_str(), 1);
      setenv("HRS_HOST_SLOTS", V.slots.c_str(), 1);
      setenv("HRS_HOST_FIRST", V.first.c_str(), 1);
      setenv("HRS_HOST_GATE", V.gate.c_str(), 1);
      setenv("HRS_HOST_NT", V.nt.c_str(), 1);
      setenv("HRS_HOST_FOLD", V.fold.c_str(), 1);
      for (const Variant& o : kVariants)  // other variants' extra keys unset, then this one's set
        for (const auto& kv : split_env(o.extra))
          if (kv.first != "ROWS") unsetenv(kv.first.c_str());
      for (const auto& kv : split_env(V.extra))
        if (kv.first != "ROWS") setenv(kv.first.c_str(), kv.second.c_str(), 1);
      for (int r = 0; r < p; ++r) memset(par[r], 0, L);
      t[v * 4 + 0].push_back(time_it([&] { ok &= hrs_encode(c, in.data(), par.data(), L) == HRS_OK; }));
      paths[v] = hrs_last_host_path(c);
      std::vector<uint8_t> got;
      for (int r = 0; r < p; ++r) got.insert(got.end(), par[r], par[r] + L);
      if (ref_par.empty()) ref_par = got;
      if (got != ref_par) {
        fprintf(stderr, "%s: parity differs from %s\n", V.name.c_str(), kVariants[0].name.c_str());
        ok = false;
      }
      for (int i = 0; i < nr; ++i) reads[to_read[i]] = rs.row[to_read[i]];
      memset(lostp, 0, L);
      t[v * 4 + 1].push_back(time_it([&] {
        ok &= hrs_decode(c, reads.data(), &lostp, erased, 1, to_read, nr, ntr.data(), static_cast<int>(ntr.size()),
                         L) == HRS_OK;
      }));
      if (memcmp(lostp, rs.row[p], L) != 0) {
        fprintf(stderr, "%s: repaired row differs\n", V.name.c_str());
        ok = false;
      }
      t[v * 4 + 2].push_back(
          time_it([&] { ok &= hrs_encode_crc(c, in.data(), par.data(), L, nullptr, crc.data()) == HRS_OK; }));
      if (ref_crc.empty()) ref_crc = crc;
      if (crc != ref_crc) {
        fprintf(stderr, "%s: encode CRCs differ\n", V.name.c_str());
        ok = false;
      }
      memset(lostp, 0, L);
      t[v * 4 + 3].push_back(time_it([&] {
        ok &= hrs_decode_crc(c, reads.data(), &lostp, erased, 1, to_read, nr, ntr.data(),
                             static_cast<int>(ntr.size()), L, nullptr, dcrc.data()) == HRS_OK;
      }));
      if (rd == 0 && v == 0) ref_dcrc = dcrc[0];
      if (dcrc[0] != ref_dcrc || memcmp(lostp, rs.row[p], L) != 0) {
        fprintf(stderr, "%s: decode CRC or repaired row differs\n", V.name.c_str());
        ok = false;
      }
    }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  for (int v = 0; v < nv; ++v)
    printf("{\"variant\": \"%s\", \"chunk\": %s, \"slots\": %s, \"first\": %s, \"gate\": %s, \"nt\": \"%s\", \"path\": \"%s\", "
           "\"L\": %zu, \"calls\": %d, \"rounds\": %d, \"encode_ms\": %.4f, \"decode_ms\": %.4f, \"encode_crc_ms\": %.4f, "
           "\"decode_crc_ms\": %.4f, \"ok\": %s}\n",
           kVariants[v].name.c_str(), kVariants[v].chunk.c_str(), kVariants[v].slots.c_str(), kVariants[v].first.c_str(),
           kVariants[v].gate.c_str(), kVariants[v].nt.c_str(), paths[v].c_str(), L, calls, rounds, med(t[v * 4]), med(t[v * 4 + 1]), med(t[v * 4 + 2]), med(t[v * 4 + 3]),
           ok ? "true" : "false");
  hrs_destroy(c);
  return ok ? 0 : 1;
}
