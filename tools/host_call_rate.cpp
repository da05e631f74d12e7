// Synchronous host-buffer call rate through the C ABI itself (what the JNI
// shim calls per Encoder / Decoder round: HrsNative.encode / decode /
// encodeCrc / decodeCrc -> hrs_encode / hrs_decode / hrs_encode_crc /
// hrs_decode_crc), without the Python mirror's per-call argument marshalling:
// one RS(k,p) stripe of L-byte pageable rows per call (default RS(10,4),
// 1 MiB), the same rows every call (Encoder.java:442 reuses its buffers),
// data shard 0 lost for decode. Checks the repaired row of each decode kind.
// Usage: host_call_rate [calls] [L] [k] [p]   (one JSON line; "path" = the
// host path hrs_last_host_path reports for the last encode)
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/hrs.h"

int main(int argc, char** argv) {
  const int calls = argc > 1 ? atoi(argv[1]) : 200;
  const size_t L = argc > 2 ? static_cast<size_t>(atol(argv[2])) : static_cast<size_t>(1) << 20;
  const int k = argc > 3 ? atoi(argv[3]) : 10, p = argc > 4 ? atoi(argv[4]) : 4, n = k + p;
  if (calls < 1 || L < 8 || k < 1 || p < 1 || n > 255) {
    fprintf(stderr, "usage: host_call_rate [calls] [L >= 8] [k] [p]\n");
    return 1;
  }
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
    for (size_t i = 0; i < L; i += 8) {
      z ^= z << 13, z ^= z >> 7, z ^= z << 17;
      memcpy(&rows[r][i], &z, 8);
    }
  std::vector<const uint8_t*> in(k);
  std::vector<uint8_t*> par(p);
  for (int i = 0; i < k; ++i) in[i] = rows[p + i].data();
  for (int r = 0; r < p; ++r) par[r] = rows[r].data();
  std::vector<uint8_t> lost(L);
  uint8_t* lostp = lost.data();
  const int erased[1] = {p};
  int to_read[16], nr = 0;
  if (hrs_locations_to_read(c, erased, 1, to_read) != HRS_OK) return 1;
  nr = k;
  std::sort(to_read, to_read + nr);
  std::vector<int> ntr;
  for (int l = 0; l < n; ++l)
    if (!std::binary_search(to_read, to_read + nr, l)) ntr.push_back(l);
  std::vector<const uint8_t*> reads(n, nullptr);
  for (int i = 0; i < nr; ++i) reads[to_read[i]] = rows[to_read[i]].data();
  std::vector<uint32_t> crc(n), dcrc(1);
  auto time_it = [&](auto&& fn) {
    for (int i = 0; i < 5; ++i) fn();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < calls; ++i) fn();
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / calls;
  };
  bool ok = true;
  const double enc = time_it([&] { ok &= hrs_encode(c, in.data(), par.data(), L) == HRS_OK; });
  const std::string path = hrs_last_host_path(c);
  const double dec = time_it([&] {
    ok &= hrs_decode(c, reads.data(), &lostp, erased, 1, to_read, nr, ntr.data(), static_cast<int>(ntr.size()), L) ==
          HRS_OK;
  });
  ok &= memcmp(lost.data(), rows[p].data(), L) == 0;  // the repaired data shard 0
  const double encc = time_it([&] { ok &= hrs_encode_crc(c, in.data(), par.data(), L, nullptr, crc.data()) == HRS_OK; });
  const double decc = time_it([&] {
    ok &= hrs_decode_crc(c, reads.data(), &lostp, erased, 1, to_read, nr, ntr.data(), static_cast<int>(ntr.size()), L,
                         nullptr, dcrc.data()) == HRS_OK;
  });
  ok &= memcmp(lost.data(), rows[p].data(), L) == 0;
  const double gib = static_cast<double>(k) * L / (1u << 30);
  const char* zc = getenv("HRS_ZEROCOPY");
  printf("{\"what\": \"C ABI synchronous host-buffer calls, one RS(k,p) stripe of pageable rows per call\", "
         "\"k\": %d, \"p\": %d, \"L\": %zu, \"path\": \"%s\", \"zero_copy\": %s, \"calls\": %d, \"encode_ms\": %.4f, \"encode_GiBps_user\": %.2f, \"decode_ms\": %.4f, "
         "\"decode_GiBps_user\": %.2f, \"encode_crc_ms\": %.4f, \"encode_crc_GiBps_user\": %.2f, "
         "\"decode_crc_ms\": %.4f, \"decode_crc_GiBps_user\": %.2f, \"ok\": %s}\n",
         k, p, L, path.c_str(), (zc && zc[0] == '0') ? "false" : "true", calls, enc, gib / (enc * 1e-3), dec, gib / (dec * 1e-3), encc,
         gib / (encc * 1e-3), decc, gib / (decc * 1e-3), ok ? "true" : "false");
  hrs_destroy(c);
  return ok ? 0 : 1;
}
