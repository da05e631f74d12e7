// Native harness: drives libhrs through include/hrs.hpp exactly as the hops
// stream drivers call the codec, and checks every byte against the oracle.
//
//  Encoder.encodeStripe (hops-erasure-coding/.../Encoder.java:397-464):
//    per bufSize round: fresh read buffers (ParallelStreamReader.java:181),
//    CRC32 of the sources (:434-436), code.encodeBulk(readBufs, writeBufs)
//    (:442), parity written out and CRC32'd (:446-452).
//  Decoder.fixErasedBlockImpl (Decoder.java:232-401):
//    erasedLocations -> locationsToReadForDecode; the three ascending arrays
//    built as at :303-338; zeros for erased / not-to-read inputs
//    (StripeReader.java:106-124); code.decodeBulk(...) per round (:352-353);
//    the repaired block's CRC32 compared with the stored one (:222-229).
//  The codec calls are the checksummed variants (encodeBulkCrc /
//  decodeBulkCrc, hrs_encode_crc / hrs_decode_crc); the engine's running
//  CRCs must equal zlib's over the same bytes (gpu_crc_mismatches).
//
// Usage: codec_harness [--host-only] [--xor | --nrs | --src=S] k p blockSize bufSize nerased seed
// --src=S drives SimpleRegeneratingCode with S SRC parities (local groups;
// a pattern the code cannot repair is redrawn).
// --nrs drives NativeReedSolomonCode semantics: rounds are checked against the
// oracle's orc_nrs_decode_bulk, and the repaired CRC against the block the Java
// actually returns in writeBufs[i] (the i-th not-to-read location in Apache
// order; "quirk" says whether that differs from erasedLocations[i]).
// Prints one JSON line; exit status 0 iff everything matched.
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "hrs.hpp"
#include "rs_oracle.h"

namespace {

uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void fill(std::vector<uint8_t>& v, uint64_t seed) {
  for (size_t i = 0; i < v.size(); i += 8) {
    uint64_t x = splitmix(seed);
    for (size_t j = 0; j < 8 && i + j < v.size(); ++j) v[i + j] = static_cast<uint8_t>(x >> (8 * j));
  }
}

uint32_t crc(uint32_t c, const uint8_t* p, size_t n) { return static_cast<uint32_t>(crc32(c, p, static_cast<uInt>(n))); }

int host_only_checks(int k, int p) {
  // locationsToReadForDecode (C++ mirror) == hrs_locations_to_read == oracle
  hrs_opts o{};
  o.device = HRS_DEVICE_NONE;
  hrs_codec* c = nullptr;
  if (hrs_create(k, p, &o, &c) != HRS_OK) return 1;
  int bad = 0;
  std::vector<int> tr(k), orc(k);
  for (int a = 0; a < k + p; ++a) {
    std::vector<int> er = {a};
    bad += hrs_locations_to_read(c, er.data(), 1, tr.data()) != HRS_OK;
    bad += orc_locations_to_read(k, p, er.data(), 1, orc.data()) != k;
    bad += tr != orc;
  }
  std::vector<uint8_t> g(static_cast<size_t>(k) * p);
  hrs_encode_matrix(c, g.data());
  std::vector<int> msg(k), par(p);
  for (int col = 0; col < k; ++col) {
    for (int j = 0; j < k; ++j) msg[j] = j == col;
    orc_rs_encode(k, p, msg.data(), par.data());
    for (int r = 0; r < p; ++r) bad += g[r * k + col] != par[r];
  }
  hrs_destroy(c);
  printf("{\"mode\": \"host-only\", \"k\": %d, \"p\": %d, \"mismatches\": %d}\n", k, p, bad);
  return bad ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
  bool host_only = false, use_xor = false, use_nrs = false, use_src = false;
  int src_s = 0;
  std::vector<std::string> pos;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--host-only")
      host_only = true;
    else if (a == "--xor")
      use_xor = true;
    else if (a == "--nrs")
      use_nrs = true;
    else if (a.rfind("--src=", 0) == 0) {
      use_src = true;
      src_s = atoi(a.c_str() + 6);
    }
    else
      pos.push_back(a);
  }
  const int k = pos.size() > 0 ? atoi(pos[0].c_str()) : 10;
  const int p = use_xor ? 1 : (pos.size() > 1 ? atoi(pos[1].c_str()) : 4);
  const size_t block = pos.size() > 2 ? strtoull(pos[2].c_str(), nullptr, 10) : (4u << 20);
  const size_t buf = pos.size() > 3 ? strtoull(pos[3].c_str(), nullptr, 10) : (1u << 20);
  const int nerased = pos.size() > 4 ? atoi(pos[4].c_str()) : 1;
  const uint64_t seed = pos.size() > 5 ? strtoull(pos[5].c_str(), nullptr, 10) : 7;
  if (host_only) return host_only_checks(k, p);
  const int n = k + p;

  try {
    std::unique_ptr<hrs::HipCode> code;
    if (use_xor)
      code.reset(new hrs::HipXORCode(k, 0));
    else if (use_nrs)
      code.reset(new hrs::HipNativeReedSolomonCode(k, p, 0));
    else if (use_src)
      code.reset(new hrs::HipSimpleRegeneratingCode(k, p, src_s, 0));
    else
      code.reset(new hrs::HipReedSolomonCode(k, p, 0));

    // one stripe of k source blocks
    std::vector<std::vector<uint8_t>> src(k, std::vector<uint8_t>(block));
    for (int i = 0; i < k; ++i) fill(src[i], seed * 1000 + i);
    std::vector<std::vector<uint8_t>> parity(p, std::vector<uint8_t>(block));
    std::vector<uint32_t> src_crc(k, 0), par_crc(p, 0);
    std::vector<uint32_t> gpu_crc(n, 0);  // the engine's own checksums (hrs_encode_crc)

    // ---- Encoder.encodeStripe
    size_t mismatches = 0;
    double t_codec = 0;
    std::vector<std::vector<uint8_t>> write_bufs(p, std::vector<uint8_t>(buf));
    for (size_t off = 0; off < block; off += buf) {
      const size_t len = std::min(buf, block - off);
      std::vector<std::vector<uint8_t>> read(k, std::vector<uint8_t>(len));  // fresh per round
      std::vector<uint8_t*> rp(k), wp(p);
      for (int i = 0; i < k; ++i) {
        std::memcpy(read[i].data(), src[i].data() + off, len);
        src_crc[i] = crc(src_crc[i], read[i].data(), len);
        rp[i] = read[i].data();
      }
      for (int r = 0; r < p; ++r) wp[r] = write_bufs[r].data();
      auto t0 = std::chrono::steady_clock::now();
      code->encodeBulkCrc(rp, wp, len, gpu_crc);
      t_codec += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      // oracle: the Java remainder on copies (it zeroes its inputs)
      std::vector<std::vector<uint8_t>> cp = read;
      std::vector<std::vector<uint8_t>> ref(p, std::vector<uint8_t>(len));
      std::vector<uint8_t*> cpp(k), refp(p);
      for (int i = 0; i < k; ++i) cpp[i] = cp[i].data();
      for (int r = 0; r < p; ++r) refp[r] = ref[r].data();
      if (use_xor)
        orc_xor_encode_bulk(k, cpp.data(), refp[0], len);
      else if (use_nrs)
        orc_nrs_encode_bulk(k, p, cpp.data(), refp.data(), len);
      else if (use_src)
        orc_src_encode_bulk(k, p, src_s, cpp.data(), refp.data(), len);
      else
        orc_rs_encode_bulk(k, p, cpp.data(), refp.data(), len);
      for (int r = 0; r < p; ++r) {
        mismatches += std::memcmp(ref[r].data(), write_bufs[r].data(), len) != 0;
        std::memcpy(parity[r].data() + off, write_bufs[r].data(), len);
        par_crc[r] = crc(par_crc[r], write_bufs[r].data(), len);
      }
    }

    // ---- lose blocks, Decoder.fixErasedBlockImpl
    std::vector<int> erased_list, to_read_list;
    uint64_t s = seed;
    for (;;) {  // SRC: redraw patterns its local groups + RS part cannot repair
      erased_list.clear();
      while (static_cast<int>(erased_list.size()) < nerased) {
        int loc = static_cast<int>(splitmix(s) % n);
        bool dup = false;
        for (int e : erased_list) dup |= e == loc;
        if (!dup) erased_list.push_back(loc);
      }
      try {
        to_read_list = code->locationsToReadForDecode(erased_list);
        break;
      } catch (const hrs::TooManyErasedLocations&) {
        if (!use_src) throw;
      }
    }
    auto contains = [](const std::vector<int>& v, int x) {
      for (int y : v)
        if (y == x) return true;
      return false;
    };
    std::vector<int> erased_arr, to_read_arr, ntr_arr;  // Decoder.java:303-338
    for (int loc = 0; loc < n; ++loc)
      if (contains(erased_list, loc)) erased_arr.push_back(loc);
    for (int loc = 0; loc < n; ++loc)
      if (contains(to_read_list, loc)) to_read_arr.push_back(loc);
    for (int loc = 0; loc < n; ++loc)
      if (!contains(to_read_list, loc) || contains(erased_list, loc)) ntr_arr.push_back(loc);

    auto stripe_row = [&](int loc) -> const uint8_t* {
      return loc < p ? parity[loc].data() : src[loc - p].data();
    };
    std::vector<uint32_t> rep_crc(erased_arr.size(), 0), gpu_rep_crc(erased_arr.size(), 0);
    size_t rep_mismatch = 0;
    const int ne = static_cast<int>(erased_arr.size());
    // the block writeBufs[i] receives: erased_arr[i], or for nrs the i-th
    // not-to-read location in Apache [data, parity] order
    std::vector<int> expect(erased_arr);
    bool quirk = false;
    if (use_nrs) {
      std::vector<int> ap;
      for (int loc : ntr_arr) ap.push_back(loc < p ? loc + k : loc - p);
      std::sort(ap.begin(), ap.end());
      for (int i = 0; i < ne; ++i) {
        expect[i] = ap[i] < k ? ap[i] + p : ap[i] - k;
        quirk |= expect[i] != erased_arr[i];
      }
    }
    std::vector<std::vector<uint8_t>> wb(ne, std::vector<uint8_t>(buf));
    for (size_t off = 0; off < block; off += buf) {
      const size_t len = std::min(buf, block - off);
      std::vector<std::vector<uint8_t>> read(n, std::vector<uint8_t>(len, 0));  // zeros: ZeroInputStream
      std::vector<uint8_t*> rp(n), wp(ne);
      for (int loc = 0; loc < n; ++loc) {
        if (contains(to_read_arr, loc) && !contains(erased_arr, loc))
          std::memcpy(read[loc].data(), stripe_row(loc) + off, len);
        rp[loc] = read[loc].data();
      }
      for (int i = 0; i < ne; ++i) wp[i] = wb[i].data();
      auto t0 = std::chrono::steady_clock::now();
      code->decodeBulkCrc(rp, wp, len, erased_arr, to_read_arr, ntr_arr, gpu_rep_crc);
      t_codec += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      for (int i = 0; i < ne; ++i) {
        rep_mismatch += std::memcmp(wb[i].data(), stripe_row(expect[i]) + off, len) != 0;
        rep_crc[i] = crc(rep_crc[i], wb[i].data(), len);
      }
      if (use_src) {  // the reference's own output for this round
        std::vector<std::vector<uint8_t>> ref(ne, std::vector<uint8_t>(len));
        std::vector<uint8_t*> refp(ne);
        for (int i = 0; i < ne; ++i) refp[i] = ref[i].data();
        if (orc_src_decode_bulk(k, p, src_s, rp.data(), refp.data(), erased_arr.data(), ne, to_read_arr.data(),
                                static_cast<int>(to_read_arr.size()), ntr_arr.data(),
                                static_cast<int>(ntr_arr.size()), len) != 0)
          ++rep_mismatch;
        for (int i = 0; i < ne; ++i) rep_mismatch += std::memcmp(ref[i].data(), wb[i].data(), len) != 0;
      }
      if (use_nrs) {  // the reference's own output for this round
        std::vector<std::vector<uint8_t>> ref(ne, std::vector<uint8_t>(len));
        std::vector<uint8_t*> refp(ne);
        for (int i = 0; i < ne; ++i) refp[i] = ref[i].data();
        if (orc_nrs_decode_bulk(k, p, rp.data(), refp.data(), erased_arr.data(), ne, ntr_arr.data(),
                                static_cast<int>(ntr_arr.size()), len) != 0)
          ++rep_mismatch;
        for (int i = 0; i < ne; ++i) rep_mismatch += std::memcmp(ref[i].data(), wb[i].data(), len) != 0;
      }
    }
    size_t crc_bad = 0;
    for (int i = 0; i < ne; ++i) {
      const int loc = expect[i];
      const uint32_t stored = loc < p ? par_crc[loc] : src_crc[loc - p];  // checksums sent to the NN
      crc_bad += stored != rep_crc[i];
    }
    size_t gpu_crc_bad = 0;  // engine checksums vs zlib over the same bytes
    for (int i = 0; i < k; ++i) gpu_crc_bad += gpu_crc[i] != src_crc[i];
    for (int r = 0; r < p; ++r) gpu_crc_bad += gpu_crc[k + r] != par_crc[r];
    for (int i = 0; i < ne; ++i) gpu_crc_bad += gpu_rep_crc[i] != rep_crc[i];
    const bool ok = mismatches == 0 && rep_mismatch == 0 && crc_bad == 0 && gpu_crc_bad == 0;
    printf("{\"code\": \"%s\", \"k\": %d, \"p\": %d, \"block\": %zu, \"buf\": %zu, \"erased\": [", use_xor ? "xor" : use_nrs ? "nrs" : use_src ? "src" : "rs",
           k, p, block, buf);
    for (int i = 0; i < ne; ++i) printf("%s%d", i ? ", " : "", erased_arr[i]);
    printf("], \"quirk\": %s, \"encode_round_mismatches\": %zu, \"repair_mismatches\": %zu, \"crc_mismatches\": %zu, "
           "\"gpu_crc_mismatches\": %zu, \"codec_seconds\": %.4f, \"ok\": %s}\n",
           quirk ? "true" : "false", mismatches, rep_mismatch, crc_bad, gpu_crc_bad, t_codec, ok ? "true" : "false");
    return ok ? 0 : 1;
  } catch (const std::exception& e) {
    printf("{\"error\": \"%s\", \"ok\": false}\n", e.what());
    return 2;
  }
}
