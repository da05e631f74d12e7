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
// --grow=R : Decoder restart (Decoder.java:373-387, readFromInputs :403-436):
// one block (erased[0]) is repaired; at round R a read of one of the
// locations to read fails (BlockMissingException), that location joins
// erasedLocations, the three arrays are rebuilt and the round is redone from
// the same offset. The repaired block and its CRC32 (chained across the
// pattern change) must match the stored ones; the decode-matrix cache must
// hand out the new pattern's matrix.
// --threads=N [--rounds=M] : N threads, one codec handle each (Encoder.java:80,
// Decoder.java:90: one ErasureCode per task), interleaving encodeBulk and
// decodeBulk of bufSize cells of RS(k,p); a checked pass (every round vs the
// oracle's parity / the original cells) then a timed pass; prints the
// aggregate user-data GiB/s (k * bufSize per call).
// --async=D : Encoder / Decoder rounds pipelined D deep through
// encodeBulkSubmit / decodeBulkSubmit / collect vs the synchronous calls
// (see async_mode).
// Prints one JSON line; exit status 0 iff everything matched.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
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


bool contains(const std::vector<int>& v, int x) {
  for (int y : v)
    if (y == x) return true;
  return false;
}

// Decoder.java:303-338: ascending erased / toRead / notToRead arrays.
void decoder_arrays(int n, const std::vector<int>& erased, const std::vector<int>& to_read, std::vector<int>& ea,
                    std::vector<int>& ta, std::vector<int>& na) {
  ea.clear();
  ta.clear();
  na.clear();
  for (int loc = 0; loc < n; ++loc)
    if (contains(erased, loc)) ea.push_back(loc);
  for (int loc = 0; loc < n; ++loc)
    if (contains(to_read, loc)) ta.push_back(loc);
  for (int loc = 0; loc < n; ++loc)
    if (!contains(to_read, loc) || contains(erased, loc)) na.push_back(loc);
}

// --grow: one block repaired, a second location lost at round `grow_round`.
int grow_mode(int k, int p, size_t block, size_t buf, int grow_round, uint64_t seed) {
  const int n = k + p;
  hrs::HipReedSolomonCode code(k, p, 0);
  std::vector<std::vector<uint8_t>> stripe(n, std::vector<uint8_t>(block));
  for (int i = 0; i < k; ++i) fill(stripe[p + i], seed * 1000 + i);
  {  // parity by the oracle (it zeroes its inputs: copies)
    std::vector<std::vector<uint8_t>> cp(stripe.begin() + p, stripe.end());
    std::vector<uint8_t*> ip(k), op(p);
    for (int i = 0; i < k; ++i) ip[i] = cp[i].data();
    for (int r = 0; r < p; ++r) op[r] = stripe[r].data();
    orc_rs_encode_bulk(k, p, ip.data(), op.data(), block);
  }
  std::vector<uint32_t> stored(n, 0);
  for (int l = 0; l < n; ++l) stored[l] = crc(0, stripe[l].data(), block);
  uint64_t s = seed;
  const int to_fix = p + static_cast<int>(splitmix(s) % k);  // a data block
  std::vector<int> erased = {to_fix};
  std::vector<int> to_read = code.locationsToReadForDecode(erased);
  // the location whose read fails mid-block: one the decoder is reading
  const int lost_later = to_read[static_cast<size_t>(splitmix(s) % to_read.size())];
  std::vector<int> ea, ta, na;
  decoder_arrays(n, erased, to_read, ea, ta, na);
  std::vector<uint8_t> repaired(block);
  uint32_t fix_crc = 0;           // java.util.zip.CRC32 of the repaired block (host zlib)
  uint32_t gpu_fix_crc = 0;       // the engine's running value (decodeBulkCrc)
  size_t mismatches = 0, restarts = 0, rounds = 0;
  int patterns = 1;
  size_t written = 0;
  while (written < block) {
    const size_t len = std::min(buf, block - written);
    if (restarts == 0 && rounds == static_cast<size_t>(grow_round)) {
      // readFromInputs: BlockMissingException in stream lost_later ->
      // erasedLocations.add, rebuild inputs from the same offset
      erased.push_back(lost_later);
      to_read = code.locationsToReadForDecode(erased);
      decoder_arrays(n, erased, to_read, ea, ta, na);
      ++restarts;
      ++patterns;
    }
    std::vector<std::vector<uint8_t>> read(n, std::vector<uint8_t>(len, 0));
    std::vector<uint8_t*> rp(n);
    for (int l = 0; l < n; ++l) {
      if (contains(ta, l) && !contains(ea, l)) std::memcpy(read[l].data(), stripe[l].data() + written, len);
      rp[l] = read[l].data();
    }
    const int ne = static_cast<int>(ea.size());
    std::vector<std::vector<uint8_t>> wb(ne, std::vector<uint8_t>(buf));
    std::vector<uint8_t*> wp(ne);
    for (int i = 0; i < ne; ++i) wp[i] = wb[i].data();
    std::vector<uint32_t> crcs(ne, 0);
    int fix_idx = -1;
    for (int i = 0; i < ne; ++i)
      if (ea[i] == to_fix) fix_idx = i;
    crcs[fix_idx] = gpu_fix_crc;
    code.decodeBulkCrc(rp, wp, len, ea, ta, na, crcs);
    gpu_fix_crc = crcs[fix_idx];
    for (int i = 0; i < ne; ++i)  // every erased cell of the round is right
      mismatches += std::memcmp(wb[i].data(), stripe[ea[i]].data() + written, len) != 0;
    std::memcpy(repaired.data() + written, wb[fix_idx].data(), len);  // out.write(writeBufs[i]) (:360-372)
    fix_crc = crc(fix_crc, wb[fix_idx].data(), len);
    written += len;
    ++rounds;
  }
  const bool block_ok = std::memcmp(repaired.data(), stripe[to_fix].data(), block) == 0;
  const bool ok = block_ok && mismatches == 0 && fix_crc == stored[to_fix] && gpu_fix_crc == fix_crc && restarts == 1;
  printf("{\"mode\": \"grow\", \"k\": %d, \"p\": %d, \"block\": %zu, \"buf\": %zu, \"to_fix\": %d, \"lost_later\": %d, "
         "\"grow_round\": %d, \"rounds\": %zu, \"restarts\": %zu, \"patterns\": %d, \"round_mismatches\": %zu, "
         "\"block_ok\": %s, \"crc_ok\": %s, \"gpu_crc_ok\": %s, \"ok\": %s}\n",
         k, p, block, buf, to_fix, lost_later, grow_round, rounds, restarts, patterns, mismatches,
         block_ok ? "true" : "false", fix_crc == stored[to_fix] ? "true" : "false",
         gpu_fix_crc == fix_crc ? "true" : "false", ok ? "true" : "false");
  return ok ? 0 : 1;
}

// --threads: concurrent handles.
int threads_mode(int k, int p, size_t buf, int nthreads, int rounds, uint64_t seed) {
  const int n = k + p;
  const int nstripes = 4;
  // stripes + oracle parity, shared read-only by every thread
  std::vector<std::vector<std::vector<uint8_t>>> st(nstripes, std::vector<std::vector<uint8_t>>(n, std::vector<uint8_t>(buf)));
  for (int s = 0; s < nstripes; ++s) {
    for (int i = 0; i < k; ++i) fill(st[s][p + i], seed * 1000 + 100 * s + i);
    std::vector<std::vector<uint8_t>> cp(st[s].begin() + p, st[s].end());
    std::vector<uint8_t*> ip(k), op(p);
    for (int i = 0; i < k; ++i) ip[i] = cp[i].data();
    for (int r = 0; r < p; ++r) op[r] = st[s][r].data();
    orc_rs_encode_bulk(k, p, ip.data(), op.data(), buf);
  }
  std::atomic<size_t> bad{0}, errors{0};
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  double timed_s = 0;
  auto body = [&](int t, bool check) {
    try {
      hrs::HipReedSolomonCode code(k, p, 0);
      std::vector<std::vector<uint8_t>> par(p, std::vector<uint8_t>(buf)), wb(p, std::vector<uint8_t>(buf));
      std::vector<uint8_t*> pp(p), wp;
      for (int r = 0; r < p; ++r) pp[r] = par[r].data();
      // warm-up (not timed): the handle's staging slots and matrices
      for (int i = -2; i < rounds; ++i) {
        if (i == 0) {
          ready.fetch_add(1);
          while (!go.load()) std::this_thread::yield();
        }
        const int s = (t + i + nstripes) % nstripes;
        std::vector<uint8_t*> in(k);
        for (int c = 0; c < k; ++c) in[c] = st[s][p + c].data();
        code.encodeBulk(in, pp, buf);
        if (check)
          for (int r = 0; r < p; ++r) bad += std::memcmp(par[r].data(), st[s][r].data(), buf) != 0;
        // lose 1..p locations (varies per round and thread: the cache sees many patterns)
        std::vector<int> erased;
        uint64_t z = seed + 7919u * t + static_cast<uint64_t>(i + 2);
        const int ne = 1 + static_cast<int>(splitmix(z) % p);
        while (static_cast<int>(erased.size()) < ne) {
          const int loc = static_cast<int>(splitmix(z) % n);
          if (!contains(erased, loc)) erased.push_back(loc);
        }
        std::vector<int> ea, ta, na;
        decoder_arrays(n, erased, code.locationsToReadForDecode(erased), ea, ta, na);
        std::vector<uint8_t*> rp(n, nullptr);
        for (int l : ta) rp[l] = st[s][l].data();  // not-to-read rows are never read: NULL
        wp.assign(ea.size(), nullptr);
        for (size_t j = 0; j < ea.size(); ++j) wp[j] = wb[j].data();
        code.decodeBulk(rp, wp, buf, ea, ta, na);
        if (check)
          for (size_t j = 0; j < ea.size(); ++j) bad += std::memcmp(wb[j].data(), st[s][ea[j]].data(), buf) != 0;
      }
    } catch (const std::exception& e) {
      fprintf(stderr, "thread %d: %s\n", t, e.what());
      errors.fetch_add(1);
    }
  };
  for (int pass = 0; pass < 2; ++pass) {  // 0: every round checked; 1: timed
    ready = 0;
    go = false;
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(body, t, pass == 0);
    while (ready.load() < nthreads && errors.load() == 0) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    go = true;
    for (auto& x : th) x.join();
    if (pass == 1) timed_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  const double user = 2.0 * k * static_cast<double>(buf) * rounds * nthreads;  // encode + decode, k cells each
  const bool ok = bad == 0 && errors == 0;
  printf("{\"mode\": \"threads\", \"k\": %d, \"p\": %d, \"buf\": %zu, \"threads\": %d, \"rounds\": %d, "
         "\"mismatches\": %zu, \"errors\": %zu, \"seconds\": %.4f, \"aggregate_GiBps\": %.3f, \"ok\": %s}\n",
         k, p, buf, nthreads, rounds, bad.load(), errors.load(), timed_s, user / (1u << 30) / timed_s,
         ok ? "true" : "false");
  return ok ? 0 : 1;
}

// --async=D : one Encoder.encodeStripe and one Decoder.fixErasedBlockImpl of a
// `block`-byte stripe in bufSize rounds, synchronous (encodeBulkCrc /
// decodeBulkCrc per round) and pipelined D rounds deep (submit round r, read
// round r + 1 while it runs, collect round r - D + 1). Both produce every
// parity / repaired cell and the chained block CRC32s; both are checked
// against the oracle and zlib; prints the user-data GiB/s of each.
int async_mode(int k, int p, size_t block, size_t buf, int nerased, int depth, uint64_t seed) {
  const int n = k + p;
  hrs::HipReedSolomonCode code(k, p, 0);
  std::vector<std::vector<uint8_t>> stripe(n, std::vector<uint8_t>(block));
  for (int i = 0; i < k; ++i) fill(stripe[p + i], seed * 1000 + i);
  {
    std::vector<std::vector<uint8_t>> cp(stripe.begin() + p, stripe.end());
    std::vector<uint8_t*> ip(k), op(p);
    for (int i = 0; i < k; ++i) ip[i] = cp[i].data();
    for (int r = 0; r < p; ++r) op[r] = stripe[r].data();
    orc_rs_encode_bulk(k, p, ip.data(), op.data(), block);
  }
  std::vector<uint32_t> stored(n);
  for (int l = 0; l < n; ++l) stored[l] = crc(0, stripe[l].data(), block);
  uint64_t z = seed;
  std::vector<int> erased;
  while (static_cast<int>(erased.size()) < nerased) {
    const int loc = static_cast<int>(splitmix(z) % n);
    if (!contains(erased, loc)) erased.push_back(loc);
  }
  std::vector<int> ea, ta, na;
  decoder_arrays(n, erased, code.locationsToReadForDecode(erased), ea, ta, na);
  const int ne = static_cast<int>(ea.size());
  const size_t nrounds = (block + buf - 1) / buf;
  // read buffers (ParallelStreamReader): the Encoder's k, the Decoder's reads
  std::vector<std::vector<uint8_t>> rbuf(n, std::vector<uint8_t>(buf));
  std::vector<std::vector<uint8_t>> wbuf(std::max(p, ne), std::vector<uint8_t>(buf));
  std::vector<uint8_t*> enc_in(k), dec_in(n, nullptr), wp;
  for (int i = 0; i < k; ++i) enc_in[i] = rbuf[p + i].data();
  for (int l : ta) dec_in[l] = rbuf[l].data();
  std::vector<std::vector<uint8_t>> parity_out(p, std::vector<uint8_t>(block)), fixed(ne, std::vector<uint8_t>(block));
  size_t bad_at[2][2] = {{0, 0}, {0, 0}};  // [sync|async][encode|decode]
  double secs[2][2] = {{0, 0}, {0, 0}};
  for (int rep = 0; rep < 2; ++rep)       // 0: warm-up, 1: timed (both checked)
    for (int mode = 0; mode < 2; ++mode) {
      // ------------------------------------------------------------ Encoder
      std::vector<uint32_t> ecrc(n, 0);
      std::vector<uint64_t> tk(nrounds);
      auto t0 = std::chrono::steady_clock::now();
      auto encode_out = [&](size_t r) {
        std::vector<uint8_t*> op(p);
        for (int o = 0; o < p; ++o) op[o] = parity_out[o].data() + r * buf;
        return op;
      };
      for (size_t r = 0; r < nrounds + (mode ? depth - 1 : 0); ++r) {
        if (r < nrounds) {
          const size_t off = r * buf, len = std::min(buf, block - off);
          for (int i = 0; i < k; ++i) std::memcpy(rbuf[p + i].data(), stripe[p + i].data() + off, len);
          if (mode == 0) {
            std::vector<uint32_t> c(ecrc);
            std::vector<uint8_t*> wb(p);
            for (int o = 0; o < p; ++o) wb[o] = wbuf[o].data();
            code.encodeBulkCrc(enc_in, wb, len, c);
            ecrc = c;
            for (int o = 0; o < p; ++o) std::memcpy(parity_out[o].data() + off, wbuf[o].data(), len);  // out.write
            continue;
          }
          tk[r] = code.encodeBulkSubmit(enc_in, len, true);
        }
        if (mode == 1 && r + 1 >= static_cast<size_t>(depth)) {
          const size_t q = r + 1 - depth;
          code.collect(tk[q], encode_out(q), &ecrc);  // collect writes straight into the output block
        }
      }
      secs[mode][0] += rep ? std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() : 0;
      for (int o = 0; o < p; ++o) bad_at[mode][0] += parity_out[o] != stripe[o];
      for (int i = 0; i < n; ++i)  // ecrc: sources then parities; stored: by location (parity first)
        bad_at[mode][0] += ecrc[i] != stored[i < k ? p + i : i - k];
      for (auto& v : parity_out) std::fill(v.begin(), v.end(), 0);
      // ------------------------------------------------------------ Decoder
      std::vector<uint32_t> dcrc(ne, 0);
      t0 = std::chrono::steady_clock::now();
      for (size_t r = 0; r < nrounds + (mode ? depth - 1 : 0); ++r) {
        if (r < nrounds) {
          const size_t off = r * buf, len = std::min(buf, block - off);
          for (int l : ta) std::memcpy(rbuf[l].data(), stripe[l].data() + off, len);
          if (mode == 0) {
            // not-to-read rows: NULL (zeros, StripeReader.java:106-124); a
            // non-NULL row would be read as the Java decode reads it
            wp.assign(ne, nullptr);
            for (int j = 0; j < ne; ++j) wp[j] = wbuf[j].data();
            code.decodeBulkCrc(dec_in, wp, len, ea, ta, na, dcrc);
            for (int j = 0; j < ne; ++j) std::memcpy(fixed[j].data() + off, wbuf[j].data(), len);
            continue;
          }
          tk[r] = code.decodeBulkSubmit(dec_in, len, ea, ta, na, true);
        }
        if (mode == 1 && r + 1 >= static_cast<size_t>(depth)) {
          const size_t q = r + 1 - depth;
          std::vector<uint8_t*> op(ne);
          for (int j = 0; j < ne; ++j) op[j] = fixed[j].data() + q * buf;
          code.collect(tk[q], op, &dcrc);
        }
      }
      secs[mode][1] += rep ? std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() : 0;
      for (int j = 0; j < ne; ++j) bad_at[mode][1] += fixed[j] != stripe[ea[j]] || dcrc[j] != stored[ea[j]];
      for (auto& v : fixed) std::fill(v.begin(), v.end(), 0);
    }
  const double user = static_cast<double>(k) * block / (1u << 30);
  const size_t bad = bad_at[0][0] + bad_at[0][1] + bad_at[1][0] + bad_at[1][1];
  const bool ok = bad == 0;
  printf("{\"mode\": \"async\", \"k\": %d, \"p\": %d, \"block\": %zu, \"buf\": %zu, \"depth\": %d, "
         "\"erased\": %d, \"mismatches\": %zu, \"bad_sync_enc_dec\": [%zu, %zu], \"bad_async_enc_dec\": [%zu, %zu], "
         "\"encode_sync_GiBps\": %.3f, \"encode_async_GiBps\": %.3f, "
         "\"decode_sync_GiBps\": %.3f, \"decode_async_GiBps\": %.3f, \"ok\": %s}\n",
         k, p, block, buf, depth, ne, bad, bad_at[0][0], bad_at[0][1], bad_at[1][0], bad_at[1][1], user / secs[0][0], user / secs[1][0], user / secs[0][1],
         user / secs[1][1], ok ? "true" : "false");
  return ok ? 0 : 1;
}

int main(int argc, char** argv) {
  bool host_only = false, use_xor = false, use_nrs = false, use_src = false;
  int src_s = 0, grow = -1, threads = 0, rounds = 16, depth = 0;
  std::vector<std::string> pos;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--host-only")
      host_only = true;
    else if (a == "--xor")
      use_xor = true;
    else if (a == "--nrs")
      use_nrs = true;
    else if (a.rfind("--grow=", 0) == 0)
      grow = atoi(a.c_str() + 7);
    else if (a.rfind("--threads=", 0) == 0)
      threads = atoi(a.c_str() + 10);
    else if (a.rfind("--async=", 0) == 0)
      depth = atoi(a.c_str() + 8);
    else if (a.rfind("--rounds=", 0) == 0)
      rounds = atoi(a.c_str() + 9);
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
  try {
    if (grow >= 0) return grow_mode(k, p, block, buf, grow, seed);
    if (threads > 0) return threads_mode(k, p, buf, threads, rounds, seed);
    if (depth > 0) return async_mode(k, p, block, buf, nerased, depth, seed);
  } catch (const std::exception& e) {
    printf("{\"error\": \"%s\", \"ok\": false}\n", e.what());
    return 2;
  }
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
