// CPU model of the CRC-32 kernels (lambdafs_amd/csrc/hrs_crc.hip): the same
// tables (crc32.hpp) and the same decomposition — per 32 KiB window, lane l
// owns the 16-byte piece at q*1024 + 16l of each 1 KiB chunk q (slicing-by-4),
// joins its pieces in chunk order with Z_1024, then a 6-level lane tree with
// Z_{16*2^t}; the window fold with G windows per lane + Z_{window*G*2^t}
// tree, the right-aligned tail window and CRC32.update chaining — emulated
// lane by lane and checked against zlib; and the fused repair + CRC's 2 KiB
// windows with its DPP lane tree (hrs_decode_crc.hip).
#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../lambdafs_amd/csrc/crc32.hpp"

using namespace hrs::crc;

static uint32_t zmul(const std::vector<uint32_t>& z, uint32_t c) {
  return z[c & 255] ^ z[256 + ((c >> 8) & 255)] ^ z[512 + ((c >> 16) & 255)] ^ z[768 + (c >> 24)];
}
static std::vector<uint32_t> tab(uint64_t n) {
  std::vector<uint32_t> t(1024);
  to_tables(zeros(n), t.data());
  return t;
}

static std::vector<uint32_t> zchunk = tab(kChunkBytes);
static const int64_t W = static_cast<int64_t>(kWindowBytes);

// pieces: chunks of 1 KiB per window (32: the 32 KiB window kernels; 2: the
// fused repair's 2 KiB task window). dpp: the lane tree's levels 0-3 move
// within 16-lane rows (DPP row_shl, 0 past the row end) and levels 4-5 keep
// the lane's own value past lane 63 (__shfl_down), as lane_tree_dpp does;
// only lane 0's result is used, which never reads a lane past its row.
static uint32_t window_raw(const Slice4& sl, const std::vector<std::vector<uint32_t>>& tree, const uint8_t* p,
                           int64_t start, int64_t lo, int64_t end, int pieces = kPieces, bool dpp = false) {
  uint32_t c[64];
  for (int lane = 0; lane < 64; ++lane) {
    uint32_t x = 0;
    for (int q = 0; q < pieces; ++q) {
      uint32_t ch = 0;  // the 16-byte piece at q*1024 + 16*lane
      for (int j = 0; j < 4; ++j) {
        uint32_t w = 0;
        for (int b = 0; b < 4; ++b) {
          const int64_t pos = start + (int64_t)q * kChunkBytes + lane * kPieceBytes + 4 * j + b;
          if (pos >= lo && pos < end) w |= (uint32_t)p[pos] << (8 * b);
        }
        const uint32_t y = ch ^ w;
        ch = sl.s[3].t[y & 255] ^ sl.s[2].t[(y >> 8) & 255] ^ sl.s[1].t[(y >> 16) & 255] ^ sl.s[0].t[y >> 24];
      }
      x = q == 0 ? ch : (zmul(zchunk, x) ^ ch);
    }
    c[lane] = x;
  }
  for (int lvl = 0; lvl < 6; ++lvl) {
    const int d = 1 << lvl;
    uint32_t n[64];
    for (int l = 0; l < 64; ++l) {
      uint32_t o = l + d < 64 ? c[l + d] : 0;
      if (dpp && lvl < 4 && (l & 15) + d >= 16) o = 0;  // row_shl: nothing from the next row
      if (dpp && lvl >= 4 && l + d >= 64) o = c[l];     // __shfl_down: own value past the wave
      n[l] = zmul(tree[lvl], c[l]) ^ o;
    }
    for (int l = 0; l < 64; ++l) c[l] = n[l];
  }
  return c[0];
}

// The fused repair + CRC (hrs_decode_crc.hip): raw CRC per 2 KiB window (two
// pieces per lane, the DPP lane tree), folded like crc_fold_kernel with
// 2 KiB windows, CRC32.update chaining; lengths are whole windows.
static int fused_repair_model(const Slice4& sl, const std::vector<std::vector<uint32_t>>& tree, int* cases) {
  const int64_t W2 = 2048;
  int bad = 0;
  uint64_t seed = 7;
  for (size_t len : {2048ul, 4096ul, 2048ul * 63, 2048ul * 64, 2048ul * 65, 2048ul * 200, 1ul << 20}) {
    std::vector<uint8_t> d(len);
    for (auto& x : d) x = (uint8_t)((seed = seed * 6364136223846793005ull + 1442695040888963407ull) >> 56);
    const uint64_t nwin = len / W2, G = (nwin + 63) / 64;
    std::vector<uint32_t> raw(nwin);
    for (uint64_t w = 0; w < nwin; ++w) raw[w] = window_raw(sl, tree, d.data(), w * W2, w * W2, (w + 1) * W2, 2, true);
    auto zw = tab(W2), zlen = tab(len);
    std::vector<std::vector<uint32_t>> ft;
    for (int t = 0; t < 6; ++t) ft.push_back(tab(W2 * G << t));
    for (uint32_t crc_in : {0u, 0x1234567u}) {
      uint32_t c[64];
      const int64_t pad = (int64_t)G * 64 - (int64_t)nwin;
      for (int l = 0; l < 64; ++l) {
        c[l] = 0;
        for (uint64_t g = 0; g < G; ++g) {
          int64_t w = (int64_t)l * G + g - pad;
          if (w >= 0) c[l] = zmul(zw, c[l]) ^ raw[w];
        }
      }
      for (int lvl = 0; lvl < 6; ++lvl) {
        uint32_t n[64];
        for (int l = 0; l < 64; ++l) n[l] = zmul(ft[lvl], c[l]) ^ (l + (1 << lvl) < 64 ? c[l + (1 << lvl)] : 0);
        for (int l = 0; l < 64; ++l) c[l] = n[l];
      }
      const uint32_t out = zmul(zlen, crc_in ^ 0xFFFFFFFFu) ^ c[0] ^ 0xFFFFFFFFu;
      const uint32_t ref = (uint32_t)crc32(crc_in, d.data(), (uInt)len);
      ++*cases;
      if (out != ref) {
        ++bad;
        printf("fused repair window model, len %zu crc_in %08x: model %08x zlib %08x\n", len, crc_in, out, ref);
      }
    }
  }
  return bad;
}

int main() {
  const Slice4 sl = make_slice4();
  std::vector<std::vector<uint32_t>> tree;
  for (int t = 0; t < 6; ++t) tree.push_back(tab((uint64_t)kPieceBytes << t));
  int bad = 0, cases = 0;
  uint64_t seed = 1;
  for (size_t len : {0ul, 1ul, 63ul, 64ul, 4095ul, 4096ul, 32767ul, 32768ul, 32769ul, 65536ul + 5,
                     65536ul * 3 + 1000, 1ul << 20, (1ul << 20) + 32768 * 70 + 33, 32768ul * 64 * 2 + 17}) {
    std::vector<uint8_t> d(len);
    for (auto& x : d) x = (uint8_t)((seed = seed * 6364136223846793005ull + 1442695040888963407ull) >> 56);
    const uint64_t nwin = len / W, tail = len % W, G = (nwin + 63) / 64;
    std::vector<uint32_t> raw(nwin + 1);
    for (uint64_t w = 0; w < nwin; ++w) raw[w] = window_raw(sl, tree, d.data(), w * W, w * W, (w + 1) * W);
    if (tail) raw[nwin] = window_raw(sl, tree, d.data(), (int64_t)len - W, nwin * W, len);
    auto zw = tab(W), ztail = tab(tail), zlen = tab(len);
    std::vector<std::vector<uint32_t>> ft;
    for (int t = 0; t < 6; ++t) ft.push_back(tab(W * G << t));
    for (uint32_t crc_in : {0u, 0xDEADBEEFu}) {
      uint32_t c[64];
      const int64_t pad = (int64_t)G * 64 - (int64_t)nwin;
      for (int l = 0; l < 64; ++l) {
        c[l] = 0;
        for (uint64_t g = 0; g < G; ++g) {
          int64_t w = (int64_t)l * G + g - pad;
          if (w >= 0) c[l] = zmul(zw, c[l]) ^ raw[w];
        }
      }
      for (int lvl = 0; lvl < 6; ++lvl) {
        uint32_t n[64];
        for (int l = 0; l < 64; ++l) n[l] = zmul(ft[lvl], c[l]) ^ (l + (1 << lvl) < 64 ? c[l + (1 << lvl)] : 0);
        for (int l = 0; l < 64; ++l) c[l] = n[l];
      }
      uint32_t r = c[0];
      if (tail) r = zmul(ztail, r) ^ raw[nwin];
      const uint32_t out = zmul(zlen, crc_in ^ 0xFFFFFFFFu) ^ r ^ 0xFFFFFFFFu;
      static const uint8_t one = 0;  // zlib returns 0 for a NULL buffer; CRC32.update(b, 0, 0) keeps the value
      const uint32_t ref = (uint32_t)crc32(crc_in, len ? d.data() : &one, (uInt)len);
      ++cases;
      if (out != ref) {
        ++bad;
        printf("len %zu crc_in %08x: model %08x zlib %08x\n", len, crc_in, out, ref);
      }
    }
  }
  bad += fused_repair_model(sl, tree, &cases);
  printf("{\"crc_model_cases\": %d, \"mismatches\": %d}\n", cases, bad);
  return bad ? 1 : 0;
}
