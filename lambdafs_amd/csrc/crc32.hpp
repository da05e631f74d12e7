// CRC-32 as java.util.zip.CRC32 computes it (the zlib / ISO-HDLC CRC: reflected
// polynomial 0xEDB88320, init and xorout 0xFFFFFFFF), which the hops stream
// drivers keep per block: Encoder.java:408-450 (sources and parity),
// Decoder.java:222-229 and :645-655 (repaired blocks).
//
// The GPU computes *raw* CRCs (zero init, no xorout), which are GF(2)-linear:
//   raw(A || B) = Z_|B|(raw(A)) ^ raw(B),      Z_n = "append n zero bytes",
//   crc(prev || M) = Z_|M|(crc_prev ^ ~0) ^ raw(M) ^ ~0   (CRC32.update chaining).
// Z_n is a 32x32 matrix over GF(2); it is applied as 4 byte-indexed tables.
#pragma once
#include <cstddef>
#include <cstdint>

namespace hrs {
namespace crc {

constexpr uint32_t kPoly = 0xEDB88320u;  // reflected 0x04C11DB7

// Window decomposition of the GPU kernels (hrs_crc.hip), shared with the CPU
// model (tests/cpp/crc_model.cpp): a window is kPieces chunks of 1 KiB; lane
// l of the window's wave owns the 16-byte piece at q * 1024 + 16 l of every
// chunk q (so each load instruction is one contiguous 1 KiB wave access).
// Its piece CRCs join in chunk order with Z_1024, and a 6-level lane tree
// joins the lanes with Z_{16 * 2^t}.
constexpr int kChunkBytes = 1024;
constexpr int kPieceBytes = 16;
constexpr int kPieces = 32;
constexpr uint64_t kWindowBytes = static_cast<uint64_t>(kChunkBytes) * kPieces;  // 32 KiB

struct ByteTable {
  uint32_t t[256];
};

// Standard byte table: raw CRC of one byte.
constexpr ByteTable make_t0() {
  ByteTable b{};
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : c >> 1;
    b.t[i] = c;
  }
  return b;
}

// Slicing-by-4 tables: s[j] advances a byte that has j more bytes after it in
// the 4-byte word (s[0] == T0).
struct Slice4 {
  ByteTable s[4];
};
constexpr Slice4 make_slice4() {
  Slice4 x{};
  x.s[0] = make_t0();
  for (int j = 1; j < 4; ++j)
    for (int i = 0; i < 256; ++i) x.s[j].t[i] = (x.s[j - 1].t[i] >> 8) ^ x.s[0].t[x.s[j - 1].t[i] & 0xFFu];
  return x;
}

// 32x32 GF(2) matrix: col[i] = image of bit i.
struct Mat {
  uint32_t col[32];
};

inline uint32_t apply(const Mat& m, uint32_t v) {
  uint32_t r = 0;
  for (int i = 0; v; ++i, v >>= 1)
    if (v & 1u) r ^= m.col[i];
  return r;
}

inline Mat mul(const Mat& a, const Mat& b) {  // a after b
  Mat r{};
  for (int i = 0; i < 32; ++i) r.col[i] = apply(a, b.col[i]);
  return r;
}

// Z_1: append one zero byte to a raw CRC state.
inline Mat zero_byte() {
  const ByteTable t0 = make_t0();
  Mat m{};
  for (int i = 0; i < 32; ++i) {
    const uint32_t v = 1u << i;
    m.col[i] = t0.t[v & 0xFFu] ^ (v >> 8);
  }
  return m;
}

// Z_n by square-and-multiply.
inline Mat zeros(uint64_t n) {
  Mat result{};
  for (int i = 0; i < 32; ++i) result.col[i] = 1u << i;
  Mat p = zero_byte();
  while (n) {
    if (n & 1u) result = mul(p, result);
    n >>= 1;
    if (n) p = mul(p, p);
  }
  return result;
}

// The 4 byte tables of a matrix: apply(m, v) == t[0][v&255] ^ t[1][(v>>8)&255] ^ ...
inline void to_tables(const Mat& m, uint32_t* out /* 4 x 256 */) {
  for (int b = 0; b < 4; ++b)
    for (uint32_t v = 0; v < 256; ++v) out[b * 256 + v] = apply(m, v << (8 * b));
}

}  // namespace crc
}  // namespace hrs
