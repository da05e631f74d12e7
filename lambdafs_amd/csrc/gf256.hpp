// GF(2^8) arithmetic and the Reed-Solomon coding matrices of hops
// `io.hops.erasure_coding.ReedSolomonCode`, written as constexpr C++ so the
// same definitions serve the host (matrix construction, decode cache) and the
// device (compile-time encode matrices baked into the gfx950 kernels).
//
// Field: GF(2^8) with primitive polynomial 285 = 0x11D, alpha = 2
//   (GaloisField.java:38-41, :84-92; ReedSolomonCode.java:33, :67-71).
// Code:  systematic cyclic RS, stripe symbol order [parity_0..p-1, data_0..k-1]
//   (ReedSolomonCode.java:87-96, ErasureCode.java:78-84); generator
//   g(x) = prod_{i<p} (x + alpha^i) (ReedSolomonCode.java:72-81).
//
// Everything the reference does on the byte path is GF(2^8)-linear, so both
// encodeBulk (ReedSolomonCode.java:103-125) and decodeBulk
// (ReedSolomonCode.java:168-211) are byte-matrix products Out = M * In. This
// header derives M in closed form (polynomial remainders for encode, an
// explicit Vandermonde inverse for decode); the test-only oracle under
// oracle/ re-runs the reference's own per-byte loops, and the parity tests
// compare the two.
#pragma once
#include <cstdint>
#include <cstddef>

#if defined(__HIPCC__)
#define HRS_HD __host__ __device__
#else
#define HRS_HD
#endif

namespace hrs {
namespace gf {

constexpr int kPrimitivePolynomial = 0x11D;  // GaloisField.java:41
constexpr int kFieldSize = 256;              // GaloisField.java:39

struct Tables {
  uint8_t exp[512];  // exp[i] = alpha^i, doubled so exp[log a + log b] needs no mod
  uint8_t log[256];  // log[0] unused
};

constexpr Tables make_tables() {
  Tables t{};
  int v = 1;
  for (int i = 0; i < 255; ++i) {
    t.exp[i] = static_cast<uint8_t>(v);
    t.exp[i + 255] = static_cast<uint8_t>(v);
    t.log[v] = static_cast<uint8_t>(i);
    v <<= 1;
    if (v & 0x100) v ^= kPrimitivePolynomial;
  }
  t.exp[510] = t.exp[0];
  t.exp[511] = t.exp[1];
  return t;
}

inline constexpr Tables kTables = make_tables();

HRS_HD constexpr uint8_t mul(uint8_t a, uint8_t b) {
  return (a == 0 || b == 0) ? 0 : kTables.exp[kTables.log[a] + kTables.log[b]];
}
// a / b; b != 0 (callers validate).
HRS_HD constexpr uint8_t div(uint8_t a, uint8_t b) {
  return (a == 0) ? 0 : kTables.exp[kTables.log[a] + 255 - kTables.log[b]];
}
HRS_HD constexpr uint8_t inv(uint8_t a) { return div(1, a); }
// alpha^e for e >= 0 (GaloisField.power(2, e), GaloisField.java:190-204).
HRS_HD constexpr uint8_t alpha_pow(long e) { return kTables.exp[e % 255]; }

// Multiply-by-constant as an 8x8 matrix over GF(2): bit q of mul(c, x) is the
// parity of (row_mask(c, q) & x). Column i of the matrix is mul(c, 1 << i).
HRS_HD constexpr uint8_t row_mask(uint8_t c, int q) {
  uint8_t m = 0;
  for (int i = 0; i < 8; ++i)
    if ((mul(c, static_cast<uint8_t>(1u << i)) >> q) & 1) m |= static_cast<uint8_t>(1u << i);
  return m;
}

// Largest parity count supported by the compile-time matrices below. The
// reference only asserts k + p < 256 (ReedSolomonCode.java:57).
constexpr int kMaxParity = 254;

// Generator polynomial coefficients g[0..p] (g[p] == 1), ReedSolomonCode.java:72-81.
struct GenPoly {
  uint8_t c[kMaxParity + 1];
};
HRS_HD constexpr GenPoly generator(int p) {
  GenPoly g{};
  g.c[0] = 1;
  for (int i = 0; i < p; ++i) {
    // multiply by (x + alpha^i)
    const uint8_t r = alpha_pow(i);
    for (int j = i + 1; j >= 0; --j) {
      const uint8_t hi = (j > 0) ? g.c[j - 1] : 0;
      g.c[j] = static_cast<uint8_t>(hi ^ mul(g.c[j], r));
    }
  }
  return g;
}

// Encode matrix: G[r][c] = coefficient r of (x^(p+c) mod g(x)); parity row r is
// sum_c G[r][c] * data_c. Equivalent to the bulk remainder in
// GaloisField.java:326-338 as driven by ReedSolomonCode.encodeBulk.
// `out` is row-major p x k.
HRS_HD constexpr void encode_matrix(int k, int p, uint8_t* out) {
  const GenPoly g = generator(p);
  uint8_t rem[kMaxParity] = {};
  // x^p mod g = g[0..p-1] (characteristic 2: -g == g)
  for (int r = 0; r < p; ++r) rem[r] = g.c[r];
  for (int c = 0; c < k; ++c) {
    for (int r = 0; r < p; ++r) out[r * k + c] = rem[r];
    // rem <- x * rem mod g
    const uint8_t top = rem[p - 1];
    for (int r = p - 1; r > 0; --r) rem[r] = static_cast<uint8_t>(rem[r - 1] ^ mul(top, g.c[r]));
    rem[0] = mul(top, g.c[0]);
  }
}

// Fixed-size compile-time encode matrix for the kernels' static variants.
template <int K, int P>
struct EncodeMatrix {
  uint8_t m[P][K];
  constexpr EncodeMatrix() : m{} {
    uint8_t flat[P * K] = {};
    encode_matrix(K, P, flat);
    for (int r = 0; r < P; ++r)
      for (int c = 0; c < K; ++c) m[r][c] = flat[r * K + c];
  }
};

// Parity rows of ISA-L gf_gen_cauchy1_matrix(m = K + P, k = K), the nrs code
// (erasure_coder.c:47-60): m[r][c] = 1 / ((K + r) ^ c).
template <int K, int P>
struct CauchyMatrix {
  uint8_t m[P][K];
  constexpr CauchyMatrix() : m{} {
    for (int r = 0; r < P; ++r)
      for (int c = 0; c < K; ++c) m[r][c] = inv(static_cast<uint8_t>((K + r) ^ c));
  }
};

}  // namespace gf
}  // namespace hrs
