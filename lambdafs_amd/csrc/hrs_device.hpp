// Device helpers shared by the gfx950 kernels: the bit-slice transform and
// GF(2^8) plane arithmetic (hrs_kernels.hip, hrs_fused.hip), the 2 KiB window
// row loads/stores, and the CRC-32 table steps (hrs_crc.hip, hrs_fused.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "gf256.hpp"
#include "hrs_crc.hpp"
#include "hrs_internal.hpp"
#include "xor_sched.hpp"

namespace hrs {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Three-input XOR in one VALU op (gfx950 v_bitop3_b32, truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Bitwise select m ? x : y in one VALU op (v_bitop3_b32, truth table 0xCA).
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t x, uint32_t y) {
  return __builtin_amdgcn_bitop3_b32(m, x, y, 0xCA);
}

// One delta-swap stage between two words: the bits of `a` at positions
// (M << SH) trade places with the bits of `b` at positions M. Two shifts +
// two selects = 4 VALU ops.
template <int SH, uint32_t M>
__device__ __forceinline__ void xchg(uint32_t& a, uint32_t& b) {
  const uint32_t na = bsel(M << SH, b << SH, a);
  const uint32_t nb = bsel(M, a >> SH, b);
  a = na;
  b = nb;
}

// Swap the 3 word-index bits with the 3 bit-in-byte bits of 8 words. Word w,
// byte j, bit i  <->  word i, byte j, bit w. Afterwards w[i] holds bit i of
// all 32 bytes (a bit-plane). Involution: applying it twice is the identity.
__device__ __forceinline__ void bitslice(uint32_t (&w)[8]) {
  xchg<1, 0x55555555u>(w[0], w[1]);
  xchg<1, 0x55555555u>(w[2], w[3]);
  xchg<1, 0x55555555u>(w[4], w[5]);
  xchg<1, 0x55555555u>(w[6], w[7]);
  xchg<2, 0x33333333u>(w[0], w[2]);
  xchg<2, 0x33333333u>(w[1], w[3]);
  xchg<2, 0x33333333u>(w[4], w[6]);
  xchg<2, 0x33333333u>(w[5], w[7]);
  xchg<4, 0x0F0F0F0Fu>(w[0], w[4]);
  xchg<4, 0x0F0F0F0Fu>(w[1], w[5]);
  xchg<4, 0x0F0F0F0Fu>(w[2], w[6]);
  xchg<4, 0x0F0F0F0Fu>(w[3], w[7]);
}

// Multiply 32 sliced bytes by alpha = 2 modulo 0x11D (x^8 = x^4+x^3+x^2+1).
__device__ __forceinline__ void xtime(uint32_t (&p)[8]) {
  const uint32_t hi = p[7];
  p[7] = p[6];
  p[6] = p[5];
  p[5] = p[4];
  p[4] = p[3] ^ hi;
  p[3] = p[2] ^ hi;
  p[2] = p[1] ^ hi;
  p[1] = p[0];
  p[0] = hi;
}

// Lane `lane` of the wave owns bytes [lane*16, +16) and [1024 + lane*16, +16)
// of the 2 KiB window at `p`. Only whole windows reach these kernels; the
// row tail (len % 2 KiB) goes to the byte-granular kernel. Every byte is
// touched once, so loads and stores are nontemporal (streaming; measured
// +4% over default-policy accesses, tools/kernel_lab.hip).
__device__ __forceinline__ void load_row(const uint8_t* p, int lane, uint32_t (&w)[8]) {
  const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + lane * 16));
  const u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + 1024 + lane * 16));
  w[0] = x[0]; w[1] = x[1]; w[2] = x[2]; w[3] = x[3];
  w[4] = y[0]; w[5] = y[1]; w[6] = y[2]; w[7] = y[3];
}

__device__ __forceinline__ void store_row(uint8_t* p, int lane, const uint32_t (&w)[8]) {
  const u32x4 x = {w[0], w[1], w[2], w[3]};
  const u32x4 y = {w[4], w[5], w[6], w[7]};
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p + lane * 16));
  __builtin_nontemporal_store(y, reinterpret_cast<u32x4*>(p + 1024 + lane * 16));
}

// Same accesses from a wave-uniform row base plus the lane's 32-bit byte
// offset (16 * lane): the compiler can then address with an SGPR base and one
// shared VGPR offset (global_load ... v_off, s[base]) instead of a 64-bit
// VGPR address per row, which in register-tight kernels it would spill.
// (The pointers are rebuilt in the global address space: a plain cast back
// from integers would make them flat accesses, which also count in lgkmcnt
// and so stall every LDS wait behind the row loads.)
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

__device__ __forceinline__ uint64_t uniform_addr(const void* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// The lane's two 16-byte pieces of a 2 KiB sub-window: base + loff and
// 1 KiB later.
__device__ __forceinline__ void load_row_u(const uint8_t* base, uint32_t loff, uint32_t (&w)[8]) {
  const g_u32x4* b = reinterpret_cast<const g_u32x4*>(uniform_addr(base) + loff);
  const u32x4 x = __builtin_nontemporal_load(b);
  const u32x4 y = __builtin_nontemporal_load(b + 64);  // + 1024 bytes
  w[0] = x[0]; w[1] = x[1]; w[2] = x[2]; w[3] = x[3];
  w[4] = y[0]; w[5] = y[1]; w[6] = y[2]; w[7] = y[3];
}

__device__ __forceinline__ void store_row_u(uint8_t* base, uint32_t loff, const uint32_t (&w)[8]) {
  g_u32x4* b = reinterpret_cast<g_u32x4*>(uniform_addr(base) + loff);
  const u32x4 x = {w[0], w[1], w[2], w[3]};
  const u32x4 y = {w[4], w[5], w[6], w[7]};
  __builtin_nontemporal_store(x, b);
  __builtin_nontemporal_store(y, b + 64);
}

__device__ __forceinline__ uint32_t wave_id_in_grid() {
  return __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
}

// The tasks (2 KiB windows, task t = stripe * nwin + window) the calling wave
// runs, in order: at(0), at(1), ... while below end. `order` (hrs_launch.hpp
// task_order) picks the window -> wave assignment:
//   C >= 1  block-cyclic: block b takes chunks b, b + G, ... of C * wpb
//           consecutive tasks, its waves interleaved within a chunk (C = 1 is
//           the grid-stride order of rounds 1-4: wave w of W takes w, w + W, ...);
//   0       block range: block b owns the b-th of G equal runs of consecutive
//           tasks (one chunk per block), so each block streams one contiguous
//           region of every row, as the fastest 1:1 copy on this pool does
//           (tools/copy_lab.hip).
// Measured (tools/sched_lab.hip, bench_order.py, order_shapes.py; profiles/
// r04/o, q, r, s): no order wins across shapes and boxes. The block range ran
// bench.py's RS(10,4) 1 MiB x 1,024 encode 3-7 % faster on four boxes and
// 6 % slower on a fifth, and lost 5-25 % on RS(12,4) and small jobs; the
// repairs prefer grid-stride or pairs (C = 2) by 0-3 %. Every family keeps
// grid-stride (hrs_launch.hpp kOrder*); the other orders stay as A/B knobs.
// Wave-uniform (SGPRs); at() is a few VALU/SALU ops per task.
struct WaveTasks {
  uint64_t t0, end, jump;  // jump: tasks between a wave's chunks (G * C * wpb)
  uint32_t chunk, wpb;     // tasks per wave per chunk (block range: 2^32 - 1)

  __device__ __forceinline__ uint64_t at(uint32_t j) const {
    if (chunk == 1) return t0 + j * jump;  // grid-stride, the default: no division
    const uint32_t q = j / chunk;
    return t0 + q * jump + static_cast<uint64_t>(j - q * chunk) * wpb;
  }
};

__device__ __forceinline__ WaveTasks wave_tasks(uint64_t ntasks, int order) {
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (order >= 1) {
    const uint32_t c = static_cast<uint32_t>(order);
    return {static_cast<uint64_t>(blockIdx.x) * c * wpb + w, ntasks, static_cast<uint64_t>(gridDim.x) * c * wpb, c, wpb};
  }
  const uint64_t per = (ntasks + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = per * blockIdx.x;
  return {lo + w, lo + per < ntasks ? lo + per : ntasks, 0, 0xFFFFFFFFu, wpb};
}

// mask[o][r][q]: the input bit-planes of data row r that feed bit-plane q of
// parity row o (gf::row_mask of G[o][r]). Evaluated by the compiler.
// MATRIX is gf::EncodeMatrix<K,P> (hops RS) or gf::CauchyMatrix<K,P> (nrs).
template <int K, int P, class MATRIX>
struct StaticPlan {
  uint8_t mask[P][K][8];
  constexpr StaticPlan() : mask{} {
    const MATRIX g;
    for (int o = 0; o < P; ++o)
      for (int r = 0; r < K; ++r)
        for (int q = 0; q < 8; ++q) mask[o][r][q] = gf::row_mask(g.m[o][r], q);
  }
};

// Accumulates the bit-sliced data row r of a window into the sliced parity
// planes: acc[o][q] ^= XOR of the planes plan.mask[o][r][q] selects, two
// planes per v_bitop3; an odd plane waits in pend for the next row. `has` is
// compile-time after unrolling.
template <int K, int P, class MATRIX>
__device__ __forceinline__ void encode_row_acc(int r, const uint32_t (&w)[8], uint32_t (&acc)[P][8],
                                               uint32_t (&pend)[P][8], bool (&has)[P][8]) {
  constexpr StaticPlan<K, P, MATRIX> plan{};
#pragma unroll
  for (int o = 0; o < P; ++o)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if ((plan.mask[o][r][q] >> i) & 1) {
          if (has[o][q]) {
            acc[o][q] = xor3(acc[o][q], pend[o][q], w[i]);
            has[o][q] = false;
          } else {
            pend[o][q] = w[i];
            has[o][q] = true;
          }
        }
      }
    }
}

// ------------------------------------------- factored XOR networks (CSE)

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Schedule family of a compile-time matrix (xor_sched.hpp): 0 = hops RS
// generator rows, 1 = ISA-L Cauchy rows.
template <class MATRIX> struct MatrixFamily;
template <int K, int P> struct MatrixFamily<gf::EncodeMatrix<K, P>> { static constexpr int value = 0; };
template <int K, int P> struct MatrixFamily<gf::CauchyMatrix<K, P>> { static constexpr int value = 1; };

// Group GI of a factored schedule (tools/gen_xor_sched.py): the group's
// sliced input planes x[g][i] are vars 8g + i; the shared temporaries are
// built first (one xor3 or XOR each), then every parity plane folds in its
// remaining terms two per xor3. Group 0 starts the planes (no running
// value). Every index is a compile-time constant, so v[] lives in registers.
// RS(10,4): 290-386 xor ops per 2 KiB window instead of 631-660 plane by
// plane, depending on the rows per group.
template <class S, int GI, int G, int P>
__device__ __forceinline__ void xor_sched_apply(const uint32_t (&x)[G][8], uint32_t (&acc)[P][8]) {
  constexpr int nin = S::kNin[GI];
  constexpr int op0 = S::kOpOff[GI];
  constexpr int nops = S::kOpOff[GI + 1] - op0;
  uint32_t v[S::kMaxVars];
#pragma unroll
  for (int i = 0; i < nin; ++i) v[i] = x[i >> 3][i & 7];
  static_for<0, nops>([&](auto j) __attribute__((always_inline)) {
    constexpr xsched::Op op = S::kOps[op0 + decltype(j)::value];
    if constexpr (op.c == 255)
      v[nin + decltype(j)::value] = v[op.a] ^ v[op.b];
    else
      v[nin + decltype(j)::value] = xor3(v[op.a], v[op.b], v[op.c]);
  });
  static_for<0, 8 * P>([&](auto pl) __attribute__((always_inline)) {
    constexpr int t0 = S::kTermOff[GI][decltype(pl)::value];
    constexpr int t1 = S::kTermOff[GI][decltype(pl)::value + 1];
    uint32_t& a = acc[decltype(pl)::value >> 3][decltype(pl)::value & 7];
    int t = t0;
    if constexpr (GI == 0) {
      if constexpr (t1 == t0) {
        a = 0u;
      } else {
        a = v[S::kTerms[t0]];
        t = t0 + 1;
      }
    }
#pragma unroll
    for (; t + 1 < t1; t += 2) a = xor3(a, v[S::kTerms[t]], v[S::kTerms[t + 1]]);
    if (t < t1) a ^= v[S::kTerms[t]];
  });
}

// ------------------------------------------------------------ CRC-32 steps

// Z(c) from a 4 x 256 table image in LDS.
__device__ __forceinline__ uint32_t zmul(const uint32_t* z, uint32_t c) {
  return z[c & 0xFFu] ^ z[256 + ((c >> 8) & 0xFFu)] ^ z[512 + ((c >> 16) & 0xFFu)] ^ z[768 + (c >> 24)];
}

// Slicing-by-4 tables in LDS, replicated kCrcRep = 32 times so lane l reads
// copy l % 32: ds_read_b32 banks are (address / 4) mod 32 per 32-lane group,
// so every data lookup is conflict-free. Layout: two 64 KiB regions; entry e
// of table j, copy c at LDS byte (j >> 1) * 65536 + 256 e + 128 (j & 1) + 4 c.
// Then one v_perm_b32 builds a lookup address from a data byte and the lane's
// copy word (byte 0 = 4 c, byte 1 = the data byte, byte 2 = region), instead
// of an extract + shift-add. The image must start at LDS address 0 (kernels
// that use it have no static LDS; the CRC tests would fail otherwise).
typedef __attribute__((address_space(3))) const uint32_t lds_u32;

struct SliceTab {
  uint32_t lw_lo;  // 4 c           (tables 0, 1)
  uint32_t lw_hi;  // 4 c | 0x10000 (tables 2, 3)
};

// rep_mask (A/B of the replication factor): lane l reads copy l & rep_mask;
// kCrcRep - 1 (31) = every lane of a 32-lane group on its own bank.
__device__ __forceinline__ SliceTab slice_tab(int lane, uint32_t rep_mask = kCrcRep - 1) {
  const uint32_t c4 = (static_cast<uint32_t>(lane) & rep_mask) * 4u;
  return SliceTab{c4, c4 | 0x10000u};
}

__device__ __forceinline__ uint32_t lds_at(uint32_t byte_addr) {
  return *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(byte_addr));
}

// One slicing-by-4 step: T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3].
__device__ __forceinline__ uint32_t slice4(const SliceTab& t, uint32_t x) {
  const uint32_t a3 = __builtin_amdgcn_perm(x, t.lw_hi, 0x0C020400u);  // [4c, x.b0, 1, 0]
  const uint32_t a2 = __builtin_amdgcn_perm(x, t.lw_hi, 0x0C020500u);  // [4c, x.b1, 1, 0]
  const uint32_t a1 = __builtin_amdgcn_perm(x, t.lw_lo, 0x0C0C0600u);  // [4c, x.b2, 0, 0]
  const uint32_t a0 = __builtin_amdgcn_perm(x, t.lw_lo, 0x0C0C0700u);  // [4c, x.b3, 0, 0]
  return xor3(lds_at(a3 + 128u), lds_at(a2), lds_at(a1 + 128u)) ^ lds_at(a0);
}

// slice4(t, x) ^ y in two VALU ops (the next word of the piece folds into
// the step's own XOR tree).
__device__ __forceinline__ uint32_t slice4_xor(const SliceTab& t, uint32_t x, uint32_t y) {
  const uint32_t a3 = __builtin_amdgcn_perm(x, t.lw_hi, 0x0C020400u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, t.lw_hi, 0x0C020500u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, t.lw_lo, 0x0C0C0600u);
  const uint32_t a0 = __builtin_amdgcn_perm(x, t.lw_lo, 0x0C0C0700u);
  return xor3(xor3(lds_at(a3 + 128u), lds_at(a2), lds_at(a1 + 128u)), lds_at(a0), y);
}

// Raw CRC of one 16-byte piece (4 little-endian words).
__device__ __forceinline__ uint32_t piece_crc(const SliceTab& s, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  uint32_t c = slice4_xor(s, w0, w1);
  c = slice4_xor(s, c, w2);
  c = slice4_xor(s, c, w3);
  return slice4(s, c);
}

// Z(c) ^ y from a 4 x 256 table image in LDS (two VALU ops for the XORs).
__device__ __forceinline__ uint32_t zmul_xor(const uint32_t* z, uint32_t c, uint32_t y) {
  return xor3(xor3(z[c & 0xFFu], z[256 + ((c >> 8) & 0xFFu)], z[512 + ((c >> 16) & 0xFFu)]), z[768 + (c >> 24)], y);
}

// Raw CRCs of the lane's two pieces of M rows (row m's words x[m][0..3] and
// x[m][4..7]), 2M chains advanced in lockstep so each step issues 8M
// independent LDS lookups before waiting on any (one chain at a time leaves
// the LDS latency exposed between its four dependent steps).
template <int M>
__device__ __forceinline__ void rows_piece_crcs(const SliceTab& t, const uint32_t (&x)[M][8], uint32_t (&c0)[M],
                                                uint32_t (&c1)[M]) {
#pragma unroll
  for (int m = 0; m < M; ++m) {
    c0[m] = x[m][0];
    c1[m] = x[m][4];
  }
#pragma unroll
  for (int st = 0; st < 4; ++st) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      c0[m] = slice4(t, c0[m]);
      c1[m] = slice4(t, c1[m]);
    }
    if (st < 3) {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        c0[m] ^= x[m][st + 1];
        c1[m] ^= x[m][st + 5];
      }
    }
  }
}

// Joins the 64 lanes' raw CRCs of a window whose lane l covered the pieces at
// 16 l + 1024 q: lane tree with Z_{16 * 2^t}; lane 0 ends with the window's.
__device__ __forceinline__ uint32_t lane_tree(const uint32_t* tree, uint32_t c) {
#pragma unroll
  for (int lvl = 0; lvl < 6; ++lvl) {
    const uint32_t o = __shfl_down(c, 1 << lvl, 64);
    c = zmul(tree + lvl * 1024, c) ^ o;
  }
  return c;
}

// Lane l receives v of lane l + N within its row of 16 lanes (0 past the
// row's end): one DPP row_shl move on the VALU instead of a ds_bpermute
// through the LDS unit.
template <int N>
__device__ __forceinline__ uint32_t dpp_down(uint32_t v) {
  static_assert(N >= 1 && N <= 15, "row_shl reaches within a row of 16 lanes");
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x100 + N, 0xF, 0xF, true));
}

// lane_tree with the levels inside a 16-lane row (2^t = 1, 2, 4, 8) moved by
// DPP: lane 0's chain only ever reads lanes of its own row at those levels
// (lanes whose partner lies past their row end compute values no later level
// reads). Same result as lane_tree in lane 0.
__device__ __forceinline__ uint32_t lane_tree_dpp(const uint32_t* tree, uint32_t c) {
  c = zmul(tree + 0 * 1024, c) ^ dpp_down<1>(c);
  c = zmul(tree + 1 * 1024, c) ^ dpp_down<2>(c);
  c = zmul(tree + 2 * 1024, c) ^ dpp_down<4>(c);
  c = zmul(tree + 3 * 1024, c) ^ dpp_down<8>(c);
  c = zmul(tree + 4 * 1024, c) ^ __shfl_down(c, 16, 64);
  c = zmul(tree + 5 * 1024, c) ^ __shfl_down(c, 32, 64);
  return c;
}

// ---------------------------------------- runtime-matrix kernel helpers

// NINB >= nin rows of the window are all loaded before any math (one
// 20 KiB-class burst per wave, like the static kernel), so a wave keeps
// nin x 2 KiB in flight; coefficients are wave-uniform kernel arguments.
// Bit loop unrolled (xtime is then a free relabel of the planes) unless the
// body would outgrow the instruction cache: unrolled, bitsliced<4,12> is
// 28 KiB of branchy code and ran 40% slower than rolled (profiles/r04/DESIGN_history.md §3).
template <int NOUT, int NINB>
struct BitLoop {
  static constexpr bool kRolled = NOUT * NINB >= 40;
};

template <int NOUT, int NINB>
__device__ __forceinline__ void mul_acc_row(uint32_t (&acc)[NOUT][8], uint32_t (&x)[8], const uint32_t (&cw)[2], int b) {
#pragma unroll
  for (int o = 0; o < NOUT; ++o)
    if ((cw[o >> 2] >> (8 * (o & 3) + b)) & 1u) {
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[o][q] ^= x[q];
    }
}

// acc[o] ^= coef[o] * x for one input row of a window: bit-slice the row,
// then for every set bit b of each output's coefficient XOR alpha^b x into it
// (wave-uniform branches). w packs the coefficients (byte o = output o); the
// empty asm keeps the per-(o, b) tests next to their use instead of hoisted
// out of the task loop (they would spill). Rolled bit loop when the unrolled
// body would outgrow the instruction cache (BitLoop). x is consumed.
template <int NOUT, int NINB>
__device__ __forceinline__ void accumulate_row(uint32_t (&acc)[NOUT][8], uint32_t (&x)[8], uint64_t w) {
  bitslice(x);
  uint32_t cw[2] = {static_cast<uint32_t>(w), static_cast<uint32_t>(w >> 32)};
  asm volatile("" : "+s"(cw[0]));
  if constexpr (NOUT > 4) asm volatile("" : "+s"(cw[1]));  // outputs 4..7 only
  if constexpr (BitLoop<NOUT, NINB>::kRolled) {
#pragma unroll 1
    for (int b = 0; b < 8; ++b) {
      mul_acc_row<NOUT, NINB>(acc, x, cw, b);
      xtime(x);
    }
  } else {
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      mul_acc_row<NOUT, NINB>(acc, x, cw, b);
      if (b < 7) xtime(x);
    }
  }
}

}  // namespace hrs
