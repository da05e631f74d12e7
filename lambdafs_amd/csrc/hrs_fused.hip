// gfx950 fused encode + CRC-32: the parity of every stripe and the
// java.util.zip.CRC32 of every source and parity cell in ONE pass over HBM —
// what Encoder.encodeStripe does per bufSize round with computeBlockChecksum
// (sourceChecksums over readBufs before encodeBulk, parityChecksums over
// writeBufs after it; Encoder.java:408-450). Run as two passes (encode, then
// hrs_crc32_dev) the cells are read twice; fused, the CRC consumes the words
// the encode already holds in registers.
//
// Decomposition: one wave per (stripe, window); a window is `subs` sub-windows
// of 2 KiB (16 = 32 KiB for large jobs; fewer when the job has too few
// 32 KiB windows to give every CU waves) — a sub-window is exactly the encode
// kernels' task (lane l holds
// the 16-byte pieces at 16 l and 1024 + 16 l of each sub-window, i.e. chunks
// 2i and 2i+1 of the window), so the CRC decomposition is identical to
// crc_window_kernel's (lane l owns the piece at 1024 q + 16 l of every chunk
// q, pieces joined in chunk order with Z_1024, lanes joined by the Z_{16*2^t}
// tree): the raw window CRCs it writes are the ones crc_window_kernel would
// write, and crc_fold_kernel finishes them unchanged. The slicing tables are
// the same 32x bank-replicated LDS image (156 KiB: one block per CU).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <string>

#include "hrs_device.hpp"
#include "hrs_launch.hpp"

namespace hrs {
namespace {

template <int K, int P, class MATRIX, int THREADS>
__global__ void __launch_bounds__(THREADS) encode_crc_kernel(const EncodeCrcArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < kCrcLdsWordsA; i += THREADS) lds[i] = a.tables[i];
  __syncthreads();
  constexpr int N = K + P;
  const int lane = threadIdx.x & 63;
  const SliceTab slices = slice_tab(lane, a.rep_mask);
  const uint32_t* zchunk = lds + kCrcSliceWords;
  const uint32_t* tree = zchunk + 1024;
  const uint64_t ntasks = a.nstripes * a.nwin;
  const WaveTasks wt = wave_tasks(ntasks, a.order);
  for (uint32_t j = 0; j < 0xFFFFFFFFu; ++j) {
    const uint64_t t = wt.at(j);
    if (t >= wt.end) break;
    const uint64_t stripe = t / a.nwin;
    const uint64_t w = t - stripe * a.nwin;
    const uint64_t in_base = stripe * a.in_stride + w * a.subs * kWindowBytes;
    const uint64_t out_base = stripe * a.out_stride + w * a.subs * kWindowBytes;
    uint32_t crc[N];
#pragma unroll
    for (int r = 0; r < N; ++r) crc[r] = 0u;  // Z(0) = 0: the first piece needs no special case
#pragma unroll 1
    for (uint32_t sub = 0; sub < a.subs; ++sub) {
      const uint64_t off = static_cast<uint64_t>(sub) * kWindowBytes;
      uint32_t acc[P][8];
      uint32_t pend[P][8];
      bool has[P][8];
#pragma unroll
      for (int o = 0; o < P; ++o)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          acc[o][q] = 0u;
          pend[o][q] = 0u;
          has[o][q] = false;
        }
#pragma unroll
      for (int r = 0; r < K; ++r) {
        uint32_t x[8];
        load_row(a.in[r] + in_base + off, lane, x);
        const uint32_t c0 = piece_crc(slices, x[0], x[1], x[2], x[3]);  // chunk 2 sub
        const uint32_t c1 = piece_crc(slices, x[4], x[5], x[6], x[7]);  // chunk 2 sub + 1
        crc[r] = zmul(zchunk, zmul(zchunk, crc[r]) ^ c0) ^ c1;
        bitslice(x);
        encode_row_acc<K, P, MATRIX>(r, x, acc, pend, has);
      }
#pragma unroll
      for (int o = 0; o < P; ++o)
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (has[o][q]) acc[o][q] ^= pend[o][q];
#pragma unroll
      for (int o = 0; o < P; ++o) {
        bitslice(acc[o]);
        store_row(a.out[o] + out_base + off, lane, acc[o]);
      }
      uint32_t p0[P], p1[P];
      rows_piece_crcs<P>(slices, acc, p0, p1);
#pragma unroll
      for (int o = 0; o < P; ++o) crc[K + o] = zmul(zchunk, zmul(zchunk, crc[K + o]) ^ p0[o]) ^ p1[o];
    }
#pragma unroll
    for (int r = 0; r < N; ++r) {
      const uint32_t c = lane_tree(tree, crc[r]);
      if (lane == 0) a.raw[(stripe * N + r) * a.nwin + w] = c;
    }
  }
}

// The scheduler otherwise interleaves the row groups for ILP until the live
// ranges spill; a scheduling barrier between them keeps each group's
// temporaries short-lived.
#ifndef HRS_NO_PHASE_FENCE
#define HRS_PHASE_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define HRS_PHASE_FENCE() ((void)0)
#endif

// Accumulates the sliced rows r0 .. r0+G-1 (those below K) into the parity
// planes: each plane's selected input planes across the whole group are
// paired into xor3s, so an odd leftover costs a lone XOR once per group
// instead of once per row.
template <int K, int P, class MATRIX, int G>
__device__ __forceinline__ void encode_group_acc(int r0, const uint32_t (&x)[G][8], uint32_t (&acc)[P][8]) {
  constexpr StaticPlan<K, P, MATRIX> plan{};
#pragma unroll
  for (int o = 0; o < P; ++o)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      uint32_t pend = 0u;
      bool has = false;
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (r0 + g < K && ((plan.mask[o][r0 + g < K ? r0 + g : 0][q] >> i) & 1)) {
            if (has) {
              acc[o][q] = xor3(acc[o][q], pend, x[g][i]);
              has = false;
            } else {
              pend = x[g][i];
              has = true;
            }
          }
      if (has) acc[o][q] ^= pend;
    }
}

// Grouped form (the default; HRS_FUSED=1 selects the row-serial one above for
// A/B runs). The same window walk, but the K data rows of a sub-window go in
// groups of G: a group's G loads issue together from wave-uniform row bases
// (SGPR base + one shared VGPR lane offset), its 2G CRC chains advance in
// lockstep (8G independent LDS lookups per slicing step), each running CRC is
// pinned in place as soon as it is updated (otherwise the compiler sinks its
// final XORs to the loop end and keeps every row's table words live:
// spills). The next word of a piece folds into each slicing step's XOR tree
// (slice4_xor), the Horner term into the zmul's (zmul_xor). G need not divide
// K (a last, smaller group).
// Parity: SCHED (the default) evaluates the group's factored XOR network
// (xor_sched.hpp: shared xor3 temporaries over the group's 8G planes), else
// each plane's selected planes are paired into xor3s across the group's rows.
// Per 2 KiB sub-window of RS(10,4), G = 2: 2,048 VALU factored, 2,313 paired
// (row-serial: 2,473); measured 3.10 vs 3.17 ms (RS(12,4), G = 4: 3.60 vs
// 3.92 ms), profiles/r02/sched.
template <int K, int P, class MATRIX, int THREADS, int G, bool SCHED>
__global__ void __launch_bounds__(THREADS) encode_crc_grouped_kernel(const EncodeCrcArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < kCrcLdsWordsA; i += THREADS) lds[i] = a.tables[i];
  __syncthreads();
  constexpr int N = K + P;
  constexpr int kGroups = (K + G - 1) / G;
  const int lane = threadIdx.x & 63;
  const uint32_t loff = static_cast<uint32_t>(lane) * 16u;
  const SliceTab slices = slice_tab(lane, a.rep_mask);
  const uint32_t* zchunk = lds + kCrcSliceWords;
  const uint32_t* tree = zchunk + 1024;
  const uint64_t ntasks = a.nstripes * a.nwin;
  const WaveTasks wt = wave_tasks(ntasks, a.order);
  for (uint32_t j = 0; j < 0xFFFFFFFFu; ++j) {
    const uint64_t t = wt.at(j);
    if (t >= wt.end) break;
    const uint64_t stripe = t / a.nwin;
    const uint64_t w = t - stripe * a.nwin;
    const uint64_t in_base = stripe * a.in_stride + w * a.subs * kWindowBytes;
    const uint64_t out_base = stripe * a.out_stride + w * a.subs * kWindowBytes;
    uint32_t crc[N];
#pragma unroll
    for (int r = 0; r < N; ++r) crc[r] = 0u;
#pragma unroll 1
    for (uint32_t sub = 0; sub < a.subs; ++sub) {
      const uint64_t off = static_cast<uint64_t>(sub) * kWindowBytes;
      uint32_t acc[P][8];
      if constexpr (!SCHED) {
#pragma unroll
        for (int o = 0; o < P; ++o)
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
      }
      static_for<0, kGroups>([&](auto gi) __attribute__((always_inline)) {
        constexpr int GI = decltype(gi)::value;
        constexpr int r0 = GI * G;
        HRS_PHASE_FENCE();
        uint32_t x[G][8];
#pragma unroll
        for (int g = 0; g < G; ++g)
          if (r0 + g < K) load_row_u(a.in[r0 + g] + in_base + off, loff, x[g]);
        uint32_t c0[G], c1[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          c0[g] = x[g][0];
          c1[g] = x[g][4];
        }
#pragma unroll
        for (int st = 0; st < 3; ++st)
#pragma unroll
          for (int g = 0; g < G; ++g)
            if (r0 + g < K) {
              c0[g] = slice4_xor(slices, c0[g], x[g][st + 1]);
              c1[g] = slice4_xor(slices, c1[g], x[g][st + 5]);
            }
#pragma unroll
        for (int g = 0; g < G; ++g)
          if (r0 + g < K) {
            c0[g] = slice4(slices, c0[g]);
            c1[g] = slice4(slices, c1[g]);
          }
#pragma unroll
        for (int g = 0; g < G; ++g)
          if (r0 + g < K) {
            crc[r0 + g] = zmul_xor(zchunk, zmul_xor(zchunk, crc[r0 + g], c0[g]), c1[g]);
            __asm__ volatile("" : "+v"(crc[r0 + g]));
          }
#pragma unroll
        for (int g = 0; g < G; ++g)
          if (r0 + g < K) bitslice(x[g]);
        if constexpr (SCHED)
          xor_sched_apply<xsched::Sched<MatrixFamily<MATRIX>::value, K, P, G>, GI, G, P>(x, acc);
        else
          encode_group_acc<K, P, MATRIX, G>(r0, x, acc);
      });
      HRS_PHASE_FENCE();
#pragma unroll
      for (int o = 0; o < P; ++o) {
        bitslice(acc[o]);
        store_row_u(a.out[o] + out_base + off, loff, acc[o]);
      }
      uint32_t p0[P], p1[P];
      rows_piece_crcs<P>(slices, acc, p0, p1);
#pragma unroll
      for (int o = 0; o < P; ++o) crc[K + o] = zmul_xor(zchunk, zmul_xor(zchunk, crc[K + o], p0[o]), p1[o]);
    }
#pragma unroll
    for (int r = 0; r < N; ++r) {
      const uint32_t c = lane_tree(tree, crc[r]);
      if (lane == 0) a.raw[(stripe * N + r) * a.nwin + w] = c;
    }
  }
}

// One 1024-thread block per CU (16 waves share the 156 KiB table image).
constexpr int kFusedThreads = 1024;
// Zero-copy jobs too small to give every CU of the grid 16 waves (a staged
// host call's 256 KiB chunk: 128 windows, 8 blocks of 1,024) take 256-thread blocks
// instead, still one per CU: 4x the CUs, so a wave's ~20 us of VALU work per
// sub-window is shared by 1 wave per SIMD instead of 4 and the last window
// finishes soon after its bytes arrive (HRS_FUSED_NARROW=0: always 1,024).
constexpr int kFusedNarrowThreads = 256;

// Rows per lockstep group, measured best (profiles/r02/sched): 2 (RS(10,4)
// 3.10 ms vs 3.06-3.28 at 4), 4 from K = 12 (RS(12,4) 3.60 vs 3.72 at 2).
template <int K>
constexpr int kFusedGroup = K >= 12 ? 4 : 2;

// HRS_FUSED (A/B runs): 1 = row-serial, 2 = grouped with the paired XOR
// network, default = grouped with the factored network. HRS_FUSED_GROUP
// overrides the rows per group (1 | 2 | 4).
int fused_variant() {
  static const int v = [] {
    const char* e = getenv("HRS_FUSED");
    if (e && e[0] == '1') return 1;
    if (e && e[0] == '2') return 2;
    return 3;
  }();
  return v;
}

bool fused_narrow_on() {  // read per launch (A/B runs in one process)
  const char* e = getenv("HRS_FUSED_NARROW");
  return !(e && e[0] == '0');
}

int fused_group() {
  static const int v = [] {
    const char* e = getenv("HRS_FUSED_GROUP");
    const int x = e ? atoi(e) : 0;
    return (x == 1 || x == 2 || x == 4) ? x : 0;
  }();
  return v;
}

using CrcKernel = void (*)(const EncodeCrcArgs);
struct CrcPick {
  CrcKernel k;
  int threads;
  const char* base;  // kernel name (rocprofv3 form: base<K, P, MATRIX, threads, G, sched>)
  int g;
  int sched;  // -1: row-serial kernel (no G / SCHED arguments)
};

template <class MATRIX> constexpr const char* kMatrixName = "";
template <int K, int P> constexpr const char* kMatrixName<gf::EncodeMatrix<K, P>> = "hrs::gf::EncodeMatrix";
template <int K, int P> constexpr const char* kMatrixName<gf::CauchyMatrix<K, P>> = "hrs::gf::CauchyMatrix";

template <int K, int P, class MATRIX>
CrcPick pick_kernel(bool narrow) {
  constexpr const char* kg = "encode_crc_grouped_kernel";
  if (fused_variant() == 1) return {encode_crc_kernel<K, P, MATRIX, kFusedThreads>, kFusedThreads, "encode_crc_kernel", 0, -1};
  const int g = fused_group() ? fused_group() : kFusedGroup<K>;
  if (fused_variant() == 3 && narrow && g == kFusedGroup<K>) {
    constexpr int G = kFusedGroup<K> == 4 ? (K > 4 ? 4 : K) : 2;
    return {encode_crc_grouped_kernel<K, P, MATRIX, kFusedNarrowThreads, G, true>, kFusedNarrowThreads, kg, G, 1};
  }
  if (fused_variant() == 3) {  // factored XOR network (xor_sched.hpp has G = 2, min(4, K), K)
    if (g == 4)
      return {encode_crc_grouped_kernel<K, P, MATRIX, kFusedThreads, (K > 4 ? 4 : K), true>, kFusedThreads, kg,
              (K > 4 ? 4 : K), 1};
    return {encode_crc_grouped_kernel<K, P, MATRIX, kFusedThreads, 2, true>, kFusedThreads, kg, 2, 1};
  }
  if (g == 4) return {encode_crc_grouped_kernel<K, P, MATRIX, kFusedThreads, 4, false>, kFusedThreads, kg, 4, 0};
  if (g == 1) return {encode_crc_grouped_kernel<K, P, MATRIX, kFusedThreads, 1, false>, kFusedThreads, kg, 1, 0};
  return {encode_crc_grouped_kernel<K, P, MATRIX, kFusedThreads, 2, false>, kFusedThreads, kg, 2, 0};
}

template <int K, int P, class MATRIX>
hipError_t launch_one(const EncodeCrcArgs& a, int cus, hipStream_t s) {
  const size_t shm = static_cast<size_t>(kCrcLdsWordsA) * 4;
  const uint64_t ntasks = a.nstripes * a.nwin;
  // zero-copy launches only (a GridCap is set): device-resident jobs keep the
  // 16 waves per CU that hide HBM latency
  const uint64_t room = capped_grid(static_cast<uint64_t>(cus));  // blocks the grid may have
  const bool narrow = t_grid_cap != 0 && fused_narrow_on() &&
                      (ntasks + kFusedThreads / 64 - 1) / (kFusedThreads / 64) < room;
  const CrcPick k = pick_kernel<K, P, MATRIX>(narrow);
  const std::string mat = std::string(kMatrixName<MATRIX>) + "<" + std::to_string(K) + ", " + std::to_string(P) + ">";
  if (k.sched < 0)
    note_kernel_t(k.base, K, P, mat.c_str(), k.threads);
  else
    note_kernel_t(k.base, K, P, mat.c_str(), k.threads, k.g, k.sched != 0);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k.k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     static_cast<int>(shm));
  if (e != hipSuccess) return e;
  const uint64_t per_block = k.threads / 64;
  uint64_t g = (ntasks + per_block - 1) / per_block;
  if (g > static_cast<uint64_t>(cus)) g = cus;
  g = capped_grid(g);  // zero-copy calls cap it (hrs::GridCap)
  hipLaunchKernelGGL(k.k, dim3(static_cast<unsigned>(g)), dim3(k.threads), shm, s, with_order(a, kOrderFusedEncode));
  return hipGetLastError();
}

}  // namespace

hipError_t launch_encode_crc(int family, int k, int p, const EncodeCrcArgs& a, int cus, hipStream_t s,
                             bool* handled) {
  *handled = true;
  if (family == kStaticCauchy) {
    if (k == 10 && p == 4) return launch_one<10, 4, gf::CauchyMatrix<10, 4>>(a, cus, s);
    if (k == 6 && p == 3) return launch_one<6, 3, gf::CauchyMatrix<6, 3>>(a, cus, s);
  } else {
    if (k == 10 && p == 4) return launch_one<10, 4, gf::EncodeMatrix<10, 4>>(a, cus, s);
    if (k == 6 && p == 3) return launch_one<6, 3, gf::EncodeMatrix<6, 3>>(a, cus, s);
    if (k == 3 && p == 2) return launch_one<3, 2, gf::EncodeMatrix<3, 2>>(a, cus, s);
    if (k == 12 && p == 4) return launch_one<12, 4, gf::EncodeMatrix<12, 4>>(a, cus, s);
  }
  *handled = false;
  return hipSuccess;
}

}  // namespace hrs
