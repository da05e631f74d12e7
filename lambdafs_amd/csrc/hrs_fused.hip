// gfx950 fused encode + CRC-32: the parity of every stripe and the
// java.util.zip.CRC32 of every source and parity cell in ONE pass over HBM —
// what Encoder.encodeStripe does per bufSize round with computeBlockChecksum
// (sourceChecksums over readBufs before encodeBulk, parityChecksums over
// writeBufs after it; Encoder.java:408-450). Run as two passes (encode, then
// hrs_crc32_dev) the cells are read twice; fused, the CRC consumes the words
// the encode already holds in registers.
//
// Decomposition: one wave per (stripe, 32 KiB window). The window is walked
// as 16 sub-windows of 2 KiB — exactly the encode kernels' task (lane l holds
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

#include "hrs_device.hpp"

namespace hrs {
namespace {

constexpr int kSubWindows = kCrcWindow / kWindowBytes;  // 16

template <int K, int P, class MATRIX, int THREADS>
__global__ void __launch_bounds__(THREADS) encode_crc_kernel(const EncodeCrcArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < kCrcLdsWordsA; i += THREADS) lds[i] = a.tables[i];
  __syncthreads();
  constexpr int N = K + P;
  const int lane = threadIdx.x & 63;
  const SliceTab slices = slice_tab(lane);
  const uint32_t* zchunk = lds + kCrcSliceWords;
  const uint32_t* tree = zchunk + 1024;
  const uint64_t ntasks = a.nstripes * a.nwin;
  const uint32_t nwaves = gridDim.x * (THREADS / 64);
  for (uint64_t t = wave_id_in_grid(); t < ntasks; t += nwaves) {
    const uint64_t stripe = t / a.nwin;
    const uint64_t w = t - stripe * a.nwin;
    const uint64_t in_base = stripe * a.in_stride + w * kCrcWindow;
    const uint64_t out_base = stripe * a.out_stride + w * kCrcWindow;
    uint32_t crc[N];
#pragma unroll
    for (int r = 0; r < N; ++r) crc[r] = 0u;  // Z(0) = 0: the first piece needs no special case
#pragma unroll 1
    for (int sub = 0; sub < kSubWindows; ++sub) {
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

// Second form (the default; HRS_FUSED=1 selects the one above for A/B):
// the row-serial kernel above waits on every row's load before touching it
// (one 2 KiB row in flight per wave: the ISA shows a vmcnt(0) per row), so
// HBM latency, not bandwidth, set its pace. Here a wave loads ALL K data rows
// of a sub-window at once (K x 8 VGPRs), CRCs them as 2K independent chains
// advanced in lockstep (8K LDS lookups in flight per slicing step), slices
// them, and then builds each parity row in turn straight from the planes
// (acc[q] = XOR of the planes G selects, no cross-row pending state), storing
// and CRC'ing it before the next. The next sub-window's K loads are issued as
// soon as the last parity's planes are built, so they overlap that row's
// un-slice, store and CRC chains, and the lane-tree / Horner updates.
#ifndef HRS_CRC_GROUP
#define HRS_CRC_GROUP 2
#endif
constexpr int kCrcGroup = HRS_CRC_GROUP;  // rows whose CRC chains advance together

template <int K, int P, class MATRIX>
__device__ __forceinline__ void parity_planes(int o, const uint32_t (&x)[K][8], uint32_t (&acc)[8]) {
  constexpr StaticPlan<K, P, MATRIX> plan{};
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    uint32_t v = 0u, pend = 0u;
    bool first = true, has = false;
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if ((plan.mask[o][r][q] >> i) & 1) {
          if (first) {
            v = x[r][i];
            first = false;
          } else if (has) {
            v = xor3(v, pend, x[r][i]);
            has = false;
          } else {
            pend = x[r][i];
            has = true;
          }
        }
    acc[q] = has ? v ^ pend : v;
  }
}

// The scheduler otherwise interleaves the phases (and the two sub-windows of
// the unrolled pair) for ILP until the live ranges spill; a scheduling
// barrier between phases keeps each phase's temporaries short-lived.
#ifndef HRS_NO_PHASE_FENCE
#define HRS_PHASE_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define HRS_PHASE_FENCE() ((void)0)
#endif

// One sub-window of the second form: source CRCs of the K rows in x
// (natural byte order), slice them, then each parity row from the planes:
// un-slice, store, CRC. x is consumed (left sliced).
template <int K, int P, class MATRIX>
__device__ __forceinline__ void encode_crc_sub(uint32_t (&x)[K][8], uint32_t (&crc)[K + P], const SliceTab& slices,
                                               const uint32_t* zchunk, const EncodeCrcArgs& a, uint64_t out_base,
                                               int lane) {
#pragma unroll
  for (int r0 = 0; r0 < K; r0 += kCrcGroup) {
    constexpr int G = kCrcGroup;
    if (r0 + G <= K) {
      uint32_t c0[G], c1[G];
      rows_piece_crcs<G>(slices, *reinterpret_cast<const uint32_t(*)[G][8]>(&x[r0][0]), c0, c1);
#pragma unroll
      for (int g = 0; g < G; ++g) crc[r0 + g] = zmul(zchunk, zmul(zchunk, crc[r0 + g]) ^ c0[g]) ^ c1[g];
    } else {  // the last K % G rows
#pragma unroll
      for (int r = r0; r < K; ++r) {
        uint32_t d0[1], d1[1];
        rows_piece_crcs<1>(slices, *reinterpret_cast<const uint32_t(*)[1][8]>(&x[r][0]), d0, d1);
        crc[r] = zmul(zchunk, zmul(zchunk, crc[r]) ^ d0[0]) ^ d1[0];
      }
    }
#pragma unroll
    for (int r = r0; r < r0 + G && r < K; ++r) bitslice(x[r]);
    HRS_PHASE_FENCE();
  }
#pragma unroll
  for (int o = 0; o < P; ++o) {
    HRS_PHASE_FENCE();
    uint32_t acc[1][8];
    parity_planes<K, P, MATRIX>(o, x, acc[0]);
    bitslice(acc[0]);
    store_row(a.out[o] + out_base, lane, acc[0]);
    uint32_t p0[1], p1[1];
    rows_piece_crcs<1>(slices, acc, p0, p1);
    crc[K + o] = zmul(zchunk, zmul(zchunk, crc[K + o]) ^ p0[0]) ^ p1[0];
  }
}

// 512 threads (8 waves, 2 per SIMD: 256 VGPRs each) so that a wave can hold
// TWO sub-windows of rows: while it works on one, the next one's K loads are
// in flight (software pipelining over the 16 sub-windows of its window).
template <int K, int P, class MATRIX, int THREADS>
__global__ void __launch_bounds__(THREADS) encode_crc2_kernel(const EncodeCrcArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < kCrcLdsWordsA; i += THREADS) lds[i] = a.tables[i];
  __syncthreads();
  constexpr int N = K + P;
  const int lane = threadIdx.x & 63;
  const SliceTab slices = slice_tab(lane);
  const uint32_t* zchunk = lds + kCrcSliceWords;
  const uint32_t* tree = zchunk + 1024;
  const uint64_t ntasks = a.nstripes * a.nwin;
  const uint32_t nwaves = gridDim.x * (THREADS / 64);
  for (uint64_t t = wave_id_in_grid(); t < ntasks; t += nwaves) {
    const uint64_t stripe = t / a.nwin;
    const uint64_t w = t - stripe * a.nwin;
    const uint64_t in_base = stripe * a.in_stride + w * kCrcWindow;
    const uint64_t out_base = stripe * a.out_stride + w * kCrcWindow;
    uint32_t crc[N];
#pragma unroll
    for (int r = 0; r < N; ++r) crc[r] = 0u;
    uint32_t xa[K][8], xb[K][8];
#pragma unroll
    for (int r = 0; r < K; ++r) load_row(a.in[r] + in_base, lane, xa[r]);
#pragma unroll 1
    for (int sub = 0; sub < kSubWindows; sub += 2) {
      const uint64_t off = static_cast<uint64_t>(sub) * kWindowBytes;
#pragma unroll
      for (int r = 0; r < K; ++r) load_row(a.in[r] + in_base + off + kWindowBytes, lane, xb[r]);
      encode_crc_sub<K, P, MATRIX>(xa, crc, slices, zchunk, a, out_base + off, lane);
      if (sub + 2 < kSubWindows) {
#pragma unroll
        for (int r = 0; r < K; ++r) load_row(a.in[r] + in_base + off + 2 * kWindowBytes, lane, xa[r]);
      }
      encode_crc_sub<K, P, MATRIX>(xb, crc, slices, zchunk, a, out_base + off + kWindowBytes, lane);
    }
#pragma unroll
    for (int r = 0; r < N; ++r) {
      const uint32_t c = lane_tree(tree, crc[r]);
      if (lane == 0) a.raw[(stripe * N + r) * a.nwin + w] = c;
    }
  }
}

// Third form: the row-serial walk of the first (1024 threads, 4 waves per
// SIMD, the CRC of row r overlapping other waves' work), but each wave keeps
// D rows of loads in flight ahead of the row it is on — a ring of D + 1 row
// buffers over the flat sequence (sub-window, row), crossing into the next
// sub-window — instead of waiting on every row's load. The registers come
// from dropping the first form's cross-row pending planes: a row's selected
// planes are paired within the row (xor3), an odd one XORs alone.
// D + 1 divides K, so each buffer index is a compile-time constant.
// Ring sizes instantiated: every B <= 4 that divides K (B = 5 at K = 10 left
// the ring in scratch memory); HRS_FUSED_RING picks
// one for A/B runs (default: kDefaultRing, or the largest divisor below it).
constexpr int kDefaultRing = 2;

template <int K, int P, class MATRIX>
__device__ __forceinline__ void encode_row_acc_local(int r, const uint32_t (&w)[8], uint32_t (&acc)[P][8]) {
  constexpr StaticPlan<K, P, MATRIX> plan{};
#pragma unroll
  for (int o = 0; o < P; ++o)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      uint32_t pend = 0u;
      bool has = false;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if ((plan.mask[o][r][q] >> i) & 1) {
          if (has) {
            acc[o][q] = xor3(acc[o][q], pend, w[i]);
            has = false;
          } else {
            pend = w[i];
            has = true;
          }
        }
      if (has) acc[o][q] ^= pend;
    }
}

template <int K, int P, class MATRIX, int THREADS, int B>
__global__ void __launch_bounds__(THREADS) encode_crc3_kernel(const EncodeCrcArgs a) {
  static_assert(K % B == 0, "ring size must divide K");
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < kCrcLdsWordsA; i += THREADS) lds[i] = a.tables[i];
  __syncthreads();
  constexpr int N = K + P;
  // B row buffers: B - 1 loads ahead
  const int lane = threadIdx.x & 63;
  const uint32_t loff = static_cast<uint32_t>(lane) * 16u;
  const SliceTab slices = slice_tab(lane);
  const uint32_t* zchunk = lds + kCrcSliceWords;
  const uint32_t* tree = zchunk + 1024;
  const uint64_t ntasks = a.nstripes * a.nwin;
  const uint32_t nwaves = gridDim.x * (THREADS / 64);
  for (uint64_t t = wave_id_in_grid(); t < ntasks; t += nwaves) {
    const uint64_t stripe = t / a.nwin;
    const uint64_t w = t - stripe * a.nwin;
    const uint64_t in_base = stripe * a.in_stride + w * kCrcWindow;
    const uint64_t out_base = stripe * a.out_stride + w * kCrcWindow;
    uint32_t crc[N];
#pragma unroll
    for (int r = 0; r < N; ++r) crc[r] = 0u;
    uint32_t ring[B][8];
#pragma unroll
    for (int r = 0; r < B - 1; ++r) load_row_u(a.in[r] + in_base, loff, ring[r]);
#pragma unroll 1
    for (int sub = 0; sub < kSubWindows; ++sub) {
      const uint64_t off = static_cast<uint64_t>(sub) * kWindowBytes;
      uint32_t acc[P][8];
#pragma unroll
      for (int o = 0; o < P; ++o)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
#pragma unroll
      for (int r = 0; r < K; ++r) {
        // keep B - 1 rows in flight: row r + B - 1 (possibly of the next sub-window)
        HRS_PHASE_FENCE();
        const int ahead = r + B - 1;
        if (ahead < K) {
          load_row_u(a.in[ahead] + in_base + off, loff, ring[ahead % B]);
        } else if (sub + 1 < kSubWindows) {
          load_row_u(a.in[ahead - K] + in_base + off + kWindowBytes, loff, ring[ahead % B]);
        }
        uint32_t(&x)[8] = ring[r % B];
        const uint32_t c0 = piece_crc(slices, x[0], x[1], x[2], x[3]);
        const uint32_t c1 = piece_crc(slices, x[4], x[5], x[6], x[7]);
        crc[r] = zmul(zchunk, zmul(zchunk, crc[r]) ^ c0) ^ c1;
        // materialize the running CRC here: otherwise its final XORs sink to
        // the loop's end and every row's table words stay live (spills)
        __asm__ volatile("" : "+v"(crc[r]));
        bitslice(x);
        encode_row_acc_local<K, P, MATRIX>(r, x, acc);
      }
      HRS_PHASE_FENCE();
#pragma unroll
      for (int o = 0; o < P; ++o) {
        bitslice(acc[o]);
        store_row_u(a.out[o] + out_base + off, loff, acc[o]);
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

int fused_variant() {  // HRS_FUSED=1|2|3 (A/B runs); default 3
  static const int v = [] {
    const char* e = getenv("HRS_FUSED");
    const int x = e ? atoi(e) : 0;
    return (x >= 1 && x <= 3) ? x : 3;
  }();
  return v;
}


// One 1024-thread block per CU (16 waves share the 156 KiB table image; the
// kernel is VALU-bound, so every wave slot counts): 3.3-3.5 ms for 1,024
// RS(10,4) 1 MiB stripes vs 4.2-4.3 ms with 512 threads, and prefetching
// the next row gained < 5% at the cost of VGPR spills (tools/bench_encode_crc.py).
constexpr int kFusedThreads = 1024;
#ifndef HRS_FUSED2_THREADS
#define HRS_FUSED2_THREADS 512
#endif
constexpr int kFused2Threads = HRS_FUSED2_THREADS;

int fused_ring() {
  static const int v = [] {
    const char* e = getenv("HRS_FUSED_RING");
    const int x = e ? atoi(e) : 0;
    return (x >= 1 && x <= 4) ? x : kDefaultRing;
  }();
  return v;
}

using CrcKernel = void (*)(const EncodeCrcArgs);

template <int K, int P, class MATRIX, int B>
CrcKernel crc3_for() {
  return encode_crc3_kernel<K, P, MATRIX, kFusedThreads, B>;
}

// The instantiated ring size closest to (not above) the requested one.
template <int K, int P, class MATRIX>
CrcKernel pick_crc3(int want) {
  if (want >= 4 && K % 4 == 0) return crc3_for<K, P, MATRIX, (K % 4 == 0 ? 4 : 1)>();
  if (want >= 3 && K % 3 == 0) return crc3_for<K, P, MATRIX, (K % 3 == 0 ? 3 : 1)>();
  if (want >= 2 && K % 2 == 0) return crc3_for<K, P, MATRIX, (K % 2 == 0 ? 2 : 1)>();
  return crc3_for<K, P, MATRIX, 1>();
}

template <int K, int P, class MATRIX>
hipError_t launch_one(const EncodeCrcArgs& a, int cus, hipStream_t s) {
  const size_t shm = static_cast<size_t>(kCrcLdsWordsA) * 4;
  const uint64_t ntasks = a.nstripes * a.nwin;
  const int v = fused_variant();
  const int threads = v == 2 ? kFused2Threads : kFusedThreads;
  const CrcKernel k = v == 1   ? encode_crc_kernel<K, P, MATRIX, kFusedThreads>
                      : v == 2 ? encode_crc2_kernel<K, P, MATRIX, kFused2Threads>
                               : pick_crc3<K, P, MATRIX>(fused_ring());
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     static_cast<int>(shm));
  if (e != hipSuccess) return e;
  const uint64_t per_block = threads / 64;
  uint64_t g = (ntasks + per_block - 1) / per_block;
  if (g > static_cast<uint64_t>(cus)) g = cus;
  if (g == 0) g = 1;
  hipLaunchKernelGGL(k, dim3(static_cast<unsigned>(g)), dim3(threads), shm, s, a);
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
