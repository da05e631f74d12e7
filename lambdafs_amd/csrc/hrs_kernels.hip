// gfx950 kernels of the Reed-Solomon engine.
//
// The reference computes parity with a bulk polynomial remainder
// (GaloisField.java:326-338, driven by ReedSolomonCode.encodeBulk,
// ReedSolomonCode.java:103-125) and repairs with per-byte syndromes plus a
// Vandermonde solve (ReedSolomonCode.java:127-166, 191-211). Both are
// GF(2^8)-linear in the stripe bytes, so every kernel here evaluates
//     out_o[col] = XOR_i  M[o][i] * in_i[col]        (GF(2^8) products)
// for every byte column `col` of every stripe, with M = the encode matrix G
// or a decode matrix D built on the host (hrs_matrix.cpp).
//
// Design (MI355X_MICROARCH.md: HBM ~6.3 TB/s achievable, VALU 64 lanes x 4
// SIMD x 256 CU): the path is HBM-bound byte streaming, so there is no MFMA
// here. A GF(2^8) multiply-by-constant is an 8x8 bit matrix over GF(2), so
// each lane bit-slices 32 bytes of a row into 8 bit-planes (3 exchange stages,
// 60 VALU ops per 32 B) and then a product becomes plain XORs of planes:
//   - static kernels: the encode matrix is a compile-time constant, each
//     output plane is an unrolled XOR of the input planes its bit matrix
//     selects (~32 XORs per coefficient per 32 B, fused into v_bitop3/xor3);
//   - runtime kernels: per input row the planes are multiplied by alpha
//     (a relabelling plus 3 XORs in the sliced domain) and accumulated into
//     the outputs whose coefficient has that bit set (wave-uniform branches).
// The bit-slice transform is an involution, applied again to the outputs.
//
// This file: the static encode, XOR and byte-granular kernels. The runtime-
// matrix kernels are in hrs_runtime.hip, the heterogeneous repair batches in
// hrs_batch.hip (separate translation units, so the build runs in parallel).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "hrs_device.hpp"
#include "hrs_launch.hpp"

namespace hrs {
namespace {

// ---------------------------------------------------------------- helpers

// bit-slice transform, plane arithmetic and window row accesses: hrs_device.hpp
__constant__ gf::Tables d_tables = gf::make_tables();

// ------------------------------------------------- static encode kernels

template <int K, int P, class MATRIX>
__device__ __forceinline__ void encode_static_body(const RowArgs& a) {
  const int lane = threadIdx.x & 63;
  const WaveTasks wt = wave_tasks(a.ntasks, a.order);
  for (uint32_t j = 0; j < 0xFFFFFFFFu; ++j) {
    const uint64_t t = wt.at(j);
    if (t >= wt.end) break;
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    uint32_t acc[P][8];
    uint32_t pend[P][8];
    bool has[P][8];  // compile-time after unrolling
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
      uint32_t w[8];
      load_row(a.in[r] + stripe * a.in_stride + off, lane, w);
      bitslice(w);
      encode_row_acc<K, P, MATRIX>(r, w, acc, pend, has);
    }
#pragma unroll
    for (int o = 0; o < P; ++o)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (has[o][q]) acc[o][q] ^= pend[o][q];
#pragma unroll
    for (int o = 0; o < P; ++o) {
      bitslice(acc[o]);
      store_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
    }
  }
}

template <int K, int P>
__global__ void __launch_bounds__(kBlockThreads) encode_static_kernel(const RowArgs a) {
  encode_static_body<K, P, gf::EncodeMatrix<K, P>>(a);
}

// nrs: the Cauchy rows of ISA-L gf_gen_cauchy1_matrix (NativeReedSolomonCode)
template <int K, int P>
__global__ void __launch_bounds__(kBlockThreads) encode_cauchy_kernel(const RowArgs a) {
  encode_static_body<K, P, gf::CauchyMatrix<K, P>>(a);
}

// ------------------------------------------------------------- XOR kernel

// out[0] = XOR of the nin input rows (XOR code, XORCode.java:99-145; also any
// single-output matrix of ones). No bit-slicing: three rows per v_bitop3.
template <int NINB>
__global__ void __launch_bounds__(kBlockThreads) xor_kernel(const RowArgs a) {
  const int lane = threadIdx.x & 63;
  const int nin = a.nin;
  const WaveTasks wt = wave_tasks(a.ntasks, a.order);
  for (uint32_t j = 0; j < 0xFFFFFFFFu; ++j) {
    const uint64_t t = wt.at(j);
    if (t >= wt.end) break;
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    const uint64_t in_base = stripe * a.in_stride + off;
    uint32_t rows[NINB][8];
#pragma unroll
    for (int r = 0; r < NINB; ++r)
      if (r < nin) load_row(a.in[r] + in_base, lane, rows[r]);
    uint32_t acc[8];
    if (a.accumulate) {
      load_row(a.out[0] + stripe * a.out_stride + off, lane, acc);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = 0u;
    }
#pragma unroll
    for (int r = 0; r < NINB; r += 2) {
      if (r + 1 < nin) {
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = xor3(acc[q], rows[r][q], rows[r + 1][q]);
      } else if (r < nin) {
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] ^= rows[r][q];
      }
    }
    store_row(a.out[0] + stripe * a.out_stride + off, lane, acc);
  }
}

// --------------------------------------------- byte-granular kernel (any alignment)

// One byte column per lane, log/antilog tables in LDS. Serves rows that are
// not 16-byte aligned; ntasks = nstripes * len here.
__global__ void __launch_bounds__(kBlockThreads) bytewise_kernel(const RowArgs a) {
  __shared__ uint8_t s_exp[512];
  __shared__ uint8_t s_log[256];
  for (int i = threadIdx.x; i < 512; i += blockDim.x) s_exp[i] = d_tables.exp[i];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_log[i] = d_tables.log[i];
  __syncthreads();
  const uint64_t nthreads = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t idx = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; idx < a.ntasks;
       idx += nthreads) {
    const uint64_t stripe = idx / a.len;
    const uint64_t col = idx - stripe * a.len;
    uint8_t acc[kMaxOut];
#pragma unroll
    for (int o = 0; o < kMaxOut; ++o)
      acc[o] = (a.accumulate && o < a.nout) ? a.out[o][stripe * a.out_stride + col] : 0;
    for (int r = 0; r < a.nin; ++r) {
      const uint8_t x = a.in[r][stripe * a.in_stride + col];
      if (x == 0) continue;
      const int lx = s_log[x];
#pragma unroll
      for (int o = 0; o < kMaxOut; ++o) {
        const uint8_t c = static_cast<uint8_t>(a.cw[r] >> (8 * o));
        if (o < a.nout && c != 0) acc[o] ^= s_exp[lx + s_log[c]];
      }
    }
#pragma unroll
    for (int o = 0; o < kMaxOut; ++o)
      if (o < a.nout) a.out[o][stripe * a.out_stride + col] = acc[o];
  }
}

template <int K, int P>
hipError_t launch_static(const RowArgs& a, hipStream_t s) {
  auto kern = encode_static_kernel<K, P>;
  note_kernel_t("encode_static_kernel", K, P);
  const unsigned g = stream_grid(a.ntasks);
  hipLaunchKernelGGL(kern, dim3(g), dim3(kBlockThreads), 0, s, with_order(a, kOrderStaticEncode));
  return hipGetLastError();
}

template <int K, int P>
hipError_t launch_cauchy(const RowArgs& a, hipStream_t s) {
  auto kern = encode_cauchy_kernel<K, P>;
  note_kernel_t("encode_cauchy_kernel", K, P);
  const unsigned g = stream_grid(a.ntasks);
  hipLaunchKernelGGL(kern, dim3(g), dim3(kBlockThreads), 0, s, with_order(a, kOrderStaticEncode));
  return hipGetLastError();
}

}  // namespace

int device_cu_count() { return device_cus(); }

namespace {
thread_local std::string t_last_kernel;
}
void note_kernel(const char* name) { t_last_kernel = name; }
const char* last_kernel() { return t_last_kernel.c_str(); }

hipError_t launch_static_encode(int family, int k, int p, const RowArgs& a, hipStream_t s, bool* handled) {
  *handled = true;
  if (family == kStaticCauchy) {
    if (k == 10 && p == 4) return launch_cauchy<10, 4>(a, s);
    if (k == 6 && p == 3) return launch_cauchy<6, 3>(a, s);
    *handled = false;
    return hipSuccess;
  }
  if (k == 10 && p == 4) return launch_static<10, 4>(a, s);
  if (k == 6 && p == 3) return launch_static<6, 3>(a, s);
  if (k == 3 && p == 2) return launch_static<3, 2>(a, s);
  if (k == 12 && p == 4) return launch_static<12, 4>(a, s);
  *handled = false;
  return hipSuccess;
}

template <int NINB>
hipError_t launch_xor_n(const RowArgs& a, hipStream_t s) {
  auto kern = xor_kernel<NINB>;
  note_kernel_t("xor_kernel", NINB);
  hipLaunchKernelGGL(kern, dim3(stream_grid(a.ntasks)), dim3(kBlockThreads), 0, s, with_order(a, kOrderStaticEncode));
  return hipGetLastError();
}

hipError_t launch_xor(const RowArgs& a, hipStream_t s) {
  if (a.nin <= 4) return launch_xor_n<4>(a, s);
  if (a.nin <= 8) return launch_xor_n<8>(a, s);
  if (a.nin <= 12) return launch_xor_n<12>(a, s);
  if (a.nin <= 16) return launch_xor_n<16>(a, s);
  return hipErrorInvalidValue;
}

hipError_t launch_bytewise(const RowArgs& a, hipStream_t s) {
  const unsigned g = grid_for(bytewise_kernel, kBlockThreads, a.ntasks);
  note_kernel("bytewise_kernel");
  hipLaunchKernelGGL(bytewise_kernel, dim3(g), dim3(kBlockThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace hrs
