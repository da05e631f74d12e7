// gfx950 kernels of the Reed-Solomon engine.
//
// The reference computes parity with a bulk polynomial remainder
// (GaloisField.java:326-338, driven by ReedSolomonCode.encodeBulk,
// ReedSolomonCode.java:103-125) and repairs with per-byte syndromes plus a
// Vandermonde solve (ReedSolomonCode.java:127-166, 191-211). Both are
// GF(2^8)-linear in the stripe bytes, so every kernel here evaluates
//     out_o[col] = XOR_i  M[o][i] * in_i[col]        (GF(2^8) products)
// for every byte column `col` of every stripe, with M = the encode matrix G
// or a decode matrix D built on the host (hrs_api.cpp).
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
#include <hip/hip_runtime.h>

#include <atomic>

#include <cstdlib>

#include "hrs_device.hpp"

namespace hrs {
namespace {

// ---------------------------------------------------------------- helpers

// bit-slice transform, plane arithmetic and window row accesses: hrs_device.hpp
__constant__ gf::Tables d_tables = gf::make_tables();

// ------------------------------------------------- static encode kernels

template <int K, int P, class MATRIX>
__device__ __forceinline__ void encode_static_body(const RowArgs& a) {
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  for (uint64_t t = wave_id_in_grid(); t < a.ntasks; t += nwaves) {
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

// ------------------------------------------ runtime-matrix bit-sliced kernel

// NINB >= nin rows of the window are all loaded before any math (one
// 20 KiB-class burst per wave, like the static kernel), so a wave keeps
// nin x 2 KiB in flight; coefficients are wave-uniform kernel arguments.
// Bit loop unrolled (xtime is then a free relabel of the planes) unless the
// body would outgrow the instruction cache: unrolled, bitsliced<4,12> is
// 28 KiB of branchy code and ran 40% slower than rolled.
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

template <int NOUT, int NINB>
__global__ void __launch_bounds__(kBlockThreads) bitsliced_kernel(const RowArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  for (uint64_t t = wave_id_in_grid(); t < a.ntasks; t += nwaves) {
    int nin = a.nin;  // opaque per task: the r < nin predicates are not hoisted (they would spill)
    asm volatile("" : "+s"(nin));
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    const uint64_t in_base = stripe * a.in_stride + off;
    uint32_t rows[NINB][8];
#pragma unroll
    for (int r = 0; r < NINB; ++r)
      if (r < nin) load_row(a.in[r] + in_base, lane, rows[r]);
    uint32_t acc[NOUT][8];
    if (a.accumulate) {
#pragma unroll
      for (int o = 0; o < NOUT; ++o) {
        load_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
        bitslice(acc[o]);
      }
    } else {
#pragma unroll
      for (int o = 0; o < NOUT; ++o)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
    }
#pragma unroll
    for (int r = 0; r < NINB; ++r) {
      if (r < nin) {
        bitslice(rows[r]);
        // one wave-uniform 64-bit word per input (byte o = coefficient of
        // output o), split in halves; the empty asm keeps the per-(o, b)
        // tests from being hoisted out of the task loop (they would spill).
        uint32_t cw[2] = {static_cast<uint32_t>(a.cw[r]), static_cast<uint32_t>(a.cw[r] >> 32)};
        asm volatile("" : "+s"(cw[0]));
        if constexpr (NOUT > 4) asm volatile("" : "+s"(cw[1]));  // outputs 4..7 only
        // acc[o] ^= sum over set bits b of coef[o][r]: alpha^b * row
        if constexpr (BitLoop<NOUT, NINB>::kRolled) {
#pragma unroll 1
          for (int b = 0; b < 8; ++b) {
            mul_acc_row<NOUT, NINB>(acc, rows[r], cw, b);
            xtime(rows[r]);
          }
        } else {
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            mul_acc_row<NOUT, NINB>(acc, rows[r], cw, b);
            if (b < 7) xtime(rows[r]);
          }
        }
      }
    }
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      bitslice(acc[o]);
      store_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
    }
  }
}

// Software-pipelined form of bitsliced_kernel for narrow outputs: two
// register sets of NINB rows, the next task's rows are loaded before the
// current task's math, so a wave keeps a window in flight while it computes
// (the plain kernel's loads sit idle during its ~1,000 VALU of slicing and
// multiplying). 2*NINB*8 + 8*NOUT VGPRs: NOUT <= 2, NINB <= 12 at 2 waves/SIMD.
template <int NOUT, int NINB>
__device__ __forceinline__ void load_task(const RowArgs& a, uint64_t t, int nin, int lane,
                                          uint32_t (&rows)[NINB][8]) {
  const uint64_t stripe = t / a.nwin;
  const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
  const uint64_t in_base = stripe * a.in_stride + off;
#pragma unroll
  for (int r = 0; r < NINB; ++r)
    if (r < nin) load_row(a.in[r] + in_base, lane, rows[r]);
}

template <int NOUT, int NINB>
__device__ __forceinline__ void apply_task(const RowArgs& a, uint64_t t, int nin, int lane,
                                           uint32_t (&rows)[NINB][8]) {
  const uint64_t stripe = t / a.nwin;
  const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
  uint32_t acc[NOUT][8];
  if (a.accumulate) {
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      load_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
      bitslice(acc[o]);
    }
  } else {
#pragma unroll
    for (int o = 0; o < NOUT; ++o)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
  }
#pragma unroll
  for (int r = 0; r < NINB; ++r) {
    if (r < nin) {
      bitslice(rows[r]);
      uint32_t cw[2] = {static_cast<uint32_t>(a.cw[r]), static_cast<uint32_t>(a.cw[r] >> 32)};
      asm volatile("" : "+s"(cw[0]));
        if constexpr (NOUT > 4) asm volatile("" : "+s"(cw[1]));  // outputs 4..7 only
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        mul_acc_row<NOUT, NINB>(acc, rows[r], cw, b);
        if (b < 7) xtime(rows[r]);
      }
    }
  }
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    bitslice(acc[o]);
    store_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
  }
}

template <int NOUT, int NINB>
__global__ void __launch_bounds__(kBlockThreads) bitsliced_pipe_kernel(const RowArgs a) {
  static_assert(!BitLoop<NOUT, NINB>::kRolled, "pipelined kernel takes the unrolled shapes only");
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  int nin = a.nin;
  asm volatile("" : "+s"(nin));
  uint64_t t = wave_id_in_grid();
  if (t >= a.ntasks) return;
  uint32_t ra[NINB][8], rb[NINB][8];
  load_task<NOUT, NINB>(a, t, nin, lane, ra);
  for (;;) {  // every wave leaves once its next task index passes ntasks
    const uint64_t t1 = t + nwaves;
    if (t1 < a.ntasks) load_task<NOUT, NINB>(a, t1, nin, lane, rb);
    apply_task<NOUT, NINB>(a, t, nin, lane, ra);
    if (t1 >= a.ntasks) break;
    const uint64_t t2 = t1 + nwaves;
    if (t2 < a.ntasks) load_task<NOUT, NINB>(a, t2, nin, lane, ra);
    apply_task<NOUT, NINB>(a, t1, nin, lane, rb);
    if (t2 >= a.ntasks) break;
    t = t2;
  }
}

// ------------------------------------------------------------- XOR kernel

// out[0] = XOR of the nin input rows (XOR code, XORCode.java:99-145; also any
// single-output matrix of ones). No bit-slicing: three rows per v_bitop3.
template <int NINB>
__global__ void __launch_bounds__(kBlockThreads) xor_kernel(const RowArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  const int nin = a.nin;
  for (uint64_t t = wave_id_in_grid(); t < a.ntasks; t += nwaves) {
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

// ------------------------------- heterogeneous batches (one pattern per stripe)

// Plans and pattern indices are read through the constant address space so
// the per-task reads are scalar loads (s_load), not vector memory traffic.
typedef const __attribute__((address_space(4))) BatchPlan* ConstPlanPtr;
typedef const __attribute__((address_space(4))) int32_t* ConstIntPtr;

// Same arithmetic as bitsliced_kernel; the wave reads its stripe's plan
// (inputs, coefficients, output count) at the start of each task.
// PATV: lane l of the wave loads the pattern index of the wave's task
// k + l (k = 0, 64, ...) in one vector load; each task then takes its index
// with a readlane instead of a scalar load that waits on HBM before any of
// the task's row loads can issue (the stripes of consecutive tasks differ).
template <int NOUT, int NINB, bool PATV>
__global__ void __launch_bounds__(kBlockThreads) batch_bitsliced_kernel(const BatchArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  const ConstPlanPtr plans = (ConstPlanPtr)a.plans;
  const ConstIntPtr pat = (ConstIntPtr)a.pat;
  int patv = 0;
  uint32_t k = 0;
  for (uint64_t t = wave_id_in_grid(); t < a.ntasks; t += nwaves, ++k) {
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    int pidx;
    if constexpr (PATV) {
      if ((k & 63u) == 0) {
        const uint64_t tl = t + static_cast<uint64_t>(lane) * nwaves;
        patv = tl < a.ntasks ? a.pat[tl / a.nwin] : 0;
      }
      pidx = __builtin_amdgcn_readlane(patv, static_cast<int>(k & 63u));
    } else {
      pidx = pat[stripe];
    }
    const ConstPlanPtr pl = plans + pidx;
    const int nin = pl->nin;
    const int nout = pl->nout;
    const uint8_t* sb = a.base + stripe * a.stripe_stride + off;
    uint32_t rows[NINB][8];
#pragma unroll
    for (int r = 0; r < NINB; ++r)
      if (r < nin) load_row(sb + static_cast<uint64_t>(pl->loc[r]) * a.row_stride, lane, rows[r]);
    uint32_t acc[NOUT][8];
#pragma unroll
    for (int o = 0; o < NOUT; ++o)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[o][q] = 0u;
#pragma unroll
    for (int r = 0; r < NINB; ++r) {
      if (r < nin) {
        bitslice(rows[r]);
        const uint64_t w = pl->cw[r];
        uint32_t cw[2] = {static_cast<uint32_t>(w), static_cast<uint32_t>(w >> 32)};
        asm volatile("" : "+s"(cw[0]));
        if constexpr (NOUT > 4) asm volatile("" : "+s"(cw[1]));  // outputs 4..7 only
        if constexpr (BitLoop<NOUT, NINB>::kRolled) {
#pragma unroll 1
          for (int b = 0; b < 8; ++b) {
            mul_acc_row<NOUT, NINB>(acc, rows[r], cw, b);
            xtime(rows[r]);
          }
        } else {
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            mul_acc_row<NOUT, NINB>(acc, rows[r], cw, b);
            if (b < 7) xtime(rows[r]);
          }
        }
      }
    }
    uint8_t* ob = a.out + stripe * a.out_stripe_stride + off;
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      if (o < nout) {
        bitslice(acc[o]);
        store_row(ob + static_cast<uint64_t>(o) * a.out_row_stride, lane, acc[o]);
      }
    }
  }
}

// Byte columns [col0, len) of every stripe (tails, unaligned batches).
__global__ void __launch_bounds__(kBlockThreads) batch_bytewise_kernel(const BatchArgs a) {
  __shared__ uint8_t s_exp[512];
  __shared__ uint8_t s_log[256];
  for (int i = threadIdx.x; i < 512; i += blockDim.x) s_exp[i] = d_tables.exp[i];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_log[i] = d_tables.log[i];
  __syncthreads();
  const uint64_t ncol = a.len - a.col0;
  const uint64_t nthreads = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t idx = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; idx < a.ntasks;
       idx += nthreads) {
    const uint64_t stripe = idx / ncol;
    const uint64_t col = a.col0 + (idx - stripe * ncol);
    const BatchPlan& pl = a.plans[a.pat[stripe]];
    const uint8_t* sb = a.base + stripe * a.stripe_stride + col;
    uint8_t acc[kMaxOut] = {};
    for (int r = 0; r < pl.nin; ++r) {
      const uint8_t x = sb[static_cast<uint64_t>(pl.loc[r]) * a.row_stride];
      if (x == 0) continue;
      const int lx = s_log[x];
      const uint64_t w = pl.cw[r];
#pragma unroll
      for (int o = 0; o < kMaxOut; ++o) {
        const uint8_t c = static_cast<uint8_t>(w >> (8 * o));
        if (c != 0) acc[o] ^= s_exp[lx + s_log[c]];
      }
    }
    uint8_t* ob = a.out + stripe * a.out_stripe_stride + col;
    for (int o = 0; o < pl.nout; ++o) ob[static_cast<uint64_t>(o) * a.out_row_stride] = acc[o];
  }
}

// ------------------------------------------------------------ launching

// CU count per device, cached; handles on several host threads may race to
// fill it (same value), hence the relaxed atomics.
int device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  static std::atomic<int> cus_of[64];
  if (dev < 0 || dev >= 64) return 256;
  int cus = cus_of[dev].load(std::memory_order_relaxed);
  if (cus == 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cus_of[dev].store(cus, std::memory_order_relaxed);
  }
  return cus;
}

// Streaming kernels: a fixed number of resident blocks per CU, grid-striding
// over the tasks. 2 x 256-thread blocks per CU (8 waves, each with a whole
// window's rows in flight) measured fastest for both the static and the
// runtime kernels (tools/kernel_lab.hip sweep, 256..1024 blocks); override
// with HRS_BLOCKS_PER_CU for experiments.
// VALU-bound shapes (the rolled bit loop: 3-4 erasure repairs, wide
// matrices) take 3 blocks per CU: the extra wave per SIMD hides more of the
// math (RS(10,4) 4-erasure decode +13%, profiles/r01/pipe/).
int blocks_per_cu(int dflt = 2) {
  static int v = [] {
    const char* e = getenv("HRS_BLOCKS_PER_CU");
    int x = e ? atoi(e) : 0;
    return (x >= 1 && x <= 32) ? x : 0;
  }();
  return v ? v : dflt;
}

unsigned stream_grid(uint64_t ntasks, int per_cu = 2) {
  const uint64_t want = static_cast<uint64_t>(blocks_per_cu(per_cu)) * device_cus();
  const uint64_t needed = (ntasks + kWavesPerBlock - 1) / kWavesPerBlock;
  uint64_t g = needed < want ? needed : want;
  return static_cast<unsigned>(g == 0 ? 1 : g);
}

template <typename Kernel>
unsigned grid_for(Kernel kernel, uint64_t work_items_per_block, uint64_t ntasks) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlockThreads, 0) != hipSuccess ||
      per_cu <= 0)
    per_cu = 2;
  const uint64_t resident = static_cast<uint64_t>(per_cu) * device_cus();
  const uint64_t needed = (ntasks + work_items_per_block - 1) / work_items_per_block;
  uint64_t g = needed < resident ? needed : resident;
  if (g == 0) g = 1;
  return static_cast<unsigned>(g);
}

// Software-pipelined runtime kernel for the unrolled shapes that fit (the 1-
// to 3-erasure repairs: RS(10,4) 1-erasure decode +3-10%, 2-3 erasures
// neutral); HRS_PIPE=0 selects the plain kernel for A/B runs. The same
// pipelining of the static encode (-1%) and of the heterogeneous batch
// kernel (-2%) measured slower and is not used (profiles/r01/pipe/ab2).
// Unrolled shapes whose two row sets + accumulators fit 2 waves/SIMD.
template <int NOUT, int NINB>
constexpr bool kPipeFits = !BitLoop<NOUT, NINB>::kRolled && 16 * NINB + 8 * NOUT <= 232;

bool use_pipe() {
  static bool v = [] {
    const char* e = getenv("HRS_PIPE");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <int K, int P>
hipError_t launch_static(const RowArgs& a, hipStream_t s) {
  auto kern = encode_static_kernel<K, P>;
  const unsigned g = stream_grid(a.ntasks);
  hipLaunchKernelGGL(kern, dim3(g), dim3(kBlockThreads), 0, s, a);
  return hipGetLastError();
}

template <int K, int P>
hipError_t launch_cauchy(const RowArgs& a, hipStream_t s) {
  auto kern = encode_cauchy_kernel<K, P>;
  const unsigned g = stream_grid(a.ntasks);
  hipLaunchKernelGGL(kern, dim3(g), dim3(kBlockThreads), 0, s, a);
  return hipGetLastError();
}

template <int NOUT, int NINB>
hipError_t launch_bits_n(const RowArgs& a, hipStream_t s) {
  auto kern = bitsliced_kernel<NOUT, NINB>;
  if constexpr (kPipeFits<NOUT, NINB>)
    if (use_pipe()) kern = bitsliced_pipe_kernel<NOUT, NINB>;
  const int per_cu = BitLoop<NOUT, NINB>::kRolled ? 3 : 2;
  hipLaunchKernelGGL(kern, dim3(stream_grid(a.ntasks, per_cu)), dim3(kBlockThreads), 0, s, a);
  return hipGetLastError();
}

template <int NOUT>
hipError_t launch_bits(const RowArgs& a, hipStream_t s) {
  if (a.nin <= 4) return launch_bits_n<NOUT, 4>(a, s);
  if (a.nin <= 8) return launch_bits_n<NOUT, 8>(a, s);
  if constexpr (NOUT < 6) {  // wider outputs would spill: the host chunks them by 8 inputs
    if (a.nin <= 12) return launch_bits_n<NOUT, 12>(a, s);
    if (a.nin <= 16) return launch_bits_n<NOUT, 16>(a, s);
  }
  return hipErrorInvalidValue;
}

// Batch kernel reads the pattern indices of its next 64 tasks with one
// vector load (PATV) instead of a dependent scalar load per task;
// HRS_BATCH_PATV=0 selects the per-task scalar read for A/B runs. (A
// software-pipelined batch kernel like bitsliced_pipe_kernel measured 3-4%
// slower, profiles/r01/pipe/batch_ab, and is not kept.)
bool use_pat_prefetch() {
  static bool v = [] {
    const char* e = getenv("HRS_BATCH_PATV");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <int NOUT, int NINB>
hipError_t launch_batch_n(const BatchArgs& a, hipStream_t s) {
  auto kern = use_pat_prefetch() ? batch_bitsliced_kernel<NOUT, NINB, true> : batch_bitsliced_kernel<NOUT, NINB, false>;
  const int per_cu = BitLoop<NOUT, NINB>::kRolled ? 3 : 2;
  hipLaunchKernelGGL(kern, dim3(stream_grid(a.ntasks, per_cu)), dim3(kBlockThreads), 0, s, a);
  return hipGetLastError();
}

template <int NOUT>
hipError_t launch_batch_nout(const BatchArgs& a, int max_nin, hipStream_t s) {
  if (max_nin <= 4) return launch_batch_n<NOUT, 4>(a, s);
  if (max_nin <= 8) return launch_batch_n<NOUT, 8>(a, s);
  if constexpr (NOUT < 6) {
    if (max_nin <= 12) return launch_batch_n<NOUT, 12>(a, s);
    if (max_nin <= 16) return launch_batch_n<NOUT, 16>(a, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace

int device_cu_count() { return device_cus(); }

hipError_t launch_batch_bitsliced(const BatchArgs& a, int max_nout, int max_nin, hipStream_t s) {
  switch (max_nout) {
    case 1: return launch_batch_nout<1>(a, max_nin, s);
    case 2: return launch_batch_nout<2>(a, max_nin, s);
    case 3: return launch_batch_nout<3>(a, max_nin, s);
    case 4: return launch_batch_nout<4>(a, max_nin, s);
    case 5: return launch_batch_nout<5>(a, max_nin, s);
    case 6: return launch_batch_nout<6>(a, max_nin, s);
    case 7: return launch_batch_nout<7>(a, max_nin, s);
    case 8: return launch_batch_nout<8>(a, max_nin, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_batch_bytewise(const BatchArgs& a, hipStream_t s) {
  const unsigned g = grid_for(batch_bytewise_kernel, kBlockThreads, a.ntasks);
  hipLaunchKernelGGL(batch_bytewise_kernel, dim3(g), dim3(kBlockThreads), 0, s, a);
  return hipGetLastError();
}

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

hipError_t launch_bitsliced(const RowArgs& a, hipStream_t s) {
  switch (a.nout) {
    case 1: return launch_bits<1>(a, s);
    case 2: return launch_bits<2>(a, s);
    case 3: return launch_bits<3>(a, s);
    case 4: return launch_bits<4>(a, s);
    case 5: return launch_bits<5>(a, s);
    case 6: return launch_bits<6>(a, s);
    case 7: return launch_bits<7>(a, s);
    case 8: return launch_bits<8>(a, s);
    default: return hipErrorInvalidValue;
  }
}

template <int NINB>
hipError_t launch_xor_n(const RowArgs& a, hipStream_t s) {
  auto kern = xor_kernel<NINB>;
  hipLaunchKernelGGL(kern, dim3(stream_grid(a.ntasks)), dim3(kBlockThreads), 0, s, a);
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
  hipLaunchKernelGGL(bytewise_kernel, dim3(g), dim3(kBlockThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace hrs
