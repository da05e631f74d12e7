// Where does the repair's access pattern lose HBM rate? (diagnostic)
// The 1-erasure repair reads 10 rows of a stripe per 2 KiB window and writes
// one (5.2-5.7 TB/s), while a plain read stream reaches 6.6-6.8 TB/s on the
// same box. Each variant below is one wave per 2 KiB window task, 256-thread
// blocks, 2 per CU, grid-stride tasks, nontemporal 16-byte accesses, over
// bench.py's 1,024 x 14 x 1 MiB stripes:
//   g<R>r<W>w      R rows read (the stripe's last R), W rows written (its
//                  first W), as hrs_probe_rows; W = 0 keeps the loads alive
//                  with a data-dependent store that is practically never taken
//   g10r1w_sep     the written row in a separate [S][L] buffer
//   c<R>           the same R x 2 KiB per task read from ONE contiguous run
//                  (task t reads bytes [t * R * 2 KiB, +R * 2 KiB)): gather vs
//                  contiguous at the same bytes per wave
//   p<R>r<W>w_b<B>_P<p>_W<w>  g<R>r<W>w with the chip's reads and writes
//                  separated in time: every wave keeps its outputs in LDS (up
//                  to B windows) and writes them only inside a write window of
//                  w ticks at the end of each p-tick period of the GPU's
//                  100 MHz real-time counter (s_memrealtime, one clock for
//                  every CU), so HBM sees long read-only and write-only phases
//                  instead of a fine read/write mix
// Usage: gather_lab [reps]   (one JSON line per variant, interleaved reps, medians)
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/gather_lab.hip -o tools/gather_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

constexpr uint64_t kL = 1u << 20;
constexpr int kN = 14;
constexpr uint64_t kS = 1024;
constexpr uint64_t kNwin = kL / 2048;

__device__ __forceinline__ uint32_t wave_gid() {
  return __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
}

// R rows read, W written, optional separate output buffer
template <int R, int W, bool SEP>
__global__ void __launch_bounds__(256) gather_kernel(uint8_t* __restrict__ base, uint8_t* __restrict__ out,
                                                     u4* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t ntasks = kS * kNwin;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4;
  u4 acc0 = {0u, 0u, 0u, 0u}, acc1 = acc0;
  for (uint64_t t = wave_gid(); t < ntasks; t += nw) {
    const uint64_t s = t / kNwin;
    const uint64_t off = (t - s * kNwin) * 2048u + lane * 16u;
    uint8_t* sb = base + s * kN * kL + off;
    u4 v[R][2];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u4* p = reinterpret_cast<const u4*>(sb + (kN - R + r) * kL);
      v[r][0] = __builtin_nontemporal_load(p);
      v[r][1] = __builtin_nontemporal_load(p + 64);
    }
    u4 a = {0u, 0u, 0u, 0u}, b = a;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      a ^= v[r][0];
      b ^= v[r][1];
    }
    if constexpr (W == 0) {
      acc0 ^= a;
      acc1 ^= b;
    } else {
#pragma unroll
      for (int o = 0; o < W; ++o) {
        u4* q = SEP ? reinterpret_cast<u4*>(out + s * kL + off) : reinterpret_cast<u4*>(sb + o * kL);
        __builtin_nontemporal_store(a + static_cast<uint32_t>(o), q);
        __builtin_nontemporal_store(b + static_cast<uint32_t>(o), q + 64);
      }
    }
  }
  if constexpr (W == 0) {
    const u4 x = acc0 ^ acc1;
    if ((x[0] ^ x[1] ^ x[2] ^ x[3]) == 0x9E3779B9u && x[0] == 0x7F4A7C15u) sink[threadIdx.x] = x;
  }
}

// R x 2 KiB contiguous per task, read-only
template <int R>
__global__ void __launch_bounds__(256) contig_kernel(const uint8_t* __restrict__ base, u4* __restrict__ sink,
                                                     uint64_t ntasks) {
  const int lane = threadIdx.x & 63;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4;
  u4 acc = {0u, 0u, 0u, 0u};
  for (uint64_t t = wave_gid(); t < ntasks; t += nw) {
    const u4* p = reinterpret_cast<const u4*>(base + t * R * 2048u + lane * 16u);
    u4 v[2 * R];
#pragma unroll
    for (int j = 0; j < 2 * R; ++j) v[j] = __builtin_nontemporal_load(p + 64 * j);
#pragma unroll
    for (int j = 0; j < 2 * R; ++j) acc ^= v[j];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9E3779B9u && acc[0] == 0x7F4A7C15u) sink[threadIdx.x] = acc;
}

__device__ __forceinline__ uint64_t rt() { return __builtin_amdgcn_s_memrealtime(); }

template <int R, int W, int B>
__global__ void __launch_bounds__(256) phased_kernel(uint8_t* __restrict__ base, uint64_t period, uint64_t wwin) {
  __shared__ u4 buf[4][B][W][2][64];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const uint64_t ntasks = kS * kNwin;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4;
  const uint64_t rstart = period - wwin;  // phase >= rstart: write window
  int nb = 0;
  uint64_t tfirst = 0;
  auto flush = [&]() {
    for (int i = 0; i < nb; ++i) {
      const uint64_t t = tfirst + i * nw;
      const uint64_t s = t / kNwin;
      const uint64_t off = (t - s * kNwin) * 2048u + lane * 16u;
      uint8_t* sb = base + s * kN * kL + off;
#pragma unroll
      for (int o = 0; o < W; ++o) {
        u4* q = reinterpret_cast<u4*>(sb + o * kL);
        __builtin_nontemporal_store(buf[wv][i][o][0][lane], q);
        __builtin_nontemporal_store(buf[wv][i][o][1][lane], q + 64);
      }
    }
    nb = 0;
  };
  for (uint64_t t = wave_gid(); t < ntasks; t += nw) {
    uint64_t ph = rt() % period;
    if (nb == B || ph >= rstart) {
      while (ph < rstart) {  // buffer full early: wait for the write window
        __builtin_amdgcn_s_sleep(2);
        ph = rt() % period;
      }
      flush();
      const uint64_t p0 = rt() / period;
      while (rt() / period == p0 && rt() % period >= rstart) __builtin_amdgcn_s_sleep(2);  // to the next read window
    }
    const uint64_t s = t / kNwin;
    const uint64_t off = (t - s * kNwin) * 2048u + lane * 16u;
    const uint8_t* sb = base + s * kN * kL + off;
    u4 v[R][2];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u4* p = reinterpret_cast<const u4*>(sb + (kN - R + r) * kL);
      v[r][0] = __builtin_nontemporal_load(p);
      v[r][1] = __builtin_nontemporal_load(p + 64);
    }
    u4 a = {0u, 0u, 0u, 0u}, b = a;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      a ^= v[r][0];
      b ^= v[r][1];
    }
    if (nb == 0) tfirst = t;
#pragma unroll
    for (int o = 0; o < W; ++o) {
      buf[wv][nb][o][0][lane] = a + static_cast<uint32_t>(o);
      buf[wv][nb][o][1][lane] = b + static_cast<uint32_t>(o);
    }
    ++nb;
  }
  flush();
}

// The same with the outputs of a group of B tasks held in registers (static
// indices): the wave reads its B windows, waits for the write window, writes
// them, waits for the next read window.
template <int R, int W, int B>
__global__ void __launch_bounds__(256) phased_reg_kernel(uint8_t* __restrict__ base, uint64_t period, uint64_t wwin) {
  const int lane = threadIdx.x & 63;
  const uint64_t ntasks = kS * kNwin;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4;
  const uint64_t rstart = period - wwin;
  for (uint64_t t0 = wave_gid(); t0 < ntasks; t0 += B * nw) {
    u4 oa[B][W], ob[B][W];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const uint64_t t = t0 + b * nw;
      if (t >= ntasks) break;
      const uint64_t s = t / kNwin;
      const uint64_t off = (t - s * kNwin) * 2048u + lane * 16u;
      const uint8_t* sb = base + s * kN * kL + off;
      u4 v[R][2];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const u4* p = reinterpret_cast<const u4*>(sb + (kN - R + r) * kL);
        v[r][0] = __builtin_nontemporal_load(p);
        v[r][1] = __builtin_nontemporal_load(p + 64);
      }
      u4 a = {0u, 0u, 0u, 0u}, c = a;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        a ^= v[r][0];
        c ^= v[r][1];
      }
#pragma unroll
      for (int o = 0; o < W; ++o) {
        oa[b][o] = a + static_cast<uint32_t>(o);
        ob[b][o] = c + static_cast<uint32_t>(o);
      }
    }
    const bool last = t0 + B * nw >= ntasks;
    if (!last)
      while (rt() % period < rstart) __builtin_amdgcn_s_sleep(2);
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const uint64_t t = t0 + b * nw;
      if (t >= ntasks) break;
      const uint64_t s = t / kNwin;
      const uint64_t off = (t - s * kNwin) * 2048u + lane * 16u;
      uint8_t* sb = base + s * kN * kL + off;
#pragma unroll
      for (int o = 0; o < W; ++o) {
        u4* q = reinterpret_cast<u4*>(sb + o * kL);
        __builtin_nontemporal_store(oa[b][o], q);
        __builtin_nontemporal_store(ob[b][o], q + 64);
      }
    }
    if (!last) {
      const uint64_t p0 = rt() / period;
      while (rt() / period == p0 && rt() % period >= rstart) __builtin_amdgcn_s_sleep(2);
    }
  }
}

struct Variant {
  std::string name;
  double bytes;
  std::function<void()> run;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 7;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned grid = 2 * cus;
  uint8_t *base = nullptr, *out = nullptr;
  u4* sink = nullptr;
  CK(hipMalloc(&base, kS * kN * kL));
  CK(hipMalloc(&out, kS * kL));
  CK(hipMalloc(&sink, 256 * sizeof(u4)));
  CK(hipMemset(base, 0x3C, kS * kN * kL));
  const double row = static_cast<double>(kS) * kL;
  std::vector<Variant> vs;
#define G(R, W, SEP, NAME)                                                                                    \
  vs.push_back({NAME, (R + W) * row, [=] {                                                                    \
                  hipLaunchKernelGGL((gather_kernel<R, W, SEP>), dim3(grid), dim3(256), 0, 0, base, out, sink); \
                }, {}})
  G(1, 0, false, "g1r0w");
  G(10, 0, false, "g10r0w");
  G(14, 0, false, "g14r0w");
  G(10, 1, false, "g10r1w");
  G(10, 1, true, "g10r1w_sep");
  G(10, 4, false, "g10r4w");
#define C(R, NAME)                                                                                        \
  vs.push_back({NAME, 10 * row, [=] {                                                                     \
                  hipLaunchKernelGGL((contig_kernel<R>), dim3(grid), dim3(256), 0, 0, base, sink,         \
                                     static_cast<uint64_t>(10 * kS * kNwin / R));                         \
                }, {}})
  C(10, "c10");
  C(1, "c1");
#define P(R, W, B, PER, WW)                                                                                 \
  vs.push_back({"p" #R "r" #W "w_b" #B "_P" #PER "_W" #WW, (R + W) * row, [=] {                            \
                  hipLaunchKernelGGL((phased_kernel<R, W, B>), dim3(grid), dim3(256), 0, 0, base,             \
                                     static_cast<uint64_t>(PER), static_cast<uint64_t>(WW));                  \
                }, {}})
  P(10, 1, 8, 5600, 700);
  P(10, 1, 8, 6000, 700);
  P(10, 1, 8, 6000, 900);
  P(10, 1, 8, 6400, 700);
  P(10, 1, 8, 6400, 900);
  P(10, 1, 8, 6800, 900);
  P(10, 1, 8, 7200, 1100);
  P(10, 1, 10, 7000, 900);
  P(10, 1, 10, 7600, 1000);
  P(10, 1, 10, 8000, 1100);
  P(10, 1, 10, 8400, 1200);
#define Q(R, W, B, PER, WW)                                                                                 \
  vs.push_back({"q" #R "r" #W "w_b" #B "_P" #PER "_W" #WW, (R + W) * row, [=] {                            \
                  hipLaunchKernelGGL((phased_reg_kernel<R, W, B>), dim3(grid), dim3(256), 0, 0, base,         \
                                     static_cast<uint64_t>(PER), static_cast<uint64_t>(WW));                  \
                }, {}})
  Q(10, 1, 8, 6400, 900);
  Q(10, 1, 8, 6800, 1000);
  Q(10, 4, 4, 3200, 1000);
  Q(10, 4, 4, 3600, 1200);
  Q(10, 4, 4, 4000, 1400);
  Q(10, 4, 6, 4800, 1500);
  Q(10, 4, 6, 5400, 1700);
  Q(10, 4, 6, 6000, 1900);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs) v.run();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < reps; ++r)
    for (auto& v : vs) {
      CK(hipEventRecord(e0, 0));
      v.run();
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    printf("{\"variant\": \"%s\", \"median_ms\": %.4f, \"GBps\": %.1f}\n", v.name.c_str(), med, v.bytes / 1e6 / med);
  }
  CK(hipFree(base));
  CK(hipFree(out));
  CK(hipFree(sink));
  return 0;
}
