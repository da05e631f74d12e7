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

// p-structure (flush whenever the write window comes) with the buffered
// outputs in registers: slot nb (wave-uniform) is written through a switch,
// so every register index is static.
template <int R, int W, int B, bool PRED = false>
__global__ void __launch_bounds__(256) phased_sw_kernel(uint8_t* __restrict__ base, uint64_t period, uint64_t wwin,
                                                        unsigned long long* stats = nullptr) {
  const int lane = threadIdx.x & 63;
  const uint64_t ntasks = kS * kNwin;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4;
  const uint64_t rstart = period - wwin;
  u4 oa[B][W], ob[B][W];
  int nb = 0;
  uint64_t tfirst = 0;
  auto flush = [&]() {
#pragma unroll
    for (int i = 0; i < B; ++i) {
      if (i >= nb) break;
      const uint64_t t = tfirst + i * nw;
      const uint64_t s = t / kNwin;
      const uint64_t off = (t - s * kNwin) * 2048u + lane * 16u;
      uint8_t* sb = base + s * kN * kL + off;
#pragma unroll
      for (int o = 0; o < W; ++o) {
        u4* q = reinterpret_cast<u4*>(sb + o * kL);
        __builtin_nontemporal_store(oa[i][o], q);
        __builtin_nontemporal_store(ob[i][o], q + 64);
      }
    }
    nb = 0;
  };
  uint64_t est = 0;  // PRED: the wave's recent task time (ticks)
  uint64_t busy = 0, ntask = 0;  // stats: read-phase task time, tasks
  for (uint64_t t = wave_gid(); t < ntasks; t += nw) {
    const uint64_t t_start = rt();
    uint64_t ph = t_start % period;
    // PRED: a task that would still be loading when the write window opens
    // is not started (its reads would mix with the other waves' writes)
    if (nb == B || ph >= rstart || (PRED && ph + est >= rstart)) {
      while (ph < rstart) {
        __builtin_amdgcn_s_sleep(2);
        ph = rt() % period;
      }
      flush();
      const uint64_t p0 = rt() / period;
      while (rt() / period == p0 && rt() % period >= rstart) __builtin_amdgcn_s_sleep(2);
    }
    const uint64_t t_go = rt();
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
    if (PRED || stats) {
      const uint64_t d = rt() - t_go;  // after the XOR: the loads are back
      est = est ? (3 * est + d) / 4 : d;
      busy += d;
      ++ntask;
    }
    if (nb == 0) tfirst = t;
#pragma unroll
    for (int i = 0; i < B; ++i)
      if (i == nb) {
#pragma unroll
        for (int o = 0; o < W; ++o) {
          oa[i][o] = a + static_cast<uint32_t>(o);
          ob[i][o] = c + static_cast<uint32_t>(o);
        }
      }
    ++nb;
  }
  flush();
  if (stats && lane == 0) {
    atomicAdd(&stats[0], static_cast<unsigned long long>(busy));
    atomicAdd(&stats[1], static_cast<unsigned long long>(ntask));
  }
}

struct Variant {
  std::string name;
  double bytes;
  std::function<void()> run;
  std::vector<float> ms;
};

// calib mode: launch the register-phased kernel `launches` times, each period
// P = slack * B * (mean read-phase task time of the previous launch) / (1 - f),
// write window W = 1.25 * f * P, f = the write share of the mix's time at the
// read / write peaks; one JSON line per launch.
template <int R, int W, int B>
void calib(uint8_t* base, unsigned grid, double slack, int launches, double f) {
  unsigned long long* st = nullptr;
  CK(hipMalloc(&st, 2 * sizeof(unsigned long long)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  double tau = 0;
  uint64_t P = 1000 * B;  // first guess: 10 us per task
  for (int l = 0; l < launches; ++l) {
    if (tau > 0) P = static_cast<uint64_t>(slack * B * tau / (1 - f));
    const uint64_t Wt = static_cast<uint64_t>(1.25 * f * P);
    CK(hipMemset(st, 0, 2 * sizeof(unsigned long long)));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((phased_sw_kernel<R, W, B, false>), dim3(grid), dim3(256), 0, 0, base, P, Wt, st);
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long h[2];
    CK(hipMemcpy(h, st, sizeof h, hipMemcpyDeviceToHost));
    tau = h[1] ? static_cast<double>(h[0]) / h[1] : 0;
    printf("{\"calib\": \"%dr%dw_b%d\", \"slack\": %.2f, \"launch\": %d, \"P\": %llu, \"W\": %llu, \"ms\": %.4f, "
           "\"GBps\": %.1f, \"tau_ticks\": %.1f}\n",
           R, W, B, slack, l, (unsigned long long)P, (unsigned long long)Wt, ms,
           static_cast<double>(R + W) * kS * kL / 1e6 / ms, tau);
  }
  CK(hipFree(st));
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 7;
  if (argc > 2 && std::string(argv[2]) == "calib") {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t* base = nullptr;
    CK(hipMalloc(&base, kS * kN * kL));
    CK(hipMemset(base, 0x3C, kS * kN * kL));
    const double f_dec = (1 / 6.1) / (10 / 6.8 + 1 / 6.1), f_enc = (4 / 6.1) / (10 / 6.8 + 4 / 6.1);
    for (double slack : {1.0, 1.2, 1.4, 1.7, 2.0, 2.4}) {
      calib<10, 1, 16>(base, 2 * cus, slack, reps, f_dec);
      calib<10, 4, 5>(base, 2 * cus, slack, reps, f_enc);
    }
    CK(hipFree(base));
    return 0;
  }
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
#define Q(R, W, B, PER, WW)                                                                                 \
  vs.push_back({"q" #R "r" #W "w_b" #B "_P" #PER "_W" #WW, (R + W) * row, [=] {                            \
                  hipLaunchKernelGGL((phased_reg_kernel<R, W, B>), dim3(grid), dim3(256), 0, 0, base,         \
                                     static_cast<uint64_t>(PER), static_cast<uint64_t>(WW));                  \
                }, {}})
#define SW(R, W, B, PER, WW)                                                                                \
  vs.push_back({"s" #R "r" #W "w_b" #B "_P" #PER "_W" #WW, (R + W) * row, [=] {                            \
                  hipLaunchKernelGGL((phased_sw_kernel<R, W, B>), dim3(grid), dim3(256), 0, 0, base,          \
                                     static_cast<uint64_t>(PER), static_cast<uint64_t>(WW));                  \
                }, {}})
#define SP(R, W, B, PER, WW)                                                                                \
  vs.push_back({"t" #R "r" #W "w_b" #B "_P" #PER "_W" #WW, (R + W) * row, [=] {                            \
                  hipLaunchKernelGGL((phased_sw_kernel<R, W, B, true>), dim3(grid), dim3(256), 0, 0, base,    \
                                     static_cast<uint64_t>(PER), static_cast<uint64_t>(WW));                  \
                }, {}})
  SW(10, 4, 5, 4800, 1500);
  SP(10, 4, 5, 3600, 1100);
  SP(10, 4, 5, 4000, 1200);
  SP(10, 4, 5, 4400, 1300);
  SP(10, 4, 5, 4800, 1450);
  SP(10, 4, 5, 5200, 1550);
  SP(10, 4, 5, 5600, 1700);
  SP(10, 4, 5, 6000, 1800);
  SW(10, 1, 16, 11000, 1500);
  SP(10, 1, 16, 8000, 1000);
  SP(10, 1, 16, 9000, 1100);
  SP(10, 1, 16, 10000, 1200);
  SP(10, 1, 16, 11000, 1300);
  SP(10, 1, 16, 12000, 1450);
  SP(10, 1, 16, 13000, 1550);
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
