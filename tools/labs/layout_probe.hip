// Layout / task-order probe for the codec's HBM access pattern (round 3).
//
// profiles/r01/lab9_task_mapping.txt measured the no-math 10-read/4-write
// window pattern at 5.64 TB/s with 1 MiB cells but 6.14 TB/s with 64 KiB
// cells (same bytes, same kernel, same task order), and row-pitch padding
// (lab5) did not move the 1 MiB case. This probe separates the candidate
// causes, each variant the same 7 GiB of stripes and the same per-wave work
// (one 2 KiB column window of K read rows and P written rows, nontemporal
// 16-byte accesses, 256-thread blocks, grid = bpc x CUs, grid-stride tasks):
//   stripe s, row r, byte o lives at
//     base + (s / G) * GS + (s % G) * SS + r * RS + o,    o < L
//   task t -> (stripe, window) by `order`: 0 = window-fastest (the product's
//   t = s * nwin + w), 1 = stripe-fastest (t = w * S + s).
// Usage: layout_probe [rounds] [layouts|spacing]   -> one line per variant, medians.
//   spacing: 64 KiB cells with the rows of a stripe D apart, D = 64 KiB .. 4 MiB.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Layout {
  uint64_t S, L, G, GS, SS, RS;
  int order;
};

__device__ __forceinline__ uint64_t gwave() {
  return __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
}

template <int K, int P>
__global__ void __launch_bounds__(256) rows_kernel(uint8_t* __restrict__ base, Layout y) {
  const int lane = threadIdx.x & 63;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * (blockDim.x >> 6);
  const uint64_t nwin = y.L / 2048;
  const uint64_t ntasks = y.S * nwin;
  for (uint64_t t = gwave(); t < ntasks; t += nw) {
    uint64_t s, w;
    if (y.order == 0) {
      s = t / nwin;
      w = t - s * nwin;
    } else {
      w = t / y.S;
      s = t - w * y.S;
    }
    uint8_t* sb = base + (s / y.G) * y.GS + (s % y.G) * y.SS + w * 2048 + lane * 16;
    u32x4 acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    u32x4 v[K][2];
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        v[r][j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sb + (P + r) * y.RS + j * 1024));
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j] ^= v[r][j];
    if (P == 0) {
      if ((acc[0][0] ^ acc[1][1]) == 0x12345678u) *reinterpret_cast<u32x4*>(sb) = acc[0];
    }
#pragma unroll
    for (int o = 0; o < P; ++o)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        __builtin_nontemporal_store(acc[j] + static_cast<uint32_t>(o),
                                    reinterpret_cast<u32x4*>(sb + o * y.RS + j * 1024));
  }
}

struct Var {
  std::string name;
  std::function<void()> run;
  double bytes;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const std::string mode = argc > 2 ? argv[2] : "layouts";
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t B = 8ull << 30;
  uint8_t* a = nullptr;
  CK(hipMalloc(&a, B));
  CK(hipMemset(a, 0x5A, B));
  std::vector<Var> vars;
  const uint64_t M = 1ull << 20, K64 = 64ull << 10;
  auto k104 = rows_kernel<10, 4>;
  auto k101 = rows_kernel<10, 1>;
  auto k100 = rows_kernel<10, 0>;
  auto add = [&](const std::string& name, Layout y, int k, int p, int bpc) {
    const unsigned g = static_cast<unsigned>(bpc * cus);
    const double bytes = static_cast<double>(k + p) * y.L * y.S;
    const std::string nm = name + " " + std::to_string(k) + "r" + std::to_string(p) + "w " + std::to_string(bpc) + "/CU";
    if (k == 10 && p == 4)
      vars.push_back({nm, [=]() { hipLaunchKernelGGL(k104, dim3(g), dim3(256), 0, 0, a, y); }, bytes, {}});
    else if (k == 10 && p == 1)
      vars.push_back({nm, [=]() { hipLaunchKernelGGL(k101, dim3(g), dim3(256), 0, 0, a, y); }, bytes, {}});
    else
      vars.push_back({nm, [=]() { hipLaunchKernelGGL(k100, dim3(g), dim3(256), 0, 0, a, y); }, bytes, {}});
  };
  if (mode == "spacing") {
    // 64 KiB cells, the rows of a stripe D apart (D a multiple of 64 KiB):
    // G = D / 64 KiB stripes interleave in each D-sized row slot, groups of G
    // stripes follow each other (14 * D bytes per group); ~7 GiB in total.
    for (uint64_t dk : {64, 128, 192, 256, 512, 960, 1024, 1088, 1536, 2048, 4096}) {
      const uint64_t D = dk << 10, G = D / K64;
      const uint64_t groups = (7ull << 30) / (14 * D);
      const Layout y{groups * G, K64, G, 14 * D, K64, D, 0};
      add("L=64K rows " + std::to_string(dk) + "K apart", y, 10, 4, 2);
      add("L=64K rows " + std::to_string(dk) + "K apart", y, 10, 1, 2);
    }
  }
  for (int kp = 0; kp < (mode == "layouts" ? 2 : 0); ++kp) {
    const int p = kp == 0 ? 4 : 1;
    for (int bpc : {2}) {
      // 1: the product layout and order, 1 MiB cells (512 stripes x 14 MiB = 7 GiB)
      add("L=1M stripe-major order0", Layout{512, M, 1, 14 * M, 0, M, 0}, 10, p, bpc);
      // 2: 64 KiB cells, same bytes
      add("L=64K stripe-major order0", Layout{8192, K64, 1, 14 * K64, 0, K64, 0}, 10, p, bpc);
      // 3: 1 MiB cells, stripe-fastest task order
      add("L=1M stripe-major order1", Layout{512, M, 1, 14 * M, 0, M, 0}, 10, p, bpc);
      // 4: 64 KiB cells whose rows are 1 MiB apart (16 stripes side by side in a 14 MiB group)
      add("L=64K rows-1M-apart order0", Layout{8192, K64, 16, 14 * M, K64, M, 0}, 10, p, bpc);
      // 5: 1 MiB cells stored as 16 interleaved 64 KiB segments per row
      //    (= the same bytes addressed as 64 KiB sub-stripes of 1 MiB stripes)
      add("L=1M as 16x64K sub-stripes", Layout{8192, K64, 1, 14 * K64, 0, K64, 0}, 10, p, bpc);
      // 6: 256 KiB cells
      add("L=256K stripe-major order0", Layout{2048, 256 * 1024, 1, 14 * 256 * 1024, 0, 256 * 1024, 0}, 10, p, bpc);
      // 7: 1 MiB cells, rows 1 MiB + 64 KiB apart (pitch padding)
      add("L=1M pitch+64K order0", Layout{480, M, 1, 14 * (M + K64), 0, M + K64, 0}, 10, p, bpc);
      // 8: 1 MiB cells, row-major [row][stripe][L] (row r of every stripe contiguous)
      add("L=1M row-major order0", Layout{512, M, 1, M, 0, 512 * M, 0}, 10, p, bpc);
    }
  }
  if (mode == "layouts") {
    add("L=1M stripe-major order0", Layout{512, M, 1, 14 * M, 0, M, 0}, 10, 4, 1);
    add("L=64K stripe-major order0", Layout{8192, K64, 1, 14 * K64, 0, K64, 0}, 10, 4, 1);
    add("L=1M stripe-major order0", Layout{512, M, 1, 14 * M, 0, M, 0}, 10, 0, 2);
    add("L=64K stripe-major order0", Layout{8192, K64, 1, 14 * K64, 0, K64, 0}, 10, 0, 2);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vars) v.run();
  CK(hipDeviceSynchronize());
  CK(hipGetLastError());
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vars) {
      CK(hipEventRecord(e0, 0));
      v.run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    printf("%-48s median %7.3f ms  min %7.3f ms  %7.1f GB/s (median)  %7.1f (best)\n", v.name.c_str(), med, mn,
           v.bytes / (med * 1e-3) / 1e9, v.bytes / (mn * 1e-3) / 1e9);
  }
  CK(hipFree(a));
  return 0;
}
