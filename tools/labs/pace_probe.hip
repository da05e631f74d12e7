// Pacing probe for the codec's 10-read / W-write window pattern (round 3).
//
// bench.py's no-math pattern probe (hrs_probe_rows: every row's loads issued
// at once, then the stores) streams the RS(10,4) encode pattern at
// 5.45 TB/s, yet the product encode kernel moves the same bytes at 5.67: the
// kernel's math spaces its loads out, and HBM serves the spaced stream better.
// This probe maps that effect, to find the pattern's real ceiling and whether
// any load schedule beats the product kernel:
//   - D: loads in flight per wave in rows (row r + D is issued before row r is
//     used; sched_barriers keep the compiler from hoisting more);
//   - M: dependent VALU work per loaded dword (2 ops per step) standing in for
//     the GF math (the product does ~12 ops per dword per row);
//   - blocks of 256 threads per CU.
// The product kernels run interleaved in the same process (libhrs).
// Usage: pace_probe [rounds]   -> one line per variant, medians.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude tools/pace_probe.hip \
//     -Llambdafs_amd -lhrs -Wl,-rpath,'$ORIGIN/../lambdafs_amd' -o tools/pace_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "hrs.h"

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t gwave() {
  return __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
}

template <int M>
__device__ __forceinline__ u32x4 work(u32x4 x) {
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = __builtin_amdgcn_alignbit(x[q], x[q], 7) ^ (0x9E3779B9u * (m + 1));
  return x;
}

// stripes [S][n][L]; read rows [n - R, n), write rows [0, W) (or out[S][W][L]).
template <int R, int W, int D, int M>
__global__ void __launch_bounds__(256) paced_kernel(uint8_t* __restrict__ base, uint8_t* __restrict__ out,
                                                     uint64_t S, int n, uint64_t L) {
  const int lane = threadIdx.x & 63;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * (blockDim.x >> 6);
  const uint64_t nwin = L / 2048;
  const uint64_t ntasks = S * nwin;
  for (uint64_t t = gwave(); t < ntasks; t += nw) {
    const uint64_t s = t / nwin;
    const uint64_t off = (t - s * nwin) * 2048 + lane * 16;
    const uint8_t* sb = base + s * n * L + off;
    u32x4 v[R][2];
    auto ld = [&](int r) {
      const u32x4* p = reinterpret_cast<const u32x4*>(sb + (n - R + r) * L);
      v[r][0] = __builtin_nontemporal_load(p);
      v[r][1] = __builtin_nontemporal_load(p + 64);
    };
#pragma unroll
    for (int r = 0; r < D && r < R; ++r) ld(r);
    u32x4 a = {0u, 0u, 0u, 0u}, b = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r + D < R) ld(r + D);
      __builtin_amdgcn_sched_barrier(0);
      a ^= work<M>(v[r][0]);
      b ^= work<M>(v[r][1]);
      __builtin_amdgcn_sched_barrier(0);
    }
    uint8_t* ob = out ? out + s * W * L + off : base + s * n * L + off;
#pragma unroll
    for (int o = 0; o < W; ++o) {
      u32x4* q = reinterpret_cast<u32x4*>(ob + o * L);
      __builtin_nontemporal_store(a + static_cast<uint32_t>(o), q);
      __builtin_nontemporal_store(b + static_cast<uint32_t>(o), q + 64);
    }
  }
}

struct Var {
  std::string name;
  std::function<void()> run;
  double bytes;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t L = 1ull << 20, S = 1024;
  const int k = 10, p = 4, n = k + p;
  uint8_t *a = nullptr, *out = nullptr;
  CK(hipMalloc(&a, S * n * L));
  CK(hipMalloc(&out, S * L));
  CK(hipMemset(a, 0x5A, S * n * L));
  hrs_codec* codec = nullptr;
  if (hrs_create(k, p, nullptr, &codec) != HRS_OK) {
    fprintf(stderr, "hrs_create failed\n");
    return 1;
  }
  std::vector<Var> vars;
  const uint8_t* in_rows[10];
  uint8_t* par_rows[4];
  const uint8_t* all_rows[14];
  for (int r = 0; r < k; ++r) in_rows[r] = a + (p + r) * L;
  for (int o = 0; o < p; ++o) par_rows[o] = a + o * L;
  for (int r = 0; r < n; ++r) all_rows[r] = a + r * L;
  uint8_t* out_rows[1] = {out};
  const int erased[1] = {4}, ntr[4] = {0, 1, 2, 4};
  vars.push_back({"product encode_static_kernel<10,4>",
                  [&]() {
                    if (hrs_encode_dev(codec, in_rows, n * L, par_rows, n * L, L, S, nullptr) != HRS_OK) exit(2);
                  },
                  14.0 * L * S, {}});
  vars.push_back({"product repair (data shard 0)",
                  [&]() {
                    if (hrs_decode_dev(codec, all_rows, n * L, out_rows, L, erased, 1, ntr, 4, L, S, nullptr) != HRS_OK)
                      exit(2);
                  },
                  11.0 * L * S, {}});
  auto add = [&](const std::string& nm, auto kern, int W, int bpc, bool sep) {
    const unsigned g = static_cast<unsigned>(bpc * cus);
    uint8_t* o = sep ? out : nullptr;
    vars.push_back({nm + " " + std::to_string(bpc) + "/CU",
                    [=]() { hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, a, o, S, n, L); },
                    double(k + W) * L * S, {}});
  };
#define ADD(W, D, M)                                                                                    \
  for (int bpc : {1, 2}) add("10r" #W "w D=" #D " M=" #M, paced_kernel<10, W, D, M>, W, bpc, W == 1);
#define ADDM(D) ADD(4, D, 0) ADD(4, D, 3) ADD(4, D, 6) ADD(4, D, 12) ADD(1, D, 0) ADD(1, D, 3) ADD(1, D, 6) ADD(1, D, 12)
  ADDM(1)
  ADDM(2)
  ADDM(3)
  ADDM(5)
  ADDM(10)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vars) v.run();
  CK(hipDeviceSynchronize());
  CK(hipGetLastError());
  for (int r = 0; r < rounds; ++r) {
    for (auto& v : vars) {
      CK(hipEventRecord(e0, 0));
      v.run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
    fprintf(stderr, "round %d done\n", r);
  }
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    printf("%-44s median %7.3f ms  min %7.3f ms  %7.1f GB/s (median)  %7.1f (best)\n", v.name.c_str(), med, mn,
           v.bytes / (med * 1e-3) / 1e9, v.bytes / (mn * 1e-3) / 1e9);
  }
  hrs_destroy(codec);
  CK(hipFree(a));
  CK(hipFree(out));
  return 0;
}
