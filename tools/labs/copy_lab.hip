// Copy-schedule lab (VERDICT r3 "validate the HBM ceiling"): which 1:1 device
// copy schedule reaches MI355X_MICROARCH.md's "6.29 TB/s measured (float4
// copy)" on this pool's boxes, and what the probes in libhrs_probe.so should
// use. Every variant copies the same 4 GiB buffer into another (bytes read +
// written / time), interleaved rep by rep in one process so box-to-box
// spread cancels; median of `reps` launches.
//
// Variants (each x {256, 512, 1024}-thread blocks x blocks/CU):
//   gs<U>   grid-stride: thread i copies elements i + j*T (T = all threads),
//           U loads in flight per thread before its U stores;
//   wc<C>   wave task of C contiguous KiB (the current probe's shape), all C
//           loads before any store;
//   bc<U>   block-contiguous: block b owns 1/grid of the buffer as one range,
//           walked block-stride with U loads in flight;
// each with load / store policy {plain, nontemporal}.
// Usage: copy_lab [reps] [GiB]   (prints one JSON line per variant)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

template <bool NT>
__device__ __forceinline__ u4 ld(const u4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u4* p, u4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// grid-stride, U elements in flight per thread (n % (U*T) handled by a tail loop)
template <int U, bool NL, bool NS>
__global__ void gs_kernel(const u4* __restrict__ a, u4* __restrict__ b, uint64_t n) {
  const uint64_t T = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  uint64_t i = gid;
  for (; i + (U - 1) * T < n; i += U * T) {
    u4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = ld<NL>(&a[i + j * T]);
#pragma unroll
    for (int j = 0; j < U; ++j) st<NS>(&b[i + j * T], v[j]);
  }
  for (; i < n; i += T) b[i] = a[i];
}

// wave task of C contiguous KiB
template <int C, bool NL, bool NS>
__global__ void wc_kernel(const u4* __restrict__ a, u4* __restrict__ b, uint64_t n) {
  const int lane = threadIdx.x & 63;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * (blockDim.x >> 6);
  const uint64_t w0 = static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t ntasks = n / (64u * C);
  for (uint64_t t = w0; t < ntasks; t += nw) {
    const uint64_t e = t * 64u * C + lane;
    u4 v[C];
#pragma unroll
    for (int j = 0; j < C; ++j) v[j] = ld<NL>(&a[e + 64u * j]);
#pragma unroll
    for (int j = 0; j < C; ++j) st<NS>(&b[e + 64u * j], v[j]);
  }
  for (uint64_t i = ntasks * 64u * C + static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    b[i] = a[i];
}

// block-contiguous range, block-stride inside it, U in flight
template <int U, bool NL, bool NS>
__global__ void bc_kernel(const u4* __restrict__ a, u4* __restrict__ b, uint64_t n) {
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = per * blockIdx.x;
  const uint64_t hi = std::min<uint64_t>(n, lo + per);
  const uint64_t B = blockDim.x;
  uint64_t i = lo + threadIdx.x;
  for (; i + (U - 1) * B < hi; i += U * B) {
    u4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = ld<NL>(&a[i + j * B]);
#pragma unroll
    for (int j = 0; j < U; ++j) st<NS>(&b[i + j * B], v[j]);
  }
  for (; i < hi; i += B) b[i] = a[i];
}

struct Variant {
  std::string name;
  void (*fn)(const u4*, u4*, uint64_t);
  int block;
  int bpc;
};

#define POLICIES(kern, P, label)                                                                             \
  do {                                                                                                       \
    for (int blk : {256, 512, 1024})                                                                         \
      for (int bpc : {1, 2, 4, 8}) {                                                                         \
        if (blk * bpc > 2048) continue;                                                                      \
        auto add = [&](auto f, const char* pol) {                                                            \
          char nm[96];                                                                                       \
          snprintf(nm, sizeof nm, "%s%d_%s_b%d_x%d", label, P, pol, blk, bpc);                               \
          vs.push_back({nm, f, blk, bpc});                                                                   \
        };                                                                                                   \
        add(kern<P, false, false>, "plain");                                                                 \
        add(kern<P, true, true>, "nt");                                                                      \
        add(kern<P, true, false>, "ntld");                                                                   \
        add(kern<P, false, true>, "ntst");                                                                   \
      }                                                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 7;
  const size_t gib = argc > 2 ? static_cast<size_t>(atol(argv[2])) : 4;
  const size_t bytes = gib << 30;
  const uint64_t n = bytes / 16;
  u4 *a = nullptr, *b = nullptr;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0x5A, bytes));
  CK(hipMemset(b, 0, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<Variant> vs;
  POLICIES(gs_kernel, 1, "gs");
  POLICIES(gs_kernel, 4, "gs");
  POLICIES(gs_kernel, 8, "gs");
  POLICIES(wc_kernel, 4, "wc");
  POLICIES(wc_kernel, 8, "wc");
  POLICIES(bc_kernel, 4, "bc");
  POLICIES(bc_kernel, 8, "bc");
  POLICIES(bc_kernel, 16, "bc");
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(vs.size());
  auto launch = [&](const Variant& v) {
    hipLaunchKernelGGL(v.fn, dim3(static_cast<unsigned>(v.bpc * cus)), dim3(v.block), 0, 0, a, b, n);
  };
  for (const Variant& v : vs) launch(v);  // warm every kernel once
  CK(hipDeviceSynchronize());
  fprintf(stderr, "copy_lab: %zu variants x %d reps, %zu GiB, %d CUs\n", vs.size(), reps, gib, cus);
  for (int r = 0; r < reps; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(e0, 0));
      launch(vs[i]);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[i].push_back(t);
    }
    fprintf(stderr, "rep %d done\n", r);
  }
  // every variant copied the same bytes: check a sample of the destination
  std::vector<uint32_t> h(1 << 20);
  CK(hipMemcpy(h.data(), reinterpret_cast<uint8_t*>(b) + bytes - (4 << 20), 4 << 20, hipMemcpyDeviceToHost));
  bool ok = std::all_of(h.begin(), h.end(), [](uint32_t x) { return x == 0x5A5A5A5Au; });
  for (size_t i = 0; i < vs.size(); ++i) {
    std::vector<float> s = ms[i];
    std::sort(s.begin(), s.end());
    const double med = s[s.size() / 2], best = s[0];
    printf("{\"variant\": \"%s\", \"block\": %d, \"blocks_per_cu\": %d, \"median_ms\": %.4f, \"min_ms\": %.4f, "
           "\"TBps_median\": %.3f, \"TBps_best\": %.3f}\n",
           vs[i].name.c_str(), vs[i].block, vs[i].bpc, med, best, 2.0 * bytes / (med * 1e-3) / 1e12,
           2.0 * bytes / (best * 1e-3) / 1e12);
  }
  printf("{\"check\": %s, \"bytes_per_buffer\": %zu, \"cus\": %d}\n", ok ? "true" : "false", bytes, cus);
  CK(hipFree(a));
  CK(hipFree(b));
  return ok ? 0 : 1;
}
