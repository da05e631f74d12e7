// Bandwidth lab: the box's HBM ceilings for the access mixes the codec kernels
// issue (read-only, write-only, copy, 10:4 and 10:1 read:write), across grid
// shapes, per-wave chunk sizes, load policies and LDS-DMA staging. Variants are
// interleaved in one process (cdna_hip_programming.md rule 24). Dev tool.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/bw_lab.hip -o build/bw_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int vmcnt(int n) { return 0x0F70 | (n & 15) | (((n >> 4) & 3) << 14); }
constexpr int kLgkm0 = 0xC07F;

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return *reinterpret_cast<const u32x4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) {
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<u32x4*>(p) = v;
}

__device__ __forceinline__ uint32_t gwave() {
  return __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
}

// Read-only: wave-task = C KiB contiguous (C loads of 1 KiB per wave, all in flight).
template <int C, bool NT>
__global__ void read_kernel(const uint8_t* __restrict__ src, uint64_t ntasks, u32x4* sink) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t t = gwave(); t < ntasks; t += nw) {
    const uint8_t* p = src + t * (C * 1024ull) + lane * 16;
    u32x4 v[C];
#pragma unroll
    for (int j = 0; j < C; ++j) v[j] = ld16<NT>(p + j * 1024);
#pragma unroll
    for (int j = 0; j < C; ++j) acc ^= v[j];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[threadIdx.x] = acc;
}

// Read-only through LDS-DMA: per-wave double buffer of 2 x C KiB; the next
// task's DMA is issued before the current one is consumed.
template <int C, int AUX>
__global__ void read_dma_kernel(const uint8_t* __restrict__ src, uint64_t ntasks, u32x4* sink) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  uint8_t* mine = smem + (threadIdx.x >> 6) * 2 * C * 1024;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  u32x4 acc = {0, 0, 0, 0};
  uint64_t t = gwave();
  int buf = 0;
  auto issue = [&](uint64_t tt, int b) {
    const uint8_t* p = src + tt * (C * 1024ull) + lane * 16;
#pragma unroll
    for (int j = 0; j < C; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(p + j * 1024), (lds_void*)(mine + (b * C + j) * 1024), 16, 0, AUX);
  };
  if (t < ntasks) issue(t, 0);
  for (; t < ntasks; t += nw) {
    const bool more = t + nw < ntasks;
    if (more) {
      issue(t + nw, buf ^ 1);
      __builtin_amdgcn_s_waitcnt(vmcnt(C));
    } else {
      __builtin_amdgcn_s_waitcnt(vmcnt(0));
    }
    const uint8_t* q = mine + buf * C * 1024 + lane * 16;
#pragma unroll
    for (int j = 0; j < C; ++j) acc ^= *reinterpret_cast<const u32x4*>(q + j * 1024);
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    buf ^= 1;
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[threadIdx.x] = acc;
}

template <int C, bool NT>
__global__ void write_kernel(uint8_t* __restrict__ dst, uint64_t ntasks) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint64_t t = gwave(); t < ntasks; t += nw) {
    uint8_t* p = dst + t * (C * 1024ull) + lane * 16;
    const u32x4 v = {(uint32_t)t, (uint32_t)lane, 1u, 2u};
#pragma unroll
    for (int j = 0; j < C; ++j) st16<NT>(p + j * 1024, v);
  }
}

template <int C, bool NT>
__global__ void copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t ntasks) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint64_t t = gwave(); t < ntasks; t += nw) {
    const uint64_t o = t * (C * 1024ull) + lane * 16;
    u32x4 v[C];
#pragma unroll
    for (int j = 0; j < C; ++j) v[j] = ld16<NT>(src + o + j * 1024);
#pragma unroll
    for (int j = 0; j < C; ++j) st16<NT>(dst + o + j * 1024, v[j]);
  }
}

// Codec-shaped probe: stripes of n = K + P rows of L bytes; a wave-task is a
// W-byte window of every row: read K rows, write P rows (XOR, no GF math).
// order 0: task -> (stripe, window) window-fastest; 1: XCD-aware (the
// workgroups that round-robin onto one XCD take adjacent windows).
template <int K, int P, int W, bool NT>
__global__ void rows_kernel(uint8_t* __restrict__ base, uint64_t nstripes, uint64_t L, int order) {
  constexpr int NP = W / 1024;
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  const uint64_t nwin = L / W;
  const uint64_t ntasks = nstripes * nwin;
  uint32_t wid = gwave();
  if (order == 1) {
    const uint32_t wpb = blockDim.x >> 6;
    const uint32_t b = blockIdx.x, nb = gridDim.x;
    const uint32_t xb = (b % 8) * (nb / 8) + b / 8;
    wid = __builtin_amdgcn_readfirstlane(xb * wpb + (threadIdx.x >> 6));
  }
  for (uint64_t t = wid; t < ntasks; t += nw) {
    const uint64_t s = t / nwin;
    const uint64_t off = (t - s * nwin) * W + lane * 16;
    uint8_t* sb = base + s * (K + P) * L;
    u32x4 acc[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) acc[j] = u32x4{0, 0, 0, 0};
    u32x4 v[K][NP];
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int j = 0; j < NP; ++j) v[r][j] = ld16<NT>(sb + (P + r) * L + off + j * 1024);
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int j = 0; j < NP; ++j) acc[j] ^= v[r][j];
#pragma unroll
    for (int o = 0; o < P; ++o)
#pragma unroll
      for (int j = 0; j < NP; ++j) st16<NT>(sb + o * L + off + j * 1024, acc[j] + (uint32_t)o);
  }
}

// Same codec shape, rows staged by LDS-DMA with a per-wave double buffer.
template <int K, int P, int AUX>
__global__ void rows_dma_kernel(uint8_t* __restrict__ base, uint64_t nstripes, uint64_t L) {
  constexpr int W = 2048;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  uint8_t* mine = smem + (threadIdx.x >> 6) * 2 * K * W;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  const uint64_t nwin = L / W;
  const uint64_t ntasks = nstripes * nwin;
  auto issue = [&](uint64_t tt, int b) {
    const uint64_t s = tt / nwin;
    const uint8_t* sb = base + s * (K + P) * L + (tt - s * nwin) * W + lane * 16;
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(sb + (P + r) * L + j * 1024),
                                         (lds_void*)(mine + (b * K + r) * W + j * 1024), 16, 0, AUX);
  };
  uint64_t t = gwave();
  int buf = 0;
  if (t < ntasks) issue(t, 0);
  for (; t < ntasks; t += nw) {
    const bool more = t + nw < ntasks;
    if (more) {
      issue(t + nw, buf ^ 1);
      __builtin_amdgcn_s_waitcnt(vmcnt(2 * K));
    } else {
      __builtin_amdgcn_s_waitcnt(vmcnt(0));
    }
    u32x4 acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    const uint8_t* q = mine + buf * K * W + lane * 16;
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j] ^= *reinterpret_cast<const u32x4*>(q + r * W + j * 1024);
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    const uint64_t s = t / nwin;
    uint8_t* ob = base + s * (K + P) * L + (t - s * nwin) * W + lane * 16;
#pragma unroll
    for (int o = 0; o < P; ++o)
#pragma unroll
      for (int j = 0; j < 2; ++j) st16<true>(ob + o * L + j * 1024, acc[j] + (uint32_t)o);
    buf ^= 1;
  }
}

// Task -> wave mappings for the codec-shaped probe (read K rows, write P rows
// of a 2 KiB window): 0 = grid-stride (consecutive waves take consecutive
// windows; a wave's next task is nw windows later, i.e. a different stripe);
// 1 = each workgroup owns a contiguous range of tasks, its waves interleave
// inside it; 2 = each wave owns a contiguous range.
template <int K, int P>
__global__ void rows_map_kernel(uint8_t* __restrict__ base, uint64_t nstripes, uint64_t L, int map) {
  constexpr int W = 2048;
  const int lane = threadIdx.x & 63;
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t nw = gridDim.x * wpb;
  const uint64_t nwin = L / W;
  const uint64_t ntasks = nstripes * nwin;
  uint64_t t0, step, tend;
  if (map == 0) {
    t0 = gwave(); step = nw; tend = ntasks;
  } else if (map == 1) {
    const uint64_t per = (ntasks + gridDim.x - 1) / gridDim.x;
    t0 = blockIdx.x * per + (threadIdx.x >> 6); step = wpb;
    tend = (blockIdx.x + 1) * per; if (tend > ntasks) tend = ntasks;
  } else {
    const uint64_t per = (ntasks + nw - 1) / nw;
    const uint32_t w = gwave();
    t0 = w * per; step = 1;
    tend = (w + 1) * per; if (tend > ntasks) tend = ntasks;
  }
  t0 = __builtin_amdgcn_readfirstlane((uint32_t)t0);
  for (uint64_t t = t0; t < tend; t += step) {
    const uint64_t s = t / nwin;
    const uint64_t off = (t - s * nwin) * W + lane * 16;
    uint8_t* sb = base + s * (K + P) * L;
    u32x4 acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    u32x4 v[K][2];
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int j = 0; j < 2; ++j) v[r][j] = ld16<true>(sb + (P + r) * L + off + j * 1024);
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j] ^= v[r][j];
    if (P == 0) {
      if ((acc[0][0] ^ acc[1][1]) == 0x12345678u) st16<true>(sb + off, acc[0]);
    }
#pragma unroll
    for (int o = 0; o < P; ++o)
#pragma unroll
      for (int j = 0; j < 2; ++j) st16<true>(sb + o * L + off + j * 1024, acc[j] + (uint32_t)o);
  }
}

// Store cache-policy variants (gfx950 sc0/sc1/nt bits) via inline asm.
template <int POL>
__device__ __forceinline__ void st_pol(uint8_t* p, u32x4 v) {
  if constexpr (POL == 0) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
  else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}

// Codec-shaped probe with load policy LNT, store policy SPOL, W-byte windows.
template <int K, int P, int W, bool LNT, int SPOL>
__global__ void rows_pol_kernel(uint8_t* __restrict__ base, uint64_t nstripes, uint64_t L) {
  constexpr int NP = W / 1024;
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  const uint64_t nwin = L / W;
  const uint64_t ntasks = nstripes * nwin;
  for (uint64_t t = gwave(); t < ntasks; t += nw) {
    const uint64_t s = t / nwin;
    const uint64_t off = (t - s * nwin) * W + lane * 16;
    uint8_t* sb = base + s * (K + P) * L;
    u32x4 acc[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) acc[j] = u32x4{0, 0, 0, 0};
    u32x4 v[K][NP];
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int j = 0; j < NP; ++j) v[r][j] = ld16<LNT>(sb + (P + r) * L + off + j * 1024);
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int j = 0; j < NP; ++j) acc[j] ^= v[r][j];
    if (P == 0) {
      if ((acc[0][0] ^ acc[NP - 1][1]) == 0x12345678u) st16<true>(sb + off, acc[0]);
    }
#pragma unroll
    for (int o = 0; o < P; ++o)
#pragma unroll
      for (int j = 0; j < NP; ++j) st_pol<SPOL>(sb + o * L + off + j * 1024, acc[j] + (uint32_t)o);
  }
}

struct Var {
  std::string name;
  std::function<void()> run;
  double bytes;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const std::string w = argc > 1 ? argv[1] : "all";
  const int rounds = argc > 2 ? atoi(argv[2]) : 7;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t B = 8ull << 30;  // 8 GiB per stream buffer
  uint8_t *a, *b;
  u32x4* sink;
  CK(hipMalloc(&a, B));
  CK(hipMalloc(&b, B));
  CK(hipMalloc(&sink, 4096 * sizeof(u32x4)));
  CK(hipMemset(a, 0x5A, B));
  CK(hipMemset(b, 0x33, B));
  std::vector<Var> vars;

  auto add_read = [&](auto kern, int C, const char* tag, int threads, int bpc) {
    const uint64_t nt = B / (C * 1024ull);
    const unsigned g = bpc * cus;
    vars.push_back({std::string("read ") + tag + " C=" + std::to_string(C) + "K " + std::to_string(threads) + "x" +
                        std::to_string(bpc) + "/CU",
                    [=]() { hipLaunchKernelGGL(kern, dim3(g), dim3(threads), 0, 0, (const uint8_t*)a, nt, sink); },
                    (double)B, {}});
  };
  auto add_dma = [&](auto kern, int C, const char* tag, int threads, int bpc) {
    const uint64_t nt = B / (C * 1024ull);
    const unsigned g = bpc * cus;
    const size_t shm = (size_t)(threads / 64) * 2 * C * 1024;
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    vars.push_back({std::string("read dma ") + tag + " C=" + std::to_string(C) + "K " + std::to_string(threads) + "x" +
                        std::to_string(bpc) + "/CU",
                    [=]() { hipLaunchKernelGGL(kern, dim3(g), dim3(threads), shm, 0, (const uint8_t*)a, nt, sink); },
                    (double)B, {}});
  };
  if (w == "read" || w == "all") {
    for (int bpc : {1, 2, 4}) {
      add_read(read_kernel<2, true>, 2, "nt", 256, bpc);
      add_read(read_kernel<8, true>, 8, "nt", 256, bpc);
      add_read(read_kernel<16, true>, 16, "nt", 256, bpc);
      add_read(read_kernel<8, false>, 8, "plain", 256, bpc);
    }
    add_read(read_kernel<8, true>, 8, "nt", 1024, 1);
    add_read(read_kernel<4, true>, 4, "nt", 1024, 2);
    add_read(read_kernel<16, true>, 16, "nt", 64, 4);
    add_dma(read_dma_kernel<8, 0>, 8, "aux0", 256, 1);
    add_dma(read_dma_kernel<8, 2>, 8, "aux2", 256, 1);
    add_dma(read_dma_kernel<4, 2>, 4, "aux2", 256, 2);
    add_dma(read_dma_kernel<8, 2>, 8, "aux2", 512, 1);
    add_dma(read_dma_kernel<16, 2>, 16, "aux2", 64, 2);
    add_dma(read_dma_kernel<16, 2>, 16, "aux2", 128, 2);
  }
  if (w == "write" || w == "all") {
    for (int bpc : {1, 2, 4}) {
      const unsigned g = bpc * cus;
      auto k8 = write_kernel<8, true>;
      auto k8p = write_kernel<8, false>;
      auto k2 = write_kernel<2, true>;
      const std::string t = " 256x" + std::to_string(bpc);
      vars.push_back({"write nt C=8K" + t, [=]() { hipLaunchKernelGGL(k8, dim3(g), dim3(256), 0, 0, b, B / 8192); }, (double)B, {}});
      vars.push_back({"write plain C=8K" + t, [=]() { hipLaunchKernelGGL(k8p, dim3(g), dim3(256), 0, 0, b, B / 8192); }, (double)B, {}});
      vars.push_back({"write nt C=2K" + t, [=]() { hipLaunchKernelGGL(k2, dim3(g), dim3(256), 0, 0, b, B / 2048); }, (double)B, {}});
      auto c8 = copy_kernel<8, true>;
      auto c2 = copy_kernel<2, true>;
      const uint64_t half = B / 2;
      vars.push_back({"copy nt C=8K" + t, [=]() { hipLaunchKernelGGL(c8, dim3(g), dim3(256), 0, 0, (const uint8_t*)a, b, half / 8192); }, (double)B, {}});
      vars.push_back({"copy nt C=2K" + t, [=]() { hipLaunchKernelGGL(c2, dim3(g), dim3(256), 0, 0, (const uint8_t*)a, b, half / 2048); }, (double)B, {}});
    }
  }
  if (w == "rows" || w == "all") {
    const uint64_t L = 1ull << 20, S = 512;  // 512 stripes x 14 MiB = 7 GiB
    for (int bpc : {1, 2}) {
      const unsigned g = bpc * cus;
      auto e = rows_kernel<10, 4, 2048, true>;
      auto d = rows_kernel<10, 1, 2048, true>;
      auto e4 = rows_kernel<10, 4, 4096, true>;
      const std::string t = " 256x" + std::to_string(bpc);
      vars.push_back({"rows 10r4w W=2K" + t, [=]() { hipLaunchKernelGGL(e, dim3(g), dim3(256), 0, 0, a, S, L, 0); }, 14.0 * L * S, {}});
      vars.push_back({"rows 10r4w W=2K xcd" + t, [=]() { hipLaunchKernelGGL(e, dim3(g), dim3(256), 0, 0, a, S, L, 1); }, 14.0 * L * S, {}});
      vars.push_back({"rows 10r4w W=4K" + t, [=]() { hipLaunchKernelGGL(e4, dim3(g), dim3(256), 0, 0, a, S, L, 0); }, 14.0 * L * S, {}});
      vars.push_back({"rows 10r1w W=2K" + t, [=]() { hipLaunchKernelGGL(d, dim3(g), dim3(256), 0, 0, a, S, L, 0); }, 11.0 * L * S, {}});
      vars.push_back({"rows 10r1w W=2K xcd" + t, [=]() { hipLaunchKernelGGL(d, dim3(g), dim3(256), 0, 0, a, S, L, 1); }, 11.0 * L * S, {}});
    }
    {
      auto e = rows_dma_kernel<10, 4, 2>;
      auto d = rows_dma_kernel<10, 1, 2>;
      const size_t per_wave = 2 * 10 * 2048;
      CK(hipFuncSetAttribute((const void*)e, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      CK(hipFuncSetAttribute((const void*)d, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      for (int waves : {2, 3}) {
        const size_t shm = per_wave * waves;
        const unsigned g = cus;
        const std::string t = " " + std::to_string(64 * waves) + "x1";
        vars.push_back({"rows dma 10r4w" + t, [=]() { hipLaunchKernelGGL(e, dim3(g), dim3(64 * waves), shm, 0, a, S, L); }, 14.0 * L * S, {}});
        vars.push_back({"rows dma 10r1w" + t, [=]() { hipLaunchKernelGGL(d, dim3(g), dim3(64 * waves), shm, 0, a, S, L); }, 11.0 * L * S, {}});
      }
    }
  }
  if (w == "map") {
    for (uint64_t L : {1ull << 20, 1ull << 16}) {
      const uint64_t S = (512ull << 20) / L;  // 7 GiB of stripes
      for (int bpc : {1, 2}) {
        const unsigned g = bpc * cus;
        auto e = rows_map_kernel<10, 4>;
        auto d = rows_map_kernel<10, 1>;
        auto r0 = rows_map_kernel<10, 0>;
        for (int map : {0, 1, 2}) {
          const std::string t = " L=" + std::to_string(L >> 10) + "K map" + std::to_string(map) + " 256x" + std::to_string(bpc);
          vars.push_back({"10r4w" + t, [=]() { hipLaunchKernelGGL(e, dim3(g), dim3(256), 0, 0, a, S, L, map); }, 14.0 * L * S, {}});
          vars.push_back({"10r1w" + t, [=]() { hipLaunchKernelGGL(d, dim3(g), dim3(256), 0, 0, a, S, L, map); }, 11.0 * L * S, {}});
          vars.push_back({"10r0w" + t, [=]() { hipLaunchKernelGGL(r0, dim3(g), dim3(256), 0, 0, a, S, L, map); }, 10.0 * L * S, {}});
        }
      }
    }
  }
  if (w == "pol") {
    const uint64_t L = 1ull << 20, S = 512;
    const unsigned g = 2 * cus;
    static const char* pn[6] = {"nt", "plain", "sc1", "sc0sc1", "sc1nt", "sc0sc1nt"};
#define POLV(K_, P_, W_, LNT_, SP_)                                                                          \
    {                                                                                                         \
      auto kk = rows_pol_kernel<K_, P_, W_, LNT_, SP_>;                                                       \
      vars.push_back({std::string(#K_ "r" #P_ "w W=" #W_ " ld=") + (LNT_ ? "nt" : "plain") + " st=" + pn[SP_], \
                      [=]() { hipLaunchKernelGGL(kk, dim3(g), dim3(256), 0, 0, a, S, L); },                   \
                      (double)(K_ + P_) * L * S, {}});                                                        \
    }
    POLV(10, 1, 2048, true, 0) POLV(10, 1, 2048, true, 1) POLV(10, 1, 2048, true, 2) POLV(10, 1, 2048, true, 3)
    POLV(10, 1, 2048, true, 4) POLV(10, 1, 2048, true, 5) POLV(10, 1, 2048, false, 0) POLV(10, 1, 2048, false, 1)
    POLV(10, 1, 4096, true, 0) POLV(10, 1, 4096, true, 1) POLV(10, 1, 8192, true, 0) POLV(10, 1, 8192, true, 1)
    POLV(10, 4, 2048, true, 0) POLV(10, 4, 2048, true, 1) POLV(10, 4, 2048, true, 2) POLV(10, 4, 2048, true, 3)
    POLV(10, 4, 2048, true, 4) POLV(10, 4, 2048, true, 5) POLV(10, 4, 2048, false, 1) POLV(10, 4, 4096, true, 1)
    POLV(10, 0, 2048, true, 0)
#undef POLV
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
    printf("%-40s median %8.3f ms  min %8.3f ms  %7.1f GB/s (median)  %7.1f (best)\n", v.name.c_str(), med, mn,
           v.bytes / (med * 1e-3) / 1e9, v.bytes / (mn * 1e-3) / 1e9);
  }
  return 0;
}
