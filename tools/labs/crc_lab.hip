// CRC-32 kernel lab: what bounds the window kernel of hrs_crc.hip?
// Variants of the per-window raw CRC (no fold; the fold is O(windows)):
//   R      slicing tables replicated R times across LDS banks (lane l uses copy l % R)
//   CH     independent chains per lane (ILP), joined with Z_{LB/CH}
//   LB     contiguous bytes per lane (window = 64 * LB)
//   SL     slicing-by-4 or slicing-by-8
// plus a no-table probe (XOR of the loaded words) for the load ceiling.
// Each variant is checked against a bitwise CPU raw CRC on sampled windows
// and timed over a 4 GiB buffer at several grid sizes.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/crc_lab.hip -o build/crc_lab
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../lambdafs_amd/csrc/crc32.hpp"

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

using namespace hrs;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t zmul(const uint32_t* z, uint32_t c) {
  return z[c & 0xFFu] ^ z[256 + ((c >> 8) & 0xFFu)] ^ z[512 + ((c >> 16) & 0xFFu)] ^ z[768 + (c >> 24)];
}

// LDS image: [SL tables][256][R] slice words, then Z_{chain} (1024), then 6 tree levels (6 x 1024)
template <int R, int SL>
constexpr int slice_words() {
  return SL * 256 * R;
}
template <int R, int SL>
constexpr int lds_words() {
  return slice_words<R, SL>() + 7 * 1024;
}

template <int R, int SL>
__device__ __forceinline__ uint32_t step4(const uint32_t* s, uint32_t c, int rep) {
  // c already XORed with the word; bytes 0..3 go through tables 3..0
  return s[(3 * 256 + (c & 0xFFu)) * R + rep] ^ s[(2 * 256 + ((c >> 8) & 0xFFu)) * R + rep] ^
         s[(1 * 256 + ((c >> 16) & 0xFFu)) * R + rep] ^ s[(0 * 256 + (c >> 24)) * R + rep];
}

template <int R>
__device__ __forceinline__ uint32_t step8(const uint32_t* s, uint32_t c, uint32_t hi, int rep) {
  // 8 bytes: c = crc ^ word0, hi = word1 (bytes 4..7)
  return s[(7 * 256 + (c & 0xFFu)) * R + rep] ^ s[(6 * 256 + ((c >> 8) & 0xFFu)) * R + rep] ^
         s[(5 * 256 + ((c >> 16) & 0xFFu)) * R + rep] ^ s[(4 * 256 + (c >> 24)) * R + rep] ^
         s[(3 * 256 + (hi & 0xFFu)) * R + rep] ^ s[(2 * 256 + ((hi >> 8) & 0xFFu)) * R + rep] ^
         s[(1 * 256 + ((hi >> 16) & 0xFFu)) * R + rep] ^ s[(0 * 256 + (hi >> 24)) * R + rep];
}

template <int R, int CH, int LB, int SL>
__global__ void __launch_bounds__(256) crc_var(const uint8_t* buf, uint64_t nwin, const uint32_t* tables,
                                               uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < lds_words<R, SL>(); i += blockDim.x) lds[i] = tables[i];
  __syncthreads();
  const uint32_t* slices = lds;
  const uint32_t* zch = lds + slice_words<R, SL>();
  const uint32_t* tree = zch + 1024;
  const int lane = threadIdx.x & 63;
  const int rep = lane % R;
  constexpr int W = LB / 4;         // words per lane
  constexpr int WPC = W / CH;       // words per chain
  const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
  for (uint64_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)); w < nwin;
       w += nwaves) {
    const u32x4* p = reinterpret_cast<const u32x4*>(buf + w * (64ull * LB) + lane * LB);
    uint32_t words[W];
#pragma unroll
    for (int j = 0; j < W / 4; ++j) {
      const u32x4 v = __builtin_nontemporal_load(p + j);
      words[4 * j] = v[0];
      words[4 * j + 1] = v[1];
      words[4 * j + 2] = v[2];
      words[4 * j + 3] = v[3];
    }
    uint32_t ch[CH];
#pragma unroll
    for (int q = 0; q < CH; ++q) ch[q] = 0u;
    if constexpr (SL == 4) {
#pragma unroll
      for (int st = 0; st < WPC; ++st)
#pragma unroll
        for (int q = 0; q < CH; ++q) ch[q] = step4<R, SL>(slices, ch[q] ^ words[q * WPC + st], rep);
    } else {
#pragma unroll
      for (int st = 0; st < WPC; st += 2)
#pragma unroll
        for (int q = 0; q < CH; ++q)
          ch[q] = step8<R>(slices, ch[q] ^ words[q * WPC + st], words[q * WPC + st + 1], rep);
    }
    uint32_t c = ch[0];
#pragma unroll
    for (int q = 1; q < CH; ++q) c = zmul(zch, c) ^ ch[q];
#pragma unroll
    for (int lvl = 0; lvl < 6; ++lvl) {
      const uint32_t o = __shfl_down(c, 1 << lvl, 64);
      c = zmul(tree + lvl * 1024, c) ^ o;
    }
    if (lane == 0) out[w] = c;
  }
}

// Coalesced layout: chain q of lane l = bytes [q*1024 + 16l, +16) of a
// window of NCH KiB; each load instruction is one contiguous 1 KiB wave
// access. The chains join with Z_1024, the lane tree with Z_{16*2^t}.
template <int R, int NCH>
__global__ void __launch_bounds__(256) crc_coal(const uint8_t* buf, uint64_t nwin, const uint32_t* tables,
                                                uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < lds_words<R, 4>(); i += blockDim.x) lds[i] = tables[i];
  __syncthreads();
  const uint32_t* slices = lds;
  const uint32_t* zch = lds + slice_words<R, 4>();
  const uint32_t* tree = zch + 1024;
  const int lane = threadIdx.x & 63;
  const int rep = lane % R;
  const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
  for (uint64_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)); w < nwin;
       w += nwaves) {
    const uint8_t* base = buf + w * (1024ull * NCH) + lane * 16;
    uint32_t words[NCH][4];
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + q * 1024));
      words[q][0] = v[0];
      words[q][1] = v[1];
      words[q][2] = v[2];
      words[q][3] = v[3];
    }
    uint32_t ch[NCH];
#pragma unroll
    for (int q = 0; q < NCH; ++q) ch[q] = 0u;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int q = 0; q < NCH; ++q) ch[q] = step4<R, 4>(slices, ch[q] ^ words[q][st], rep);
    uint32_t c = ch[0];
#pragma unroll
    for (int q = 1; q < NCH; ++q) c = zmul(zch, c) ^ ch[q];
#pragma unroll
    for (int lvl = 0; lvl < 6; ++lvl) {
      const uint32_t o = __shfl_down(c, 1 << lvl, 64);
      c = zmul(tree + lvl * 1024, c) ^ o;
    }
    if (lane == 0) out[w] = c;
  }
}

// Bank-private tables: slicing tables replicated 32x, lane l reads copy
// l % 32 (ds_read_b32 banks are (a/4) mod 32 per 32-lane group), so data
// lookups never conflict; Z tables unreplicated. Windows of NCH KiB, chains
// processed GROUP at a time (Horner join with Z_1024), BLOCK threads per
// block sharing one 156 KiB table image.
constexpr int kBigSliceWords = 4 * 256 * 32;
constexpr int kBigWords = kBigSliceWords + 7 * 1024;

template <int NCH, int GROUP, int BLOCK>
__global__ void __launch_bounds__(BLOCK) crc_big(const uint8_t* buf, uint64_t nwin, const uint32_t* tables,
                                                 uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < kBigWords; i += blockDim.x) lds[i] = tables[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t* slices = lds + (lane & 31);  // this lane's copy: entry e at e * 32
  const uint32_t* zj = lds + kBigSliceWords;
  const uint32_t* tree = zj + 1024;
  const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
  for (uint64_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)); w < nwin;
       w += nwaves) {
    const uint8_t* base = buf + w * (1024ull * NCH) + lane * 16;
    uint32_t c = 0;
#pragma unroll 1
    for (int g = 0; g < NCH; g += GROUP) {
      uint32_t words[GROUP][4];
#pragma unroll
      for (int q = 0; q < GROUP; ++q) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (g + q) * 1024));
        words[q][0] = v[0];
        words[q][1] = v[1];
        words[q][2] = v[2];
        words[q][3] = v[3];
      }
      uint32_t ch[GROUP];
#pragma unroll
      for (int q = 0; q < GROUP; ++q) ch[q] = 0u;
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int q = 0; q < GROUP; ++q) {
          const uint32_t x = ch[q] ^ words[q][st];
          ch[q] = slices[(3 * 256 + (x & 0xFFu)) * 32] ^ slices[(2 * 256 + ((x >> 8) & 0xFFu)) * 32] ^
                  slices[(1 * 256 + ((x >> 16) & 0xFFu)) * 32] ^ slices[(0 * 256 + (x >> 24)) * 32];
        }
#pragma unroll
      for (int q = 0; q < GROUP; ++q) c = (g + q == 0) ? ch[q] : (zmul(zj, c) ^ ch[q]);
    }
#pragma unroll
    for (int lvl = 0; lvl < 6; ++lvl) {
      const uint32_t o = __shfl_down(c, 1 << lvl, 64);
      c = zmul(tree + lvl * 1024, c) ^ o;
    }
    if (lane == 0) out[w] = c;
  }
}

template <int NCH>
__global__ void __launch_bounds__(256) probe_coal(const uint8_t* buf, uint64_t nwin, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
  for (uint64_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)); w < nwin;
       w += nwaves) {
    const uint8_t* base = buf + w * (1024ull * NCH) + lane * 16;
    uint32_t x = 0;
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + q * 1024));
      x ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    for (int o = 32; o; o >>= 1) x ^= __shfl_down(x, o, 64);
    if (lane == 0) out[w] = x;
  }
}

// load ceiling: same access pattern, XOR of the words, no tables
template <int LB>
__global__ void __launch_bounds__(256) probe(const uint8_t* buf, uint64_t nwin, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
  for (uint64_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)); w < nwin;
       w += nwaves) {
    const u32x4* p = reinterpret_cast<const u32x4*>(buf + w * (64ull * LB) + lane * LB);
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < LB / 16; ++j) {
      const u32x4 v = __builtin_nontemporal_load(p + j);
      x ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    for (int o = 32; o; o >>= 1) x ^= __shfl_down(x, o, 64);
    if (lane == 0) out[w] = x;
  }
}

static uint32_t raw_crc_cpu(const uint8_t* d, size_t n) {
  uint32_t c = 0;
  for (size_t i = 0; i < n; ++i) {
    c ^= d[i];
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ crc::kPoly : c >> 1;
  }
  return c;
}

template <int R, int SL, int CH, int LB>
std::vector<uint32_t> make_tables() {
  std::vector<uint32_t> h(lds_words<R, SL>());
  // slicing-by-SL tables: s[j] advances a byte with j more bytes after it in the SL-byte group
  crc::ByteTable t[8];
  t[0] = crc::make_t0();
  for (int j = 1; j < 8; ++j)
    for (int i = 0; i < 256; ++i) t[j].t[i] = (t[j - 1].t[i] >> 8) ^ t[0].t[t[j - 1].t[i] & 0xFFu];
  for (int j = 0; j < SL; ++j)
    for (int v = 0; v < 256; ++v)
      for (int r = 0; r < R; ++r) h[(j * 256 + v) * R + r] = t[j].t[v];
  crc::to_tables(crc::zeros(LB / CH), &h[slice_words<R, SL>()]);
  for (int l = 0; l < 6; ++l)
    crc::to_tables(crc::zeros(static_cast<uint64_t>(LB) << l), &h[slice_words<R, SL>() + (1 + l) * 1024]);
  return h;
}

static uint8_t* g_buf = nullptr;
static std::vector<uint8_t> g_host_sample;  // first 256 KiB
static const uint64_t kBytes = 4ull << 30;
static uint32_t* g_out = nullptr;
static int g_cus = 256;

template <int R, int CH, int LB, int SL>
void run(const char* name) {
  auto h = make_tables<R, SL, CH, LB>();
  uint32_t* dt;
  CHECK(hipMalloc(&dt, h.size() * 4));
  CHECK(hipMemcpy(dt, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const uint64_t win = 64ull * LB, nwin = kBytes / win;
  auto k = crc_var<R, CH, LB, SL>;
  const size_t shm = h.size() * 4;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(shm)));
  // correctness on the first windows
  hipLaunchKernelGGL(k, dim3(g_cus * 2), dim3(256), shm, 0, g_buf, nwin, dt, g_out);
  CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> got(4);
  CHECK(hipMemcpy(got.data(), g_out, 16, hipMemcpyDeviceToHost));
  bool ok = true;
  for (int i = 0; i < 4; ++i) ok &= got[i] == raw_crc_cpu(g_host_sample.data() + i * win, win);
  printf("%-28s lds=%6zu B ok=%d  GB/s by blocks/CU:", name, shm, ok ? 1 : 0);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int bpc : {1, 2, 3, 4, 6, 8}) {
    if (shm * bpc > 160 * 1024) {
      printf("      -");
      continue;
    }
    hipLaunchKernelGGL(k, dim3(g_cus * bpc), dim3(256), shm, 0, g_buf, nwin, dt, g_out);
    CHECK(hipEventRecord(a));
    for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k, dim3(g_cus * bpc), dim3(256), shm, 0, g_buf, nwin, dt, g_out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf(" %6.0f", kBytes / (ms / 5 * 1e-3) / 1e9);
  }
  printf("\n");
  fflush(stdout);
  CHECK(hipFree(dt));
}

template <int R, int NCH>
void run_coal(const char* name) {
  // tables: slicing-by-4 (R copies), Z_1024 join, tree Z_{16 * 2^t}
  std::vector<uint32_t> h(lds_words<R, 4>());
  crc::Slice4 sl = crc::make_slice4();
  for (int j = 0; j < 4; ++j)
    for (int v = 0; v < 256; ++v)
      for (int r = 0; r < R; ++r) h[(j * 256 + v) * R + r] = sl.s[j].t[v];
  crc::to_tables(crc::zeros(1024), &h[slice_words<R, 4>()]);
  for (int l = 0; l < 6; ++l) crc::to_tables(crc::zeros(16ull << l), &h[slice_words<R, 4>() + (1 + l) * 1024]);
  uint32_t* dt;
  CHECK(hipMalloc(&dt, h.size() * 4));
  CHECK(hipMemcpy(dt, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const uint64_t win = 1024ull * NCH, nwin = kBytes / win;
  auto k = crc_coal<R, NCH>;
  const size_t shm = h.size() * 4;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(shm)));
  hipLaunchKernelGGL(k, dim3(g_cus * 2), dim3(256), shm, 0, g_buf, nwin, dt, g_out);
  CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> got(4);
  CHECK(hipMemcpy(got.data(), g_out, 16, hipMemcpyDeviceToHost));
  bool ok = true;
  for (int i = 0; i < 4; ++i) ok &= got[i] == raw_crc_cpu(g_host_sample.data() + i * win, win);
  printf("%-28s lds=%6zu B ok=%d  GB/s by blocks/CU:", name, shm, ok ? 1 : 0);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int bpc : {1, 2, 3, 4, 6, 8}) {
    if (shm * bpc > 160 * 1024) {
      printf("      -");
      continue;
    }
    hipLaunchKernelGGL(k, dim3(g_cus * bpc), dim3(256), shm, 0, g_buf, nwin, dt, g_out);
    CHECK(hipEventRecord(a));
    for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k, dim3(g_cus * bpc), dim3(256), shm, 0, g_buf, nwin, dt, g_out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf(" %6.0f", kBytes / (ms / 5 * 1e-3) / 1e9);
  }
  printf("\n");
  fflush(stdout);
  CHECK(hipFree(dt));
}

template <int NCH, int GROUP, int BLOCK>
void run_big(const char* name) {
  std::vector<uint32_t> h(kBigWords);
  crc::Slice4 sl = crc::make_slice4();
  for (int j = 0; j < 4; ++j)
    for (int v = 0; v < 256; ++v)
      for (int r = 0; r < 32; ++r) h[(j * 256 + v) * 32 + r] = sl.s[j].t[v];
  crc::to_tables(crc::zeros(1024), &h[kBigSliceWords]);
  for (int l = 0; l < 6; ++l) crc::to_tables(crc::zeros(16ull << l), &h[kBigSliceWords + (1 + l) * 1024]);
  uint32_t* dt;
  CHECK(hipMalloc(&dt, h.size() * 4));
  CHECK(hipMemcpy(dt, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const uint64_t win = 1024ull * NCH, nwin = kBytes / win;
  auto k = crc_big<NCH, GROUP, BLOCK>;
  const size_t shm = h.size() * 4;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(shm)));
  hipLaunchKernelGGL(k, dim3(g_cus), dim3(BLOCK), shm, 0, g_buf, nwin, dt, g_out);
  CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> got(4);
  CHECK(hipMemcpy(got.data(), g_out, 16, hipMemcpyDeviceToHost));
  bool ok = true;
  for (int i = 0; i < 4; ++i) ok &= got[i] == raw_crc_cpu(g_host_sample.data() + i * win, win);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(g_cus), dim3(BLOCK), shm, 0, g_buf, nwin, dt, g_out);
  CHECK(hipEventRecord(a));
  for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k, dim3(g_cus), dim3(BLOCK), shm, 0, g_buf, nwin, dt, g_out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  printf("%-36s lds=%6zu B ok=%d  %6.0f GB/s (1 block/CU)\n", name, shm, ok ? 1 : 0, kBytes / (ms / 5 * 1e-3) / 1e9);
  fflush(stdout);
  CHECK(hipFree(dt));
}

template <int NCH>
void run_probe_coal() {
  const uint64_t nwin = kBytes / (1024ull * NCH);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  printf("probe coalesced NCH=%-2d                      GB/s by blocks/CU:", NCH);
  for (int bpc : {1, 2, 3, 4, 6, 8}) {
    hipLaunchKernelGGL(probe_coal<NCH>, dim3(g_cus * bpc), dim3(256), 0, 0, g_buf, nwin, g_out);
    CHECK(hipEventRecord(a));
    for (int it = 0; it < 5; ++it)
      hipLaunchKernelGGL(probe_coal<NCH>, dim3(g_cus * bpc), dim3(256), 0, 0, g_buf, nwin, g_out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf(" %6.0f", kBytes / (ms / 5 * 1e-3) / 1e9);
  }
  printf("\n");
  fflush(stdout);
}

template <int LB>
void run_probe() {
  const uint64_t nwin = kBytes / (64ull * LB);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  printf("probe LB=%-3d (no tables)                    GB/s by blocks/CU:", LB);
  for (int bpc : {1, 2, 3, 4, 6, 8}) {
    hipLaunchKernelGGL(probe<LB>, dim3(g_cus * bpc), dim3(256), 0, 0, g_buf, nwin, g_out);
    CHECK(hipEventRecord(a));
    for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(probe<LB>, dim3(g_cus * bpc), dim3(256), 0, 0, g_buf, nwin, g_out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf(" %6.0f", kBytes / (ms / 5 * 1e-3) / 1e9);
  }
  printf("\n");
  fflush(stdout);
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  g_cus = prop.multiProcessorCount;
  CHECK(hipMalloc(&g_buf, kBytes));
  CHECK(hipMalloc(&g_out, (kBytes / 2048) * 4));
  g_host_sample.resize(256 << 10);
  uint64_t s = 12345;
  for (auto& x : g_host_sample) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    x = static_cast<uint8_t>(s >> 56);
  }
  for (uint64_t off = 0; off < kBytes; off += g_host_sample.size())
    CHECK(hipMemcpy(g_buf + off, g_host_sample.data(), g_host_sample.size(), hipMemcpyHostToDevice));
  printf("CUs %d, buffer %llu GiB\n", g_cus, (unsigned long long)(kBytes >> 30));
  run_probe<64>();
  run_probe_coal<2>();
  run_probe_coal<4>();
  run_probe_coal<8>();
  run_big<8, 8, 1024>("big R32 NCH8 G8 B1024");
  run_big<16, 8, 1024>("big R32 NCH16 G8 B1024");
  run_big<32, 8, 1024>("big R32 NCH32 G8 B1024");
  run_big<16, 4, 1024>("big R32 NCH16 G4 B1024");
  run_big<16, 8, 512>("big R32 NCH16 G8 B512");
  run_big<32, 16, 1024>("big R32 NCH32 G16 B1024");
  run_big<64, 8, 1024>("big R32 NCH64 G8 B1024");
  run_coal<1, 4>("coalesced R1 NCH4");
  run_coal<4, 4>("coalesced R4 NCH4");
  run_coal<1, 8>("coalesced R1 NCH8");
  run_coal<4, 8>("coalesced R4 NCH8");
  run_coal<1, 2>("coalesced R1 NCH2");
  run_coal<2, 4>("coalesced R2 NCH4");
  run<4, 4, 64, 4>("R4 CH4 LB64 S4 (product)");
  run<1, 4, 64, 4>("R1 CH4 LB64 S4");
  run<4, 2, 64, 4>("R4 CH2 LB64 S4");
  return 0;
}
