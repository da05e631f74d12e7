// Kernel lab: times encode-kernel variants against a no-math probe with the
// same HBM access pattern, interleaved in one process (cdna_hip_programming.md
// §5.4 rule 24). Dev tool, not part of the product.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/kernel_lab.hip -o build/kernel_lab
#include "../lambdafs_amd/csrc/hrs_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

using namespace hrs;

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

namespace lab {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void ld(const uint8_t* p, int lane, uint32_t (&w)[8]) {
  const u32x4* a = reinterpret_cast<const u32x4*>(p + lane * 16);
  const u32x4* b = reinterpret_cast<const u32x4*>(p + 1024 + lane * 16);
  u32x4 x, y;
  if (NT) {
    x = __builtin_nontemporal_load(a);
    y = __builtin_nontemporal_load(b);
  } else {
    x = *a;
    y = *b;
  }
  w[0] = x[0]; w[1] = x[1]; w[2] = x[2]; w[3] = x[3];
  w[4] = y[0]; w[5] = y[1]; w[6] = y[2]; w[7] = y[3];
}

template <bool NT>
__device__ __forceinline__ void st(uint8_t* p, int lane, const uint32_t (&w)[8]) {
  u32x4* a = reinterpret_cast<u32x4*>(p + lane * 16);
  u32x4* b = reinterpret_cast<u32x4*>(p + 1024 + lane * 16);
  u32x4 x = {w[0], w[1], w[2], w[3]}, y = {w[4], w[5], w[6], w[7]};
  if (NT) {
    __builtin_nontemporal_store(x, a);
    __builtin_nontemporal_store(y, b);
  } else {
    *a = x;
    *b = y;
  }
}

// Same decomposition, no GF math: out_o = XOR of the rows (pattern ceiling).
template <int K, int P, bool NT>
__global__ void __launch_bounds__(kBlockThreads) probe_kernel(const RowArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  for (uint64_t t = wave_id_in_grid(); t < a.ntasks; t += nwaves) {
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < K; ++r) {
      uint32_t w[8];
      ld<NT>(a.in[r] + stripe * a.in_stride + off, lane, w);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] ^= w[q];
    }
#pragma unroll
    for (int o = 0; o < P; ++o) {
      uint32_t v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = acc[q] + o;
      st<NT>(a.out[o] + stripe * a.out_stride + off, lane, v);
    }
  }
}

// The product's static encode body with load/store policy knobs.
template <int K, int P, bool NT>
__global__ void __launch_bounds__(kBlockThreads) encode_var_kernel(const RowArgs a) {
  constexpr StaticPlan<K, P, gf::EncodeMatrix<K, P>> plan{};
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  for (uint64_t t = wave_id_in_grid(); t < a.ntasks; t += nwaves) {
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
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
      uint32_t w[8];
      ld<NT>(a.in[r] + stripe * a.in_stride + off, lane, w);
      bitslice(w);
#pragma unroll
      for (int o = 0; o < P; ++o)
#pragma unroll
        for (int q = 0; q < 8; ++q)
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if ((plan.mask[o][r][q] >> i) & 1) {
              if (has[o][q]) {
                acc[o][q] = xor3(acc[o][q], pend[o][q], w[i]);
                has[o][q] = false;
              } else {
                pend[o][q] = w[i];
                has[o][q] = true;
              }
            }
    }
#pragma unroll
    for (int o = 0; o < P; ++o)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (has[o][q]) acc[o][q] ^= pend[o][q];
#pragma unroll
    for (int o = 0; o < P; ++o) {
      bitslice(acc[o]);
      st<NT>(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
    }
  }
}

// The round-1 runtime kernel (one row of prefetch), kept for A/B.
template <int NOUT>
__global__ void __launch_bounds__(kBlockThreads) bitsliced_old_kernel(const RowArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  for (uint64_t t = wave_id_in_grid(); t < a.ntasks; t += nwaves) {
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    const uint64_t in_base = stripe * a.in_stride + off;
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
    uint32_t cur[8];
    load_row(a.in[0] + in_base, lane, cur);
    for (int r = 0; r < a.nin; ++r) {
      uint32_t nxt[8];
      if (r + 1 < a.nin) load_row(a.in[r + 1] + in_base, lane, nxt);
      bitslice(cur);
      uint32_t c[NOUT];
#pragma unroll
      for (int o = 0; o < NOUT; ++o) c[o] = static_cast<uint8_t>(a.cw[r] >> (8 * o));
#pragma unroll
      for (int b = 0; b < 8; ++b) {
#pragma unroll
        for (int o = 0; o < NOUT; ++o) {
          if ((c[o] >> b) & 1u) {
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[o][q] ^= cur[q];
          }
        }
        if (b < 7) xtime(cur);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) cur[q] = nxt[q];
    }
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      bitslice(acc[o]);
      store_row(a.out[o] + stripe * a.out_stride + off, lane, acc[o]);
    }
  }
}

// Classic grid-stride float4 copy (the MI355X_MICROARCH.md copy-peak shape).
template <bool NT>
__global__ void __launch_bounds__(256) copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
    else dst[i] = src[i];
  }
}
typedef __attribute__((address_space(3))) void lds_void;

// Probe with W-byte windows: lane owns W/64 bytes of each row as W/1024 16-B pieces
// (each piece-instruction a coalesced 1 KiB wave access).
template <int K, int P, int W>
__global__ void __launch_bounds__(kBlockThreads) probe_wide_kernel(const RowArgs a, uint64_t nwin_w) {
  constexpr int NP = W / 1024;
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  const uint64_t ntasks = nwin_w * (a.ntasks / a.nwin);
  for (uint64_t t = wave_id_in_grid(); t < ntasks; t += nwaves) {
    const uint64_t stripe = t / nwin_w;
    const uint64_t off = (t - stripe * nwin_w) * W;
    u32x4 acc[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) acc[j] = u32x4{0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int j = 0; j < NP; ++j)
        acc[j] ^= __builtin_nontemporal_load(
            reinterpret_cast<const u32x4*>(a.in[r] + stripe * a.in_stride + off + j * 1024 + lane * 16));
#pragma unroll
    for (int o = 0; o < P; ++o)
#pragma unroll
      for (int j = 0; j < NP; ++j)
        __builtin_nontemporal_store(acc[j] + (uint32_t)o,
                                    reinterpret_cast<u32x4*>(a.out[o] + stripe * a.out_stride + off + j * 1024 + lane * 16));
  }
}

// Probe with rows staged by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction), then read back with ds_read_b128: is the DMA read path faster?
template <int K, int P>
__global__ void __launch_bounds__(kBlockThreads) probe_glds_kernel(const RowArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  uint8_t* mine = smem + (threadIdx.x >> 6) * K * kWindowBytes;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  for (uint64_t t = wave_id_in_grid(); t < a.ntasks; t += nwaves) {
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const uint8_t* g = a.in[r] + stripe * a.in_stride + off + lane * 16;
      __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)(mine + r * kWindowBytes), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(g + 1024), (lds_void*)(mine + r * kWindowBytes + 1024), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x3F70);  // vmcnt(0): this wave's DMA has landed
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const uint4 x = *reinterpret_cast<const uint4*>(mine + r * kWindowBytes + lane * 16);
      const uint4 y = *reinterpret_cast<const uint4*>(mine + r * kWindowBytes + 1024 + lane * 16);
      acc[0] ^= x.x; acc[1] ^= x.y; acc[2] ^= x.z; acc[3] ^= x.w;
      acc[4] ^= y.x; acc[5] ^= y.y; acc[6] ^= y.z; acc[7] ^= y.w;
    }
#pragma unroll
    for (int o = 0; o < P; ++o) {
      uint32_t v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = acc[q] + o;
      st<true>(a.out[o] + stripe * a.out_stride + off, lane, v);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) before the slot is refilled
  }
}

// Register-load probe that prefetches the next task's rows while finishing the current one.
template <int K, int P>
__global__ void __launch_bounds__(kBlockThreads) probe_prefetch_kernel(const RowArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  uint64_t t = wave_id_in_grid();
  if (t >= a.ntasks) return;
  uint32_t cur[K][8];
  {
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
#pragma unroll
    for (int r = 0; r < K; ++r) ld<true>(a.in[r] + stripe * a.in_stride + off, lane, cur[r]);
  }
  for (; t < a.ntasks; t += nwaves) {
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] ^= cur[r][q];
    const uint64_t tn = t + nwaves;
    if (tn < a.ntasks) {
      const uint64_t sn = tn / a.nwin;
      const uint64_t on = (tn - sn * a.nwin) * kWindowBytes;
#pragma unroll
      for (int r = 0; r < K; ++r) ld<true>(a.in[r] + sn * a.in_stride + on, lane, cur[r]);
    }
#pragma unroll
    for (int o = 0; o < P; ++o) {
      uint32_t v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = acc[q] + o;
      st<true>(a.out[o] + stripe * a.out_stride + off, lane, v);
    }
  }
}
}  // namespace lab

int main(int argc, char** argv) {
  const int S = argc > 1 ? atoi(argv[1]) : 1024;
  const size_t L = 1 << 20;
  const int k = 10, p = 4, n = 14;
  const int rounds = argc > 2 ? atoi(argv[2]) : 15;
  uint8_t* buf;
  const size_t buf_bytes = (size_t)S * n * (L + 65536 + 2048);
  CK(hipMalloc(&buf, buf_bytes));
  CK(hipMemset(buf, 0x3c, buf_bytes));
  uint8_t* copy_dst;
  CK(hipMalloc(&copy_dst, (size_t)S * 7 * L + (size_t)S * (65536 + 2048)));
  RowArgs a{};
  for (int c = 0; c < k; ++c) a.in[c] = buf + (size_t)(p + c) * L;
  for (int r = 0; r < p; ++r) a.out[r] = buf + (size_t)r * L;
  a.in_stride = a.out_stride = (uint64_t)n * L;
  a.len = L;
  a.nwin = L / kWindowBytes;
  a.ntasks = a.nwin * S;
  a.nin = k;
  a.nout = p;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));

  struct Var {
    std::string name;
    std::function<void()> run;
    double bytes;
    std::vector<float> ms;
  };
  auto occ = [&](const void* f) {
    int b = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, f, kBlockThreads, 0));
    return b;
  };
  const double enc_bytes = (double)(k + p) * L * S;
  std::vector<Var> vars;
  auto add_grid = [&](const char* nm, auto kern, unsigned grid) {
    vars.push_back({std::string(nm) + " grid=" + std::to_string(grid),
                    [=]() { hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlockThreads), 0, 0, a); }, enc_bytes, {}});
  };
  const unsigned all_tasks = (unsigned)((a.ntasks + kWavesPerBlock - 1) / kWavesPerBlock);
  const char* which = argc > 3 ? argv[3] : "sweep";
  if (std::string(which) == "sweep") {
    for (unsigned g : {256u, 512u, 768u, 1024u, 2048u})
      add_grid("product encode_static NT", encode_static_kernel<10, 4>, g);
    for (unsigned g : {512u, 1024u}) add_grid("lab encode NT", lab::encode_var_kernel<10, 4, true>, g);
    add_grid("probe10x4 NT", lab::probe_kernel<10, 4, true>, 512);
  }
  vars.push_back({"hipMemcpyAsync D2D 7/14 of batch", [=]() {
                    (void)hipMemcpyAsync(copy_dst, buf, (size_t)S * 7 * L, hipMemcpyDeviceToDevice, 0);
                  }, 2.0 * S * 7 * L, {}});
  {
    RowArgs d = a;  // decode 1 erasure through the runtime kernels
    d.nout = 1;
    for (int c = 0; c < k; ++c) set_coef(d, 0, c, (uint8_t)(17 * c + 3));
    d.out[0] = copy_dst;
    d.out_stride = L;
    auto knew = bitsliced_kernel<1, 12>;
    auto kold = lab::bitsliced_old_kernel<1>;
    for (unsigned g : {512u, 768u, 1024u, 2048u}) {
      vars.push_back({"product bitsliced<1,12> (decode) grid=" + std::to_string(g), [=]() {
                        hipLaunchKernelGGL(knew, dim3(g), dim3(kBlockThreads), 0, 0, d);
                      }, (double)(k + 1) * L * S, {}});
      vars.push_back({"old bitsliced<1> (decode) grid=" + std::to_string(g), [=]() {
                        hipLaunchKernelGGL(kold, dim3(g), dim3(kBlockThreads), 0, 0, d);
                      }, (double)(k + 1) * L * S, {}});
    }
  }
  if (std::string(which) == "sweep") {
    // classic copy at several grids: 7/14 of the batch
    const size_t nvec = (size_t)S * 7 * L / 16;
    auto cnt = lab::copy_kernel<true>;
    auto cpl = lab::copy_kernel<false>;
    for (unsigned g : {1024u, 2048u, 4096u, 16384u}) {
      vars.push_back({"classic copy NT grid=" + std::to_string(g), [=]() {
                        hipLaunchKernelGGL(cnt, dim3(g), dim3(256), 0, 0, (const lab::u32x4*)buf, (lab::u32x4*)copy_dst, nvec);
                      }, 2.0 * S * 7 * L, {}});
      vars.push_back({"classic copy plain grid=" + std::to_string(g), [=]() {
                        hipLaunchKernelGGL(cpl, dim3(g), dim3(256), 0, 0, (const lab::u32x4*)buf, (lab::u32x4*)copy_dst, nvec);
                      }, 2.0 * S * 7 * L, {}});
    }
    // decode right after encode, reading parity location 3 the encode just wrote
    RowArgs d = a;
    d.nout = 1;
    const int locs[10] = {3, 5, 6, 7, 8, 9, 10, 11, 12, 13};
    for (int c = 0; c < k; ++c) {
      d.in[c] = buf + (size_t)locs[c] * L;
      set_coef(d, 0, c, (uint8_t)(17 * c + 3));
    }
    d.out[0] = copy_dst;
    d.out_stride = L;
    auto kenc = encode_static_kernel<10, 4>;
    auto kdec = bitsliced_kernel<1, 12>;
    for (unsigned g : {512u, 768u}) {
      vars.push_back({"PAIR encode+decode(loc3) dec grid=" + std::to_string(g), [=]() {
                        hipLaunchKernelGGL(kenc, dim3(512), dim3(kBlockThreads), 0, 0, a);
                        hipLaunchKernelGGL(kdec, dim3(g), dim3(kBlockThreads), 0, 0, d);
                      }, enc_bytes + (double)(k + 1) * L * S, {}});
      vars.push_back({"decode(loc3) alone grid=" + std::to_string(g), [=]() {
                        hipLaunchKernelGGL(kdec, dim3(g), dim3(kBlockThreads), 0, 0, d);
                      }, (double)(k + 1) * L * S, {}});
    }
  }
  if (std::string(which) == "pitch") {
    // row pitch sweep: rows at buf + (stripe * n + r) * (L + pad); buffer sized for the max pad
    auto kenc = encode_static_kernel<10, 4>;
    auto kdec = bitsliced_kernel<1, 12>;
    auto kread = lab::probe_kernel<10, 1, true>;
    for (size_t pad : {(size_t)0, (size_t)256, (size_t)2048, (size_t)4096, (size_t)6144, (size_t)8192,
                       (size_t)12288, (size_t)65536 + 2048}) {
      const size_t P = L + pad;
      if ((size_t)S * n * P > (size_t)S * n * L + (size_t)S * n * (65536 + 2048)) continue;
      RowArgs e = a;
      for (int c = 0; c < k; ++c) e.in[c] = buf + (size_t)(p + c) * P;
      for (int r = 0; r < p; ++r) e.out[r] = buf + (size_t)r * P;
      e.in_stride = e.out_stride = (uint64_t)n * P;
      RowArgs d = e;
      d.nout = 1;
      for (int c = 0; c < k; ++c) set_coef(d, 0, c, (uint8_t)(17 * c + 3));
      d.out[0] = copy_dst;
      d.out_stride = P;
      const std::string t = " pad=" + std::to_string(pad);
      vars.push_back({"encode grid=512" + t, [=]() { hipLaunchKernelGGL(kenc, dim3(512), dim3(kBlockThreads), 0, 0, e); },
                      enc_bytes, {}});
      vars.push_back({"decode<1,12> grid=512" + t, [=]() { hipLaunchKernelGGL(kdec, dim3(512), dim3(kBlockThreads), 0, 0, d); },
                      (double)(k + 1) * L * S, {}});
      vars.push_back({"probe read10x1 grid=512" + t, [=]() { hipLaunchKernelGGL(kread, dim3(512), dim3(kBlockThreads), 0, 0, d); },
                      (double)(k + 1) * L * S, {}});
    }
  }
  if (std::string(which) == "glds") {
    auto pg = lab::probe_glds_kernel<10, 4>;
    auto pg1 = lab::probe_glds_kernel<10, 1>;
    auto pr = lab::probe_kernel<10, 4, true>;
    auto pr1 = lab::probe_kernel<10, 1, true>;
    auto pp = lab::probe_prefetch_kernel<10, 4>;
    const size_t shm = (size_t)kWavesPerBlock * 10 * kWindowBytes;  // 80 KiB per block
    CK(hipFuncSetAttribute((const void*)pg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    CK(hipFuncSetAttribute((const void*)pg1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    RowArgs d = a;
    d.out[0] = copy_dst;
    d.out_stride = L;
    for (unsigned g : {256u, 512u}) {
      const std::string t = " grid=" + std::to_string(g);
      vars.push_back({"glds probe 10x4" + t, [=]() { hipLaunchKernelGGL(pg, dim3(g), dim3(kBlockThreads), shm, 0, a); }, enc_bytes, {}});
      vars.push_back({"reg probe 10x4" + t, [=]() { hipLaunchKernelGGL(pr, dim3(g), dim3(kBlockThreads), 0, 0, a); }, enc_bytes, {}});
      vars.push_back({"reg prefetch probe 10x4" + t, [=]() { hipLaunchKernelGGL(pp, dim3(g), dim3(kBlockThreads), 0, 0, a); }, enc_bytes, {}});
      vars.push_back({"glds probe 10x1" + t, [=]() { hipLaunchKernelGGL(pg1, dim3(g), dim3(kBlockThreads), shm, 0, d); }, (double)(k + 1) * L * S, {}});
      vars.push_back({"reg probe 10x1" + t, [=]() { hipLaunchKernelGGL(pr1, dim3(g), dim3(kBlockThreads), 0, 0, d); }, (double)(k + 1) * L * S, {}});
    }
    auto pe = encode_static_kernel<10, 4>;
    vars.push_back({"product encode grid=512", [=]() {
                      hipLaunchKernelGGL(pe, dim3(512), dim3(kBlockThreads), 0, 0, a); }, enc_bytes, {}});
  }
  if (std::string(which) == "wide") {
    auto w2 = lab::probe_wide_kernel<10, 4, 2048>;
    auto w4 = lab::probe_wide_kernel<10, 4, 4096>;
    auto w8 = lab::probe_wide_kernel<10, 4, 8192>;
    auto w1 = lab::probe_wide_kernel<10, 4, 1024>;
    auto pe = encode_static_kernel<10, 4>;
    for (unsigned g : {256u, 512u, 1024u}) {
      const std::string t = " grid=" + std::to_string(g);
      vars.push_back({"wide probe W=1K" + t, [=]() { hipLaunchKernelGGL(w1, dim3(g), dim3(kBlockThreads), 0, 0, a, (uint64_t)(L / 1024)); }, enc_bytes, {}});
      vars.push_back({"wide probe W=2K" + t, [=]() { hipLaunchKernelGGL(w2, dim3(g), dim3(kBlockThreads), 0, 0, a, (uint64_t)(L / 2048)); }, enc_bytes, {}});
      vars.push_back({"wide probe W=4K" + t, [=]() { hipLaunchKernelGGL(w4, dim3(g), dim3(kBlockThreads), 0, 0, a, (uint64_t)(L / 4096)); }, enc_bytes, {}});
      vars.push_back({"wide probe W=8K" + t, [=]() { hipLaunchKernelGGL(w8, dim3(g), dim3(kBlockThreads), 0, 0, a, (uint64_t)(L / 8192)); }, enc_bytes, {}});
    }
    vars.push_back({"product encode grid=512", [=]() { hipLaunchKernelGGL(pe, dim3(512), dim3(kBlockThreads), 0, 0, a); }, enc_bytes, {}});
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vars) v.run();  // warm
  CK(hipDeviceSynchronize());
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
    printf("%-48s median %8.3f ms  min %8.3f ms  %7.1f GB/s (median)\n", v.name.c_str(), med, mn,
           v.bytes / (med * 1e-3) / 1e9);
  }
  return 0;
}
