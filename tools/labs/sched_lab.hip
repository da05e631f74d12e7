// Task-order lab for the headline encode (encode_static_kernel<10,4>, RS(10,4)
// 1 MiB cells x 1024 stripes, bench.py's workload): does the block-range
// schedule that made the fastest 1:1 copy (tools/copy_lab.hip, +5-7 % over
// grid-stride) also speed up the coding kernel and its no-math pattern?
// The kernel body is the product's (encode_row_acc / bitslice / load_row /
// store_row from hrs_kernels.hip); only the window -> wave assignment and the
// block shape change. Interleaved rep by rep, median of `reps`; every
// variant's parity is compared with the product kernel's.
//
// Orders (task t = stripe * nwin + window):
//   gs   wave w takes t = w, w + W, ...            (the product's order)
//   br   block b owns tasks [b*per, (b+1)*per), its waves interleaved
//   wr   wave w owns tasks [w*per, (w+1)*per)
//   gsx  gs with blocks renumbered XCD-major (the blocks one XCD runs
//        take consecutive tasks: logical id = (b % 8) * (G / 8) + b / 8)
// Block shapes: 256 threads x {2,3,4,8} per CU, 512 x 1, 1024 x {1,2}.
// Usage: sched_lab [reps]   (one JSON line per variant)
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/sched_lab.hip -o tools/sched_lab
#include "../lambdafs_amd/csrc/hrs_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace hrs;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

namespace lab {

enum { GS = 0, BR = 1, WR = 2, GSX = 3 };

// First task, step and end of the calling wave under order O.
template <int O>
__device__ __forceinline__ void task_range(uint64_t ntasks, uint64_t& t, uint64_t& step, uint64_t& end) {
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * wpb;
  if constexpr (O == GS || O == GSX) {
    uint32_t b = blockIdx.x;
    if constexpr (O == GSX) {
      const uint32_t per_xcd = gridDim.x / 8;  // host launches multiples of 8 blocks
      b = (b % 8) * per_xcd + b / 8;
    }
    t = static_cast<uint64_t>(b) * wpb + w;
    step = nw;
    end = ntasks;
  } else if constexpr (O == BR) {
    const uint64_t per = (ntasks + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = per * blockIdx.x;
    t = lo + w;
    step = wpb;
    end = lo + per < ntasks ? lo + per : ntasks;
  } else {
    const uint64_t per = (ntasks + nw - 1) / nw;
    const uint64_t lo = per * (static_cast<uint64_t>(blockIdx.x) * wpb + w);
    t = lo;
    step = 1;
    end = lo + per < ntasks ? lo + per : ntasks;
  }
}

template <int K, int P, int O, int B>
__global__ void __launch_bounds__(B) enc_kernel(const RowArgs a) {
  const int lane = threadIdx.x & 63;
  uint64_t t, step, end;
  task_range<O>(a.ntasks, t, step, end);
  for (; t < end; t += step) {
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
      load_row(a.in[r] + stripe * a.in_stride + off, lane, w);
      bitslice(w);
      encode_row_acc<K, P, gf::EncodeMatrix<K, P>>(r, w, acc, pend, has);
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

// The same accesses without the math: all K rows loaded, XOR-folded, the
// fold (+o) stored to the P outputs (hrs_probe_rows schedule 0).
template <int K, int P, int O, int B>
__global__ void __launch_bounds__(B) pat_kernel(const RowArgs a) {
  const int lane = threadIdx.x & 63;
  uint64_t t, step, end;
  task_range<O>(a.ntasks, t, step, end);
  for (; t < end; t += step) {
    const uint64_t stripe = t / a.nwin;
    const uint64_t off = (t - stripe * a.nwin) * kWindowBytes;
    uint32_t w[K][8];
#pragma unroll
    for (int r = 0; r < K; ++r) load_row(a.in[r] + stripe * a.in_stride + off, lane, w[r]);
    uint32_t x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      x[q] = 0u;
#pragma unroll
      for (int r = 0; r < K; ++r) x[q] ^= w[r][q];
    }
#pragma unroll
    for (int o = 0; o < P; ++o) {
      uint32_t y[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) y[q] = x[q] + o;
      store_row(a.out[o] + stripe * a.out_stride + off, lane, y);
    }
  }
}

struct Variant {
  std::string name;
  void (*kern)(const RowArgs);
  int block;
  int per_cu;
  bool math;
  std::vector<float> ms;
};

template <int O, int B>
void add(std::vector<Variant>& v, const char* oname, int per_cu) {
  char nm[64];
  snprintf(nm, sizeof nm, "enc_%s_b%d_x%d", oname, B, per_cu);
  v.push_back({nm, enc_kernel<10, 4, O, B>, B, per_cu, true, {}});
  snprintf(nm, sizeof nm, "pat_%s_b%d_x%d", oname, B, per_cu);
  v.push_back({nm, pat_kernel<10, 4, O, B>, B, per_cu, false, {}});
}

template <int O>
void add_order(std::vector<Variant>& v, const char* oname) {
  add<O, 256>(v, oname, 2);
  add<O, 256>(v, oname, 3);
  add<O, 256>(v, oname, 4);
  add<O, 256>(v, oname, 8);
  add<O, 512>(v, oname, 1);
  add<O, 1024>(v, oname, 1);
  add<O, 1024>(v, oname, 2);
}

}  // namespace lab

int main(int argc, char** argv) {
  using namespace lab;
  const int reps = argc > 1 ? atoi(argv[1]) : 7;
  const int K = 10, P = 4, n = K + P;
  const uint64_t L = 1u << 20, S = 1024;
  const uint64_t bytes = S * n * L;
  uint8_t* buf = nullptr;
  CK(hipMalloc(&buf, bytes));
  {
    std::vector<uint64_t> h(L / 8);
    uint64_t z = 0x9E3779B97F4A7C15ull;
    for (uint64_t s = 0; s < S; ++s)
      for (int r = P; r < n; ++r) {
        for (auto& x : h) {
          z ^= z << 13, z ^= z >> 7, z ^= z << 17;
          x = z;
        }
        CK(hipMemcpy(buf + (s * n + r) * L, h.data(), L, hipMemcpyHostToDevice));
      }
  }
  RowArgs a{};
  for (int i = 0; i < K; ++i) a.in[i] = buf + (P + i) * L;
  for (int o = 0; o < P; ++o) a.out[o] = buf + o * L;
  a.in_stride = a.out_stride = n * L;
  a.len = L;
  a.nwin = L / kWindowBytes;
  a.ntasks = S * a.nwin;
  a.nin = K;
  a.nout = P;
  a.order = 1;  // the product kernel in its grid-stride order (hrs_device.hpp wave_tasks)
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));

  std::vector<Variant> vs;
  vs.push_back({"product_b256_x2", encode_static_kernel<10, 4>, kBlockThreads, 2, true, {}});
  add_order<GS>(vs, "gs");
  add_order<BR>(vs, "br");
  add_order<WR>(vs, "wr");
  add_order<GSX>(vs, "gsx");

  // reference parity: the product kernel (vs[0]), sampled stripes
  const uint64_t sample[] = {0, 1, 333, 512, 777, 1023};
  auto snap = [&](std::vector<uint8_t>& out) {
    out.resize(sizeof(sample) / sizeof(sample[0]) * P * L);
    size_t at = 0;
    for (uint64_t s : sample)
      for (int o = 0; o < P; ++o, at += L) CK(hipMemcpy(out.data() + at, buf + (s * n + o) * L, L, hipMemcpyDeviceToHost));
  };
  auto launch = [&](const Variant& v) {
    const unsigned g = static_cast<unsigned>(v.per_cu * cus);
    hipLaunchKernelGGL(v.kern, dim3(g), dim3(v.block), 0, 0, a);
    CK(hipGetLastError());
  };
  std::vector<uint8_t> want, got;
  CK(hipMemset(buf, 0, L));  // stripe 0's parity row 0 starts wrong
  launch(vs[0]);
  CK(hipDeviceSynchronize());
  snap(want);
  std::vector<int> ok(vs.size(), 1);
  for (size_t i = 0; i < vs.size(); ++i) {
    if (!vs[i].math) continue;
    for (uint64_t s : sample) CK(hipMemset(buf + s * n * L, 0, P * L));
    launch(vs[i]);
    CK(hipDeviceSynchronize());
    snap(got);
    ok[i] = memcmp(got.data(), want.data(), want.size()) == 0;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs) launch(v);  // warm
  CK(hipDeviceSynchronize());
  for (int r = 0; r < reps; ++r)
    for (auto& v : vs) {
      CK(hipEventRecord(e0, 0));
      launch(v);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  const double moved = static_cast<double>(S) * n * L;
  for (size_t i = 0; i < vs.size(); ++i) {
    auto& v = vs[i];
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    printf("{\"variant\": \"%s\", \"median_ms\": %.4f, \"min_ms\": %.4f, \"GBps\": %.1f, \"ok\": %s}\n",
           v.name.c_str(), med, v.ms[0], moved / 1e6 / med, v.math ? (ok[i] ? "true" : "false") : "null");
  }
  CK(hipFree(buf));
  return 0;
}
