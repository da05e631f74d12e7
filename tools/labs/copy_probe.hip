// The classic STREAM-copy shape of MI355X_MICROARCH.md ("6.29 TB/s measured
// (float4 copy)"): a grid-stride float4 copy of one large buffer into another,
// timed with HIP events; rate = read + write bytes / time. Run once per round
// on the pool to settle what "the HBM ceiling" is on these boxes (VERDICT r1
// item 8). Also the same loop with nontemporal accesses, as the codec uses.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void copy_f4(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x)
    b[i] = a[i];
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void copy_f4_nt(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  const f32x4* x = reinterpret_cast<const f32x4*>(a);
  f32x4* y = reinterpret_cast<f32x4*>(b);
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(&x[i]), &y[i]);
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const size_t bytes = size_t(4) << 30;  // 4 GiB per buffer: far past the 256 MiB Infinity Cache
  const size_t n = bytes / sizeof(float4);
  float4 *a = nullptr, *b = nullptr;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("{\"probe\": \"float4 grid-stride copy\", \"bytes_per_buffer\": %zu, \"cus\": %d, \"runs\": [", bytes, cus);
  const int blocks_per_cu[] = {4, 8, 16};
  bool first = true;
  for (int nt = 0; nt < 2; ++nt)
    for (int bpc : blocks_per_cu) {
      const unsigned grid = static_cast<unsigned>(bpc * cus);
      auto launch = [&] {
        if (nt)
          hipLaunchKernelGGL(copy_f4_nt, dim3(grid), dim3(256), 0, 0, a, b, n);
        else
          hipLaunchKernelGGL(copy_f4, dim3(grid), dim3(256), 0, 0, a, b, n);
      };
      launch();
      CK(hipDeviceSynchronize());
      float best = 1e30f, sum = 0;
      const int reps = 10;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(t0, 0));
        launch();
        CK(hipEventRecord(t1, 0));
        CK(hipEventSynchronize(t1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, t0, t1));
        best = ms < best ? ms : best;
        sum += ms;
      }
      printf("%s{\"kernel\": \"%s\", \"grid\": %u, \"block\": 256, \"mean_ms\": %.4f, \"best_ms\": %.4f, "
             "\"mean_TBps\": %.3f, \"best_TBps\": %.3f}",
             first ? "" : ", ", nt ? "copy_f4_nt" : "copy_f4", grid, sum / reps, best,
             2.0 * bytes / (sum / reps * 1e-3) / 1e12, 2.0 * bytes / (best * 1e-3) / 1e12);
      first = false;
    }
  printf("]}\n");
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
