// Cost of registering pageable host rows with HIP (hipHostRegister) per call,
// vs staging them through pinned memory with memcpy: decides whether the
// synchronous host-buffer calls (one 1 MiB-cell stripe per JNI call) could DMA
// straight from the caller's rows. Prints one JSON line per row size.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const int rows = 14;
  for (size_t len : {size_t(256) << 10, size_t(1) << 20, size_t(4) << 20}) {
    std::vector<void*> host(rows);
    for (auto& h : host) {
      h = aligned_alloc(4096, len);
      memset(h, 1, len);
    }
    void* dev = nullptr;
    void* pin = nullptr;
    if (hipMalloc(&dev, rows * len) != hipSuccess || hipHostMalloc(&pin, rows * len, 0) != hipSuccess) return 1;
    hipStream_t s;
    (void)hipStreamCreate(&s);
    double reg = 0, unreg = 0, dma_reg = 0, cpy = 0, dma_pin = 0;
    const int reps = 20;
    for (int it = 0; it < reps + 2; ++it) {
      double t0 = now_us();
      for (auto h : host)
        if (hipHostRegister(h, len, hipHostRegisterDefault) != hipSuccess) return 2;
      double t1 = now_us();
      for (int r = 0; r < rows; ++r) {
        void* dp = nullptr;
        (void)hipHostGetDevicePointer(&dp, host[r], 0);
        (void)hipMemcpyAsync(static_cast<char*>(dev) + r * len, host[r], len, hipMemcpyHostToDevice, s);
      }
      (void)hipStreamSynchronize(s);
      double t2 = now_us();
      for (auto h : host) (void)hipHostUnregister(h);
      double t3 = now_us();
      for (int r = 0; r < rows; ++r) memcpy(static_cast<char*>(pin) + r * len, host[r], len);
      double t4 = now_us();
      (void)hipMemcpyAsync(dev, pin, rows * len, hipMemcpyHostToDevice, s);
      (void)hipStreamSynchronize(s);
      double t5 = now_us();
      if (it >= 2) {
        reg += t1 - t0;
        dma_reg += t2 - t1;
        unreg += t3 - t2;
        cpy += t4 - t3;
        dma_pin += t5 - t4;
      }
    }
    printf("{\"rows\": %d, \"row_bytes\": %zu, \"register_us\": %.1f, \"dma_registered_us\": %.1f, "
           "\"unregister_us\": %.1f, \"memcpy_to_pinned_1thread_us\": %.1f, \"dma_pinned_us\": %.1f}\n",
           rows, len, reg / reps, dma_reg / reps, unreg / reps, cpy / reps, dma_pin / reps);
    for (auto h : host) free(h);
    (void)hipFree(dev);
    (void)hipHostFree(pin);
  }
  return 0;
}
