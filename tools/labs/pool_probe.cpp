// The host copy pool itself (lambdafs_amd/csrc/hrs_host.hpp CopyPool::run),
// as the synchronous calls use it: one chunk's copy-in, 10 rows x 512 KiB of
// pageable rows into pinned staging (hipHostMalloc), calls spaced like a
// call's copy-in / launch / copy-out rhythm. Compared with the raw memcpy
// rate of tools/memcpy_probe.cpp, this says whether the pool parallelizes.
// Usage: HRS_HOST_THREADS=N pool_probe   (JSON lines)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../lambdafs_amd/csrc/hrs_host.hpp"

int main() {
  const size_t rows = 10, len = 512 << 10;
  std::vector<std::vector<uint8_t>> src(rows, std::vector<uint8_t>(len, 1));
  uint8_t* dst = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&dst), rows * len, hipHostMallocDefault) != hipSuccess) return 1;
  hrs::CopyPool& pool = hrs::CopyPool::instance();
  std::vector<hrs::CopyJob> jobs;
  for (size_t r = 0; r < rows; ++r) jobs.push_back({dst + r * len, src[r].data(), len});
  const char* e = getenv("HRS_HOST_THREADS");
  for (int gap_us : {0, 50, 200}) {
    std::vector<double> t;
    for (int i = 0; i < 300; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      pool.run(jobs);
      const auto t1 = std::chrono::steady_clock::now();
      if (i >= 20) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      const auto t2 = t1 + std::chrono::microseconds(gap_us);
      while (std::chrono::steady_clock::now() < t2) {
      }
    }
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2];
    printf("{\"threads\": \"%s\", \"gap_us\": %d, \"median_us\": %.1f, \"p90_us\": %.1f, \"GBps\": %.1f}\n",
           e ? e : "default", gap_us, med, t[t.size() * 9 / 10], rows * len / med / 1e3);
  }
  hipHostFree(dst);
  return 0;
}
