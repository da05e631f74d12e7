// Host copy ceiling of the synchronous host-buffer calls:
// one RS(10,4) 1 MiB-cell encodeBulk moves 10 MiB of pageable rows into
// pinned staging and 4 MiB of parity back out — 14 MiB of host memcpy per
// call. How fast can this box's CPU share do that, by thread count?
//   - "warm": the same 14 rows every call (bench_host_api.py's case);
//   - "cold": rows cycled over 1 GiB, so they come from DRAM (a DataNode's
//     freshly read block).
// Threads split each call's rows into 256 KiB pieces (the copy pool's piece
// size) and are released by a spin barrier per call, so this is the memcpy
// rate itself, not a thread pool's wake-up cost.
// Usage: memcpy_probe [calls]   (one JSON line per (mode, threads))
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

int main(int argc, char** argv) {
  const int calls = argc > 1 ? atoi(argv[1]) : 60;
  const size_t row = 1 << 20, piece = 256 << 10;
  const int rows_per_call = 14;
  const size_t call_bytes = row * rows_per_call;
  const size_t cold_bytes = size_t(1) << 30;
  uint8_t* pin = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&pin), call_bytes, hipHostMallocDefault) != hipSuccess) {
    fprintf(stderr, "hipHostMalloc failed\n");
    return 1;
  }
  std::vector<uint8_t> src(cold_bytes);
  for (size_t i = 0; i < cold_bytes; i += 4096) src[i] = static_cast<uint8_t>(i >> 12);
  memset(pin, 0, call_bytes);
  const size_t npieces = call_bytes / piece;
  for (int mode = 0; mode < 2; ++mode) {
    for (int nt : {1, 2, 4, 8, 12, 16}) {
      std::atomic<int> go{0}, done{0};
      std::atomic<size_t> next{0};
      std::atomic<bool> stop{false};
      size_t base = 0;
      auto work = [&](int) {
        int seen = 0;
        for (;;) {
          while (go.load(std::memory_order_acquire) == seen && !stop.load(std::memory_order_relaxed)) {
          }
          if (stop.load()) return;
          seen = go.load();
          for (;;) {
            const size_t i = next.fetch_add(1);
            if (i >= npieces) break;
            memcpy(pin + i * piece, src.data() + base + i * piece, piece);
          }
          done.fetch_add(1);
        }
      };
      std::vector<std::thread> th;
      for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
      std::vector<double> us;
      for (int c = 0; c < calls + 3; ++c) {
        base = mode == 0 ? 0 : (static_cast<size_t>(c) * call_bytes) % (cold_bytes - call_bytes);
        next.store(0);
        done.store(0);
        const auto t0 = std::chrono::steady_clock::now();
        go.fetch_add(1, std::memory_order_release);
        for (;;) {  // the caller copies too, as in CopyPool::run
          const size_t i = next.fetch_add(1);
          if (i >= npieces) break;
          memcpy(pin + i * piece, src.data() + base + i * piece, piece);
        }
        while (done.load() < nt - 1) {
        }
        const auto t1 = std::chrono::steady_clock::now();
        if (c >= 3) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      }
      stop.store(true);
      go.fetch_add(1);
      for (auto& t : th) t.join();
      std::sort(us.begin(), us.end());
      const double med = us[us.size() / 2];
      printf("{\"mode\": \"%s\", \"threads\": %d, \"call_bytes\": %zu, \"median_us\": %.1f, \"min_us\": %.1f, "
             "\"GBps\": %.2f}\n",
             mode == 0 ? "warm" : "cold", nt, call_bytes, med, us[0], call_bytes / (med * 1e-6) / 1e9);
      fflush(stdout);
    }
  }
  hipHostFree(pin);
  return 0;
}
