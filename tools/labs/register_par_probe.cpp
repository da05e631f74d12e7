// Does registering a call's rows with HIP (hipHostRegister, mapped) go faster
// from several threads at once? The direct synchronous call registers its 14
// RS(10,4) rows (1 MiB each, pageable, 16 bytes past a page boundary as a
// JVM's byte[]) one after another before its launch and unregisters them after
// (~0.9 us + ~0.4 us per row, profiles/r05/NOTES.md). Here: the same 14
// whole-page ranges registered / unregistered serially, then split over T
// pre-started threads released together (a spin barrier, no thread start in
// the timed part). Per T, median microseconds per call.
// Usage: register_par_probe [calls]   (one JSON line)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Range {
  void* p;
  size_t n;
};

int main(int argc, char** argv) {
  const int calls = argc > 1 ? atoi(argv[1]) : 200;
  const int rows = 14;
  const size_t L = 1 << 20, P = 4096;
  if (hipSetDevice(0) != hipSuccess) return 1;
  std::vector<uint8_t*> bufs;
  std::vector<Range> rg;
  for (int r = 0; r < rows; ++r) {
    uint8_t* b = static_cast<uint8_t*>(aligned_alloc(2u << 20, 2u << 20));
    for (size_t i = 0; i < (2u << 20); i += P) b[i] = 1;  // resident
    bufs.push_back(b);
    const uintptr_t a = reinterpret_cast<uintptr_t>(b) + 16;
    const uintptr_t lo = (a + P - 1) & ~(P - 1), hi = (a + L) & ~(P - 1);
    rg.push_back({reinterpret_cast<void*>(lo), hi - lo});
  }
  std::atomic<int> bad{0};
  auto op = [&](int ph, int i) {
    const hipError_t e = ph == 0 ? hipHostRegister(rg[i].p, rg[i].n, hipHostRegisterMapped) : hipHostUnregister(rg[i].p);
    if (e != hipSuccess) bad.fetch_add(1);
  };
  printf("{\"what\": \"hipHostRegister / hipHostUnregister of 14 x 1 MiB rows per call, serial vs split over T threads\", "
         "\"calls\": %d, \"by_threads\": [", calls);
  for (int T : {1, 2, 4, 7}) {
    // T - 1 helper threads spin on a generation counter; thread 0 is the caller
    std::atomic<int> gen{0}, done{0};
    std::atomic<bool> quit{false};
    std::atomic<int> phase{0};  // 0 = register, 1 = unregister
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t)
      th.emplace_back([&, t] {
        int seen = 0;
        while (!quit.load()) {
          const int g = gen.load();
          if (g == seen) continue;
          seen = g;
          if (quit.load()) break;
          for (int i = t; i < rows; i += T) op(phase.load(), i);
          done.fetch_add(1);
        }
      });
    auto run = [&](int ph) {
      phase = ph;
      done = 0;
      gen.fetch_add(1);
      for (int i = 0; i < rows; i += T) op(ph, i);
      while (done.load() < T - 1) {
      }
    };
    std::vector<double> tr, tu;
    for (int c = -5; c < calls; ++c) {
      const double t0 = now_us();
      run(0);
      const double t1 = now_us();
      run(1);
      const double t2 = now_us();
      if (c >= 0) {
        tr.push_back(t1 - t0);
        tu.push_back(t2 - t1);
      }
    }
    quit = true;  // before the last release: the helpers leave without acting
    gen.fetch_add(1);
    for (auto& x : th) x.join();
    std::sort(tr.begin(), tr.end());
    std::sort(tu.begin(), tu.end());
    printf("%s{\"threads\": %d, \"register_us\": %.2f, \"unregister_us\": %.2f}", T == 1 ? "" : ", ", T,
           tr[tr.size() / 2], tu[tu.size() / 2]);
  }
  const bool ok = bad.load() == 0;
  printf("], \"ok\": %s}\n", ok ? "true" : "false");
  for (auto* b : bufs) free(b);
  return ok ? 0 : 1;
}
