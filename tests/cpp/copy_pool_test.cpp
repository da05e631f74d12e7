// CPU test of the host copy pool (lambdafs_amd/csrc/hrs_host.hpp): several
// caller threads post batches of pieces of random sizes at once (the
// synchronous calls of concurrent codec handles); every byte must land, no
// batch may return before its pieces are done, and the workers must drain
// batches they join. Prints one JSON line; exit status 0 = ok.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../lambdafs_amd/csrc/hrs_host.hpp"

int main(int argc, char** argv) {
  const int callers = argc > 1 ? atoi(argv[1]) : 4;
  const int rounds = argc > 2 ? atoi(argv[2]) : 200;
  std::atomic<long> bad{0}, bytes{0};
  std::vector<std::thread> th;
  for (int c = 0; c < callers; ++c)
    th.emplace_back([&, c] {
      std::mt19937_64 rng(1234 + c);
      for (int r = 0; r < rounds; ++r) {
        const int njobs = 1 + static_cast<int>(rng() % 14);
        std::vector<std::vector<uint8_t>> src(njobs), dst(njobs);
        std::vector<hrs::CopyJob> jobs;
        for (int j = 0; j < njobs; ++j) {
          const size_t n = rng() % 3 == 0 ? rng() % 4096 : (rng() % (1u << 20));
          src[j].resize(n);
          dst[j].assign(n, 0xEE);
          for (size_t i = 0; i < n; i += 64) src[j][i] = static_cast<uint8_t>(rng());
          jobs.push_back({dst[j].data(), src[j].data(), n});
          bytes += static_cast<long>(n);
        }
        hrs::CopyPool::instance().run(jobs);
        for (int j = 0; j < njobs; ++j)
          if (src[j] != dst[j]) ++bad;
      }
    });
  for (auto& t : th) t.join();
  printf("{\"callers\": %d, \"rounds\": %d, \"bytes\": %ld, \"bad_jobs\": %ld, \"ok\": %s}\n", callers, rounds,
         bytes.load(), bad.load(), bad.load() == 0 ? "true" : "false");
  return bad.load() == 0 ? 0 : 1;
}
