// CPU test of the host copy pool (lambdafs_amd/csrc/hrs_host.hpp): several
// caller threads post batches of pieces of random sizes at once (the
// synchronous calls of concurrent codec handles); every byte must land, no
// batch may return before its pieces are done, and the workers must drain
// batches they join. Jobs take every store mode (cached, nontemporal, and
// nontemporal off the pool's home NUMA node, set to node 0 before the pool's
// first use), at odd offsets and sizes; half the callers hold the pool (the
// synchronous calls' spin path). Prints one JSON line; exit status 0 = ok.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <thread>
#include <vector>

#include "../../lambdafs_amd/csrc/hrs_host.hpp"

int main(int argc, char** argv) {
  const int callers = argc > 1 ? atoi(argv[1]) : 4;
  const int rounds = argc > 2 ? atoi(argv[2]) : 200;
  std::atomic<long> bad{0}, bytes{0};
  hrs::CopyPool::set_home_node(0);
  std::vector<std::thread> th;
  for (int c = 0; c < callers; ++c)
    th.emplace_back([&, c] {
      std::mt19937_64 rng(1234 + c);
      for (int r = 0; r < rounds; ++r) {
        std::unique_ptr<hrs::CopyPool::Hold> hold;
        if (c % 2 == 1) hold.reset(new hrs::CopyPool::Hold());
        const int njobs = 1 + static_cast<int>(rng() % 14);
        std::vector<std::vector<uint8_t>> src(njobs), dst(njobs);
        std::vector<hrs::CopyJob> jobs;
        for (int j = 0; j < njobs; ++j) {
          const size_t n = rng() % 3 == 0 ? rng() % 4096 : (rng() % (1u << 20));
          const size_t off = rng() % 48;  // destination misalignment for the streamed head
          src[j].resize(n);
          dst[j].assign(n + off, 0xEE);
          for (size_t i = 0; i < n; i += 64) src[j][i] = static_cast<uint8_t>(rng());
          const uint8_t mode = static_cast<uint8_t>(rng() % 3);  // kStorePlain / kStoreStream / kStoreRemote
          jobs.push_back({dst[j].data() + off, src[j].data(), n, mode});
          bytes += static_cast<long>(n);
        }
        hrs::CopyPool::instance().run(jobs);
        for (int j = 0; j < njobs; ++j) {
          const size_t off = dst[j].size() - src[j].size();
          bool ok = std::memcmp(dst[j].data() + off, src[j].data(), src[j].size()) == 0;
          for (size_t i = 0; i < off; ++i) ok &= dst[j][i] == 0xEE;  // nothing written before the job
          if (!ok) ++bad;
        }
      }
    });
  for (auto& t : th) t.join();
  printf("{\"callers\": %d, \"rounds\": %d, \"bytes\": %ld, \"bad_jobs\": %ld, \"ok\": %s}\n", callers, rounds,
         bytes.load(), bad.load(), bad.load() == 0 ? "true" : "false");
  return bad.load() == 0 ? 0 : 1;
}
