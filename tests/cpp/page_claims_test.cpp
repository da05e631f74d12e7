// hrs::PageClaims (hrs_host.hpp): the process-wide claims on host page ranges
// the synchronous direct calls register with HIP (hrs_hostpath.cpp). Checks the
// overlap rules single-threaded, then N threads claiming random ranges of a
// small page space at once: a claimed page is never claimed by a second
// holder, and every claim is released. Then hrs::inner_stripes (the stripes
// of a pageable host batch that lie inside whole pages, hrs_batch_api.cpp)
// against a brute-force scan over random layouts. CPU only (also under
// `make tsan`).
// Usage: page_claims_test [threads] [iterations]   (one JSON line)
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "../../lambdafs_amd/csrc/hrs_host.hpp"

using Ranges = std::vector<std::pair<uintptr_t, uintptr_t>>;

int main(int argc, char** argv) {
  const int nthreads = argc > 1 ? atoi(argv[1]) : 4;
  const int iters = argc > 2 ? atoi(argv[2]) : 20000;
  const uintptr_t P = 4096, base = uintptr_t(1) << 40;
  hrs::PageClaims& pc = hrs::PageClaims::instance();
  int bad = 0;
  auto R = [&](int a, int b) { return std::make_pair(base + a * P, base + b * P); };
  // rules: overlap fails, adjacency is fine, release frees, all-or-nothing
  bad += !pc.claim({R(10, 20)});
  bad += pc.claim({R(15, 16)});           // inside
  bad += pc.claim({R(5, 11)});            // overlaps the start
  bad += pc.claim({R(19, 30)});           // overlaps the end
  bad += pc.claim({R(0, 100)});           // covers it
  bad += !pc.claim({R(20, 21), R(9, 10)});  // adjacent on both sides
  bad += pc.claim({R(30, 31), R(12, 13)});  // one of two overlaps: nothing claimed
  bad += !pc.claim({R(30, 31)});            // ... so this one is still free
  pc.release({R(10, 20)});
  bad += !pc.claim({R(15, 16)});
  pc.release({R(15, 16)});
  pc.release({R(20, 21), R(9, 10)});
  pc.release({R(30, 31)});
  bad += !pc.claim({R(0, 100)});
  pc.release({R(0, 100)});
  // concurrent holders over a 64-page space
  const int npages = 64;
  std::vector<std::atomic<int>> owner(npages);
  for (auto& o : owner) o = -1;
  std::atomic<int> violations{0};
  std::atomic<long> granted{0}, refused{0};
  auto body = [&](int t) {
    std::mt19937 rng(1234 + t);
    for (int it = 0; it < iters; ++it) {
      Ranges rg;
      const int nr = 1 + rng() % 3;
      for (int r = 0; r < nr; ++r) {
        const int a = rng() % (npages - 4), len = 1 + rng() % 4;
        bool dup = false;  // ranges of one call are disjoint (the caller merges them)
        for (auto& x : rg) dup |= !(R(a, a + len).second <= x.first || x.second <= R(a, a + len).first);
        if (!dup) rg.push_back(R(a, a + len));
      }
      if (!pc.claim(rg)) {
        refused++;
        continue;
      }
      granted++;
      for (auto& x : rg)
        for (uintptr_t pg = (x.first - base) / P; pg < (x.second - base) / P; ++pg) {
          int expect = -1;
          if (!owner[pg].compare_exchange_strong(expect, t)) violations++;
        }
      for (auto& x : rg)
        for (uintptr_t pg = (x.first - base) / P; pg < (x.second - base) / P; ++pg) owner[pg] = -1;
      pc.release(rg);
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) th.emplace_back(body, t);
  for (auto& x : th) x.join();
  bad += !pc.claim({R(0, npages)});  // every claim was released
  pc.release({R(0, npages)});
  // inner_stripes vs brute force: stripe s is inside iff its first byte is at
  // or past the first whole page and its last byte before the span's last
  // partial page; the inside stripes must be exactly [lo, hi)
  std::mt19937 rng(99);
  int inner_bad = 0;
  for (int it = 0; it < 20000; ++it) {
    const uintptr_t b = base + rng() % (3 * P);
    const size_t ext = 1 + rng() % (5 * P);
    const size_t ns = rng() % 12;
    const size_t stride = (rng() % 8 == 0) ? rng() % (ext + 1) : ext + (rng() % 3) * (rng() % (2 * P));
    const hrs::InnerStripes r = hrs::inner_stripes(reinterpret_cast<const void*>(b), stride, ext, ns);
    const bool overl = ns > 1 && stride < ext;
    const uintptr_t p0 = (b + P - 1) / P * P, p1 = ns ? (b + (ns - 1) * stride + ext) / P * P : 0;
    for (size_t s = 0; s < ns; ++s) {
      const bool in = !overl && ns && b + s * stride >= p0 && b + s * stride + ext <= p1;
      const bool said = s >= r.lo && s < r.hi;
      if (in != said) inner_bad++;
      if (said && (r.p0 != p0 || r.p1 != p1)) inner_bad++;
    }
    if (r.hi > ns) inner_bad++;
  }
  bad += inner_bad;
  const bool ok = bad == 0 && violations == 0;
  printf("{\"threads\": %d, \"iterations\": %d, \"inner_stripes_failures\": %d, \"rule_failures\": %d, "
         "\"violations\": %d, \"granted\": %ld, \"refused\": %ld, \"ok\": %s}\n",
         nthreads, iters, inner_bad, bad - inner_bad, violations.load(), granted.load(), refused.load(),
         ok ? "true" : "false");
  return ok ? 0 : 1;
}
