// Host copy rates of the staged synchronous calls (lambdafs_amd/csrc/hrs_host.hpp
// CopyPool), on the box's own CPUs: one 256 KiB chunk of an RS(10,4) 1 MiB-cell
// call copied into pinned staging (10 rows, 2.5 MiB; plain or nontemporal
// stores) and its outputs copied out (4 rows, 1 MiB), through the pool with
// and without a call holding it, and by one thread; plus the NUMA nodes of the
// calling CPU, the pageable rows and the pinned staging (move_pages query).
// Usage: host_copy_probe [reps]   (one JSON line per case, medians in us)
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <vector>

#include "../lambdafs_amd/csrc/hrs_host.hpp"

static int node_of(const void* p) {
  void* pages[1] = {const_cast<void*>(p)};
  int status[1] = {-1};
  if (syscall(SYS_move_pages, 0, 1, pages, nullptr, status, 0) != 0) return -1;
  return status[0];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  const size_t L = 256 << 10;
  std::vector<std::vector<uint8_t>> rows(14, std::vector<uint8_t>(1 << 20, 7));
  uint8_t* stage = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&stage), 14 * L, hipHostMallocDefault) != hipSuccess) return 1;
  for (size_t i = 0; i < 14 * L; i += 4096) stage[i] = 1;
  unsigned cpu = 0, node = 0;
  syscall(SYS_getcpu, &cpu, &node, nullptr);
  printf("{\"cpu\": %u, \"cpu_node\": %u, \"rows_node\": %d, \"staging_node\": %d, \"nprocs_onln\": %ld}\n", cpu, node,
         node_of(rows[0].data()), node_of(stage), sysconf(_SC_NPROCESSORS_ONLN));
  hrs::CopyPool& pool = hrs::CopyPool::instance();
  auto run_case = [&](const char* name, bool in, bool nt, bool hold, bool single) {
    std::vector<hrs::CopyJob> jobs;
    if (in)
      for (int r = 0; r < 10; ++r) jobs.push_back({stage + r * L, rows[r].data() + L, L, nt});
    else
      for (int r = 0; r < 4; ++r) jobs.push_back({rows[10 + r].data() + L, stage + (10 + r) * L, L, false});
    std::vector<double> t;
    std::unique_ptr<hrs::CopyPool::Hold> held;  // a call holds the pool across its copies
    if (hold) held.reset(new hrs::CopyPool::Hold());
    for (int i = 0; i < reps; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      if (single) {
        for (const auto& j : jobs) hrs::copy_job(j.dst, j.src, j.bytes, j.stream);
      } else {
        pool.run(jobs);
      }
      const auto t1 = std::chrono::steady_clock::now();
      t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      const auto t2 = t1 + std::chrono::microseconds(40);  // a call's launch / wait between copies
      while (std::chrono::steady_clock::now() < t2) {
      }
    }
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2];
    const double bytes = in ? 10.0 * L : 4.0 * L;
    printf("{\"case\": \"%s\", \"median_us\": %.1f, \"p90_us\": %.1f, \"GBps\": %.1f}\n", name, med,
           t[t.size() * 9 / 10], bytes / med / 1e3);
  };
  run_case("in_pool", true, false, false, false);
  run_case("in_pool_hold", true, false, true, false);
  run_case("in_pool_nt", true, true, false, false);
  run_case("in_pool_hold_nt", true, true, true, false);
  run_case("in_single", true, false, false, true);
  run_case("in_single_nt", true, true, false, true);
  run_case("out_pool", false, false, false, false);
  run_case("out_pool_hold", false, false, true, false);
  run_case("out_single", false, false, false, true);
  (void)hipHostFree(stage);
  return 0;
}
