// Host copy rates of the staged synchronous calls (lambdafs_amd/csrc/hrs_host.hpp
// CopyPool), on the box's own CPUs: one 256 KiB chunk of an RS(10,4) 1 MiB-cell
// call copied into pinned staging (10 rows, 2.5 MiB; plain or nontemporal
// stores) and its outputs copied out (4 rows, 1 MiB), through the pool with
// and without a call holding it, and by one thread; plus the NUMA nodes of the
// calling CPU, the pageable rows and the pinned staging (move_pages query)
// and of the GPU (sysfs).
// Usage: host_copy_probe [reps]   (one JSON line per case, medians in us)
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <thread>
#include <cctype>
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

// NUMA node of device 0's PCI function (sysfs), -1 if unknown.
static int gpu_node() {
  char bus[64] = {0}, path[160];
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), 0) != hipSuccess) return -1;
  for (char* q = bus; *q; ++q) *q = static_cast<char>(tolower(*q));
  snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE* f = fopen(path, "r");
  if (!f) return -1;
  int n = -1;
  if (fscanf(f, "%d", &n) != 1) n = -1;
  fclose(f);
  return n;
}

// The calling thread's allowed CPUs, each with the id of its L3 (one per CCD).
static std::vector<std::pair<int, int>> cpus_by_l3() {
  std::vector<std::pair<int, int>> v;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) != 0) return v;
  for (int c = 0; c < CPU_SETSIZE; ++c) {
    if (!CPU_ISSET(c, &set)) continue;
    char path[128];
    snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/id", c);
    FILE* f = fopen(path, "r");
    int id = -1;
    if (f) {
      if (fscanf(f, "%d", &id) != 1) id = -1;
      fclose(f);
    }
    v.emplace_back(c, id);
  }
  return v;
}

// T threads, each pinned to one CPU of `cpus`, copy `jobs` split evenly
// (static split by row), timed from the first start to the last end.
static double pinned_threads_copy(const std::vector<int>& cpus, const std::vector<hrs::CopyJob>& jobs) {
  const int T = static_cast<int>(cpus.size());
  std::vector<std::thread> th;
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::vector<std::chrono::steady_clock::time_point> t1(T);
  for (int i = 0; i < T; ++i)
    th.emplace_back([&, i] {
      cpu_set_t one;
      CPU_ZERO(&one);
      CPU_SET(cpus[i], &one);
      sched_setaffinity(0, sizeof(one), &one);
      ready.fetch_add(1);
      while (!go.load()) {
      }
      for (size_t j = 0; j < jobs.size(); ++j) {
        const size_t per = (jobs[j].bytes + T - 1) / T, off = per * i;
        if (off < jobs[j].bytes)
          hrs::copy_job(static_cast<uint8_t*>(jobs[j].dst) + off, static_cast<const uint8_t*>(jobs[j].src) + off,
                        std::min(per, jobs[j].bytes - off), false);
      }
      t1[i] = std::chrono::steady_clock::now();
    });
  while (ready.load() < T) {
  }
  const auto t0 = std::chrono::steady_clock::now();
  go.store(true);
  for (auto& x : th) x.join();
  auto end = t0;
  for (const auto& x : t1) end = std::max(end, x);
  return std::chrono::duration<double, std::micro>(end - t0).count();
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
  printf("{\"cpu\": %u, \"cpu_node\": %u, \"rows_node\": %d, \"staging_node\": %d, \"gpu_node\": %d, \"nprocs_onln\": %ld}\n",
         cpu, node, node_of(rows[0].data()), node_of(stage), gpu_node(), sysconf(_SC_NPROCESSORS_ONLN));
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
  // CPUs grouped by L3: copy-in of the 2.5 MiB chunk by 1-4 pinned threads on
  // one L3, and by the same number spread over distinct L3s.
  const auto cl = cpus_by_l3();
  std::map<int, std::vector<int>> by_l3;
  for (const auto& x : cl) by_l3[x.second].push_back(x.first);
  printf("{\"cpus\": %zu, \"l3_groups\": %zu, \"groups\": [", cl.size(), by_l3.size());
  bool first = true;
  for (const auto& g : by_l3) {
    printf("%s{\"l3\": %d, \"cpus\": [", first ? "" : ", ", g.first);
    for (size_t i = 0; i < g.second.size(); ++i) printf("%s%d", i ? ", " : "", g.second[i]);
    printf("]}");
    first = false;
  }
  printf("]}\n");
  std::vector<hrs::CopyJob> in_jobs;
  for (int r = 0; r < 10; ++r) in_jobs.push_back({stage + r * L, rows[r].data() + L, L, false});
  for (int T : {1, 2, 3, 4}) {
    std::vector<int> same, spread;
    const auto& g0 = by_l3.begin()->second;
    for (int i = 0; i < T && i < static_cast<int>(g0.size()); ++i) same.push_back(g0[i]);
    for (const auto& g : by_l3)
      if (static_cast<int>(spread.size()) < T) spread.push_back(g.second[0]);
    for (int mode = 0; mode < 2; ++mode) {
      const auto& cpus = mode ? spread : same;
      if (static_cast<int>(cpus.size()) < T) continue;
      std::vector<double> t;
      for (int i = 0; i < reps; ++i) t.push_back(pinned_threads_copy(cpus, in_jobs));
      std::sort(t.begin(), t.end());
      const double med = t[t.size() / 2];
      printf("{\"case\": \"in_threads_%s\", \"threads\": %d, \"median_us\": %.1f, \"GBps\": %.1f}\n",
             mode ? "spread_l3" : "same_l3", T, med, 10.0 * L / med / 1e3);
    }
  }
  (void)hipHostFree(stage);
  return 0;
}
