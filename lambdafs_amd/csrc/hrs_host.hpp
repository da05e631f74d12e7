// Host-side copy pool for the synchronous host-buffer calls (hrs_encode /
// hrs_decode, the JNI path): rows arrive in pageable memory (a JNI-pinned Java
// heap array), are copied by a few threads into pinned staging, and DMA'd from
// there, chunk by chunk, while the GPU works on the previous chunk
// (hrs_hostpath.cpp: host_apply).
//
// Several codec handles may call concurrently (one codec per mapper / repair
// thread: Encoder.java:80, Decoder.java:90, MapReduceBlockRepairManager.java:426),
// so run() never serializes callers: each call posts its pieces as a batch,
// copies its own pieces on the calling thread, and the shared workers join
// the open batches in turn, each taking pieces of the batch it joined until
// none is left (a piece per lock round trip cost a 5 MiB copy-in 40-80 us on
// the MI355X hosts whatever the worker count: tools/pool_probe.cpp). A call
// returns once all its pieces are copied and no worker still holds its batch;
// it spins for that (a condition-variable sleep at the end of every batch cost
// about as much as the copy).
//
// Placement (round 6, tools/host_copy_probe): a host copy is bound by the CPU
// complex (CCD) it runs on, about 70 GB/s each; threads on distinct CCDs add
// up (4 threads copying a 2.5 MiB chunk: 188 GB/s on one L3, 271 GB/s over
// four). So each worker is bound to the CPUs of its own L3 within the
// process's affinity set, away from the constructing thread's L3, on the
// GPU's NUMA node first, where the pinned staging lives (set_home_node;
// HRS_HOST_HOME=caller: the constructing thread's node), the GPU ordinal
// choosing where on that node's L3s a process starts (HRS_HOST_PIN=0: no
// binding). With an affinity set inside one L3 nothing is bound.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <immintrin.h>
#include <pthread.h>
#include <sched.h>

namespace hrs {

// CopyJob::stream: how the destination lines are stored
enum : uint8_t {
  kStorePlain = 0,   // through this CPU's caches
  kStoreStream = 1,  // nontemporal: dst is read next by a device, not by this CPU
  kStoreRemote = 2,  // nontemporal only from a CPU off the pool's home NUMA node
};

struct CopyJob {
  void* dst;
  const void* src;
  size_t bytes;
  uint8_t stream = kStorePlain;
};

// The NUMA node the copy pool works for: the node of the GPU whose pinned
// staging it fills (set by the library before the pool's first use; -1 none).
inline std::atomic<int>& pool_home_node() {
  static std::atomic<int> node{-1};
  return node;
}

// The GPU's ordinal, so processes driving different GPUs of one node start
// their workers on different L3s of it (one process per GPU).
inline std::atomic<int>& pool_home_ordinal() {
  static std::atomic<int> ordinal{0};
  return ordinal;
}

// NUMA node of the CPU the calling thread runs on, -1 if unknown.
inline int current_node() {
  unsigned cpu = 0, node = 0;
  return getcpu(&cpu, &node) == 0 ? static_cast<int>(node) : -1;
}

// memcpy with nontemporal (streaming) stores: the destination lines go to
// memory instead of this CPU's caches, so a device reading them next across
// the host link does not snoop them out of a CPU cache, and the copy does not
// evict the caller's working set. AVX2 where the CPU has it, else memcpy.
__attribute__((target("avx2"))) inline void stream_copy_avx2(uint8_t* d, const uint8_t* s, size_t n) {
  const size_t head = (32 - (reinterpret_cast<uintptr_t>(d) & 31)) & 31;
  if (head >= n) {
    std::memcpy(d, s, n);
    return;
  }
  std::memcpy(d, s, head);
  d += head, s += head, n -= head;
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
    const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
  }
  std::memcpy(d + i, s + i, n - i);
  _mm_sfence();  // the streamed lines are in memory before this copy counts as done
}

inline void copy_job(void* d, const void* s, size_t n, uint8_t mode) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  bool stream = mode == kStoreStream;
  if (mode == kStoreRemote) {
    const int home = pool_home_node().load(std::memory_order_relaxed);
    stream = home >= 0 && current_node() != home;
  }
  if (stream && avx2)
    stream_copy_avx2(static_cast<uint8_t*>(d), static_cast<const uint8_t*>(s), n);
  else
    std::memcpy(d, s, n);
}

class CopyPool {
 public:
  static CopyPool& instance() {
    static CopyPool pool;
    return pool;
  }

  // The GPU's NUMA node, for the workers' placement (first caller wins; call
  // before the pool's first use for it to count).
  static void set_home_node(int node, int ordinal = 0) {
    int none = -1;
    if (node >= 0 && pool_home_node().compare_exchange_strong(none, node))
      pool_home_ordinal().store(ordinal > 0 ? ordinal : 0);
  }

  void run(const std::vector<CopyJob>& jobs) {
    size_t total = 0;
    for (const CopyJob& j : jobs) total += j.bytes;
    if (nthreads_ == 0 || total < (256u << 10)) {
      for (const CopyJob& j : jobs) copy_job(j.dst, j.src, j.bytes, j.stream);
      return;
    }
    Batch b;
    for (const CopyJob& j : jobs)
      for (size_t off = 0; off < j.bytes; off += piece_) {
        const size_t n = std::min(piece_, j.bytes - off);
        b.pieces.push_back({static_cast<uint8_t*>(j.dst) + off, static_cast<const uint8_t*>(j.src) + off, n, j.stream});
      }
    {
      std::lock_guard<std::mutex> lk(mu_);
      open_.push_back(&b);
      nopen_.store(open_.size(), std::memory_order_release);
    }
    cv_.notify_all();
    drain(b);
    {
      std::lock_guard<std::mutex> lk(mu_);
      close(&b);  // no new worker may join
    }
    // the last pieces are in other threads' hands: spin for them (held: as
    // long as it takes; else a while) before sleeping
    auto finished = [&] {
      return b.done.load(std::memory_order_acquire) == b.pieces.size() && b.users.load(std::memory_order_acquire) == 0;
    };
    const auto t0 = std::chrono::steady_clock::now();
    const bool held = holders_.load(std::memory_order_acquire) > 0;
    while (!finished() && (held || std::chrono::steady_clock::now() - t0 < kSpin)) __builtin_ia32_pause();
    if (finished()) return;
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, finished);
  }

  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : threads_) t.join();
  }

 private:
  // A synchronous call holds the pool for its duration (Hold): its copy-ins
  // and copy-outs come every few tens of microseconds, and a worker woken
  // through the condition variable joins a batch that late (round 6 trace: a
  // 2.5 MiB copy-in took 35-50 us, single-thread speed). While any call holds
  // the pool, idle workers spin instead of sleeping.
 public:
  class Hold {
   public:
    Hold() : p_(CopyPool::instance()) { p_.holders_.fetch_add(1, std::memory_order_acq_rel); }
    ~Hold() { p_.holders_.fetch_sub(1, std::memory_order_acq_rel); }
    Hold(const Hold&) = delete;
    Hold& operator=(const Hold&) = delete;

   private:
    CopyPool& p_;
  };

 private:

  struct Batch {
    std::vector<CopyJob> pieces;
    std::atomic<size_t> next{0};
    std::atomic<size_t> done{0};
    std::atomic<int> users{0};  // workers inside drain(): raised under mu_ while the batch is open
  };

  // CPUs this process may run on: its affinity set, capped by a cgroup v2 CPU
  // quota (the GPU boxes give one GPU's job 16 CPUs of a larger machine).
  static int cpu_share() {
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long period = 0;
      if (fscanf(f, "%31s %ld", q, &period) == 2 && q[0] != 'm' && period > 0) {
        const long quota = atol(q) / period;
        if (quota > 0 && (n == 0 || quota < n)) n = static_cast<int>(quota);
      }
      fclose(f);
    }
    return n > 0 ? n : 2;
  }

  CopyPool() {
    const char* e = getenv("HRS_HOST_THREADS");
    // default 3 workers (2 on a share under 8 CPUs, 1 under 4): with the
    // caller, 4 threads copy a 1.25 MiB chunk at ~200 GB/s on the MI355X hosts
    // (one thread ~75 GB/s); RS(10,4) 1 MiB staged encode 0.267 ms with 3,
    // 0.274 with 2 (r06r). Each spins while a call holds the pool, so more
    // only burn the job's CPU share (profiles/r06/NOTES.md).
    const int share = cpu_share();
    int n = e ? atoi(e) : (share >= 8 ? 3 : share >= 4 ? 2 : 1);
    if (n < 0) n = 0;
    if (n > 32) n = 32;
    nthreads_ = n;
    // Piece size: the unit a thread claims (HRS_HOST_PIECE, bytes; default
    // 256 KiB, measured ahead of 64 and 32 KiB, profiles/r06/NOTES.md)
    const char* pe = getenv("HRS_HOST_PIECE");
    const long pc = pe ? atol(pe) : 0;
    piece_ = pc >= 4096 ? static_cast<size_t>(pc) : static_cast<size_t>(256) << 10;
    const char* pin = getenv("HRS_HOST_PIN");
    const std::vector<cpu_set_t> homes = (pin && pin[0] == '0') ? std::vector<cpu_set_t>() : worker_homes(n);
    for (int i = 0; i < n; ++i) {
      threads_.emplace_back([this] { worker(); });
      if (!homes.empty())
        (void)pthread_setaffinity_np(threads_.back().native_handle(), sizeof(cpu_set_t), &homes[i % homes.size()]);
    }
  }

  // "0-7,128-135" -> CPU numbers
  static std::vector<int> parse_cpulist(const char* text) {
    std::vector<int> v;
    const char* q = text;
    while (*q) {
      char* e = nullptr;
      const long a = strtol(q, &e, 10);
      if (e == q) break;
      long b = a;
      q = e;
      if (*q == '-') {
        b = strtol(q + 1, &e, 10);
        q = e;
      }
      for (long x = a; x <= b; ++x) v.push_back(static_cast<int>(x));
      while (*q == ',' || *q == '\n' || *q == ' ') ++q;
    }
    return v;
  }

  static int read_int(const std::string& path) {
    int x = -1;
    if (FILE* f = fopen(path.c_str(), "r")) {
      if (fscanf(f, "%d", &x) != 1) x = -1;
      fclose(f);
    }
    return x;
  }

  // One CPU set per worker: the allowed CPUs of one L3 each, the L3s on the
  // home NUMA node first (the GPU's, set_home_node; HRS_HOST_HOME=caller or no
  // home: the constructing thread's node) starting at the GPU ordinal's n-th,
  // the constructing thread's own L3 last. Empty when the affinity set spans
  // fewer than two L3s or sysfs says nothing.
  static std::vector<cpu_set_t> worker_homes(int n) {
    std::vector<cpu_set_t> homes;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (n <= 0 || sched_getaffinity(0, sizeof set, &set) != 0) return homes;
    std::map<int, int> node_of;  // cpu -> NUMA node
    for (int node = 0; node < 64; ++node) {
      FILE* f = fopen(("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
      if (!f) continue;
      char buf[4096] = {0};
      const size_t got = fread(buf, 1, sizeof buf - 1, f);
      fclose(f);
      buf[got] = 0;
      for (int cpu : parse_cpulist(buf)) node_of[cpu] = node;
    }
    std::map<int, std::vector<int>> l3;  // L3 id -> allowed CPUs
    for (int cpu = 0; cpu < CPU_SETSIZE; ++cpu) {
      if (!CPU_ISSET(cpu, &set)) continue;
      const int id = read_int("/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/cache/index3/id");
      if (id < 0) return homes;
      l3[id].push_back(cpu);
    }
    if (l3.size() < 2) return homes;
    const int me = sched_getcpu();
    const int my_l3 = me >= 0 ? read_int("/sys/devices/system/cpu/cpu" + std::to_string(me) + "/cache/index3/id") : -1;
    const char* he = getenv("HRS_HOST_HOME");
    const int home = pool_home_node().load();
    const int want_node = (home >= 0 && !(he && strcmp(he, "caller") == 0)) ? home : node_of.count(me) ? node_of[me] : -1;
    std::vector<std::pair<int, int>> order;  // (rank, L3 id): wanted node 0, other node 1, own L3 2
    for (const auto& g : l3) {
      const int node = node_of.count(g.second[0]) ? node_of[g.second[0]] : -1;
      order.push_back({g.first == my_l3 ? 2 : node == want_node ? 0 : 1, g.first});
    }
    std::stable_sort(order.begin(), order.end(),
                     [](const std::pair<int, int>& a, const std::pair<int, int>& b) { return a.first < b.first; });
    // the wanted node's L3s from the GPU ordinal's n-th one on: with one
    // process per GPU, the pools of a node's GPUs spread over its L3s
    const int nwant = static_cast<int>(std::count_if(order.begin(), order.end(),
                                                     [](const std::pair<int, int>& o) { return o.first == 0; }));
    if (nwant > 1)
      std::rotate(order.begin(), order.begin() + (pool_home_ordinal().load() * n) % nwant, order.begin() + nwant);
    for (int i = 0; i < n && i < static_cast<int>(order.size()); ++i) {
      cpu_set_t h;
      CPU_ZERO(&h);
      for (int cpu : l3[order[i].second]) CPU_SET(cpu, &h);
      homes.push_back(h);
    }
    return homes;
  }

  // Copies pieces of b until none is left unclaimed.
  static void drain(Batch& b) {
    for (;;) {
      const size_t i = b.next.fetch_add(1);
      if (i >= b.pieces.size()) return;
      copy_job(b.pieces[i].dst, b.pieces[i].src, b.pieces[i].bytes, b.pieces[i].stream);
      b.done.fetch_add(1);
    }
  }

  void close(Batch* b) {  // mu_ held
    auto it = std::find(open_.begin(), open_.end(), b);
    if (it != open_.end()) open_.erase(it);
    nopen_.store(open_.size(), std::memory_order_release);
  }

  // A worker that just ran out of work spins this long for the next batch
  // before it sleeps on the condition variable: a synchronous call posts a
  // batch every few tens of microseconds (copy-in, then copy-out, per chunk),
  // and a wake-up through the condition variable costs about as much.
  static constexpr auto kSpin = std::chrono::microseconds(30);

  void spin_for_work() {
    const auto t0 = std::chrono::steady_clock::now();
    while (nopen_.load(std::memory_order_acquire) == 0 &&
           (holders_.load(std::memory_order_acquire) > 0 || std::chrono::steady_clock::now() - t0 < kSpin))
      __builtin_ia32_pause();
  }

  void worker() {
    size_t turn = 0;
    for (;;) {
      spin_for_work();
      Batch* b = nullptr;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !open_.empty(); });
        if (stop_) return;
        b = open_[turn++ % open_.size()];  // interleave concurrent callers
        if (b->next.load() >= b->pieces.size()) {
          close(b);  // fully claimed: its caller finishes it
          continue;
        }
        b->users.fetch_add(1, std::memory_order_relaxed);
      }
      drain(*b);  // every piece left; one lock round trip per batch, not per piece
      b->users.fetch_sub(1, std::memory_order_release);  // b may be gone after this
      { std::lock_guard<std::mutex> lk(mu_); }            // a caller between its check and its wait is waiting now
      done_cv_.notify_all();
    }
  }

  int nthreads_ = 0;
  size_t piece_ = static_cast<size_t>(256) << 10;
  std::atomic<int> holders_{0};  // calls holding the pool (Hold): idle workers spin
  std::vector<std::thread> threads_;
  std::vector<Batch*> open_;
  std::atomic<size_t> nopen_{0};  // open_.size(), readable without mu_ (spin_for_work)
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  bool stop_ = false;
};

}  // namespace hrs
