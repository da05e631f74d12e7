// Host-side copy pool for the synchronous host-buffer calls (hrs_encode /
// hrs_decode, the JNI path): rows arrive in pageable memory (a JNI-pinned Java
// heap array), are copied by a few threads into pinned staging, and DMA'd from
// there, chunk by chunk, while the GPU works on the previous chunk
// (hrs_api.cpp: host_apply).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace hrs {

struct CopyJob {
  void* dst;
  const void* src;
  size_t bytes;
};

// A fixed set of worker threads; run() splits the jobs into <= 256 KiB
// pieces, the caller joins in, and returns when every byte is copied.
class CopyPool {
 public:
  static CopyPool& instance() {
    static CopyPool pool;
    return pool;
  }

  void run(const std::vector<CopyJob>& jobs) {
    size_t total = 0;
    for (const CopyJob& j : jobs) total += j.bytes;
    if (nthreads_ == 0 || total < (256u << 10)) {
      for (const CopyJob& j : jobs) std::memcpy(j.dst, j.src, j.bytes);
      return;
    }
    std::lock_guard<std::mutex> one_at_a_time(run_mu_);
    pieces_.clear();
    for (const CopyJob& j : jobs)
      for (size_t off = 0; off < j.bytes; off += kPiece) {
        const size_t b = j.bytes - off < kPiece ? j.bytes - off : kPiece;
        pieces_.push_back({static_cast<uint8_t*>(j.dst) + off, static_cast<const uint8_t*>(j.src) + off, b});
      }
    next_.store(0);
    {
      std::lock_guard<std::mutex> lk(mu_);
      busy_ = nthreads_;
      ++generation_;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return busy_ == 0; });
  }

  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++generation_;
    }
    cv_.notify_all();
    for (std::thread& t : threads_) t.join();
  }

 private:
  static constexpr size_t kPiece = 256u << 10;

  CopyPool() {
    const char* e = getenv("HRS_HOST_THREADS");
    int n = e ? atoi(e) : 2;  // measured best on the MI355X hosts (tools/host_sweep.sh)
    if (n < 0) n = 0;
    if (n > 32) n = 32;
    nthreads_ = n;
    for (int i = 0; i < n; ++i) threads_.emplace_back([this] { worker(); });
  }

  void drain() {
    for (;;) {
      const size_t i = next_.fetch_add(1);
      if (i >= pieces_.size()) return;
      std::memcpy(pieces_[i].dst, pieces_[i].src, pieces_[i].bytes);
    }
  }

  void worker() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return generation_ != seen; });
        seen = generation_;
        if (stop_) return;
      }
      drain();
      std::lock_guard<std::mutex> lk(mu_);
      if (--busy_ == 0) done_cv_.notify_all();
    }
  }

  int nthreads_ = 0;
  std::vector<std::thread> threads_;
  std::vector<CopyJob> pieces_;
  std::atomic<size_t> next_{0};
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  uint64_t generation_ = 0;
  int busy_ = 0;
  bool stop_ = false;
};

}  // namespace hrs
