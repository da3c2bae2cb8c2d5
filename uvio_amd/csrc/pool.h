// A small persistent pool of host worker threads for the per-feature loops of the feature database
// (undistortion of a TrackSIM frame, the selection scans and the marginalization cleanup over every
// tracked feature, VioManager.cpp:366-596).  Those loops are independent per element and memory-latency
// bound at the 20k-40k features of configs 4-5; everything order-dependent (database inserts, erasures,
// the selected lists) stays sequential in the caller, so results do not depend on the thread count.
// Threads: UVIO_HP_THREADS, default min(8, hardware threads).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace uvhp {

class WorkPool {
 public:
  WorkPool() {
    int n = (int)std::thread::hardware_concurrency();
    n = n > 0 ? std::min(n, 8) : 1;
    if (const char *e = std::getenv("UVIO_HP_THREADS")) n = std::max(1, std::atoi(e));
    for (int i = 1; i < n; i++) th_.emplace_back([this] { worker(); });
  }
  ~WorkPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  int threads() const { return (int)th_.size() + 1; }

  // fn(begin, end) over [0, n) in chunks of `chunk`; the caller works too and returns when all are done.
  // An exception thrown by fn (on any thread) is rethrown here, after every chunk has finished.
  void parallel_for(size_t n, size_t chunk, const std::function<void(size_t, size_t)> &fn) {
    if (n == 0) return;
    if (th_.empty() || n <= chunk) {
      fn(0, n);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &fn;
      n_ = n;
      chunk_ = chunk;
      next_.store(0);
      active_ = (int)th_.size();
      err_ = nullptr;
      gen_++;
    }
    cv_.notify_all();
    run_chunks();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return active_ == 0; });
    job_ = nullptr;
    if (err_) std::rethrow_exception(err_);
  }

 private:
  void run_chunks() {
    for (;;) {
      size_t b = next_.fetch_add(chunk_);
      if (b >= n_) break;
      try {
        (*job_)(b, std::min(n_, b + chunk_));
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu_);
        if (!err_) err_ = std::current_exception();
      }
    }
  }
  void worker() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      run_chunks();
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--active_ == 0) done_cv_.notify_one();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t, size_t)> *job_ = nullptr;
  size_t n_ = 0, chunk_ = 1;
  std::atomic<size_t> next_{0};
  int active_ = 0;
  std::exception_ptr err_;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace uvhp
