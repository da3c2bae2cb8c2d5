// A small persistent pool of host worker threads for the per-feature loops of the feature database
// (undistortion of a TrackSIM frame, the selection scans and the marginalization cleanup over every
// tracked feature, VioManager.cpp:366-596).  Those loops are independent per element and memory-latency
// bound at the 20k-40k features of configs 4-5; everything order-dependent (database inserts, erasures,
// the selected lists) stays sequential in the caller, so results do not depend on the thread count.
// Threads: UVIO_HP_THREADS, default min(16, hardware threads) (the box's CPU share per GPU; cfg4 186 vs 175
// frames/s against 8 threads in the same-box A/B profiles/r04o_env_ab.txt).
//
// A frame issues a dozen parallel loops a few tens of microseconds apart, so a worker that finishes one
// spins for a while (spin_us_) on the job generation before it sleeps on the condition variable, and the
// caller never waits for a worker that has not joined the job: it closes the job when its own share of
// chunks runs out and waits only for the workers that took part (a late sleeper wakes to a closed job).
#pragma once
#include <atomic>
#include <chrono>
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
    n = n > 0 ? std::min(n, 16) : 1;
    if (const char *e = std::getenv("UVIO_HP_THREADS")) n = std::max(1, std::atoi(e));
    if (const char *e = std::getenv("UVIO_HP_SPIN_US")) spin_us_ = std::max(0, std::atoi(e));
    for (int i = 1; i < n; i++) th_.emplace_back([this] { worker(); });
  }
  ~WorkPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_.store(true);
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
    Job job;
    job.fn = &fn;
    job.n = n;
    job.chunk = chunk;
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &job;
      gen_.fetch_add(1, std::memory_order_release);
      if (sleeping_ > 0) cv_.notify_all();
    }
    run(job);
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = nullptr;  // closed: no worker joins from here on
    }
    while (job.refs.load(std::memory_order_acquire) != 0) relax();
    if (job.err) std::rethrow_exception(job.err);
  }

 private:
  struct Job {
    const std::function<void(size_t, size_t)> *fn = nullptr;
    size_t n = 0, chunk = 1;
    std::atomic<size_t> next{0};
    std::atomic<int> refs{0};  // workers inside run()
    std::mutex err_mu;
    std::exception_ptr err;
  };
  int spin_us_ = 200;  // kept spinning after a job (UVIO_HP_SPIN_US: A/B runs)
  static void relax() { __builtin_ia32_pause(); }
  static void run(Job &job) {
    for (;;) {
      const size_t b = job.next.fetch_add(job.chunk);
      if (b >= job.n) break;
      try {
        (*job.fn)(b, std::min(job.n, b + job.chunk));
      } catch (...) {
        std::lock_guard<std::mutex> lk(job.err_mu);
        if (!job.err) job.err = std::current_exception();
      }
    }
  }
  void worker() {
    uint64_t seen = gen_.load(std::memory_order_acquire);
    for (;;) {
      // spin for a new job, then sleep
      const auto t0 = std::chrono::steady_clock::now();
      while (gen_.load(std::memory_order_acquire) == seen && !stop_.load(std::memory_order_relaxed)) {
        relax();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) break;
      }
      Job *j = nullptr;
      {
        std::unique_lock<std::mutex> lk(mu_);
        if (gen_.load(std::memory_order_relaxed) == seen && !stop_.load()) {
          sleeping_++;
          cv_.wait(lk, [&] { return stop_.load() || gen_.load(std::memory_order_relaxed) != seen; });
          sleeping_--;
        }
        if (stop_.load()) return;
        seen = gen_.load(std::memory_order_relaxed);
        j = job_;
        if (j) j->refs.fetch_add(1, std::memory_order_relaxed);
      }
      if (j) {
        run(*j);
        j->refs.fetch_sub(1, std::memory_order_release);
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  Job *job_ = nullptr;           // the open job (guarded by mu_)
  std::atomic<uint64_t> gen_{0};  // incremented (under mu_) per job
  int sleeping_ = 0;             // workers waiting on cv_ (guarded by mu_)
  std::atomic<bool> stop_{false};
};

}  // namespace uvhp
