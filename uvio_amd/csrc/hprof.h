// Host-side section timer for profiling the per-frame loop (debug only).  Enabled by the environment
// variable UVIO_HP_HOST_PROF; the accumulated wall time per section is printed to stderr when the
// engine is destroyed.  Disabled, a section costs one branch.
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>

namespace uvhp {

struct HostProf {
  bool on = std::getenv("UVIO_HP_HOST_PROF") != nullptr;
  std::map<std::string, std::pair<double, long>> acc, cnt;
  std::mutex mu;  // sections may close on a worker thread (the TrackSIM feed's propagation task)
  // a per-frame quantity (sizes, counts) averaged over the calls
  void count(const char *name, double v) {
    if (!on) return;
    std::lock_guard<std::mutex> lk(mu);
    auto &a = cnt[name];
    a.first += v;
    a.second++;
  }
  ~HostProf() {
    if (!on) return;
    for (auto &kv : acc)
      std::fprintf(stderr, "hprof %-28s %10.3f ms  %8ld calls  %8.2f us/call\n", kv.first.c_str(),
                   1e3 * kv.second.first, kv.second.second, 1e6 * kv.second.first / std::max(1L, kv.second.second));
    for (auto &kv : cnt)
      std::fprintf(stderr, "hcount %-27s mean %12.1f over %8ld calls\n", kv.first.c_str(),
                   kv.second.first / std::max(1L, kv.second.second), kv.second.second);
  }
};

struct HostProfScope {
  HostProf &p;
  const char *name;
  std::chrono::steady_clock::time_point t0;
  HostProfScope(HostProf &p_, const char *n) : p(p_), name(n) {
    if (p.on) t0 = std::chrono::steady_clock::now();
  }
  ~HostProfScope() {
    if (!p.on) return;
    std::lock_guard<std::mutex> lk(p.mu);
    auto &a = p.acc[name];
    a.first += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    a.second++;
  }
};

#define HPROF_CAT2(a, b) a##b
#define HPROF_CAT(a, b) HPROF_CAT2(a, b)
#define HPROF(name) HostProfScope HPROF_CAT(hprof_scope_, __LINE__)(hprof_, name)

}  // namespace uvhp
