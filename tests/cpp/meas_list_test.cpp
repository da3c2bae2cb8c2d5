// Host unit test of the feature database's per-camera measurement storage (uvio_amd/csrc/engine.h MeasList /
// TrackSet), of the host work pool (pool.h) and of the database's slab node allocator: random push / trim / erase sequences against a plain vector
// model, checking every query and the cached first / last times; many back-to-back pool jobs.  Built and run by tests/test_host_structs.py (no GPU needed).
#include <cstdio>
#include <random>
#include <vector>

#include "engine.h"

using uvhp::FeatMeas;
using uvhp::MeasList;

static int fails = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);         \
      if (++fails > 20) return 1;                                     \
    }                                                                 \
  } while (0)

int main() {
  std::mt19937 rng(7);
  for (int trial = 0; trial < 400; trial++) {
    MeasList m;
    std::vector<FeatMeas> ref;
    const bool ordered = trial % 3 != 0;
    double t = 0;
    for (int step = 0; step < 200; step++) {
      const int op = (int)(rng() % 10);
      if (op < 5) {  // append
        t += ordered ? 1.0 + (rng() % 2) : 0.0;
        const double tt = ordered ? t : (double)(rng() % 40);
        FeatMeas x{(float)step, 0.f, 0.f, 0.f, tt};
        m.push_back(x);
        ref.push_back(x);
      } else if (op < 7) {  // drop everything at or before a time
        const double c = ordered ? t - (double)(rng() % 6) : (double)(rng() % 40);
        m.drop_through(c);
        std::vector<FeatMeas> r2;
        for (auto &x : ref)
          if (!(x.t <= c)) r2.push_back(x);
        ref.swap(r2);
      } else if (op < 8) {  // remove one time (the zero-velocity exact cleanup)
        const double c = ordered ? t - (double)(rng() % 4) : (double)(rng() % 40);
        m.erase(std::remove_if(m.begin(), m.end(), [c](const FeatMeas &x) { return x.t == c; }), m.end());
        ref.erase(std::remove_if(ref.begin(), ref.end(), [c](const FeatMeas &x) { return x.t == c; }), ref.end());
      } else if (op < 9) {  // drop the k oldest
        const size_t k = std::min(ref.size(), (size_t)(rng() % 3));
        m.drop_front(k);
        ref.erase(ref.begin(), ref.begin() + (std::ptrdiff_t)k);
      } else {
        // queries below
      }
      CHECK(m.size() == ref.size());
      CHECK(m.empty() == ref.empty());
      for (size_t i = 0; i < ref.size(); i++) CHECK(m[i].t == ref[i].t && m[i].u == ref[i].u);
      if (!ref.empty()) {
        CHECK(m.last_t() == ref.back().t);
        CHECK(m.front().t == ref.front().t);
      }
      for (double q = -1; q <= t + 1 && q < 60; q += 1.0) {
        bool has = false;
        for (auto &x : ref) has = has || x.t == q;
        CHECK(m.contains(q) == has);
      }
    }
  }
  // tracks: a camera's first measurement inserts its track at the front (reverse first-insertion order)
  uvhp::Feature f;
  f.track(2).m.push_back(FeatMeas{0, 0, 0, 0, 1.0});
  f.track(0).m.push_back(FeatMeas{0, 0, 0, 0, 1.0});
  f.track(2).m.push_back(FeatMeas{0, 0, 0, 0, 2.0});
  f.track(1).m.push_back(FeatMeas{0, 0, 0, 0, 2.0});
  std::vector<size_t> order;
  for (auto &c : f.tracks) order.push_back(c.cam);
  CHECK(order.size() == 3 && order[0] == 1 && order[1] == 0 && order[2] == 2);
  CHECK(f.count() == 4);
  CHECK(f.find(2) && f.find(2)->m.size() == 2 && f.find(2)->m.last_t() == 2.0);
  // the work pool: every index exactly once over many back-to-back jobs of varied sizes, an exception in a
  // chunk reaches the caller after the job, and the pool stays usable afterwards
  {
    uvhp::WorkPool pool;
    std::vector<int> hits;
    for (int job = 0; job < 2000; job++) {
      const size_t n = 1 + (size_t)(rng() % 5000), chunk = 1 + (size_t)(rng() % 300);
      hits.assign(n, 0);
      pool.parallel_for(n, chunk, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; i++) hits[i]++;
      });
      bool ok = true;
      for (int h : hits) ok = ok && h == 1;
      CHECK(ok);
    }
    bool thrown = false;
    try {
      pool.parallel_for(10000, 16, [&](size_t b, size_t) {
        if (b == 4096) throw std::runtime_error("chunk");
      });
    } catch (const std::runtime_error &) {
      thrown = true;
    }
    CHECK(thrown);
    std::atomic<long> sum{0};
    pool.parallel_for(100000, 64, [&](size_t b, size_t e) {
      long s = 0;
      for (size_t i = b; i < e; i++) s += (long)i;
      sum += s;
    });
    CHECK(sum.load() == 100000L * 99999L / 2);
  }
  // the feature database's slab node allocator (engine.h NodeSlabs / SlabAlloc): a map on the slabs and a plain
  // std::unordered_map under the same operation sequence (a sliding window of consecutive ids, as the
  // simulated feeds insert and erase them, plus random keys) iterate in the same order with the same values
  {
    uvhp::NodeSlabs slabs;
    using SMap = std::unordered_map<size_t, long, std::hash<size_t>, std::equal_to<size_t>,
                                    uvhp::SlabAlloc<std::pair<const size_t, long>>>;
    SMap a{uvhp::SlabAlloc<std::pair<const size_t, long>>(&slabs)};
    std::unordered_map<size_t, long> b;
    size_t next = 1000, oldest = 1000;
    for (int frame = 0; frame < 300; frame++) {
      const int nnew = 500 + (int)(rng() % 1500);
      for (int i = 0; i < nnew; i++, next++) {
        a.emplace(next, (long)next * 3);
        b.emplace(next, (long)next * 3);
      }
      for (int i = 0; i < 50; i++) {  // random keys, some present
        const size_t k = rng() % (next + 5000);
        a.emplace(k, -(long)k);
        b.emplace(k, -(long)k);
      }
      while (next - oldest > 40000) {  // the window's oldest features leave
        a.erase(oldest);
        b.erase(oldest);
        oldest++;
      }
      for (int i = 0; i < 300; i++) {  // scattered erasures
        const size_t k = oldest + rng() % (next - oldest);
        a.erase(k);
        b.erase(k);
      }
      CHECK(a.size() == b.size() && a.bucket_count() == b.bucket_count());
      auto ia = a.begin();
      auto ib = b.begin();
      bool same = true;
      for (; ia != a.end() && ib != b.end(); ++ia, ++ib) same = same && ia->first == ib->first && ia->second == ib->second;
      CHECK(same && ia == a.end() && ib == b.end());
    }
    a.clear();
  }
  std::printf(fails ? "meas_list_test: %d failures\n" : "meas_list_test: ok\n", fails);
  return fails ? 1 : 0;
}
