// ORACLE — test infrastructure only (see la.h header).
// Rounding-tie witness for the lock-step parity tests.
//
// The reference quantizes two kinds of double values to float on the state path:
//   * the predicted normalized coordinates of the feature refinement, z = (float)(h1/h3)
//     (FeatureInitializer.cpp:273-275 and its cost, :414-416), and
//   * every predicted pixel: distort_d casts the normalized point to float and distort_f returns a
//     float pixel (CamBase.h:130, CamRadtan.h / CamEqui.h distort_f).
// Two implementations whose doubles agree to rounding (different summation order) round such a cast
// to different floats only when its double input lies within that rounding difference of a float
// rounding midpoint.  fcast() is the one place the oracle performs these casts; under a FlipCtl it
// numbers them in execution order, records the ones whose relative distance to the midpoint is below
// `thresh` (the candidates), and can round one chosen cast to the other neighbouring float.  The
// steering in updater.cpp uses it to show that a feature on which the device and the oracle differ
// is explained by exactly one such cast: re-running the reference algorithm with that single cast
// rounded the other way reproduces the device's result to the strict bounds.
#pragma once
#include <cmath>
#include <vector>

namespace orc {

struct FlipCtl {
  long counter = 0;     // casts seen so far (execution order)
  long force = -1;      // index of the cast to round to the other neighbour
  double thresh = 1e-9; // record casts whose relative distance to the rounding midpoint is below this
  std::vector<std::pair<long, double>> near;  // (index, margin) of the recorded casts
};

extern thread_local FlipCtl *g_flip;

// (float)q, instrumented
inline float fcast(double q) {
  float f = (float)q;
  FlipCtl *c = g_flip;
  if (!c) return f;
  const long idx = c->counter++;
  const double fd = (double)f;
  if (fd == q || !std::isfinite(q)) return f;  // exactly representable: no tie to break
  const float other = fd < q ? std::nextafterf(f, INFINITY) : std::nextafterf(f, -INFINITY);
  const double mid = 0.5 * (fd + (double)other);
  const double margin = std::fabs(q - mid) / std::fabs(q);
  if (margin < c->thresh) c->near.push_back({idx, margin});
  return idx == c->force ? other : f;
}

// RAII: install a FlipCtl for one scope
struct FlipScope {
  FlipCtl *prev;
  explicit FlipScope(FlipCtl *c) : prev(g_flip) { g_flip = c; }
  ~FlipScope() { g_flip = prev; }
};

}  // namespace orc
