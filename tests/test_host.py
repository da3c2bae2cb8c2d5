"""Host-side building blocks of the product compiled for the CPU (no GPU needed): the worker pool that
runs the feature-database loops (uvio_amd/csrc/pool.h) -- every index visited exactly once, results
independent of the thread count, exceptions rethrown on the caller, many back-to-back jobs."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r'''
#include "pool.h"
#include <cstdio>
#include <stdexcept>
#include <vector>
using namespace uvhp;
int main() {
  WorkPool pool;
  int bad = 0;
  for (int rep = 0; rep < 2000; rep++) {
    size_t n = 1 + (rep * 7919) % 50000;
    std::vector<int> hit(n, 0);
    pool.parallel_for(n, 1 + rep % 300, [&](size_t b, size_t e) { for (size_t i = b; i < e; i++) hit[i]++; });
    for (size_t i = 0; i < n; i++) bad += hit[i] != 1;
  }
  int caught = 0;
  try {
    pool.parallel_for(100000, 64, [&](size_t b, size_t e) { if (b <= 5000 && 5000 < e) throw std::runtime_error("x"); });
  } catch (const std::runtime_error &) { caught = 1; }
  std::vector<int> after(1000, 0);
  pool.parallel_for(1000, 10, [&](size_t b, size_t e) { for (size_t i = b; i < e; i++) after[i] = 1; });
  for (int v : after) bad += v != 1;
  std::printf("%d %d %d\n", bad, caught, pool.threads());
  return 0;
}
'''


def test_work_pool(tmp_path):
    c = tmp_path / "pool_test.cpp"
    c.write_text(SRC)
    exe = tmp_path / "pool_test"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "uvio_amd", "csrc"),
                           str(c), "-o", str(exe)])
    for threads in ["1", "3", "8"]:
        env = dict(os.environ, UVIO_HP_THREADS=threads)
        bad, caught, nthreads = map(int, subprocess.check_output([str(exe)], env=env, timeout=120).split())
        assert bad == 0 and caught == 1 and nthreads == int(threads)
