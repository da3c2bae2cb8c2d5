"""GPU: the FAST cell selection in Grider_GRID.h:128's std::sort order (kernels_track.hip grid_introsort,
k_fast_select) against the oracle, which calls libstdc++'s std::sort itself (tests/test_grid_sort.py pins the
oracle to the libstdc++ algorithm and the device's formulation to the oracle on the CPU).

  * the probe (uvio_hp_debug_grid_order, the same __device__ code as k_fast_select) on random cells with many
    tied responses: the introsort loop's arrangement, stably ordered, equals std::sort's order bit for bit; the
    pruned top-k the kernel uses equals std::sort's first k; depth 0 (the heap-sort fallback) equals
    std::partial_sort;
  * the tracker on a corner-dense image pair: ids and points equal the oracle's after every frame, with most
    cells on the introsort path (uvio_hp_debug_grid_stats) and cells whose std::sort pick differs from the
    stable pick (the order rounds 1-5 used).
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _cells(rng, count, nmax):
    out = []
    for _ in range(count):
        n = int(rng.integers(1, nmax))
        spread = int(rng.choice([2, 5, 12, 40, 200]))
        out.append(rng.integers(21, 21 + spread, n))
    return out


def test_probe_arrangement_is_std_sort():
    from uvio_amd.manager import grid_order
    from oracle import oracle as O
    rng = np.random.default_rng(21)
    cells = _cells(rng, 1500, 700) + [rng.integers(20, 23, 2000), rng.integers(20, 255, 4000), np.full(300, 40)]
    arrs, _ = grid_order(cells, kmax=0)
    intro = 0
    for c, a in zip(cells, arrs):
        a = np.asarray(a)
        assert sorted(a.tolist()) == list(range(len(c)))
        got = a[np.argsort(-np.asarray(c)[a], kind="stable")]
        ref = O.grid_order(np.asarray(c, dtype=np.float32), 0)
        assert np.array_equal(got, ref), len(c)
        intro += len(c) > 16
    print("cells %d, on the introsort path %d" % (len(cells), intro))


@pytest.mark.parametrize("kmax", [1, 2, 9, 17, 64])
def test_probe_top_k_is_std_sort(kmax):
    from uvio_amd.manager import grid_order
    from oracle import oracle as O
    rng = np.random.default_rng(100 + kmax)
    cells = _cells(rng, 1000, 500)
    _, tops = grid_order(cells, kmax=kmax)
    differ = 0
    for c, top in zip(cells, tops):
        r = np.asarray(c, dtype=np.float32)
        ref = O.grid_order(r, 0)[:min(kmax, len(c))]
        assert np.array_equal(top, ref), (len(c), kmax)
        differ += not np.array_equal(ref, O.grid_order(r, 1)[:min(kmax, len(c))])
    print("kmax %d: std::sort pick != stable pick in %d of %d cells" % (kmax, differ, len(cells)))
    if kmax > 1:
        assert differ > 0


def test_probe_heap_sort_fallback():
    from uvio_amd.manager import grid_order
    from oracle import oracle as O
    rng = np.random.default_rng(7)
    cells = [c for c in _cells(rng, 300, 300) if len(c) > 16]
    arrs, _ = grid_order(cells, kmax=0, depth=0)
    for c, a in zip(cells, arrs):
        a = np.asarray(a)
        got = a[np.argsort(-np.asarray(c)[a], kind="stable")]
        assert np.array_equal(got, O.grid_order(np.asarray(c, dtype=np.float32), 2)), len(c)


def _dense_pair(w, h, seed):
    """A binary block texture (every block edge a FAST corner candidate, responses tied in small integers) and
    the same texture shifted by a sub-block offset."""
    rng = np.random.default_rng(seed)
    base = (rng.integers(0, 2, (h // 3 + 4, w // 3 + 4)) * 150 + 50).astype(np.uint8)
    big = np.kron(base, np.ones((3, 3), dtype=np.uint8))
    noise = rng.integers(0, 3, big.shape).astype(np.uint8)
    big = big + noise
    return [big[2 + d:2 + d + h, 3 + d:3 + d + w].copy() for d in range(4)]


def test_tracks_bit_exact_dense_corners(euroc_yaml):
    """The stereo tracker on corner-dense frames: nearly every cell has more than 16 FAST candidates with tied
    responses, so the kept corners and their ids depend on std::sort's order; the device equals the oracle."""
    import uvio_amd as U
    from oracle import oracle as O
    from test_gpu_track import _compare_tracks
    opts = U.load_options(euroc_yaml, init_max_features=200)
    w, h = opts.cams[0].width, opts.cams[0].height
    g, o = U.VioManager(opts), O.OracleManager(opts)
    frames = _dense_pair(w, h, 4)
    total = bad = 0
    for i, img in enumerate(frames):
        t = 0.05 * (i + 1)
        imgs = [img, np.roll(img, 2, axis=1)]
        g.feed_measurement_camera(t, [0, 1], imgs, allow_uninit=True)
        o.feed_measurement_camera(t, [0, 1], imgs, allow_uninit=True)
        n, b = _compare_tracks(g, o, [0, 1])
        total += n
        bad += b
    cells, intro = g.grid_stats()
    print("dense corners: %d tracks, %d FAST cells, %d on the introsort path" % (total, cells, intro))
    assert intro > 0.5 * cells > 0
    assert total > 200
    assert bad == 0, (bad, total)
