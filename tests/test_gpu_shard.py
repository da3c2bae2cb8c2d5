"""Feature-sharded MSCKF update on the GPU (UpdaterMSCKF.cpp:118-286).

* world 1 over a real RCCL communicator (ncclCommInitRank with one rank, ncclAllReduce on the library's
  stream): the sharded update path in lock-step against the oracle, same bounds as test_gpu_parity.py, on a
  EuRoC stream and at the BASELINE sizes it exists for (bench.py cfg4: 800 MSCKF features x 52 measurements,
  cfg5: 1500 features, IMU intrinsics, UWB), where the tiled T GEMM (m >= 4096), the MFMA Gram (m >= 8192),
  the chunked batch build (>= 256 features) and the n > 135 information-form factors run.
* world 2 and 4 on one MI355X at cfg4 / cfg5, and world 8 at cfg5 (BASELINE.json's "8xMI355X sharded
  compression" split, 8 ranks of the 1500-feature update) (one fresh process per rank, host all-reduce over
  gloo, since RCCL needs one GPU per rank): EVERY rank runs its own oracle in lock-step at the strict bounds (its MSCKF
  per-feature results are its shard of the oracle's), the replicas' states and covariances are bit-identical
  after every frame, and the shards are disjoint and together make up the oracle's update.
* world 2 on the EuRoC stream: the sharded run agrees with an unsharded run of the same stream.
* world 4 with at most 2 MSCKF features per update: every update leaves ranks with an empty chunk (no feature
  kernel, no rows, a zero Gram and a zero accepted count in the all-reduce); the replicas stay bit-identical and
  agree with an unsharded run.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from test_gpu_parity import _check_lockstep, _features_updated, _rel, _snap, _steer_cap, run_lockstep

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EUROC = os.path.join(ROOT, "configs", "euroc_mav", "estimator_config.yaml")
N_FRAMES = 30


def _opts(U, max_msckf=200):
    return U.load_options(EUROC, max_msckf_in_update=max_msckf, max_slam_features=20, max_slam_in_update=10,
                          dt_slam_delay=0.3)


def _stream(opts):
    from uvio_amd.sim import SimStream
    return SimStream(opts, duration=N_FRAMES / opts.track_frequency + 1.2, seed=5, spawn=120, frac_long=0.2)


def test_sharded_world1_rccl_lockstep():
    import uvio_amd as U
    from oracle import oracle as O
    from uvio_amd.manager import shard_unique_id
    opts = _opts(U)
    s = _stream(opts)
    g = U.VioManager(opts)
    g.enable_feature_sharding(0, 1, backend="rccl", unique_id=shard_unique_id(), min_features=1)
    steps = run_lockstep(opts, s, N_FRAMES, mgr=g)
    g.close()
    assert sum(a["timing"]["n_msckf"] for a, _ in steps) > 300
    _check_lockstep(steps)


def _free_port():
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    p = sk.getsockname()[1]
    sk.close()
    return p


def _rank(rank, world, port, q, max_msckf=200):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import uvio_amd as U
    opts = _opts(U, max_msckf)
    s = _stream(opts)
    g = U.VioManager(opts, device=0)
    g.enable_feature_sharding(rank, world, backend="host", min_features=1)
    frames = []

    def after(nf, t):
        x, _ = g.get_state_vector()
        tm = g.get_timing()
        frames.append((x, g.get_cov(), tm["n_msckf"], tm["msckf_rows"], len(g.debug_last_msckf()[0])))

    s.run(g, n_frames=N_FRAMES, on_frame=after)
    g.close()
    q.put((rank, frames))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_world2_gloo_one_gpu():
    import uvio_amd as U
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=240) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    f0, f1 = out[0][1], out[1][1]
    assert len(f0) == len(f1) == N_FRAMES
    local = 0
    for a, b in zip(f0, f1):
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), "replicas diverged"
        assert a[2] == b[2] and a[3] == b[3]  # global update set and accepted rows
        local += a[4]
        assert a[4] + b[4] <= a[2]  # each rank linearized only its chunk of the update's features
    assert local > 0 and sum(b[4] for b in f1) > 0  # both ranks did work
    # an unsharded run of the same stream
    opts = _opts(U)
    s = _stream(opts)
    g = U.VioManager(opts)
    ref = []
    s.run(g, n_frames=N_FRAMES, on_frame=lambda nf, t: ref.append((g.get_state_vector()[0], g.get_timing())))
    g.close()
    for (x, _, nm, rows, _), (xr, tr) in zip(f0, ref):
        assert nm == tr["n_msckf"]
    assert _rel(f0[-1][0], ref[-1][0]) < 1e-6


def test_sharded_more_ranks_than_features():
    import uvio_amd as U
    world, cap = 4, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, cap)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=240) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    frames = [o[1] for o in out]
    assert all(len(f) == N_FRAMES for f in frames)
    empty = updates = 0
    for k in range(N_FRAMES):
        frs = [f[k] for f in frames]
        assert all(np.array_equal(frs[0][0], fr[0]) and np.array_equal(frs[0][1], fr[1]) for fr in frs), ("replicas diverged", k)
        assert len({(fr[2], fr[3]) for fr in frs}) == 1
        assert frs[0][2] <= cap
        if frs[0][2] > 0:
            assert sum(fr[4] for fr in frs) <= frs[0][2]  # each rank linearized only its chunk
            updates += 1
            empty += sum(1 for fr in frs if fr[4] == 0)
    assert updates > 10 and empty >= 2 * updates  # >= 2 of the 4 ranks without a feature in every update
    opts = _opts(U, cap)
    s = _stream(opts)
    g = U.VioManager(opts)
    ref = []
    s.run(g, n_frames=N_FRAMES, on_frame=lambda nf, t: ref.append((g.get_state_vector()[0], g.get_timing())))
    g.close()
    for fr, (xr, tr) in zip(frames[0], ref):
        assert fr[2] == tr["n_msckf"]
    assert _rel(frames[0][-1][0], ref[-1][0]) < 1e-6


# ---- BASELINE sizes (bench.py cfg4 / cfg5 TrackSIM streams) ----
BIG = {"cfg4": 30, "cfg5": 35}


def _bench():
    import sys
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    return bench


def _big(wl):
    import uvio_amd as U
    B = _bench()
    opts = B.workload_options(U, wl)
    n = BIG[wl]
    return opts, B.make_stream(opts, n + 2, seed=5, workload=wl), n


def _assert_big(steps, wl):
    assert max(a["timing"]["n_msckf"] for a, _ in steps) == {"cfg4": 800, "cfg5": 1500}[wl]
    assert max(a["timing"]["msckf_rows"] for a, _ in steps) >= 8192


@pytest.mark.parametrize("wl", ["cfg4", "cfg5"])
def test_sharded_world1_rccl_lockstep_baseline_size(wl):
    import uvio_amd as U
    from uvio_amd.manager import shard_unique_id
    opts, s, n = _big(wl)
    g = U.VioManager(opts)
    g.enable_feature_sharding(0, 1, backend="rccl", unique_id=shard_unique_id(), min_features=1)
    steps = run_lockstep(opts, s, n, mgr=g)
    g.close()
    _assert_big(steps, wl)
    _check_lockstep(steps)


def _digest(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()


def _rank_lockstep(rank, world, port, q, wl):
    """one rank of a feature-sharded run over gloo, in lock-step with its own oracle"""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"rank": rank, "err": None}
    try:
        import uvio_amd as U
        opts, s, n = _big(wl)
        g = U.VioManager(opts, device=0)
        g.enable_feature_sharding(rank, world, backend="host", min_features=1)
        steps = run_lockstep(opts, s, n, mgr=g)
        g.close()
        out["frames"] = [(_digest(a["x"]), _digest(a["P"]), a["timing"]["n_msckf"], a["timing"]["msckf_rows"],
                          sorted(int(i) for i in a["feats"][0]), sorted(int(i) for i in b["feats"][0]))
                         for a, b in steps]
        out["steer"] = list(steps.steer)
        out["n_features"] = _features_updated(steps)
        try:
            out["worst"] = _check_lockstep(steps, max_events=None, sharded=True)
        except AssertionError as e:
            out["err"] = repr(e)[:4000]
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        out["err"] = "exception: " + repr(e)[:4000]
    q.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("wl,world", [("cfg4", 2), ("cfg4", 4), ("cfg5", 2), ("cfg5", 4), ("cfg5", 8)])
def test_sharded_gloo_lockstep_baseline_size(wl, world):
    from conftest import record_steer
    from test_gpu_parity import STEER_MARGIN
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_lockstep, args=(r, world, port, q, wl)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=280) for _ in range(world)], key=lambda o: o["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for o in outs:
        assert o["err"] is None, (o["rank"], o["err"])
    n = BIG[wl]
    f0 = outs[0]["frames"]
    assert all(len(o["frames"]) == n for o in outs)
    assert max(fr[2] for fr in f0) == {"cfg4": 800, "cfg5": 1500}[wl]
    assert max(fr[3] for fr in f0) >= 8192
    per_rank = [0] * world
    for k in range(n):
        frs = [o["frames"][k] for o in outs]
        # replicas: bit-identical state and covariance, same update set and accepted rows
        assert len({(fr[0], fr[1], fr[2], fr[3]) for fr in frs}) == 1, ("replicas diverged", k)
        # the shards: disjoint, and together the oracle's MSCKF update (every rank's oracle saw the same one)
        union = []
        for r, fr in enumerate(frs):
            union += fr[4]
            per_rank[r] += len(fr[4])
        assert len(union) == len(set(union)), ("shards overlap", k)
        assert sorted(union) == frs[0][5] and all(fr[5] == frs[0][5] for fr in frs), ("shards != update", k)
    assert min(per_rank) > 0, per_rank
    # the oracles' rounding-tie steering: every event one near tie, at most 1 % of the features updated
    ev = [e for o in outs for e in o["steer"]]
    nf = sum(o["n_features"] for o in outs)
    cap = _steer_cap(nf)
    record_steer(ev, nf, cap)
    assert all(e["found"] and e["margin"] < STEER_MARGIN for e in ev), ev
    assert len(ev) <= cap, (len(ev), cap)
    print("worst per rank", [o["worst"] for o in outs])
