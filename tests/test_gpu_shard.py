"""Feature-sharded MSCKF update on the GPU.

* world 1 over a real RCCL communicator (ncclCommInitRank with one rank, ncclAllReduce on the library's
  stream): the sharded update path in lock-step against the oracle, same bounds as test_gpu_parity.py.
* world 2 on one MI355X (two processes, host all-reduce over gloo, since RCCL needs one GPU per rank):
  both replicas hold bit-identical states after every frame, each rank linearized only its chunk, and
  the run agrees with an unsharded run of the same stream (same update sets; final state within 1e-6
  relative: the Gram sums in a different association, and the filter carries the rounding forward).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from test_gpu_parity import _check_lockstep, _rel, _snap, run_lockstep

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EUROC = os.path.join(ROOT, "configs", "euroc_mav", "estimator_config.yaml")
N_FRAMES = 30


def _opts(U):
    return U.load_options(EUROC, max_msckf_in_update=200, max_slam_features=20, max_slam_in_update=10,
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


def _rank(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import uvio_amd as U
    opts = _opts(U)
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
