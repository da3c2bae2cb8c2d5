"""Multi-rank plumbing of bench.py on CPU (gloo, world_size 2): each rank runs an independent
estimator replica; the job's wall time is the max over ranks (DESIGN.md "Multi-GPU")."""
import os
import socket

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    t = bench.max_over_ranks(1.5 + rank, device="cpu")
    # each replica runs its own stream: seeds differ per rank, shapes do not
    import uvio_amd as U
    opts = bench.cfg2_options(U)
    sim = bench.make_stream(opts, 12, seed=5 + rank)
    q.put((rank, t, len(sim.frames), sim.frames[3][0][1][:2].tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_max_over_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    assert [o[1] for o in out] == [2.5, 2.5]
    assert out[0][2] == out[1][2]
    assert out[0][3] != out[1][3]
