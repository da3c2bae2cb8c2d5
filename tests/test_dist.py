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


WORKER = r'''
import json, os, sys
import torch, torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
t = torch.tensor([float(r + 1)])
dist.all_reduce(t)
assert int(os.environ["LOCAL_RANK"]) == r and os.environ["MASTER_ADDR"] == "127.0.0.1"
if r == 0:
    print(json.dumps({"n_gpus": w, "sum": float(t.item()), "argv": sys.argv[1:]}))
dist.destroy_process_group()
'''


def test_bench_launcher_spawns_world(tmp_path, capsys):
    """bench.py --gpus N without torch.distributed.run spawns N ranks itself (env rendezvous on 127.0.0.1)
    and passes rank 0's JSON line through; here the workers are a gloo stand-in for the GPU bench."""
    import json
    import sys
    sys.path.insert(0, ROOT)
    import bench
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    rc = bench.spawn_workers(2, ["--gpus", "2", "--steps", "3"], script=str(script))
    assert rc == 0
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["n_gpus"] == 2 and out["sum"] == 3.0
    assert out["argv"] == ["--gpus", "2", "--steps", "3"]
