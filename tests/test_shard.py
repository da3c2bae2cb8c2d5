"""Feature sharding host logic on CPU: the row-balanced contiguous partition the sharded
MSCKF update uses (uvio_hp_shard_partition, C ABI) and the host all-reduce callback over a gloo process
group with world_size 2 (the path the GPU test uses when two ranks share one MI355X)."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_partition_contiguous_and_balanced(seed):
    from uvio_amd.manager import shard_partition
    rng = np.random.default_rng(seed)
    for n in [0, 1, 7, 200, 1500]:
        rows = 2 * rng.integers(2, 60, n) - 3
        for world in [1, 2, 3, 4, 8]:
            b = shard_partition(rows, world)
            assert b[0] == 0 and b[-1] == n and np.all(np.diff(b) >= 0)
            if n == 0:
                continue
            total = rows.sum()
            sums = [rows[b[r]:b[r + 1]].sum() for r in range(world)]
            assert sum(sums) == total
            # every chunk within one feature of its share (midpoint rule)
            assert max(abs(s - total / world) for s in sums) <= rows.max() + 1e-9


def test_partition_matches_reference_order():
    """Uniform rows split evenly and in order (features stay in the selection's sorted order)."""
    from uvio_amd.manager import shard_partition
    assert list(shard_partition([101] * 10, 3)) == [0, 3, 7, 10]
    assert list(shard_partition([5, 5], 4)) == [0, 0, 1, 1, 2]
    assert list(shard_partition([1, 1, 1, 50, 1, 1], 2)) == [0, 3, 6]


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
    from uvio_amd.manager import host_allreduce_callback, shard_partition
    # the library's view: a host buffer of doubles handed to the callback
    cb = host_allreduce_callback()
    n = 173 * 173 + 2
    buf = (C.c_double * n)()
    vals = np.arange(n, dtype=np.float64) * (rank + 1) + 0.25 * rank
    for i in range(n):
        buf[i] = vals[i]
    rc = cb(buf, n, None)
    out = np.ctypeslib.as_array(buf)
    # every rank splits the same feature list and takes its own chunk
    rows = 2 * np.random.default_rng(3).integers(2, 53, 800) - 3
    b = shard_partition(rows, world)
    q.put((rank, rc, out.copy(), (int(b[rank]), int(b[rank + 1]))))
    dist.barrier()
    dist.destroy_process_group()


def test_host_allreduce_callback_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=240) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 173 * 173 + 2
    want = np.arange(n, dtype=np.float64) * 3 + 0.25
    for rank, rc, arr, _ in out:
        assert rc == 0
        assert np.array_equal(arr, want)
    # both ranks hold bit-identical sums (the replicas apply the same update)
    assert np.array_equal(out[0][2], out[1][2])
    # the chunks tile the feature list
    (a0, a1), (b0, b1) = out[0][3], out[1][3]
    assert a0 == 0 and a1 == b0 and b1 == 800
