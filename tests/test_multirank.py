"""Multi-GPU path on CPU: world_size-2 gloo ranks exercise the bench's channel
sharding (distinct channels per rank, no data-path collective) and its timing
reduction (MAX over ranks of the timed region, SUM of channels)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

import bench


def test_shard_weak_and_strong():
    assert [bench.shard(65536, 8, r, False) for r in (0, 7)] == [(65536, 0), (65536, 7 * 65536)]
    parts = [bench.shard(65536, 3, r, True) for r in range(3)]
    assert sum(n for n, _ in parts) == 65536
    assert [c0 for _, c0 in parts] == [0, parts[0][0], parts[0][0] + parts[1][0]]
    assert bench.shard(10, 4, 3, True) == (2, 8)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nch, c0 = bench.shard(1000, world, rank, strong=True)
    # synthetic per-rank inputs are distinct channel ids: same generator, offset c0
    import singlecarrier_amd as sc
    x = sc.synth(5, nch, 2, c0=c0)
    tmax, total = bench.reduce_step(dist, 0.5 + rank, nch, torch.device("cpu"))
    q.put((rank, nch, c0, tmax, total, int(x[0, 0, :100].astype("int64").sum())))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_sharding_and_reduction():
    if not os.path.exists(os.path.join(os.path.dirname(bench.__file__), "singlecarrier_amd",
                                       "libqpsk_hip.so")):
        pytest.skip("library not built")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, n0, c00, t0, tot0, s0), (r1, n1, c01, t1, tot1, s1) = res
    assert (n0, n1, c00, c01) == (500, 500, 0, 500)
    assert t0 == t1 == 1.5 and tot0 == tot1 == 1000      # MAX of times, SUM of channels
    import singlecarrier_amd as sc
    assert s1 == int(sc.synth(5, 1, 2, c0=500)[0, 0, :100].astype("int64").sum())
