"""Multi-GPU path on CPU: world_size-2 gloo ranks exercise the bench's channel
sharding (C4: one 65,536-channel batch split into contiguous channel shards,
no data-path collective), its launcher (`bench.py --gpus N` without torchrun
spawns one process per GPU) and its timing reduction (MAX over ranks of the
timed region, SUM of channels) over the host gloo group."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_strong_is_c4_split():
    # C4: shard g = channels [g*C/N, (g+1)*C/N)
    for n in (1, 2, 4, 8):
        parts = [bench.shard(65536, n, r) for r in range(n)]
        assert parts == [(65536 // n, r * 65536 // n) for r in range(n)]
    parts = [bench.shard(65536, 3, r, True) for r in range(3)]
    assert sum(n for n, _ in parts) == 65536
    assert [c0 for _, c0 in parts] == [0, parts[0][0], parts[0][0] + parts[1][0]]
    assert bench.shard(10, 4, 3, True) == (2, 8)


def test_shard_weak():
    assert [bench.shard(65536, 8, r, False) for r in (0, 7)] == [(65536, 0), (65536, 7 * 65536)]


WORKER = textwrap.dedent('''
    import json, os, sys
    sys.path.insert(0, {root!r})
    import bench
    import singlecarrier_amd as sc
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["LOCAL_RANK"]) == rank
    dist = bench.init_host_group(rank, world)
    nch, c0 = bench.shard(1000, world, rank)
    # a rank's synthetic shard = the same channels of the whole batch (c0 offset)
    x = sc.synth(5, nch, 2, c0=c0)
    tmax, total = bench.reduce_step(dist, 0.5 + rank, nch)
    rows = [None] * world
    dist.all_gather_object(rows, {{"rank": rank, "ok": True}})
    with open(os.path.join({out!r}, f"r{{rank}}.json"), "w") as f:
        json.dump([rank, nch, c0, tmax, total, int(x[0, 0, :100].astype("int64").sum()), rows], f)
    dist.barrier()
    dist.destroy_process_group()
''')


def test_launcher_two_rank_gloo_sharding_and_reduction(tmp_path, capfd):
    """bench.launch() is what `python bench.py --gpus 2` runs without torchrun:
    two child processes with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, gloo on
    127.0.0.1, MAX of times and SUM of channels on every rank.  The group's
    setup writes nothing to stdout (rank 0's stdout is the bench's one JSON
    line)."""
    if not os.path.exists(os.path.join(ROOT, "singlecarrier_amd", "libqpsk_hip.so")):
        pytest.skip("library not built")
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT, out=str(tmp_path)))
    assert bench.launch(2, [], script=str(script)) == 0
    assert capfd.readouterr().out == ""
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(2)]
    (r0, n0, c00, t0, tot0, s0, g0), (r1, n1, c01, t1, tot1, s1, g1) = res
    assert (n0, n1, c00, c01) == (500, 500, 0, 500)
    assert t0 == t1 == 1.5 and tot0 == tot1 == 1000      # MAX of times, SUM of channels
    assert g0 == g1 == [{"rank": 0, "ok": True}, {"rank": 1, "ok": True}]
    import singlecarrier_amd as sc
    assert s1 == int(sc.synth(5, 1, 2, c0=500)[0, 0, :100].astype("int64").sum())


def test_launcher_reports_a_failing_rank(tmp_path):
    script = tmp_path / "fail.py"
    script.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    assert bench.launch(2, [], script=str(script)) == 3


def test_launcher_stops_the_peers_of_a_failed_rank(tmp_path):
    """A rank that fails early must not leave its peers blocked (in gloo's
    rendezvous, a barrier or a reduction) until a timeout: launch() watches
    every child, terminates the rest and returns the failing status."""
    import time
    script = tmp_path / "hang.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1':\n    sys.exit(5)\n"
                      "time.sleep(600)\n")
    t = time.perf_counter()
    assert bench.launch(3, [], script=str(script)) == 5
    assert time.perf_counter() - t < 60


def test_launcher_kills_a_peer_that_ignores_sigterm(tmp_path):
    """A peer that ignores SIGTERM is killed after the grace period instead of
    holding the launcher; a rank ended by a signal reports
    128 + signum, never a negative status."""
    import time
    script = tmp_path / "stubborn.py"
    script.write_text("import os, signal, sys, time\n"
                      "signal.signal(signal.SIGTERM, signal.SIG_IGN)\n"
                      "if os.environ['RANK'] == '1':\n    time.sleep(0.5)\n    sys.exit(4)\n"
                      "time.sleep(600)\n")
    t = time.perf_counter()
    assert bench.launch(2, [], script=str(script), grace_s=1.0) == 4
    assert time.perf_counter() - t < 30
    sig = tmp_path / "sig.py"
    sig.write_text("import os, signal\n"
                   "if os.environ['RANK'] == '0':\n    os.kill(os.getpid(), signal.SIGKILL)\n")
    assert bench.launch(2, [], script=str(sig)) == 128 + 9


def test_bench_gpus_flag_spawns_ranks():
    """`bench.py --gpus 2` with no WORLD_SIZE runs itself as 2 ranks through
    bench.launch(); --dry-run takes every rank through the host gloo group,
    its C4 shard and the MAX/SUM reduction, and stops before any GPU call.
    Rank 0's stdout is the one JSON line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["dry_run"] and out["world"] == 2 and out["channels_total"] == 65536
    assert out["max_time_s"] == 0.002 and out["scaling"] == "strong"
    assert out["shards"] == [{"rank": 0, "local_rank": 0, "channels": [0, 32768]},
                             {"rank": 1, "local_rank": 1, "channels": [32768, 65536]}]


def test_host_cpus_honours_the_cgroup_quota(monkeypatch):
    """The all-cores CPU baseline runs one reference process per CPU this job
    may use: the affinity set, capped by the cgroup quota (the GPU boxes show
    256 CPUs of affinity and a cpu.max of 16 CPUs)."""
    base = {"nproc": 256, "cpu_model": "x", "omp_num_threads": None}
    monkeypatch.setattr(bench, "cpu_info", lambda: {**base, "affinity_cpus": 256, "cgroup_cpu_quota": 16.0})
    assert bench.host_cpus() == 16
    monkeypatch.setattr(bench, "cpu_info", lambda: {**base, "affinity_cpus": 8, "cgroup_cpu_quota": None})
    assert bench.host_cpus() == 8
    monkeypatch.setattr(bench, "cpu_info", lambda: {**base, "affinity_cpus": 4, "cgroup_cpu_quota": 0.5})
    assert bench.host_cpus() == 1
