"""bench.py on hardware (run with -m gpu): the N = 1 line and the N = 2
launcher.  On a one-GPU box both ranks share the GPU (`shared_gpus` in the
line; the time is not a scaling figure): what is checked is the contract the
driver reads -- rank 0's stdout is exactly one JSON line -- and per-rank
parity of the timed outputs against the oracle."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "2", "--warmup", "1", "--channels", "4096", "--cpu-channels", "0",
         "--cpu-all-channels", "0", "--stream-chunks", "0", "--verify", "64"]


def _run(args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_one_gpu_line():
    d = _run(SMALL)
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["verified_vs_oracle"] is True
    assert d["config"]["channels_total"] == 4096 and d["roofline"]["kernels_us"]["rx_kernel"] > 0


def test_bench_two_ranks_one_json_line():
    d = _run(["--gpus", "2", *SMALL])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["channels_per_gpu"] == 2048 and d["config"]["channels_total"] == 4096
    assert [v["channels"][0] for v in d["verified_per_rank"]] == [0, 2048]
    assert d["verified_vs_oracle"] is True
