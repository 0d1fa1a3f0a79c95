"""bench.py's multi-rank contract on CPU (no GPU): ``python bench.py --gpus
N`` started as one process launches N ranks itself, they rendezvous (gloo
here, RCCL on the node), time with a barrier and a max over ranks, and rank 0
prints one JSON line with ``n_gpus`` = N.  ``--selftest`` swaps the flash
step for a CPU matmul so the launch path runs without a device."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {}, PLI_BENCH_BACKEND="gloo")
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=ROOT)


@pytest.mark.timeout(300)
def test_bench_gpus2_launches_two_ranks():
    r = _run(["--gpus", "2", "--selftest", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    # gloo itself prints "[Gloo] Rank i is connected ..." lines to stdout
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON line, from rank 0
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["backend"] == "gloo"
    assert d["steps"] == 3 and d["warmup"] == 1 and d["value"] > 0
    assert d["data"].startswith("SELFTEST")


@pytest.mark.timeout(120)
def test_bench_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--selftest"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 3 and "WORLD_SIZE 1 != --gpus 2" in r.stderr
