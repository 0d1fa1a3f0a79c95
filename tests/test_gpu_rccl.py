"""RCCL ("nccl" backend) and the HIP library in one process (reference
ch09/tensor_parallel.py:43-68; worker: tests/rccl_worker.py).

* one rank on the one-GPU box: a one-rank process group passed explicitly to
  RowParallelLinear and row_parallel_forward_overlapped, so the all-reduce
  (identity at one rank) runs on RCCL's stream after pli_gemm /
  pli_gemm_f32out -- every result bitwise equal to the same GEMMs without the
  group;
* two ranks on two GPUs where the box has them (the row-parallel sum).

Each rank is a child process (fresh HIP context per rank, a free port)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

WORKER = os.path.join(os.path.dirname(__file__), "rccl_worker.py")


def _run(world: int):
    with socket.socket() as sk:  # a free port: a stale listener on a fixed one would fail the rendezvous
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, WORKER, str(r), str(world)], env=env, stdout=subprocess.PIPE,
                              text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    results = [json.loads(o.strip().splitlines()[-1]) for o in outs if o.strip()]
    print(results)
    assert [p.returncode for p in procs] == [0] * world, results
    return results


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a ROCm device")
@pytest.mark.timeout(120)
def test_rccl_one_rank_with_hip_library():
    (r,) = _run(1)
    assert r["backend"] == "nccl" and r["ok"], r
    assert r["checks"]["overlapped_eq_chunked_gemm"] and r["checks"]["f32_overlapped_eq_chunked"], r


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="needs >= 2 visible GPUs (RCCL all-reduce of the row-parallel partials)")
@pytest.mark.timeout(120)
def test_rccl_two_ranks_row_parallel():
    res = _run(2)
    assert all(r["ok"] for r in res), res
