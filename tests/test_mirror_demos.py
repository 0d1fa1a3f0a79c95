"""The reference modules' public demo helpers and __main__ blocks exist on
the mirrors too (explain_* texts, verify_tensor_core_usage,
benchmark_graph_vs_eager, compare_generation_methods, the chapter demos):
CPU checks here (no device: the GPU legs return None / are skipped), the
device legs in test_gpu_mirror_demos below."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest
import torch

from conftest import PKG

MAINS = ["ch05.memory_coalescing", "ch06.flash_attention", "ch06.attention_memory", "ch06.online_softmax", "ch09.nccl_primitives",
         "ch09.tensor_parallel", "ch05.tensor_cores", "ch05.triton_matmul", "ch05.shared_memory",
         "ch08.cuda_graph", "ch09.moe_layer"]


def test_explain_texts():
    from ch05.tensor_cores import explain_tensor_cores
    from ch05.triton_matmul import triton_matmul_explained
    from ch09.nccl_primitives import explain_nccl
    from ch09.tensor_parallel import explain_tensor_parallelism
    for f in (explain_tensor_cores, triton_matmul_explained, explain_nccl, explain_tensor_parallelism):
        text = f()
        assert isinstance(text, str) and len(text) > 200


@pytest.mark.skipif(torch.cuda.is_available(), reason="CPU-only behaviour")
def test_device_helpers_without_device():
    from ch05.tensor_cores import verify_tensor_core_usage
    from ch08.cuda_graph import benchmark_graph_vs_eager
    assert verify_tensor_core_usage(256) is None
    assert benchmark_graph_vs_eager(torch.relu, (16,)) is None


@pytest.mark.parametrize("mod", MAINS)
def test_demo_main_runs(mod):
    """`python -m <module>` as the reference's __main__ (CPU: the device legs skip)"""
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([PKG, os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-m", mod], cwd=PKG, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(r.stdout) > 100


@pytest.mark.gpu
def test_gpu_mirror_demos():
    from ch05.tensor_cores import verify_tensor_core_usage
    from ch08.cuda_graph import benchmark_graph_vs_eager
    v = verify_tensor_core_usage(1024)
    assert v["likely_tensor_cores"] and v["speedup"] > 1.5
    fn = lambda t: torch.sigmoid(torch.relu(t) * 2.0)  # noqa: E731
    r = benchmark_graph_vs_eager(fn, (1024,), batch_size=4, iterations=50)
    assert r["eager_us"] > 0 and r["graph_us"] > 0
    assert set(r) == {"batch_size", "input_shape", "eager_us", "graph_us", "speedup"} and r["input_shape"] == (1024,)
    # the replayed graph computes what the eager call does (checked here, not in the helper)
    x = torch.randn(4, 1024, device="cuda")
    static_in = torch.zeros_like(x)
    fn(static_in)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static_out = fn(static_in)
    static_in.copy_(x)
    g.replay()
    torch.testing.assert_close(static_out, fn(x))
