#!/usr/bin/env python3
"""Graph-replayed ch02 decode steps (tools/tune.py's 0.85B Llama shape) for a
rocprofv3 kernel-trace: python tools/decode_prof.py [batch] [steps]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import torch  # noqa: E402

from ch02 import CachedTransformerModel  # noqa: E402
from ch08 import DecodeStepGraph  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
prompt = 512
torch.manual_seed(0)
model = CachedTransformerModel(32000, 2048, 16, 32, 8, 5632).cuda().bfloat16().eval()
ids = torch.randint(0, 32000, (B, prompt), device="cuda")
tok = torch.randint(0, 32000, (B, 1), device="cuda")
with torch.no_grad():
    g = DecodeStepGraph(model, B, prompt + steps + 8, torch.bfloat16)
    g.prefill(ids)
    g.step(tok)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.step(tok)
    torch.cuda.synchronize()
print(f"batch {B}: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms/token", flush=True)
