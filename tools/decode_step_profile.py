#!/usr/bin/env python3
"""Run graph-replayed decode steps of the Llama-shaped model (tools/tune.py
graph) for a rocprofv3 kernel trace:  rocprofv3 --kernel-trace --stats -- \\
python tools/decode_step_profile.py [batch] [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]

import torch  # noqa: E402

from ch02 import CachedTransformerModel  # noqa: E402
from ch08 import DecodeStepGraph  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
torch.manual_seed(0)
model = CachedTransformerModel(32000, 2048, 16, 32, 8, 5632).cuda().bfloat16().eval()
g = DecodeStepGraph(model, B, 512 + N + 8, torch.bfloat16)
g.prefill(torch.randint(0, 32000, (B, 512), device="cuda"))
tok = torch.randint(0, 32000, (B, 1), device="cuda")
for _ in range(N):
    g.step(tok)
torch.cuda.synchronize()
print("steps", N, "seq_len", g.seq_len)
