#!/usr/bin/env python3
"""GB/s of each pli_hbm_read_probe layout (GPU box): grid-stride vs one
contiguous slice per workgroup, several workgroups per CU, 2 x 1 GiB buffers."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]
import pli_hip  # noqa: E402

nbytes = 1 << 30
bufs = [torch.empty(nbytes // 4, device="cuda", dtype=torch.int32).fill_(i + 1) for i in range(2)]
res = {}
for mode, per_cu in ((0, 4), (0, 8), (0, 16), (1, 1), (1, 2), (1, 4), (1, 8), (1, 16)):
    blocks = 256 * per_cu
    out = torch.empty(blocks * 256, device="cuda", dtype=torch.int32)
    for b in bufs:
        pli_hip.hbm_read_probe(b, out, blocks, mode)
    best = 1e9
    for i in range(10):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        pli_hip.hbm_read_probe(bufs[i & 1], out, blocks, mode)
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / 1e3)
    res[f"mode{mode}_wg_per_cu{per_cu}"] = round(nbytes / best / 1e9, 1)
print(json.dumps(res))
