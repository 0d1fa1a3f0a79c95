import os, sys
sys.path[:0] = ["physics-llm-inference_amd", "."]
import torch, pli_hip
from bench import paired_time_ms
st = torch.cuda.current_stream()
for (n, k) in ([(16384, 1024), (8192, 1024), (32000, 1024), (4096, 1024), (32000, 2048)] if os.environ.get('GV_SHORT') else [(8192, 8192), (2048, 5632), (2048, 2048), (3072, 2048), (32000, 2048), (4096, 4096), (32000, 4096), (16384, 1024), (128256, 2048)]):
    # rotate over enough copies to exceed the 256 MiB MALL
    copies = max(2, (768 << 20) // (n * k * 2))
    ws = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
    x = torch.randn(1, k, device="cuda", dtype=torch.bfloat16)
    y = torch.empty(1, n, device="cuda", dtype=torch.bfloat16)
    yv = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    it = {"i": 0}
    def nxt():
        it["i"] = (it["i"] + 1) % copies
        return ws[it["i"]]
    fns = {"gemv": lambda: pli_hip.gemv(nxt(), x[0], out=yv),
           "torch": lambda: torch.nn.functional.linear(x, nxt())}
    for v in (8, 9, 10, 15, 16):
        fns[f"gemv_v{v}"] = (lambda v=v: pli_hip.gemv(nxt(), x[0], out=yv, variant=v))
    t = paired_time_ms(fns, 4 * copies, st, rounds=5)
    print(n, k, {kk: round(n * k * 2 / (v * 1e-3) / 1e9) for kk, v in t.items()}, "GB/s", flush=True)
    del ws
