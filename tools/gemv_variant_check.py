"""Every pli_gemv variant agrees with the fp32 product on a few shapes (GPU)."""
import sys
sys.path[:0] = ["physics-llm-inference_amd", "."]
import torch, pli_hip
torch.manual_seed(0)
for (m, k, dt) in [(4096, 4096, torch.bfloat16), (2048, 2048, torch.bfloat16), (333, 520, torch.float16),
                   (16385, 2048, torch.bfloat16), (7, 8192, torch.float16)]:
    w = torch.randn(m, k, device="cuda", dtype=dt)
    x = torch.randn(k, device="cuda", dtype=dt)
    ref = (w.float() @ x.float())
    for v in range(17):
        y = pli_hip.gemv(w, x, variant=v).float()
        err = ((y - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-2, (m, k, dt, v, err)
    print("ok", m, k, dt, flush=True)
