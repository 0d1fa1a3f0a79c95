import os, sys, json, torch
sys.path[:0] = [os.path.join(os.getcwd(), "physics-llm-inference_amd"), os.getcwd()]
import pli_hip
g = torch.Generator(device="cuda").manual_seed(5)
for Nk in (64, 128, 192):
    q = torch.randn(1, 1, 256, 128, device="cuda", dtype=torch.bfloat16, generator=g)
    k = torch.randn(1, 1, Nk, 128, device="cuda", dtype=torch.bfloat16, generator=g)
    v = torch.randn(1, 1, Nk, 128, device="cuda", dtype=torch.bfloat16, generator=g)
    a = pli_hip.flash_attn_fwd(q, k, v, variant=55).float()[0, 0]
    b = pli_hip.flash_attn_fwd(q, k, v, variant=70).float()[0, 0]
    r = (b / a)
    out = {"Nk": Nk}
    for row in (0, 1, 31, 32, 33, 63, 64):
        rr = r[row]
        out[f"row{row}"] = [round(rr.median().item(), 4), round(rr.min().item(), 3), round(rr.max().item(), 3),
                            round((b[row]-a[row]).abs().max().item(), 4)]
    print(json.dumps(out), flush=True)
