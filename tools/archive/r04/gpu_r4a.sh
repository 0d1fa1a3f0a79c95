# v13 first hardware run: smoke (small shape vs f64), the v13 GPU tests, A/B vs v12
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 120 python -u - > $O/smoke.log 2>&1 <<'PY'
import sys, os, torch
sys.path[:0] = [os.path.join(os.getcwd(), "physics-llm-inference_amd"), os.getcwd(), os.path.join(os.getcwd(), "tests")]
import pli_hip
for (B, H, Nq, Nk) in ((1, 1, 256, 128), (1, 1, 256, 256), (1, 2, 300, 192), (2, 8, 1024, 1024)):
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, n, 128, device="cuda", dtype=torch.bfloat16, generator=g) for n in (Nq, Nk, Nk))
    ref = torch.softmax((q.double() @ k.double().transpose(-1, -2)) * 128 ** -0.5, -1) @ v.double()
    for var in (80, 81, 82):
        o = pli_hip.flash_attn_fwd(q, k, v, variant=var)
        torch.cuda.synchronize()
        print(B, H, Nq, Nk, var, "max err", (o.double() - ref).abs().max().item(), flush=True)
    if Nq == Nk:
        s = (q.double() @ k.double().transpose(-1, -2)) * 128 ** -0.5
        s = s.masked_fill(torch.ones(Nq, Nk, device="cuda", dtype=torch.bool).triu(1), float("-inf"))
        ref = torch.softmax(s, -1) @ v.double()
        for var in (83, 84, 85):
            o = pli_hip.flash_attn_fwd(q, k, v, causal=True, variant=var)
            torch.cuda.synchronize()
            print(B, H, Nq, Nk, "causal", var, "max err", (o.double() - ref).abs().max().item(), flush=True)
PY
rc=$?; cat $O/smoke.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_flash_v13.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_v13.log 2>&1
rc=$?; tail -5 $O/pytest_v13.log; [ $rc -eq 0 ] || exit $rc
LIBS=physics-llm-inference_amd/pli_hip/libpli_hip.so VARIANTS=71,80,81 ROUNDS=8 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; [ $rc -eq 0 ] || exit $rc
CAUSAL=1 LIBS=physics-llm-inference_amd/pli_hip/libpli_hip.so VARIANTS=74,83 ROUNDS=8 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_causal.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab_causal.log; exit $rc
