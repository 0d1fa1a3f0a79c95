# gemm_w5 SwiGLU prefill route: GPU SwiGLU tests, then timing vs the phased 256x128 tile and torch
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zn
mkdir -p $O
PLI_W5_SWIGLU_CHECK=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_swiglu.py -q -p no:cacheprovider --timeout 200 --timeout-method thread -rf > $O/pytest_swiglu.log 2>&1
rc=$?; tail -4 $O/pytest_swiglu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u - > $O/swiglu_timing.log 2>&1 <<'PY'
import sys, os, json, statistics, torch
sys.path[:0] = [os.path.join(os.getcwd(), "physics-llm-inference_amd"), os.getcwd()]
import pli_hip
import torch.nn.functional as F
for (m, n, k) in ((4096, 14336, 4096), (16384, 14336, 4096), (4096, 1792, 4096), (2048, 5632, 2048)):
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    wg = torch.randn(n, k, device="cuda", dtype=torch.bfloat16); wu = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    h = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    fns = {"w5": lambda: pli_hip.gemm_swiglu(x, wg, wu, out=h, variant=3),
           "phased": lambda: pli_hip.gemm_swiglu(x, wg, wu, out=h, variant=4),
           "torch": lambda: F.silu(x @ wg.t()) * (x @ wu.t())}
    for f in fns.values():
        for _ in range(3): f()
    res = {kk: [] for kk in fns}
    for _ in range(5):
        for kk, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10): f()
            e.record(); e.synchronize()
            res[kk].append(4 * m * n * k / (s.elapsed_time(e) / 10 * 1e-3) / 1e12)
    print(json.dumps({"m": m, "n": n, "k": k, "TFLOP/s": {kk: round(statistics.median(v), 1) for kk, v in res.items()}}), flush=True)
PY
rc=$?; grep -v amdgpu $O/swiglu_timing.log; exit $rc
