# gemm_w5 fp32 epilogue (pli_gemm_f32out): parity tests, TP parity tests, then bench TP leg timing
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zm
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gemm_1wave.py -k "f32out or row_parallel or w5 or w4v" -q -p no:cacheprovider --timeout 200 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u - > $O/f32out_timing.log 2>&1 <<'PY'
import sys, os, json, torch
sys.path[:0] = [os.path.join(os.getcwd(), "physics-llm-inference_amd"), os.getcwd()]
import pli_hip
for (m, n, k) in ((8192, 8192, 1024), (8192, 8192, 8192)):
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16); w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    for _ in range(5): pli_hip.gemm_f32out(x, w); pli_hip.gemm(x, w, trans_b=True)
    res = {}
    for name, fn in (("f32out", lambda: pli_hip.gemm_f32out(x, w)), ("bf16", lambda: pli_hip.gemm(x, w, trans_b=True))):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20): fn()
        e.record(); e.synchronize()
        res[name + "_us"] = round(s.elapsed_time(e) / 20 * 1e3, 1)
    print(json.dumps({"m": m, "n": n, "k": k, **res}), flush=True)
PY
rc=$?; cat $O/f32out_timing.log | grep -v amdgpu; exit $rc
