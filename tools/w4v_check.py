#!/usr/bin/env python3
"""GPU box: gemm_w4v (variant 40) correctness against the 256 tile (variant 2,
same MFMA chain order: bitwise) and an f64 product, then interleaved timing
against the default route and torch (hipBLASLt) on the bench shapes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]

import torch  # noqa: E402

import pli_hip  # noqa: E402

VAR = int(os.environ.get("VARIANT", "40"))  # 40 gemm_w4v, 41 gemm_w5 (K % 64 shapes only)


def ev_ms(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def check(m, n, k, tb, dt=torch.bfloat16, bias=False):
    g = torch.Generator(device="cuda").manual_seed(m * 7 + n * 3 + k)
    a = torch.randn(m, k, device="cuda", dtype=dt, generator=g)
    b = torch.randn(n, k, device="cuda", dtype=dt, generator=g) if tb else torch.randn(k, n, device="cuda", dtype=dt,
                                                                                        generator=g)
    bs = torch.randn(n, device="cuda", dtype=dt, generator=g) if bias else None
    o = pli_hip.gemm(a, b, trans_b=tb, bias=bs, variant=VAR)
    ref = a.double() @ (b.double().t() if tb else b.double())
    if bias:
        ref = ref + bs.double()
    err = ((o.double() - ref).abs() / (ref.abs() + 1)).max().item()
    res = {"m": m, "n": n, "k": k, "nt": tb, "dtype": str(dt), "bias": bias, "max_rel_err_f64": err}
    if k % 64 == 0 and m >= 512 and n >= 512:
        o2 = pli_hip.gemm(a, b, trans_b=tb, bias=bs, variant=2)
        res["bitwise_eq_v2"] = bool(torch.equal(o, o2))
        res["max_diff_v2"] = (o.float() - o2.float()).abs().max().item()
    print(json.dumps(res), flush=True)
    return err


def main():
    bad = 0
    for (m, n, k) in ((512, 512, 64), (256, 256, 32), (4096, 4096, 4096), (300, 520, 96), (1000, 776, 4096),
                      (777, 1032, 160), (2048, 8192, 1024)):
        if VAR in (41, 43) and (k % 64 or (VAR == 43 and (m % 256 or n % 256))):
            continue
        for tb in (True, False):
            e = check(m, n, k, tb)
            bad += e > 1e-2
    bad += check(1024, 1024, 512, True, bias=True) > 1e-2
    bad += check(1024, 1024, 512, False, dt=torch.float16) > 1e-2
    if bad:
        print("FAILED", bad)
        sys.exit(1)
    shapes = [tuple(int(x) for x in s.split("x")) for s in
              os.environ.get("SHAPES", "4096x4096x4096,8192x8192x8192,8192x8192x1024").split(",")]
    for (m, n, k) in shapes:
        a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        bt = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
        bn = torch.randn(k, n, device="cuda", dtype=torch.bfloat16)
        c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        fns = {"nt_w4v": lambda: pli_hip.gemm(a, bt, trans_b=True, out=c, variant=VAR),
               "nt_v0": lambda: pli_hip.gemm(a, bt, trans_b=True, out=c),
               "nt_torch": lambda: torch.mm(a, bt.t(), out=c),
               "nn_w4v": lambda: pli_hip.gemm(a, bn, out=c, variant=VAR),
               "nn_v0": lambda: pli_hip.gemm(a, bn, out=c),
               "nn_torch": lambda: torch.mm(a, bn, out=c)}
        for f in fns.values():
            for _ in range(3):
                f()
        res = {kk: [] for kk in fns}
        for _ in range(int(os.environ.get("ROUNDS", "5"))):
            for kk, f in fns.items():
                res[kk].append(ev_ms(f, 10))
        row = {kk: round(2 * m * n * k / sorted(v)[len(v) // 2] / 1e9, 1) for kk, v in res.items()}
        print(json.dumps({"m": m, "n": n, "k": k, "TFLOP/s": row}), flush=True)


if __name__ == "__main__":
    main()
