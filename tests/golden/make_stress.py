#!/usr/bin/env python3
"""Record the REFERENCE's own bf16 flash output on the adversarial inputs of
tests/stress_cases.py (build container only; imports /root/reference, copies
none of it).

    python tests/golden/make_stress.py [--ref /root/reference]

Writes stress_flash.npz: for each case, the reference ch06
flash_attention_forward output (bf16 bits; small cases only) and its max
|error| against the float64 naive attention.  The GPU tests hold the prescaled default kernel to
"no worse than the reference's own bf16 path" on these inputs.
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.dirname(HERE)]

from oracle import attention as oatt  # noqa: E402
from oracle.numerics import bf16_bits  # noqa: E402
from stress_cases import STRESS, stress_inputs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    import torch
    spec = importlib.util.spec_from_file_location("ref_flash", os.path.join(a.ref, "ch06", "flash_attention.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = {}
    for name in STRESS:
        q, k, v = stress_inputs(name)
        g = q.shape[1] // k.shape[1]  # GQA: the reference takes K/V at the query heads
        t = [torch.from_numpy(np.ascontiguousarray(x)).to(torch.bfloat16)
             for x in (q, np.repeat(k, g, axis=1), np.repeat(v, g, axis=1))]
        y = mod.flash_attention_forward(*t).float().numpy()
        ref = oatt.naive_attention(q, k, v)
        if q.size <= 1 << 20:  # the large seam cases keep only their error (fixture size)
            out[f"{name}_ref_flash"] = bf16_bits(y)
        out[f"{name}_ref_err"] = np.float64(np.abs(y.astype(np.float64) - ref).max())
        print(name, "reference bf16 flash max|err| vs f64:", float(out[f"{name}_ref_err"]))
    np.savez_compressed(os.path.join(HERE, "stress_flash.npz"), **out)


if __name__ == "__main__":
    main()
