#!/usr/bin/env python3
"""Build libpli_hip.so for gfx950 with hipcc (no cmake, no JIT cache).

    python physics-llm-inference_amd/build.py [--force] [--jobs N]

Compiles every ``csrc/*.hip`` / ``csrc/*.cpp`` into an object under
``build/`` and links ``pli_hip/libpli_hip.so`` in-tree, so the library
travels with the repository snapshot to the GPU box.  Objects are rebuilt
only when a source or header is newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "pli_hip", "libpli_hip.so")
ARCH = os.environ.get("PLI_OFFLOAD_ARCH", "gfx950")

# -fvisibility=hidden: only the entry points include/pli.h declares (inside its
# visibility push(default)) are exported (tests/test_capi.py checks the set)
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"--offload-arch={ARCH}", "-I" + INCLUDE, "-I" + CSRC,
          "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]
# per-source extra flags.  flash_v7: no NaN ever reaches the softmax (masks
# use -inf), so fmaxf on MFMA results folds into v_max3_f32 without the
# canonicalising v_max_f32 hipcc otherwise puts in front of each one.
EXTRA = {"flash_v7.hip": ["-fno-honor-nans"], "flash_v12.hip": ["-fno-honor-nans"]}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    raise RuntimeError("hipcc not found")


def _newest(paths):
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= _newest([src] + headers):
        return obj
    cmd = [hipcc(), *CFLAGS, *EXTRA.get(os.path.basename(src), []), "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < _newest(objs):
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[pli build] {LIB} ({len(objs)} objects, {ARCH})")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    try:
        build(force=a.force, jobs=a.jobs)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
