#!/usr/bin/env python3
"""Build libpli_hip.so for gfx950 with hipcc (no cmake, no JIT cache).

    python physics-llm-inference_amd/build.py [--force] [--jobs N]
    python physics-llm-inference_amd/build.py --asan   # CPU sanitizer build

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


# ---- SURVEY.md §5 sanitizer build (CPU checks only, never shipped) ---------
# Every source compiled with AddressSanitizer on the HOST side (each
# -fsanitize= directly after -Xarch_host: the device code is the product's,
# and GPU ASan is not used on this pool), linked into
# build_asan/libpli_hip_asan.so, plus tests/asan/abi_check.c linked against
# it: the argument checks, empty-operand rules, workspace sizing, debug-mode
# switch and error strings of the entry points, run with the ASan runtime in
# the executable (tests/test_capi.py::test_abi_checks_under_asan).
ASAN_DIR = os.path.join(PKG, "build_asan")
ASAN_FLAGS = ["-O1", "-g", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"--offload-arch={ARCH}",
              "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer",
              "-I" + INCLUDE, "-I" + CSRC]
ASAN_LIB = os.path.join(ASAN_DIR, "libpli_hip_asan.so")
ASAN_CHECK = os.path.join(ASAN_DIR, "abi_check")


def _clang() -> str:
    for cand in ("/opt/rocm/lib/llvm/bin/clang", "/opt/rocm/llvm/bin/clang"):
        if os.path.exists(cand):
            return cand
    raise RuntimeError("ROCm clang not found")


def build_asan(jobs: int = 8, verbose: bool = True) -> str:
    """host-side AddressSanitizer build: returns the abi_check executable"""
    os.makedirs(ASAN_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))

    def one(src):
        obj = os.path.join(ASAN_DIR, os.path.basename(src) + ".o")
        if os.path.exists(obj) and os.path.getmtime(obj) >= _newest([src] + headers):
            return obj
        cmd = [hipcc(), *ASAN_FLAGS, *EXTRA.get(os.path.basename(src), []), "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"asan compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
        objs = list(ex.map(one, srcs))
    if not os.path.exists(ASAN_LIB) or os.path.getmtime(ASAN_LIB) < _newest(objs):
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", ASAN_LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"asan link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    check_src = os.path.join(ROOT, "tests", "asan", "abi_check.c")
    if not os.path.exists(ASAN_CHECK) or os.path.getmtime(ASAN_CHECK) < _newest([ASAN_LIB, check_src] + headers):
        cmd = [_clang(), "-O1", "-g", "-fsanitize=address", "-fno-omit-frame-pointer", "-I" + INCLUDE, check_src,
               ASAN_LIB, "-Wl,-rpath," + ASAN_DIR, "-o", ASAN_CHECK]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"abi_check link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[pli build --asan] {ASAN_LIB}, {ASAN_CHECK}")
    return ASAN_CHECK


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--asan", action="store_true",
                    help="host-side AddressSanitizer build + tests/asan/abi_check (CPU only)")
    a = ap.parse_args()
    try:
        if a.asan:
            build_asan(jobs=a.jobs)
        else:
            build(force=a.force, jobs=a.jobs)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
