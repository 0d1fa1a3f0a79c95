"""C ABI checks that need no GPU: the library loads, exports every entry point
include/pli.h declares, validates arguments before touching the device, and
the product path has no route to the oracle or to a CPU fallback."""
from __future__ import annotations

import ctypes
import os
import re

import pytest
import torch

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "pli.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(pli_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_hot_path():
    syms = declared_symbols()
    for s in ("pli_flash_attn_fwd", "pli_gemv", "pli_gemm", "pli_scale_copy", "pli_softmax_rows",
              "pli_online_softmax_with_output", "pli_attn_decode", "pli_attn_decode_workspace_size",
              "pli_last_error", "pli_version"):
        assert s in syms


def test_library_exports_every_declared_symbol(built_lib):
    lib = ctypes.CDLL(built_lib)
    for s in declared_symbols():
        assert hasattr(lib, s), f"{s} declared in pli.h but not exported"


def test_library_exports_exactly_the_header(built_lib):
    """Built with -fvisibility=hidden: the dynamic symbol table holds the
    pli.h entry points and nothing else of ours (no C++-internal pli::
    functions); hipcc's per-translation-unit __hip_cuid_* markers aside."""
    import shutil
    import subprocess
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    out = subprocess.run([nm, "-D", "--defined-only", built_lib], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    ours = {s for s in exported if not s.startswith("__hip_cuid_")}
    assert ours == set(declared_symbols()), sorted(ours ^ set(declared_symbols()))


def test_version_and_error_strings(built_lib):
    import pli_hip
    L = pli_hip.lib()
    assert L.pli_version().decode().startswith("pli_hip")
    assert L.pli_last_error() is not None


def test_argument_validation_without_gpu(built_lib):
    """Null pointers / bad shapes are rejected with PLI_EINVAL and a message,
    before any HIP call (so this runs on a GPU-less host)."""
    import pli_hip
    L = pli_hip.lib()
    EINVAL = 1000
    rc = L.pli_gemv(None, None, None, 16, 16, 16, 2, None)
    assert rc == EINVAL and b"null" in L.pli_last_error()
    p = ctypes.c_void_p(16)  # never dereferenced: validation fails first
    assert L.pli_gemv(p, p, p, 16, 32, 16, 2, None) == EINVAL  # ldw < k
    assert b"bad shape" in L.pli_last_error()
    assert L.pli_gemm(p, p, p, None, 8, 8, 8, 8, 8, 8, 0, 7, None) == EINVAL  # bad dtype
    st = (ctypes.c_int64 * 12)(*([0] * 12))
    assert L.pli_flash_attn_fwd(p, p, p, p, 1, 6, 4, 8, 8, 64, st, 0.1, 0, 2, None) == EINVAL
    assert b"multiple of kv_heads" in L.pli_last_error()
    assert L.pli_flash_attn_fwd(p, p, p, p, 1, 4, 4, 8, 8, 64, st, float("nan"), 0, 2, None) == EINVAL
    assert L.pli_scale_copy(p, p, 16, 0, None) == EINVAL
    assert L.pli_softmax_rows(p, p, 4, -1, 0, None) == EINVAL
    dec = lambda *shape, causal=0, ws=0: L.pli_attn_decode(p, p, p, p, *shape, st, 0.1, causal,
                                                           None, ws, 2, None)
    assert dec(1, 6, 4, 1, 64, 64) == EINVAL and b"multiple of kv_heads" in L.pli_last_error()
    assert dec(1, 8, 2, 4, 2, 64, causal=1) == EINVAL  # causal chunk longer than the cache
    assert b"n_q" in L.pli_last_error()
    # split-K needs its workspace: refused (not silently single-split) when short
    need = L.pli_attn_decode_workspace_size(1, 32, 8, 1, 32768, 128)
    assert need > 0
    st_dec = (ctypes.c_int64 * 12)(*([8] * 12))
    rc = L.pli_attn_decode(p, p, p, p, 1, 32, 8, 1, 32768, 128, st_dec, 0.1, 0, None, need - 1, 2, None)
    assert rc == EINVAL and b"workspace" in L.pli_last_error()
    # fused decode projection: at most 128 rows (k % 128 == 0 past 16), whole batches, 1..3 groups
    P3, I3, L3 = ctypes.c_void_p * 3, ctypes.c_int * 3, ctypes.c_int64 * 3
    w3, n3, ld3 = P3(16, 16, 16), I3(64, 64, 64), L3(64, 64, 64)
    multi = lambda m, tpb, ng: L.pli_gemm_multi_nt(p, 64, m, 64, tpb, w3, w3, n3, ld3, ld3, ld3,
                                                   P3(None, None, None), I3(9, 9, 9), ng, 2, None)
    assert multi(129, 1, 3) == EINVAL and b"m <= 128" in L.pli_last_error()
    assert multi(17, 1, 3) == EINVAL and b"k % 128" in L.pli_last_error()  # k = 64
    assert multi(6, 4, 3) == EINVAL  # 6 rows are not whole batches of 4
    assert multi(4, 1, 4) == EINVAL and b"groups" in L.pli_last_error()
    # fused norm + projection: <= 4 rows, k <= 8192
    rms = lambda m, k: L.pli_rms_gemm_nt(p, 8192, None, 0, p, 1e-6, None, 0, m, k, 1, w3, None, w3,
                                         n3, ld3, ld3, ld3, P3(None, None, None), I3(9, 9, 9), 3, 2, None)
    assert rms(5, 64) == EINVAL and b"m <= 4" in L.pli_last_error()
    assert rms(1, 16384) == EINVAL and b"k <= 8192" in L.pli_last_error()


def test_empty_operands_without_gpu(built_lib):
    """pli.h: an operand with zero elements may be NULL (torch's data_ptr of
    an empty tensor) and a call whose output is empty returns PLI_OK before
    any HIP call; a non-empty output still needs its pointer"""
    import pli_hip
    L = pli_hip.lib()
    EINVAL = 1000
    st = (ctypes.c_int64 * 12)(*([8] * 12))
    for B, Nq in ((0, 8), (2, 0)):  # no output rows
        assert L.pli_flash_attn_fwd(None, None, None, None, B, 4, 4, Nq, 8, 64, None, 0.1, 0, 2, None) == 0
        assert L.pli_attn_decode(None, None, None, None, B, 4, 4, Nq, 8, 64, None, 0.1, 0, None, 0, 2, None) == 0
    assert L.pli_flash_attn_fwd(None, None, None, None, 1, 4, 4, 8, 0, 64, st, 0.1, 0, 2, None) == EINVAL
    assert b"null" in L.pli_last_error()  # no keys, but 8 output rows: O is needed
    for m, n, k in ((0, 8, 8), (8, 0, 8), (0, 0, 0)):
        assert L.pli_gemm(None, None, None, None, m, n, k, 8, 8, 8, 1, 2, None) == 0
        assert L.pli_gemm_f32out(None, None, None, m, n, k, 8, 8, 2, None) == 0
        assert L.pli_gemm_swiglu(None, None, None, None, m, n, k, 8, 8, 8, 8, 2, None) == 0
        assert L.pli_gemm_naive(None, None, None, m, n, k, 8, 8, 8, None) == 0
    assert L.pli_gemm(None, None, None, None, 8, 8, 0, 8, 8, 8, 1, 2, None) == EINVAL  # C = bias / 0: C needed
    assert L.pli_gemv(None, None, None, 0, 16, 16, 2, None) == 0
    assert L.pli_gemv(None, None, None, 16, 0, 16, 2, None) == EINVAL  # y = 0 has 16 rows
    assert L.pli_rmsnorm(None, None, None, None, None, 0, 64, 64, 64, 64, 64, 1e-6, 2, None) == 0
    assert L.pli_softmax_rows(None, None, 0, 64, 2, None) == 0
    assert L.pli_softmax_rows(None, None, 4, 0, 2, None) == 0
    assert L.pli_online_softmax_with_output(None, None, None, None, 0, 64, 64, 2, None) == 0
    assert L.pli_scale_copy(None, None, 0, 1, None) == 0
    assert L.pli_kv_append(None, None, None, None, 2, 0, 4, 64, 128, None, None, 2, None) == 0
    assert L.pli_moe_combine(None, 64, None, None, None, 64, 0, 2, 64, 2, None) == 0
    assert L.pli_gemm_grouped(None, None, None, None, None, None, 4, 0, 64, 128, 128, 128, 64, 2, None) == 0


def test_decode_workspace_plan(built_lib):
    """Split-K plan (host arithmetic, no GPU): one chunk per head when the
    (batch, kv head) grid alone fills the chip; fp32 partials otherwise."""
    import pli_hip
    ws = pli_hip.attn_decode_workspace_bytes
    assert ws(64, 32, 8, 1, 4096, 128) == 512 * 2 * 4 * (128 + 2) * 4  # 512 heads x 2 chunks
    assert ws(128, 32, 8, 1, 4096, 128) == 0         # 1024 (b, kv head) pairs fill the grid
    n = ws(1, 32, 8, 1, 32768, 128)                  # 8 heads -> 128 chunks each
    assert n == 8 * 128 * 4 * (128 + 2) * 4
    assert ws(1, 32, 8, 1, 100, 128) == 0            # one 128-key chunk
    assert ws(1, 64, 2, 1, 4096, 128) == 0           # 32 rows per kv head: prefill kernel
    assert ws(1, 8, 8, 1, 4096, 80) == 0             # head_dim 80: prefill kernel


def test_hip_path_refuses_cpu_tensors(built_lib):
    import pli_hip
    x = torch.randn(4, 4)
    with pytest.raises(pli_hip.PliError):
        pli_hip.gemm(x, x)
    with pytest.raises(pli_hip.PliError):
        pli_hip.flash_attn_fwd(x[None, None], x[None, None], x[None, None])


def test_product_never_imports_the_oracle():
    """Nothing under physics-llm-inference_amd/ may import or reach oracle/."""
    offenders = []
    for dirpath, _, files in os.walk(PKG):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                if re.search(r"^\s*(from|import)\s+oracle\b", src, re.M) or "oracle/" in src:
                    offenders.append(os.path.join(dirpath, f))
    assert not offenders, offenders


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    import pli_hip
    monkeypatch.setattr(pli_hip, "_lib", None)
    monkeypatch.setattr(pli_hip, "_LIB_PATH", str(tmp_path / "absent.so"))
    with pytest.raises(pli_hip.PliError, match="not built"):
        pli_hip.lib()
    assert not pli_hip.available()


def test_debug_sync_switch(built_lib):
    """PLI_SYNC debug mode: off unless the environment says
    so, switchable through pli_debug_sync; PLI_SYNC=1 turns it on at load"""
    import subprocess
    import sys
    import pli_hip
    prev = pli_hip.debug_sync(-1)
    try:
        assert pli_hip.debug_sync(1) == prev and pli_hip.debug_sync(-1) is True
        assert pli_hip.debug_sync(0) is True and pli_hip.debug_sync(-1) is False
    finally:
        pli_hip.debug_sync(int(prev))
    code = "import ctypes, sys; L = ctypes.CDLL(sys.argv[1]); print(L.pli_debug_sync(-1))"
    for name, env_val, want in (("PLI_SYNC", "1", "1"), ("PLI_SYNC", "0", "0"), ("PLI_SYNC", None, "0"),
                                ("HIP_LAUNCH_BLOCKING", "1", "1")):
        env = {k: v for k, v in os.environ.items() if k not in ("PLI_SYNC", "HIP_LAUNCH_BLOCKING")}
        if env_val is not None:
            env[name] = env_val
        out = subprocess.run([sys.executable, "-c", code, built_lib], capture_output=True, text=True, env=env,
                             check=True).stdout.strip()
        assert out == want, (env_val, out)


@pytest.mark.timeout(1500)
def test_abi_checks_under_asan():
    """build.py --asan: every source with AddressSanitizer on the host side,
    and tests/asan/abi_check.c (the argument checks, empty operands,
    workspace sizing and error strings above, from C) run against it"""
    import subprocess
    import sys
    sys.path.insert(0, PKG)
    import build as pli_build
    exe = pli_build.build_asan(jobs=8, verbose=False)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "all checks passed under AddressSanitizer" in r.stdout
