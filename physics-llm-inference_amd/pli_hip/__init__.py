"""ctypes binding of ``libpli_hip.so`` (the C ABI declared in ``include/pli.h``).

Every wrapper takes torch tensors that already live on a ROCm device, passes
raw ``data_ptr()`` values plus sizes/strides and the current HIP stream across
the C ABI, and raises ``PliError`` on a non-zero status.  There is no CPU or
torch fallback in here: if the library is missing or a tensor is not on the
GPU, the call fails loudly.
"""
from __future__ import annotations

import ctypes
import os

import torch

__all__ = [
    "PliError", "lib", "library_path", "available", "DTYPE_CODE",
    "flash_attn_fwd", "gemv", "gemm", "gemm_f32out", "scale_copy", "mfma_probe", "hbm_read_probe", "softmax_rows",
    "online_softmax_with_output",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
# PLI_HIP_LIB: an alternate in-tree build (A/B tooling); default the package .so
_LIB_PATH = os.environ.get("PLI_HIP_LIB") or os.path.join(_HERE, "libpli_hip.so")
_lib = None

DTYPE_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}

_c_int, _c_i64, _c_f32, _vp = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p

# name -> argtypes, mirroring include/pli.h
_SIGS = {
    "pli_version": [],
    "pli_last_error": [],
    "pli_last_route": [],
    "pli_debug_sync": [_c_int],
    "pli_flash_attn_fwd": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                           ctypes.POINTER(_c_i64), _c_f32, _c_int, _c_int, _vp],
    "pli_gemv": [_vp, _vp, _vp, _c_int, _c_int, _c_i64, _c_int, _vp],
    "pli_gemm": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _c_i64, _c_int,
                 _c_int, _vp],
    "pli_gemm_workspace_size": [_c_int, _c_int, _c_int, _c_int, _c_int],
    "pli_gemm_ws": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _c_i64, _c_int,
                    _c_int, _vp, ctypes.c_size_t, _vp],
    "pli_gemm_swiglu_workspace_size": [_c_int, _c_int, _c_int, _c_int],
    "pli_gemm_swiglu_ws": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _c_i64,
                           _c_i64, _c_int, _vp, ctypes.c_size_t, _vp],
    "pli_gemm_swiglu_ws_variant": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_i64, _c_i64,
                                   _c_i64, _c_i64, _c_int, _vp, ctypes.c_size_t, _vp, _c_int],
    "pli_gemm_swiglu": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _c_i64,
                        _c_i64, _c_int, _vp],
    "pli_rmsnorm": [_vp, _vp, _vp, _vp, _vp, _c_i64, _c_int, _c_i64, _c_i64, _c_i64, _c_i64,
                    _c_f32, _c_int, _vp],
    "pli_gemm_multi_nt": [_vp, _c_i64, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                          _vp, _c_int, _c_int, _vp],
    "pli_rms_gemm_nt": [_vp, _c_i64, _vp, _c_i64, _vp, _c_f32, _vp, _c_i64, _c_int, _c_int, _c_int,
                        _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _vp],
    "pli_moe_route": [_vp, _c_i64, _c_int, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp,
                      _vp, _vp, _vp],
    "pli_gemm_grouped": [_vp, _vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_i64,
                         _c_i64, _c_i64, _c_int, _vp],
    "pli_gemm_grouped_variant": [_vp, _vp, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int,
                                 _c_i64, _c_i64, _c_i64, _c_int, _vp, _c_int],
    "pli_moe_combine": [_vp, _c_i64, _vp, _vp, _vp, _c_i64, _c_int, _c_int, _c_int, _c_int, _vp],
    "pli_scale_copy": [_vp, _vp, _c_i64, _c_int, _vp],
    "pli_gemm_naive": [_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _c_i64, _vp],
    "pli_gemm_f32out": [_vp, _vp, _vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _c_int, _vp],
    "pli_mfma_probe": [_vp, _vp, _c_int, _c_int, _c_int, _vp],
    "pli_hbm_read_probe": [_vp, _c_i64, _vp, _c_int, _c_int, _vp],
    "pli_softmax_rows": [_vp, _vp, _c_i64, _c_int, _c_int, _vp],
    "pli_online_softmax_with_output": [_vp, _vp, _vp, _vp, _c_i64, _c_int, _c_int, _c_int, _vp],
    "pli_attn_decode_workspace_size": [_c_int] * 6,
    "pli_kv_append": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int,
                      ctypes.POINTER(_c_i64), _vp, _c_int, _vp],
    "pli_attn_decode_dev": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                            ctypes.POINTER(_c_i64), _c_f32, _c_int, _vp, _c_int, _vp,
                            ctypes.c_size_t, _c_int, _vp],
    "pli_attn_decode": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                        ctypes.POINTER(_c_i64), _c_f32, _c_int, _vp, ctypes.c_size_t, _c_int, _vp],
    # tuning entry points (include/pli.h tuning section): explicit kernel variant
    "pli_flash_attn_fwd_variant": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int,
                                   _c_int, ctypes.POINTER(_c_i64), _c_f32, _c_int, _c_int, _vp,
                                   _c_int],
    "pli_gemv_variant": [_vp, _vp, _vp, _c_int, _c_int, _c_i64, _c_int, _vp, _c_int],
    "pli_gemm_variant": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _c_i64,
                         _c_int, _c_int, _vp, _c_int],
    "pli_gemm_ws_variant": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_i64, _c_i64, _c_i64,
                            _c_int, _c_int, _vp, ctypes.c_size_t, _vp, _c_int],
    "pli_attn_decode_variant": [_vp, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                                ctypes.POINTER(_c_i64), _c_f32, _c_int, _vp, ctypes.c_size_t,
                                _c_int, _vp, _c_int, _c_int],
}


class PliError(RuntimeError):
    """A libpli_hip entry point returned a non-zero status."""


def library_path() -> str:
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    """Load libpli_hip.so (after torch, so both share torch's HIP runtime)."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise PliError(
                f"{_LIB_PATH} is not built; run `python physics-llm-inference_amd/build.py` "
                "(or __graft_entry__.build())")
        L = ctypes.CDLL(_LIB_PATH)
        for name, argtypes in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = argtypes
            fn.restype = (ctypes.c_char_p if name in ("pli_version", "pli_last_error", "pli_last_route") else
                          ctypes.c_size_t if name.endswith("_workspace_size") else _c_int)
        _lib = L
    return _lib


def available() -> bool:
    """True when the library loads AND a ROCm device is visible."""
    try:
        lib()
    except (PliError, OSError):
        return False
    return torch.cuda.is_available()


def last_route() -> str:
    """the kernels this thread's last library call launched ('+'-separated;
    pli_last_route)"""
    return lib().pli_last_route().decode()


def debug_sync(mode: int = -1) -> bool:
    """the library's synchronous debug mode (pli_debug_sync; PLI_SYNC=1 in the
    environment turns it on at load): mode 1 / 0 sets it, -1 only queries;
    returns the previous state.  When on, every launch is synchronised and
    checked, and a failing kernel's name is in the raised PliError."""
    return bool(lib().pli_debug_sync(int(mode)))


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().pli_last_error().decode(errors="replace")
        raise PliError(f"{what} failed with status {rc}: {msg}")


def _dtype_code(t: torch.Tensor) -> int:
    try:
        return DTYPE_CODE[t.dtype]
    except KeyError:
        raise PliError(f"unsupported dtype {t.dtype} (HIP path supports fp32/fp16/bf16)") from None


def _require_gpu(*ts: torch.Tensor) -> torch.device:
    dev = ts[0].device
    for t in ts:
        if not t.is_cuda:
            raise PliError("HIP path called with a CPU tensor")
        if t.device != dev:
            raise PliError(f"tensors on different devices: {t.device} vs {dev}")
        if t.dtype != ts[0].dtype:
            raise PliError(f"mixed dtypes {t.dtype} vs {ts[0].dtype}")
    return dev


def _check_out(out: torch.Tensor, ref: torch.Tensor, shape: tuple, what: str) -> None:
    """A caller-supplied output: same device and dtype as ``ref``, exactly
    ``shape``, unit inner stride, rows not overlapping (the kernels write
    ``shape[0]`` rows of ``shape[-1]`` elements at the row stride)."""
    _require_gpu(ref, out)
    if tuple(out.shape) != tuple(shape):
        raise PliError(f"{what}: out has shape {tuple(out.shape)}, expected {tuple(shape)}")
    if out.dim() > 0 and out.stride(-1) != 1:
        raise PliError(f"{what}: out needs a unit inner stride, got strides {out.stride()}")
    if out.dim() == 2 and out.shape[0] > 1 and out.stride(0) < out.shape[1]:
        raise PliError(f"{what}: out rows overlap (row stride {out.stride(0)} < {out.shape[1]})")


def _stream(dev: torch.device) -> int:
    # raw hipStream_t of the current stream (cheaper than building a Stream object)
    return torch._C._cuda_getCurrentRawStream(dev.index)


class _on_device:
    """Device guard that costs nothing when ``dev`` is already current."""

    __slots__ = ("dev", "prev")

    def __init__(self, dev: torch.device):
        self.dev, self.prev = dev, None

    def __enter__(self):
        cur = torch.cuda.current_device()
        if self.dev.index is not None and cur != self.dev.index:
            self.prev = cur
            torch.cuda.set_device(self.dev.index)

    def __exit__(self, *exc):
        if self.prev is not None:
            torch.cuda.set_device(self.prev)


def _ptr(t: torch.Tensor | None):
    return t.data_ptr() if t is not None else None


# ------------------------------------------------------------------ attention
def flash_attn_fwd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float | None = None,
                   causal: bool = False, out: torch.Tensor | None = None,
                   variant: int | None = None) -> torch.Tensor:
    """O = softmax(Q K^T * scale [+ causal]) V on [B, H, N, D] tensors (any
    strides with a unit head_dim stride); K/V may have fewer (GQA) heads."""
    dev = _require_gpu(q, k, v)
    if q.dim() != 4 or k.dim() != 4 or v.dim() != 4:
        raise PliError("flash_attn_fwd expects [B, H, N, D] tensors")
    B, H, Nq, D = q.shape
    Bk, Hkv, Nk, Dk = k.shape
    if (Bk, Dk) != (B, D) or tuple(v.shape) != tuple(k.shape):
        raise PliError(f"shape mismatch q{tuple(q.shape)} k{tuple(k.shape)} v{tuple(v.shape)}")
    if H % Hkv != 0:
        raise PliError(f"heads {H} not a multiple of kv heads {Hkv}")
    q, k, v = (t if t.stride(-1) == 1 else t.contiguous() for t in (q, k, v))
    if out is None:
        out = torch.empty_like(q, memory_format=torch.contiguous_format)
    _require_gpu(q, out)
    if tuple(out.shape) != tuple(q.shape) or out.stride(-1) != 1:
        raise PliError("bad output tensor")
    if scale is None:
        scale = D ** -0.5
    st = (_c_i64 * 12)(*(int(x) for t in (q, k, v, out) for x in t.stride()[:3]))
    args = (_ptr(q), _ptr(k), _ptr(v), _ptr(out), B, H, Hkv, Nq, Nk, D, st, float(scale),
            int(bool(causal)), _dtype_code(q), _stream(dev))
    with _on_device(dev):
        if variant is None:
            rc = lib().pli_flash_attn_fwd(*args)
        else:
            rc = lib().pli_flash_attn_fwd_variant(*args, int(variant))
    _check(rc, "pli_flash_attn_fwd")
    return out


# ------------------------------------------------------- decode attention
def attn_decode_workspace_bytes(B: int, H: int, Hkv: int, Sq: int, n_kv: int, D: int) -> int:
    return int(lib().pli_attn_decode_workspace_size(B, H, Hkv, Sq, n_kv, D))


def attn_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, n_kv: int,
                scale: float | None = None, causal: bool = True,
                out: torch.Tensor | None = None, variant: int | None = None,
                target_wgs: int = 0) -> torch.Tensor:
    """Attention of the new tokens over a KV cache, in the cache layout of
    ch02/kv_cache.py:25-35: q [B, Sq, Hq, D], k/v caches [B, S_max, Hkv, D]
    of which the first n_kv positions are valid (the current token's K/V
    already appended).  Returns [B, Sq, Hq, D].  causal masks bottom-right
    (ch02/kv_cache.py:91-95); with Sq == 1 it changes nothing."""
    dev = _require_gpu(q, k_cache, v_cache)
    if q.dim() != 4 or k_cache.dim() != 4 or v_cache.dim() != 4:
        raise PliError("attn_decode expects q [B, Sq, Hq, D] and caches [B, S, Hkv, D]")
    B, Sq, H, D = q.shape
    Bk, S_max, Hkv, Dk = k_cache.shape
    if (Bk, Dk) != (B, D) or tuple(v_cache.shape) != tuple(k_cache.shape):
        raise PliError(f"shape mismatch q{tuple(q.shape)} k{tuple(k_cache.shape)} "
                       f"v{tuple(v_cache.shape)}")
    if H % Hkv != 0:
        raise PliError(f"heads {H} not a multiple of kv heads {Hkv}")
    if not 0 <= n_kv <= S_max:
        raise PliError(f"n_kv {n_kv} outside the cache [0, {S_max}]")
    q, k_cache, v_cache = (t if t.stride(-1) == 1 else t.contiguous() for t in (q, k_cache, v_cache))
    if out is None:
        out = torch.empty((B, Sq, H, D), device=q.device, dtype=q.dtype)
    _require_gpu(q, out)
    if tuple(out.shape) != (B, Sq, H, D) or out.stride(-1) != 1:
        raise PliError("bad output tensor")
    if scale is None:
        scale = D ** -0.5
    # [b, h, n] strides of the [B, N, H, D] tensors
    st = (_c_i64 * 12)(*(int(x) for t in (q, k_cache, v_cache, out)
                         for x in (t.stride(0), t.stride(2), t.stride(1))))
    ws_bytes = int(lib().pli_attn_decode_workspace_size(B, H, Hkv, Sq, n_kv, D))
    if target_wgs:  # tuning: room for the finest split (one 128-key chunk per block)
        ws_bytes = B * Hkv * -(-n_kv // 128) * Sq * (H // Hkv) * (D + 2) * 4
    ws = torch.empty(max(ws_bytes // 4, 1), device=q.device, dtype=torch.float32)
    args = (_ptr(q), _ptr(k_cache), _ptr(v_cache), _ptr(out), B, H, Hkv, Sq, int(n_kv), D, st,
            float(scale), int(bool(causal)), _ptr(ws), ws_bytes, _dtype_code(q), _stream(dev))
    with _on_device(dev):
        if variant is None and not target_wgs:
            rc = lib().pli_attn_decode(*args)
        else:
            rc = lib().pli_attn_decode_variant(*args, -1 if variant is None else int(variant),
                                               int(target_wgs))
    _check(rc, "pli_attn_decode")
    return out


def kv_append(k_new: torch.Tensor, v_new: torch.Tensor, k_cache: torch.Tensor,
              v_cache: torch.Tensor, pos: torch.Tensor) -> None:
    """Write [B, T, Hkv, D] K/V into [B, S, Hkv, D] caches at rows pos[0] +
    (0..T-1), pos an int32 device tensor (graph-replayable KVCache.update)."""
    dev = _require_gpu(k_new, v_new, k_cache, v_cache)
    if pos.dtype != torch.int32 or not pos.is_cuda:
        raise PliError("pos must be an int32 device tensor")
    B, T, Hkv, D = k_new.shape
    if tuple(v_new.shape) != tuple(k_new.shape) or k_cache.shape[0] != B or \
            tuple(k_cache.shape[2:]) != (Hkv, D) or tuple(v_cache.shape) != tuple(k_cache.shape):
        raise PliError(f"kv_append shape mismatch new{tuple(k_new.shape)} cache{tuple(k_cache.shape)}")
    st = (_c_i64 * 12)(*(int(x) for t in (k_new, k_cache, v_cache, v_new)
                         for x in (t.stride(0), t.stride(2), t.stride(1))))
    with _on_device(dev):
        rc = lib().pli_kv_append(_ptr(k_new), _ptr(v_new), _ptr(k_cache), _ptr(v_cache), B, T, Hkv,
                                 D, k_cache.shape[1], st, _ptr(pos), _dtype_code(k_new), _stream(dev))
    _check(rc, "pli_kv_append")


def attn_decode_dev(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                    n_kv_dev: torch.Tensor, n_kv_add: int = 0, n_kv_max: int | None = None,
                    scale: float | None = None, causal: bool = True,
                    out: torch.Tensor | None = None, workspace: torch.Tensor | None = None
                    ) -> torch.Tensor:
    """attn_decode with the valid length n_kv_dev[0] + n_kv_add read on the
    device (graph-replayable); the grid is planned for n_kv_max (default: the
    cache capacity)."""
    dev = _require_gpu(q, k_cache, v_cache)
    B, Sq, H, D = q.shape
    Hkv = k_cache.shape[2]
    n_max = k_cache.shape[1] if n_kv_max is None else int(n_kv_max)
    if out is None:
        out = torch.empty((B, Sq, H, D), device=q.device, dtype=q.dtype)
    if scale is None:
        scale = D ** -0.5
    st = (_c_i64 * 12)(*(int(x) for t in (q, k_cache, v_cache, out)
                         for x in (t.stride(0), t.stride(2), t.stride(1))))
    ws_bytes = int(lib().pli_attn_decode_workspace_size(B, H, Hkv, Sq, n_max, D))
    if workspace is None or workspace.numel() * 4 < ws_bytes:
        workspace = torch.empty(max(ws_bytes // 4, 1), device=q.device, dtype=torch.float32)
    with _on_device(dev):
        rc = lib().pli_attn_decode_dev(_ptr(q), _ptr(k_cache), _ptr(v_cache), _ptr(out), B, H, Hkv,
                                       Sq, n_max, D, st, float(scale), int(bool(causal)),
                                       _ptr(n_kv_dev), int(n_kv_add), _ptr(workspace), ws_bytes,
                                       _dtype_code(q), _stream(dev))
    _check(rc, "pli_attn_decode_dev")
    return out


# ---------------------------------------------------------------------- MoE
def moe_route(logits: torch.Tensor, top_k: int, normalize: bool = True):
    """Router tail of ch09/moe_layer.py:24-33 on the device: returns
    (weights [T, k] fp32, expert_idx [T, k] int32, pos [T, k] int32,
    gather [T*k] int32, offsets [E+1] int32)."""
    dev = _require_gpu(logits)
    T, E = logits.shape
    if logits.stride(1) != 1:
        logits = logits.contiguous()
    i32 = dict(device=logits.device, dtype=torch.int32)
    weights = torch.empty(T, top_k, device=logits.device, dtype=torch.float32)
    idx = torch.empty(T, top_k, **i32)
    pos = torch.empty(T, top_k, **i32)
    gather = torch.empty(max(T * top_k, 1), **i32)
    offsets = torch.empty(E + 1, **i32)
    ws = torch.empty(E + T * top_k, **i32)
    with _on_device(dev):
        rc = lib().pli_moe_route(_ptr(logits), logits.stride(0), T, E, int(top_k), int(bool(normalize)),
                                 _dtype_code(logits), _ptr(weights), _ptr(idx), _ptr(pos),
                                 _ptr(gather), _ptr(offsets), _ptr(ws), _stream(dev))
    _check(rc, "pli_moe_route")
    return weights, idx, pos, gather, offsets


def weight_table(weights: list[torch.Tensor]) -> torch.Tensor:
    """Device int64 array of the weights' data pointers (for pli_gemm_grouped)."""
    return torch.tensor([w.data_ptr() for w in weights], dtype=torch.int64,
                        device=weights[0].device)


def gemm_grouped(x: torch.Tensor, gather: torch.Tensor | None, w_table: torch.Tensor,
                 offsets: torch.Tensor, rows: int, n: int, k: int, ldw: int,
                 wu_table: torch.Tensor | None = None, out: torch.Tensor | None = None,
                 variant: int | None = None) -> torch.Tensor:
    """Per-expert NT GEMM over expert-sorted rows (see include/pli.h)."""
    dev = _require_gpu(x)
    E = offsets.numel() - 1
    if out is None:
        out = torch.empty(max(rows, 1), n, device=x.device, dtype=x.dtype)
    args = (_ptr(x), _ptr(gather), _ptr(w_table), _ptr(wu_table), _ptr(out), _ptr(offsets), E,
            int(rows), int(n), int(k), x.stride(0), int(ldw), out.stride(0), _dtype_code(x), _stream(dev))
    with _on_device(dev):
        if variant is None:
            rc = lib().pli_gemm_grouped(*args)
        else:
            rc = lib().pli_gemm_grouped_variant(*args, int(variant))
    _check(rc, "pli_gemm_grouped")
    return out


def moe_combine(y: torch.Tensor, pos: torch.Tensor, weights: torch.Tensor, tokens: int,
                out: torch.Tensor | None = None) -> torch.Tensor:
    dev = _require_gpu(y)
    H = y.shape[1]
    k = pos.shape[1]
    if out is None:
        out = torch.empty(tokens, H, device=y.device, dtype=y.dtype)
    with _on_device(dev):
        rc = lib().pli_moe_combine(_ptr(y), y.stride(0), _ptr(pos), _ptr(weights), _ptr(out),
                                   out.stride(0), tokens, k, H, _dtype_code(y), _stream(dev))
    _check(rc, "pli_moe_combine")
    return out


# ------------------------------------------------------------------ RMSNorm
def rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-6,
            residual: torch.Tensor | None = None, out: torch.Tensor | None = None):
    """y = h / sqrt(mean(h^2) + eps) * weight over the last dim, h = x (+ residual).
    Returns y, or (h, y) when a residual is given (h = x + residual in x.dtype)."""
    dev = _require_gpu(x, weight)
    n = x.shape[-1]
    if weight.shape != (n,):
        raise PliError(f"weight {tuple(weight.shape)} for rows of {n}")
    x2 = x.reshape(-1, n)
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    r2 = None
    if residual is not None:
        _require_gpu(x, residual)
        if residual.shape != x.shape:
            raise PliError("residual shape mismatch")
        r2 = residual.reshape(-1, n)
        if r2.stride(-1) != 1:
            r2 = r2.contiguous()
    weight = weight.contiguous()
    if out is not None:
        _check_out(out, x, tuple(x.shape), "rmsnorm")
        if not out.is_contiguous():
            raise PliError("rmsnorm: out must be contiguous")
    y = torch.empty_like(x2) if out is None else out.view(-1, n)
    h = torch.empty_like(x2) if residual is not None else None
    rows = x2.shape[0]
    with _on_device(dev):
        rc = lib().pli_rmsnorm(_ptr(x2), _ptr(r2), _ptr(weight), _ptr(y), _ptr(h), rows, n,
                               x2.stride(0), r2.stride(0) if r2 is not None else n, y.stride(0),
                               h.stride(0) if h is not None else n, float(eps), _dtype_code(x),
                               _stream(dev))
    _check(rc, "pli_rmsnorm")
    y = y.view(x.shape)
    return y if residual is None else (h.view(x.shape), y)


def qkv_into_cache(x: torch.Tensor, wq: torch.Tensor, wk: torch.Tensor, wv: torch.Tensor,
                   q_out: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                   pos: torch.Tensor) -> torch.Tensor:
    """Decode-step projections in one launch (pli_gemm_multi_nt): x [B, S, hidden]
    (B*S <= 128; above 16 rows hidden % 128 == 0) -> q_out [B, S, Hq*D]; k / v
    rows written into [B, S_max, Hkv, D] caches at rows pos[0] + s.  Returns
    q_out."""
    dev = _require_gpu(x, wq, wk, wv, q_out, k_cache, v_cache)
    B, S, hidden = x.shape
    x2 = x.reshape(B * S, hidden)
    if x2.stride(1) != 1:
        x2 = x2.contiguous()
    S_max, Hkv, D = k_cache.shape[1:]
    if pos.dtype != torch.int32 or not pos.is_cuda:
        raise PliError("pos must be an int32 device tensor")
    for name, t in (("k_cache", k_cache), ("v_cache", v_cache)):
        if t.shape[0] != B or t.stride(3) != 1 or t.stride(2) != D:
            raise PliError(f"{name} must be [B, S_max, Hkv, D] with contiguous (Hkv, D) rows")
    if tuple(v_cache.shape) != tuple(k_cache.shape):
        raise PliError("k_cache / v_cache shape mismatch")
    if wk.shape[0] != Hkv * D or wv.shape[0] != Hkv * D or q_out.shape[-1] != wq.shape[0]:
        raise PliError("projection widths do not match the cache / output")
    if q_out.dim() != 3 or tuple(q_out.shape[:2]) != (B, S) or q_out.stride(2) != 1:
        raise PliError("q_out must be [B, S, Hq*D] with unit inner stride")
    if any(w.stride(1) != 1 or w.shape[1] != hidden for w in (wq, wk, wv)):
        raise PliError("weights must be [n, hidden] with unit inner stride")
    P = ctypes.c_void_p
    w = (P * 3)(*(t.data_ptr() for t in (wq, wk, wv)))
    c = (P * 3)(q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr())
    n = (_c_int * 3)(wq.shape[0], wk.shape[0], wv.shape[0])
    ldw = (_c_i64 * 3)(wq.stride(0), wk.stride(0), wv.stride(0))
    sb = (_c_i64 * 3)(q_out.stride(0), k_cache.stride(0), v_cache.stride(0))
    stok = (_c_i64 * 3)(q_out.stride(1), k_cache.stride(1), v_cache.stride(1))
    ro = (P * 3)(None, pos.data_ptr(), pos.data_ptr())
    cap = (_c_int * 3)(S, S_max, S_max)
    with _on_device(dev):
        rc = lib().pli_gemm_multi_nt(_ptr(x2), x2.stride(0), B * S, hidden, S, w, c, n, ldw, sb, stok,
                                     ro, cap, 3, _dtype_code(x), _stream(dev))
    _check(rc, "pli_gemm_multi_nt")
    return q_out


def _rows(t: torch.Tensor) -> torch.Tensor:
    t2 = t.reshape(-1, t.shape[-1])
    return t2 if t2.stride(1) == 1 and t2.stride(0) % 8 == 0 else t2.contiguous()


def _rms_gemm(a: torch.Tensor, norm_weight: torch.Tensor, eps: float, groups: list,
              residual: torch.Tensor | None, h_out: torch.Tensor | None, tokens_per_batch: int,
              swiglu: bool) -> None:
    """pli_rms_gemm_nt.  groups: (w, w_up | None, c, n, stride_batch, stride_token,
    pos | None, capacity) with c the output base tensor."""
    dev = _require_gpu(a, norm_weight, *(g[0] for g in groups))
    a2 = _rows(a)
    r2 = _rows(residual) if residual is not None else None
    if h_out is not None and (h_out.stride(-1) != 1 or tuple(h_out.shape[-1:]) != (a2.shape[1],)):
        raise PliError("h_out must have unit inner stride and the hidden width")
    h2 = h_out.view(-1, h_out.shape[-1]) if h_out is not None else None
    m, k = a2.shape
    ng = len(groups)
    P = ctypes.c_void_p
    w = (P * ng)(*(g[0].data_ptr() for g in groups))
    wu = (P * ng)(*(g[1].data_ptr() for g in groups)) if swiglu else None
    c = (P * ng)(*(g[2].data_ptr() for g in groups))
    n = (_c_int * ng)(*(int(g[3]) for g in groups))
    ldw = (_c_i64 * ng)(*(g[0].stride(0) for g in groups))
    sb = (_c_i64 * ng)(*(int(g[4]) for g in groups))
    stok = (_c_i64 * ng)(*(int(g[5]) for g in groups))
    ro = (P * ng)(*((g[6].data_ptr() if g[6] is not None else None) for g in groups))
    cap = (_c_int * ng)(*(int(g[7]) for g in groups))
    for g in groups:
        if g[0].stride(1) != 1 or (g[1] is not None and (g[1].stride(1) != 1 or g[1].stride(0) != g[0].stride(0))):
            raise PliError("weights must be [n, k] with unit inner stride (up weight: same ldw)")
    with _on_device(dev):
        rc = lib().pli_rms_gemm_nt(_ptr(a2), a2.stride(0), _ptr(r2), r2.stride(0) if r2 is not None else 0,
                                   _ptr(norm_weight), float(eps), _ptr(h2),
                                   h2.stride(0) if h2 is not None else 0, m, k, int(tokens_per_batch),
                                   w, wu, c, n, ldw, sb, stok, ro, cap, ng, _dtype_code(a), _stream(dev))
    _check(rc, "pli_rms_gemm_nt")


def rms_linear(a: torch.Tensor, norm_weight: torch.Tensor, eps: float, w: torch.Tensor,
               residual: torch.Tensor | None = None, h_out: torch.Tensor | None = None,
               out: torch.Tensor | None = None) -> torch.Tensor:
    """rmsnorm(a (+ residual)) @ w^T in one launch (decode: <= 4 rows)."""
    a2 = a.reshape(-1, a.shape[-1])
    if out is None:
        out = torch.empty(a2.shape[0], w.shape[0], device=a.device, dtype=a.dtype)
    # one token per "batch": row bb lands at out + bb * stride(0)
    _rms_gemm(a, norm_weight, eps, [(w, None, out, w.shape[0], out.stride(0), 0, None, 1 << 30)],
              residual, h_out, 1, False)
    return out.view(*a.shape[:-1], w.shape[0])


def rms_swiglu(a: torch.Tensor, norm_weight: torch.Tensor, eps: float, wg: torch.Tensor,
               wu: torch.Tensor, residual: torch.Tensor | None = None,
               h_out: torch.Tensor | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """silu(y wg^T) * (y wu^T) with y = rmsnorm(a (+ residual)), one launch."""
    a2 = a.reshape(-1, a.shape[-1])
    if out is None:
        out = torch.empty(a2.shape[0], wg.shape[0], device=a.device, dtype=a.dtype)
    _rms_gemm(a, norm_weight, eps, [(wg, wu, out, wg.shape[0], out.stride(0), 0, None, 1 << 30)],
              residual, h_out, 1, True)
    return out.view(*a.shape[:-1], wg.shape[0])


def rms_qkv_into_cache(a: torch.Tensor, norm_weight: torch.Tensor, eps: float,
                       wq: torch.Tensor, wk: torch.Tensor, wv: torch.Tensor, q_out: torch.Tensor,
                       k_cache: torch.Tensor, v_cache: torch.Tensor, pos: torch.Tensor,
                       residual: torch.Tensor | None = None,
                       h_out: torch.Tensor | None = None) -> torch.Tensor:
    """qkv_into_cache on rmsnorm(a (+ residual)), one launch; a [B, S, hidden]."""
    B, S, _ = a.shape
    S_max, Hkv, D = k_cache.shape[1:]
    if pos.dtype != torch.int32 or not pos.is_cuda:
        raise PliError("pos must be an int32 device tensor")
    for t in (k_cache, v_cache):
        if t.shape[0] != B or t.stride(3) != 1 or t.stride(2) != D:
            raise PliError("caches must be [B, S_max, Hkv, D] with contiguous (Hkv, D) rows")
    if q_out.dim() != 3 or tuple(q_out.shape[:2]) != (B, S) or q_out.stride(2) != 1:
        raise PliError("q_out must be [B, S, Hq*D] with unit inner stride")
    groups = [(wq, None, q_out, wq.shape[0], q_out.stride(0), q_out.stride(1), None, S),
              (wk, None, k_cache, wk.shape[0], k_cache.stride(0), k_cache.stride(1), pos, S_max),
              (wv, None, v_cache, wv.shape[0], v_cache.stride(0), v_cache.stride(1), pos, S_max)]
    _rms_gemm(a, norm_weight, eps, groups, residual, h_out, S, False)
    return q_out


# ------------------------------------------------------------ fused SwiGLU
def gemm_swiglu(x: torch.Tensor, w_gate: torch.Tensor, w_up: torch.Tensor,
                out: torch.Tensor | None = None, split_k: bool = True,
                variant: int | None = None) -> torch.Tensor:
    """h = silu(x W_gate^T) * (x W_up^T) in one launch; x [m, k], W_* [n, k]
    (unit column stride; any row stride, e.g. the two halves of a fused
    gate_up weight)."""
    dev = _require_gpu(x, w_gate, w_up)
    if x.dim() != 2 or w_gate.dim() != 2 or tuple(w_up.shape) != tuple(w_gate.shape) \
            or w_gate.shape[1] != x.shape[1]:
        raise PliError(f"gemm_swiglu shape mismatch x{tuple(x.shape)} wg{tuple(w_gate.shape)} "
                       f"wu{tuple(w_up.shape)}")
    x, w_gate, w_up = (t if t.stride(1) == 1 else t.contiguous() for t in (x, w_gate, w_up))
    m, k = x.shape
    n = w_gate.shape[0]
    if out is None:
        out = torch.empty(m, n, device=x.device, dtype=x.dtype)
    _require_gpu(x, out)
    if tuple(out.shape) != (m, n) or out.stride(1) != 1:
        raise PliError("bad output tensor")
    head = (_ptr(x), _ptr(w_gate), _ptr(w_up), _ptr(out), m, n, k, x.stride(0), w_gate.stride(0),
            w_up.stride(0), out.stride(0), _dtype_code(x))
    with _on_device(dev):
        wsb = lib().pli_gemm_swiglu_workspace_size(m, n, k, _dtype_code(x)) if split_k else 0
        if variant is not None:  # an explicit route (A/B, tests); no workspace when none is needed
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev) if wsb else None
            rc = lib().pli_gemm_swiglu_ws_variant(*head, _ptr(ws), wsb, _stream(dev), int(variant))
        elif wsb:
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            rc = lib().pli_gemm_swiglu_ws(*head, _ptr(ws), wsb, _stream(dev))
        else:
            rc = lib().pli_gemm_swiglu(*head, _stream(dev))
    _check(rc, "pli_gemm_swiglu")
    return out


# ---------------------------------------------------------------------- GEMV
def gemv(w: torch.Tensor, x: torch.Tensor, out: torch.Tensor | None = None,
         variant: int | None = None) -> torch.Tensor:
    """y = W x (torch.mv semantics), W [m, k] with unit column stride."""
    dev = _require_gpu(w, x)
    if w.dim() != 2 or x.dim() != 1 or w.shape[1] != x.shape[0]:
        raise PliError(f"gemv shape mismatch {tuple(w.shape)} x {tuple(x.shape)}")
    if w.stride(1) != 1:
        w = w.contiguous()
    x = x.contiguous()
    m, k = w.shape
    if out is None:
        out = torch.empty(m, dtype=w.dtype, device=dev)
    else:
        _check_out(out, w, (m,), "gemv")
    args = (_ptr(w), _ptr(x), _ptr(out), m, k, max(w.stride(0), k), _dtype_code(w), _stream(dev))
    with _on_device(dev):
        if variant is None:
            rc = lib().pli_gemv(*args)
        else:
            rc = lib().pli_gemv_variant(*args, int(variant))
    _check(rc, "pli_gemv")
    return out


# ---------------------------------------------------------------------- GEMM
def gemm(a: torch.Tensor, b: torch.Tensor, trans_b: bool = False,
         bias: torch.Tensor | None = None, out: torch.Tensor | None = None,
         variant: int | None = None) -> torch.Tensor:
    """C = A B (trans_b=False, torch.mm) or A B^T (+ bias) (trans_b=True, F.linear)."""
    ts = (a, b) if bias is None else (a, b, bias)
    dev = _require_gpu(*ts)
    if a.dim() != 2 or b.dim() != 2:
        raise PliError("gemm expects 2-D operands")
    m, k = a.shape
    n, kb = (b.shape if trans_b else (b.shape[1], b.shape[0]))
    if kb != k:
        raise PliError(f"gemm inner dims differ: {tuple(a.shape)} vs {tuple(b.shape)} trans_b={trans_b}")
    if a.stride(1) != 1:
        a = a.contiguous()
    if b.stride(1) != 1:
        b = b.contiguous()
    if bias is not None:
        bias = bias.contiguous()
        if bias.shape != (n,):
            raise PliError(f"bias must be [{n}]")
    if out is None:
        out = torch.empty((m, n), dtype=a.dtype, device=dev)
    else:
        _check_out(out, a, (m, n), "gemm")
    lda = a.stride(0) if m > 1 else k
    ldb = b.stride(0) if b.shape[0] > 1 else b.shape[1]
    head = (_ptr(a), _ptr(b), _ptr(out), _ptr(bias), m, n, k, max(lda, 1), max(ldb, 1),
            max(out.stride(0), n), int(bool(trans_b)), _dtype_code(a))
    with _on_device(dev):
        # decode-batch NT shapes split K over workgroups through a scratch
        # workspace from torch's caching allocator (pli_gemm_ws)
        wsb = lib().pli_gemm_workspace_size(m, n, k, int(bool(trans_b)), _dtype_code(a)) \
            if variant in (None, 0, 22, 24, 25, 26, 27, 28, 29) else 0
        if wsb:
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            if variant is None:
                rc = lib().pli_gemm_ws(*head, _ptr(ws), wsb, _stream(dev))
            else:
                rc = lib().pli_gemm_ws_variant(*head, _ptr(ws), wsb, _stream(dev), int(variant))
        elif variant is None:
            rc = lib().pli_gemm(*head, _stream(dev))
        else:
            rc = lib().pli_gemm_variant(*head, _stream(dev), int(variant))
    _check(rc, "pli_gemm")
    return out


def gemm_naive(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """C = A B for fp32 [M,K] x [K,N] with the ch05 naive kernel
    (pli_gemm_naive, one thread per output) -- the demo's contrast, not a
    production path."""
    dev = _require_gpu(a, b)
    if a.dtype != torch.float32 or b.dtype != torch.float32 or a.dim() != 2 or b.dim() != 2:
        raise PliError("gemm_naive expects 2-D fp32 operands")
    if a.shape[1] != b.shape[0]:
        raise PliError(f"gemm_naive inner dims differ: {tuple(a.shape)} vs {tuple(b.shape)}")
    a, b = a.contiguous(), b.contiguous()
    m, k = a.shape
    n = b.shape[1]
    if out is None:
        out = torch.empty((m, n), dtype=torch.float32, device=dev)
    else:
        _check_out(out, a, (m, n), "gemm_naive")
    with _on_device(dev):
        rc = lib().pli_gemm_naive(_ptr(a), _ptr(b), _ptr(out), m, n, k, max(k, 1), max(n, 1),
                                  max(out.stride(0), n), _stream(dev))
    _check(rc, "pli_gemm_naive")
    return out


# -------------------------------------------------------------- calibration
def scale_copy(inp: torch.Tensor, out: torch.Tensor, stride: int = 1) -> torch.Tensor:
    """out[i] = 2 * inp[i * stride] (fp32), the ch05/coalescing.cu probes."""
    dev = _require_gpu(inp, out)
    if inp.dtype != torch.float32 or not inp.is_contiguous() or not out.is_contiguous():
        raise PliError("scale_copy expects contiguous fp32 tensors")
    n_out = out.numel()
    if (n_out - 1) * stride >= inp.numel() and n_out > 0:
        raise PliError("scale_copy: input too short for stride")
    with _on_device(dev):
        rc = lib().pli_scale_copy(_ptr(inp), _ptr(out), n_out, int(stride), _stream(dev))
    _check(rc, "pli_scale_copy")
    return out


# ------------------------------------------------------------------ softmax
def gemm_f32out(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 [m, n] = x [m, k] @ w [n, k]^T for bf16 / fp16 x, w (pli_gemm_f32out):
    the row-parallel partial kept unrounded for the all-reduce."""
    dev = _require_gpu(x, w)
    if x.dim() != 2 or w.dim() != 2 or x.shape[1] != w.shape[1]:
        raise PliError(f"gemm_f32out: x {tuple(x.shape)} and w {tuple(w.shape)} must be [m, k] and [n, k]")
    if x.dtype not in (torch.bfloat16, torch.float16):
        raise PliError("gemm_f32out: bf16 / fp16 inputs only")
    x = x if x.stride(1) == 1 else x.contiguous()
    w = w if w.stride(1) == 1 else w.contiguous()
    m, k = x.shape
    n = w.shape[0]
    if out is None:
        out = torch.empty(m, n, dtype=torch.float32, device=dev)
    if out.dtype != torch.float32 or tuple(out.shape) != (m, n) or not out.is_contiguous() or out.device != dev:
        raise PliError("gemm_f32out: out must be a contiguous fp32 [m, n] tensor on the inputs' device")
    with _on_device(dev):
        rc = lib().pli_gemm_f32out(_ptr(x), _ptr(w), _ptr(out), m, n, k, x.stride(0), w.stride(0),
                                   _dtype_code(x), _stream(dev))
    _check(rc, "pli_gemm_f32out")
    return out


def mfma_probe(out: torch.Tensor, blocks: int, iters: int, shape: int = 0,
               clocks: torch.Tensor | None = None) -> torch.Tensor:
    """Launch the MFMA calibration kernel (pli_mfma_probe): ``blocks`` x 256
    threads, one workgroup per CU, ``iters`` rounds of 262,144 bf16 MFMA FLOP
    per wave (shape 0: 8 x 32x32x16, 1: 16 x 16x16x32); FLOPs = blocks * 4 *
    iters * 262144.  ``clocks`` (int64, >= blocks * 8, optional) receives per
    wave the s_memtime and s_memrealtime (100 MHz) ticks around the loop."""
    dev = _require_gpu(out)
    if out.dtype != torch.float32 or not out.is_contiguous() or out.numel() < blocks * 256:
        raise PliError("mfma_probe: out must be contiguous fp32 with >= blocks*256 elements")
    if clocks is not None:
        if _require_gpu(clocks) != dev:
            raise PliError("mfma_probe: clocks on another device")
        if clocks.dtype != torch.int64 or not clocks.is_contiguous() or clocks.numel() < blocks * 8:
            raise PliError("mfma_probe: clocks must be contiguous int64 with >= blocks*8 elements")
    with _on_device(dev):
        rc = lib().pli_mfma_probe(_ptr(out), _ptr(clocks), int(blocks), int(iters), int(shape), _stream(dev))
    _check(rc, "pli_mfma_probe")
    return out


def hbm_read_probe(buf: torch.Tensor, out: torch.Tensor, blocks: int, mode: int = 0) -> torch.Tensor:
    """Stream ``buf`` (contiguous, 16-byte multiple) with non-temporal 16-byte
    loads, ``blocks`` x 256 threads (pli_hbm_read_probe; mode 0 grid-stride,
    1 one contiguous slice per block); out: contiguous int32 >= blocks*256 on
    the same device."""
    dev = _require_gpu(buf)
    if _require_gpu(out) != dev:
        raise PliError("hbm_read_probe: out on another device")
    nbytes = buf.numel() * buf.element_size()
    if not buf.is_contiguous() or nbytes % 16:
        raise PliError("hbm_read_probe: buf must be contiguous with a multiple of 16 bytes")
    if out.dtype != torch.int32 or not out.is_contiguous() or out.numel() < blocks * 256:
        raise PliError("hbm_read_probe: out must be contiguous int32 with >= blocks*256 elements")
    with _on_device(dev):
        rc = lib().pli_hbm_read_probe(_ptr(buf), nbytes, _ptr(out), int(blocks), int(mode), _stream(dev))
    _check(rc, "pli_hbm_read_probe")
    return out


def softmax_rows(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Softmax over the last dim with the single-pass online (m, d) recurrence."""
    dev = _require_gpu(x)
    x = x.contiguous()
    n = x.shape[-1] if x.dim() > 0 else 1
    rows = x.numel() // max(n, 1)
    if out is None:
        out = torch.empty_like(x)
    with _on_device(dev):
        rc = lib().pli_softmax_rows(_ptr(x), _ptr(out), rows, n, _dtype_code(x), _stream(dev))
    _check(rc, "pli_softmax_rows")
    return out


def online_softmax_with_output(x: torch.Tensor, v: torch.Tensor):
    """(o, d): softmax(x)-weighted rows of v, and the denominator at the final max."""
    dev = _require_gpu(x, v)
    x, v = x.contiguous(), v.contiguous()
    n, dv = x.shape[-1], v.shape[-1]
    if tuple(v.shape[:-1]) != tuple(x.shape):
        raise PliError(f"v shape {tuple(v.shape)} does not match x {tuple(x.shape)}")
    rows = x.numel() // n
    o = torch.empty(x.shape[:-1] + (dv,), dtype=x.dtype, device=dev)
    d = torch.empty(x.shape[:-1], dtype=x.dtype, device=dev)
    with _on_device(dev):
        rc = lib().pli_online_softmax_with_output(_ptr(x), _ptr(v), _ptr(o), _ptr(d), rows, n, dv,
                                                  _dtype_code(x), _stream(dev))
    _check(rc, "pli_online_softmax_with_output")
    return o, d
