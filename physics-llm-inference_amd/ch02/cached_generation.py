"""Cached generation -- mirror of ``ch02/cached_generation.py``.

Module names, constructor signatures, parameter names and creation order
follow the reference (``ch02/cached_generation.py:20-201``), so seeded models
and ``state_dict``s are interchangeable.  On a ROCm device:

* ``CachedGQA`` projects on ``pli_gemm`` and attends over the cache with
  ``pli_attn_decode`` (split-K flash-decoding in place on the
  [B, S_max, Hkv, hd] buffer; the prompt goes to the prefill flash kernel
  through the same entry point), replacing ``:71-94``;
* ``SwiGLUFFN`` runs gate + up + silu·mul as one ``pli_gemm_swiglu`` launch
  and down on ``pli_gemm``;
* ``CachedTransformerModel``'s ``lm_head`` runs on ``pli_gemm``.
* ``RMSNorm`` is one ``pli_rmsnorm`` launch, and the model folds every
  residual add into the following norm's launch (2 launches per layer
  instead of 14 elementwise/reduce kernels).
Embedding lookup and sampling stay in torch.  CPU tensors keep the
reference math.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

import pli_hip

from .kv_cache import _proj, attend_cached


def _lin(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return _proj(x, w) if x.is_cuda else F.linear(x, w)


@dataclass
class LayerKVCache:
    """One layer's cache: k, v [batch, max_seq_len, num_kv_heads, head_dim].

    ``pos`` (optional, this build): an int32 [1] device tensor holding the
    number of valid rows, shared by all layers of a model and advanced by
    ``CachedTransformerModel.forward``.  With it the append and the
    single-token attention read the length on the device, so a decode step
    can be captured once and replayed (``ch08.DecodeStepGraph``)."""
    k: torch.Tensor
    v: torch.Tensor
    seq_len: int = 0
    pos: torch.Tensor | None = None

    def reserve(self, n: int) -> None:
        """Raise when appending ``n`` rows would overrun ``max_seq_len`` -- the
        reference raises there too (its slice assignment shapes stop matching,
        ``:27-33``).  The device-length paths need the check on the host: the
        append and attention kernels clamp to the capacity and would otherwise
        return wrong logits silently."""
        cap = self.k.shape[1]
        if self.seq_len + n > cap:
            raise RuntimeError(f"KV cache overflow: {self.seq_len} cached + {n} new rows > "
                               f"max_seq_len {cap}")

    def update(self, k_new: torch.Tensor, v_new: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """Append new K/V and return the valid prefixes (``:27-33``).  With a
        device ``pos`` the rows go to ``*pos``, which this method does NOT
        advance: ``CachedTransformerModel.forward`` advances the one ``pos``
        all layers share, once per forward (``seq_len`` is advanced here)."""
        n = k_new.shape[1]
        self.reserve(n)
        if self.pos is not None:
            pli_hip.kv_append(k_new, v_new, self.k, self.v, self.pos)
        else:
            self.k[:, self.seq_len:self.seq_len + n] = k_new
            self.v[:, self.seq_len:self.seq_len + n] = v_new
        self.seq_len += n
        return self.k[:, :self.seq_len], self.v[:, :self.seq_len]


class CachedGQA(nn.Module):
    def __init__(self, hidden_dim: int, num_heads: int, num_kv_heads: int):
        super().__init__()
        self.num_heads = num_heads
        self.num_kv_heads = num_kv_heads
        self.num_groups = num_heads // num_kv_heads
        self.head_dim = hidden_dim // num_heads
        self.hidden_dim = hidden_dim
        self.q_proj = nn.Linear(hidden_dim, num_heads * self.head_dim, bias=False)
        self.k_proj = nn.Linear(hidden_dim, num_kv_heads * self.head_dim, bias=False)
        self.v_proj = nn.Linear(hidden_dim, num_kv_heads * self.head_dim, bias=False)
        self.o_proj = nn.Linear(hidden_dim, hidden_dim, bias=False)

    def forward(self, x: torch.Tensor, cache: LayerKVCache | None = None, start_pos: int = 0
                ) -> torch.Tensor:
        B, S, _ = x.shape
        if (cache is not None and cache.pos is not None and x.is_cuda
                and (B * S <= 16 or (B * S <= 32 and x.shape[-1] % 128 == 0))
                and _device_len_ok_shape(x, S, self.num_heads, self.num_kv_heads, self.head_dim)):
            # decode step, device-resident length: q/k/v projections in one
            # launch with k/v written straight into the cache rows at pos
            # (skinny kernel up to 16 rows, small-M MFMA kernel up to 32: above
            # that the mid-M kernel of the packed GEMM + the append win)
            cache.reserve(S)
            q = torch.empty(B, S, self.num_heads * self.head_dim, device=x.device, dtype=x.dtype)
            pli_hip.qkv_into_cache(x, self.q_proj.weight, self.k_proj.weight, self.v_proj.weight,
                                   q, cache.k, cache.v, cache.pos)
            cache.seq_len += S
            o = pli_hip.attn_decode_dev(q.view(B, S, self.num_heads, self.head_dim), cache.k,
                                        cache.v, cache.pos, n_kv_add=S, causal=S > 1)
            return _lin(o.reshape(B, S, self.hidden_dim), self.o_proj.weight)
        if x.is_cuda:
            # q, k and v from one GEMM over the packed [Wq; Wk; Wv] (views of
            # the output columns feed the cache append and attention in place)
            nq, nk = self.num_heads * self.head_dim, self.num_kv_heads * self.head_dim
            qkv = _lin(x, self._packed_qkv())
            q = qkv[..., :nq].unflatten(-1, (self.num_heads, self.head_dim))
            k = qkv[..., nq:nq + nk].unflatten(-1, (self.num_kv_heads, self.head_dim))
            v = qkv[..., nq + nk:].unflatten(-1, (self.num_kv_heads, self.head_dim))
        else:
            q = _lin(x, self.q_proj.weight).view(B, S, self.num_heads, self.head_dim)
            k = _lin(x, self.k_proj.weight).view(B, S, self.num_kv_heads, self.head_dim)
            v = _lin(x, self.v_proj.weight).view(B, S, self.num_kv_heads, self.head_dim)
        if cache is not None:
            cache.update(k, v)
            if cache.pos is not None and _device_len_ok(q, cache):
                # length read on the device: replayable inside a captured step
                o = pli_hip.attn_decode_dev(q, cache.k, cache.v, cache.pos, n_kv_add=S,
                                            causal=S > 1)
                return _lin(o.reshape(B, S, self.hidden_dim), self.o_proj.weight)
            k_buf, v_buf, n_kv = cache.k, cache.v, cache.seq_len
        else:
            k_buf, v_buf, n_kv = k, v, S
        o = attend_cached(q, k_buf, v_buf, n_kv).reshape(B, S, self.hidden_dim)
        return _lin(o, self.o_proj.weight)


    def _packed_qkv(self) -> torch.Tensor:
        """[Wq; Wk; Wv] as one contiguous [(H + 2 Hkv) hd, hidden] tensor whose
        row blocks ARE the three projections' weights: the first call packs
        them and re-points the parameters' data at the blocks (no second
        copy is kept); a parameter replaced later (load, dtype / device move)
        is detected by address and packed again."""
        wq, wk, wv = self.q_proj.weight, self.k_proj.weight, self.v_proj.weight
        buf = getattr(self, "_qkv_buf", None)
        nq, nk = wq.shape[0], wk.shape[0]
        if (buf is not None and buf.device == wq.device and buf.dtype == wq.dtype
                and wq.data_ptr() == buf.data_ptr() and wk.data_ptr() == buf[nq].data_ptr()
                and wv.data_ptr() == buf[nq + nk].data_ptr()):
            return buf
        with torch.no_grad():
            buf = torch.cat([wq.data, wk.data, wv.data]).contiguous()
            wq.data, wk.data, wv.data = buf[:nq], buf[nq:nq + nk], buf[nq + nk:]
        self._qkv_buf = buf
        return buf


def _device_len_ok_shape(x: torch.Tensor, S: int, H: int, Hkv: int, D: int) -> bool:
    return (x.dtype in (torch.bfloat16, torch.float16) and D in (64, 128)
            and S * (H // Hkv) <= 16 and x.shape[-1] % 8 == 0)


def _device_len_ok(q: torch.Tensor, cache: LayerKVCache) -> bool:
    """Shapes the device-length decode kernel takes (the prompt, with more
    query rows per kv head, goes through the host-length path)."""
    B, S, H, D = q.shape
    return (q.dtype in (torch.bfloat16, torch.float16) and D in (64, 128)
            and S * (H // cache.k.shape[2]) <= 16)


class RMSNorm(nn.Module):
    def __init__(self, hidden_dim: int, eps: float = 1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_dim))
        self.eps = eps

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:  # one launch (pli_rmsnorm) instead of six elementwise/reduce kernels
            return pli_hip.rmsnorm(x, self.weight, self.eps)
        return x / torch.sqrt(torch.mean(x ** 2, dim=-1, keepdim=True) + self.eps) * self.weight


class SwiGLUFFN(nn.Module):
    def __init__(self, hidden_dim: int, intermediate_dim: int):
        super().__init__()
        self.gate_proj = nn.Linear(hidden_dim, intermediate_dim, bias=False)
        self.up_proj = nn.Linear(hidden_dim, intermediate_dim, bias=False)
        self.down_proj = nn.Linear(intermediate_dim, hidden_dim, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:  # gate, up and silu*mul in one launch (pli_gemm_swiglu)
            lead = x.shape[:-1]
            h = pli_hip.gemm_swiglu(x.reshape(-1, x.shape[-1]), self.gate_proj.weight,
                                    self.up_proj.weight)
            return _lin(h.view(*lead, h.shape[-1]), self.down_proj.weight)
        h = F.silu(_lin(x, self.gate_proj.weight)) * _lin(x, self.up_proj.weight)
        return _lin(h, self.down_proj.weight)


class CachedTransformerBlock(nn.Module):
    def __init__(self, hidden_dim: int, num_heads: int, num_kv_heads: int, intermediate_dim: int):
        super().__init__()
        self.input_norm = RMSNorm(hidden_dim)
        self.attn = CachedGQA(hidden_dim, num_heads, num_kv_heads)
        self.post_attn_norm = RMSNorm(hidden_dim)
        self.ffn = SwiGLUFFN(hidden_dim, intermediate_dim)

    def forward(self, x: torch.Tensor, cache: LayerKVCache | None = None, start_pos: int = 0
                ) -> torch.Tensor:
        if x.is_cuda:
            h, n2 = self.attn_half(x, None, cache, start_pos)
            return h + self.ffn(n2)
        h = x + self.attn(self.input_norm(x), cache, start_pos)
        return h + self.ffn(self.post_attn_norm(h))

    def decode_fused(self, x: torch.Tensor, pending: torch.Tensor | None, cache: LayerKVCache
                     ) -> tuple[torch.Tensor, torch.Tensor]:
        """Decode step of the layer in 5 launches: input norm (+ the pending
        residual add) fused into q/k/v (k/v straight into the cache at the
        device position), attention, o_proj, post-attention norm (+ residual)
        fused into gate/up/silu*mul, down_proj.  Returns (residual stream,
        pending FFN output)."""
        B, S, hd = x.shape
        at = self.attn
        cache.reserve(S)
        q = torch.empty(B, S, at.num_heads * at.head_dim, device=x.device, dtype=x.dtype)
        if pending is None:
            pli_hip.rms_qkv_into_cache(x, self.input_norm.weight, self.input_norm.eps,
                                       at.q_proj.weight, at.k_proj.weight, at.v_proj.weight, q,
                                       cache.k, cache.v, cache.pos)
        else:
            h = torch.empty_like(x)
            pli_hip.rms_qkv_into_cache(pending, self.input_norm.weight, self.input_norm.eps,
                                       at.q_proj.weight, at.k_proj.weight, at.v_proj.weight, q,
                                       cache.k, cache.v, cache.pos, residual=x, h_out=h)
            x = h
        cache.seq_len += S
        o = pli_hip.attn_decode_dev(q.view(B, S, at.num_heads, at.head_dim), cache.k, cache.v,
                                    cache.pos, n_kv_add=S, causal=S > 1)
        a = _lin(o.reshape(B, S, hd), at.o_proj.weight)
        h2 = torch.empty_like(x)
        f = self.ffn
        g = pli_hip.rms_swiglu(a, self.post_attn_norm.weight, self.post_attn_norm.eps,
                               f.gate_proj.weight, f.up_proj.weight, residual=x, h_out=h2)
        return h2, _lin(g, f.down_proj.weight)

    def attn_half(self, x: torch.Tensor, pending: torch.Tensor | None,
                  cache: LayerKVCache | None, start_pos: int):
        """Device path: x (+ the previous layer's pending FFN output, added in
        the input norm's launch) -> attention -> (h, post_attn_norm(h)), the
        residual add fused into the post-attention norm's launch."""
        if pending is None:
            n1 = pli_hip.rmsnorm(x, self.input_norm.weight, self.input_norm.eps)
        else:
            x, n1 = pli_hip.rmsnorm(pending, self.input_norm.weight, self.input_norm.eps,
                                    residual=x)
        a = self.attn(n1, cache, start_pos)
        return pli_hip.rmsnorm(a, self.post_attn_norm.weight, self.post_attn_norm.eps, residual=x)


# decode steps (<= 4 rows, device-resident cache length): every RMSNorm fused
# into the projection that consumes it (pli_rms_gemm_nt); tests flip it off
# to compare with the unfused launches
FUSED_DECODE = True


class CachedTransformerModel(nn.Module):
    """Decoder-only transformer whose layers append to per-layer KV caches."""

    def __init__(self, vocab_size: int, hidden_dim: int, num_layers: int, num_heads: int,
                 num_kv_heads: int, intermediate_dim: int):
        super().__init__()
        self.embed = nn.Embedding(vocab_size, hidden_dim)
        self.layers = nn.ModuleList([
            CachedTransformerBlock(hidden_dim, num_heads, num_kv_heads, intermediate_dim)
            for _ in range(num_layers)
        ])
        self.norm = RMSNorm(hidden_dim)
        self.lm_head = nn.Linear(hidden_dim, vocab_size, bias=False)
        self.hidden_dim = hidden_dim
        self.num_layers = num_layers
        self.num_kv_heads = num_kv_heads
        self.head_dim = hidden_dim // num_heads

    def forward(self, input_ids: torch.Tensor, caches: list[LayerKVCache] | None = None,
                start_pos: int = 0) -> torch.Tensor:
        x = self.embed(input_ids)
        if x.is_cuda and self._fused_decode_ok(x, caches):
            pending = None
            for i, layer in enumerate(self.layers):
                x, pending = layer.decode_fused(x, pending, caches[i])
            caches[0].pos.add_(input_ids.shape[1])
            return pli_hip.rms_linear(pending, self.norm.weight, self.norm.eps, self.lm_head.weight,
                                      residual=x)
        if x.is_cuda:
            # residual stream with the adds folded into the norms: per layer one
            # norm(+add) before attention, one after; the FFN output stays
            # pending until the next layer's (or the final) norm adds it
            pending = None
            for i, layer in enumerate(self.layers):
                x, n2 = layer.attn_half(x, pending, caches[i] if caches is not None else None,
                                        start_pos)
                pending = layer.ffn(n2)
            if caches is not None and caches[0].pos is not None:
                caches[0].pos.add_(input_ids.shape[1])  # one length shared by every layer
            if pending is None:  # no layers
                xn = pli_hip.rmsnorm(x, self.norm.weight, self.norm.eps)
            else:
                _, xn = pli_hip.rmsnorm(pending, self.norm.weight, self.norm.eps, residual=x)
            return _lin(xn, self.lm_head.weight)
        for i, layer in enumerate(self.layers):
            x = layer(x, caches[i] if caches is not None else None, start_pos)
        return _lin(self.norm(x), self.lm_head.weight)

    def _fused_decode_ok(self, x: torch.Tensor, caches) -> bool:
        if not FUSED_DECODE or caches is None or caches[0].pos is None or not self.layers:
            return False
        B, S, hd = x.shape
        at = self.layers[0].attn
        return (B * S <= 4 and hd % 8 == 0 and hd <= 8192 and B * S * hd * 2 <= 65536
                and _device_len_ok_shape(x, S, at.num_heads, at.num_kv_heads, at.head_dim))

    def create_caches(self, batch_size: int, max_seq_len: int, device: torch.device,
                      dtype: torch.dtype, device_pos: bool = False) -> list[LayerKVCache]:
        """Per-layer caches (``:187-201``).  ``device_pos`` (this build) gives them
        one shared device-resident length for graph-captured decode steps."""
        shape = (batch_size, max_seq_len, self.num_kv_heads, self.head_dim)
        pos = torch.zeros(1, device=device, dtype=torch.int32) if device_pos else None
        return [LayerKVCache(k=torch.zeros(shape, device=device, dtype=dtype),
                             v=torch.zeros(shape, device=device, dtype=dtype), seq_len=0, pos=pos)
                for _ in range(self.num_layers)]


def _sync(device: torch.device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize()


def cached_generate(model: CachedTransformerModel, input_ids: torch.Tensor, max_new_tokens: int,
                    temperature: float = 1.0) -> tuple[torch.Tensor, dict]:
    """Prefill the prompt once, then decode one token per step over the caches
    (``ch02/cached_generation.py:204-274``).  Returns the prompt followed by
    the sampled tokens, and {prefill_ms, decode_ms[], total_ms}."""
    model.eval()
    device = input_ids.device
    dtype = next(model.parameters()).dtype
    batch_size, prompt_len = input_ids.shape
    caches = model.create_caches(batch_size, prompt_len + max_new_tokens, device, dtype)
    timings = {"prefill_ms": 0, "decode_ms": [], "total_ms": 0}
    out = [input_ids]

    def sample(logits):
        probs = F.softmax(logits[:, -1, :] / temperature, dim=-1)
        return torch.multinomial(probs, num_samples=1)

    with torch.no_grad():
        _sync(device)
        t0 = time.perf_counter()
        logits = model(input_ids, caches, start_pos=0)
        _sync(device)
        timings["prefill_ms"] = (time.perf_counter() - t0) * 1000
        token = sample(logits)
        out.append(token)
        for i in range(max_new_tokens - 1):
            _sync(device)
            t0 = time.perf_counter()
            logits = model(token, caches, start_pos=prompt_len + i)
            _sync(device)
            timings["decode_ms"].append((time.perf_counter() - t0) * 1000)
            token = sample(logits)
            out.append(token)

    timings["total_ms"] = timings["prefill_ms"] + sum(timings["decode_ms"])
    return torch.cat(out, dim=1), timings


def compare_generation_methods():
    """The chapter's comparison run (ch02/cached_generation.py:277-314): a
    small GQA model, prefill vs per-token decode timings of cached_generate."""
    device = "cuda" if torch.cuda.is_available() else "cpu"
    dtype = torch.float16 if device == "cuda" else torch.float32
    model = CachedTransformerModel(vocab_size=1000, hidden_dim=512, num_layers=8, num_heads=8, num_kv_heads=2,
                                   intermediate_dim=1024).to(device, dtype)
    prompt_len, new_tokens = 50, 50
    ids = torch.randint(0, 1000, (1, prompt_len), device=device)
    print(f"Generation Comparison (device={device})\nPrompt: {prompt_len} tokens, Generate: {new_tokens} tokens")
    print("=" * 60)
    _, t = cached_generate(model, ids, new_tokens)
    print(f"\nCached Generation:\n  Prefill:     {t['prefill_ms']:.2f} ms ({prompt_len} tokens)\n"
          f"  Decode avg:  {sum(t['decode_ms']) / len(t['decode_ms']):.2f} ms/token\n  Total:       {t['total_ms']:.2f} ms")
    print("\n" + "=" * 60 + "\n\nKey insight:\n"
          f"  Prefill processes {prompt_len} tokens in one pass (GEMMs, flash attention: compute bound)\n"
          "  Decode processes 1 token at a time (GEMVs, attention over the cache: memory bound)\n"
          "  Per-token decode time barely grows with the cache at this length")


if __name__ == "__main__":
    compare_generation_methods()
