"""Decode-path ops: split-KV GQA decode attention and the fused top-k/top-p sampler.

GPU tensors run `torch.ops.dla.decode_attn` / `torch.ops.dla.sample_tokens` (csrc/decode.hip,
csrc/sampling.hip); both take their lengths / RNG counter from device memory so a decode step can
be captured once in a hipGraph and replayed per token. CPU tensors use PyTorch references.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from . import _ext


def decode_supported(q_heads: int, kv_heads: int, head_dim: int) -> bool:
    return head_dim in (64, 128) and q_heads % kv_heads == 0 and (q_heads // kv_heads) in (1, 2, 4, 8)


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                     kv_len: torch.Tensor, kv_start: Optional[torch.Tensor] = None, window: int = 0,
                     scale: Optional[float] = None) -> torch.Tensor:
    """q [B, Hq, D] (the newest token), caches [B, Tmax, Hkv, D]; keys [kv_start, kv_len) are
    attended (kv_len: int32 [1] on device). Returns [B, Hq, D]."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if _ext.use_native(q):
        return _ext.require().decode_attn(q, k_cache, v_cache, kv_len.to(torch.int32),
                                          kv_start.to(torch.int32) if kv_start is not None else None,
                                          int(window), float(scale))
    return ref_decode_attention(q, k_cache, v_cache, int(kv_len.reshape(-1)[0]), kv_start, window, scale)


def ref_decode_attention(q, k_cache, v_cache, L: int, kv_start=None, window: int = 0, scale=None):
    B, Hq, D = q.shape
    Hkv = k_cache.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    k = k_cache[:, :L].float().repeat_interleave(Hq // Hkv, dim=2)  # [B, L, Hq, D]
    v = v_cache[:, :L].float().repeat_interleave(Hq // Hkv, dim=2)
    s = torch.einsum("bhd,blhd->bhl", q.float(), k) * scale
    idx = torch.arange(L, device=q.device)
    lo = kv_start.view(B, 1).long() if kv_start is not None else torch.zeros(B, 1, dtype=torch.long, device=q.device)
    if window and window > 0:
        lo = torch.clamp(lo, min=L - window)
    mask = idx.view(1, L) < lo
    s = s.masked_fill(mask.view(B, 1, L), float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("bhl,blhd->bhd", p, v).to(q.dtype)


def sample_tokens(logits: torch.Tensor, temperature: float, top_k: int, top_p: float, greedy: bool,
                  rng: torch.Tensor, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """logits [B, V] -> token ids [B] (int64). rng: int64 [2] device tensor (seed, counter) for
    the fused kernel; CPU falls back to `models.generation.sample_next` semantics."""
    if _ext.use_native(logits):
        return _ext.require().sample_tokens(logits, float(temperature), int(top_k), float(top_p),
                                            bool(greedy), rng)
    from ..models.generation import sample_next

    return sample_next(logits.float(), not greedy, temperature, top_p, top_k, generator)
