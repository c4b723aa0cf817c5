"""Fused AdamW + grad-norm clipping over flat buffers.

The reference builds `torch.optim.AdamW` per trainer (src/training/train_dpo.py:73-77 wd=0.01,
train_sft.py:89-94 betas (0.9, 0.95), ...) and clips with `accelerator.clip_grad_norm_`
(src/training/utils.py:121-123). Here the update is ONE HIP kernel launch over the whole flat
(or ZeRO-sharded) buffer: fp32 master + fp32 moments, bf16 weights written back, clip
coefficient read from device memory (no host sync).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..ops import _ext


def adamw_update(param: Optional[torch.Tensor], master: Optional[torch.Tensor], grad: torch.Tensor,
                 m: torch.Tensor, v: torch.Tensor, lr: float, beta1: float, beta2: float, eps: float,
                 weight_decay: float, step: int, clip: Optional[torch.Tensor] = None,
                 grad_scale: float = 1.0) -> None:
    """In-place AdamW on flat tensors. `param` (bf16) receives the updated weights; `master`
    (fp32, optional) is the authoritative copy when present."""
    if _ext.use_native(grad):
        _ext.require().adamw_step(param, master, grad, m, v, float(lr), float(beta1), float(beta2),
                                  float(eps), float(weight_decay), int(step), clip, float(grad_scale))
        return
    g = grad.float() * grad_scale
    if clip is not None:
        g = g * clip.float()
    w = master if master is not None else param.float()
    w.mul_(1 - lr * weight_decay)
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    w.addcdiv_(m, denom, value=-lr / bc1)
    if param is not None:
        param.copy_(w.to(param.dtype))


def grad_sumsq(grad: torch.Tensor, out: torch.Tensor, accumulate: bool = False) -> torch.Tensor:
    """out[0] (+)= sum(grad^2) in fp32 (deterministic fixed-grid reduction on the GPU)."""
    if _ext.use_native(grad):
        _ext.require().grad_sumsq(grad, out, accumulate)
        return out
    s = grad.float().pow(2).sum()
    if accumulate:
        out.add_(s)
    else:
        out.copy_(s.reshape(out.shape))
    return out


def clip_coefficient(sumsq: torch.Tensor, max_norm: float):
    """(norm, coef) with coef = min(1, max_norm / (norm + 1e-6)) — torch clip_grad_norm_ rule."""
    if _ext.use_native(sumsq):
        return _ext.require().clip_coef(sumsq.contiguous(), float(max_norm))
    norm = sumsq.reshape(()).sqrt()
    coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0) if max_norm > 0 else torch.ones_like(norm)
    return norm, coef
