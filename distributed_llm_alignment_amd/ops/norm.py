"""Fused residual-add + RMSNorm / LayerNorm.

`add_norm(x, residual, weight, bias, eps, rms)` returns `(y, s)` where `s = x + residual` (the
new residual stream, bf16-rounded as in HF) and `y = norm(s)`. With `residual=None`, `s = x`.
Reference semantics: HF LlamaRMSNorm / nn.LayerNorm as used by the reference's models
(src/models/base_model.py:30-34 -> transformers modeling).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _ext


def _ref_norm(s: torch.Tensor, weight, bias, eps: float, rms: bool) -> torch.Tensor:
    xf = s.float()
    if rms:
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    else:
        mu = xf.mean(-1, keepdim=True)
        y = (xf - mu) * torch.rsqrt((xf - mu).pow(2).mean(-1, keepdim=True) + eps)
    y = y * weight.float()
    if bias is not None:
        y = y + bias.float()
    return y.to(s.dtype)


class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps, rms, keep_stream=False):
        ops = _ext.require()
        H = x.shape[-1]
        x2 = x.reshape(-1, H)
        r2 = residual.reshape(-1, H) if residual is not None else None
        y, s, rstd, mean = ops.norm_fwd(x2, r2, weight, bias, float(eps), bool(rms))
        if residual is None:
            s = x2
        ctx.save_for_backward(s, weight, rstd, mean if not rms else None)
        ctx.rms = rms
        ctx.has_res = residual is not None
        ctx.has_bias = bias is not None
        ctx.shape = x.shape
        # keep_stream: the stream s (= x when there is no residual) leaves as a second output of
        # THIS node, so whoever adds the next branch onto it (a GEMM with s as its C input,
        # ops.linear.linear_add) hands its gradient back here, where norm_bwd folds it in as
        # `dres` -- one kernel, no separate autograd accumulation of the two gradients of s
        out_s = s.view(x.shape) if (residual is not None or keep_stream) else None
        ctx.mark_non_differentiable(rstd)
        return y.view(x.shape), out_s

    @staticmethod
    def backward(ctx, dy, ds_out):
        ops = _ext.require()
        s, weight, rstd, mean = ctx.saved_tensors
        H = ctx.shape[-1]
        dres = ds_out.reshape(-1, H).contiguous() if ds_out is not None else None
        ds, dw, db = ops.norm_bwd(dy.reshape(-1, H).contiguous(), s, weight, rstd, mean, dres,
                                  ctx.has_bias, ctx.rms)
        ds = ds.view(ctx.shape)
        return ds, (ds if ctx.has_res else None), dw, (db if ctx.has_bias else None), None, None, None


def add_norm(x: torch.Tensor, residual: Optional[torch.Tensor], weight: torch.Tensor,
             bias: Optional[torch.Tensor] = None, eps: float = 1e-5,
             rms: bool = True, keep_stream: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """`keep_stream`: return the stream s as an output of the norm node even without a
    residual (see _NormFn), for a caller that feeds s to ops.linear.linear_add."""
    if _ext.use_native(x):
        y, s = _NormFn.apply(x.contiguous(), residual.contiguous() if residual is not None else None,
                             weight, bias, eps, rms, keep_stream)
        return y, (s if s is not None else x)
    s = x if residual is None else (x + residual)
    return _ref_norm(s, weight, bias, eps, rms), s


def rms_norm(x, weight, eps=1e-6):
    return add_norm(x, None, weight, None, eps, True)[0]


def layer_norm(x, weight, bias, eps=1e-5):
    return add_norm(x, None, weight, bias, eps, False)[0]
