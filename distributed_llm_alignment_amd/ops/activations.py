"""Fused MLP activations: SwiGLU over a fused gate|up GEMM output, tanh-GELU.

Reference: HF LlamaMLP `down_proj(act(gate_proj(x)) * up_proj(x))`, GPT-2 / phi-2 `gelu_new`.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _ext


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        ops = _ext.require()
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        return ops.swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dout):
        (gu,) = ctx.saved_tensors
        return _ext.require().swiglu_bwd(gu, dout.contiguous())


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    """silu(gu[..., :F]) * gu[..., F:]."""
    if _ext.use_native(gu):
        return _SwiGLUFn.apply(gu)
    g, u = gu.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gu.dtype)


class _GeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        ctx.save_for_backward(x)
        return _ext.require().gelu_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return _ext.require().gelu_bwd(x, dy.contiguous())


def gelu_new(x: torch.Tensor) -> torch.Tensor:
    if _ext.use_native(x):
        return _GeluFn.apply(x)
    xf = x.float()
    y = 0.5 * xf * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (xf + 0.044715 * xf.pow(3))))
    return y.to(x.dtype)
