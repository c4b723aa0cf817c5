"""Linear layer whose weight gradient is accumulated straight into the flat fp32/bf16 grad
buffer by the GEMM itself (C = A^T B + C, beta = 1).

Eager autograd computes each weight gradient into a fresh tensor and then launches a separate
elementwise add into `.grad` on every micro-batch (≈1.5 % of a Llama-3-8B DPO step on MI355X,
measured: profiles/r1_baseline_kernel_stats.md). When the training engine has attached
`param.main_grad` (a view of its flat gradient buffer) this op instead issues
`main_grad.addmm_(dY^T, X)` — hipBLASLt folds the accumulation into the GEMM epilogue, no
temporary, one rounding — and notifies the engine's bucket scheduler itself.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def accumulate_weight_grad(weight: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor) -> bool:
    """main_grad += dy2^T @ x2 if the engine attached a main_grad; returns True if handled."""
    mg = getattr(weight, "main_grad", None)
    if mg is None or getattr(weight, "_dla_shared", False):
        return False
    mg.addmm_(dy2.t(), x2)
    hook = getattr(weight, "_dla_grad_hook", None)
    if hook is not None:
        hook(weight)
    return True


class _LinearMainGradFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        K, N = x.shape[-1], dy.shape[-1]
        dy2 = dy.reshape(-1, N)
        dx = (dy2 @ weight).view(x.shape) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, K)
            if not accumulate_weight_grad(weight, dy2, x2):
                dw = dy2.t() @ x2
        db = dy2.sum(0) if (ctx.has_bias and ctx.needs_input_grad[2]) else None
        return dx, dw, db


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None) -> torch.Tensor:
    if (weight.requires_grad and torch.is_grad_enabled() and getattr(weight, "main_grad", None) is not None
            and not getattr(weight, "_dla_shared", False)):
        return _LinearMainGradFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)
