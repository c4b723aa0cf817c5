"""Fused MLP activations: SwiGLU over a fused gate|up GEMM output, tanh-GELU.

Reference: HF LlamaMLP `down_proj(act(gate_proj(x)) * up_proj(x))`, GPT-2 / phi-2 `gelu_new`.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

import os

from . import _ext
from .linear import accumulate_weight_grad, add_gemm, input_grad, uses_main_grad
from ..parallel import collectives as coll

FUSED_MLP = os.environ.get("DLA_FUSED_MLP", "1") != "0"


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


class _SwiGLUMLPFn(torch.autograd.Function):
    """down(swiglu(h @ Wgu^T)) as ONE autograd node for weights that accumulate into the engine's
    main_grad. The HIP SwiGLU kernels also emit m^T (forward) and dgu^T (backward), the operands
    the TN weight-gradient GEMMs (ops/linear.py) would otherwise transpose in separate passes:
    per Llama-3-8B layer and micro-batch that removes a read+write of [M, 3F] bf16."""

    @staticmethod
    def forward(ctx, h, w_up, w_down, tp_group=None, chunks=1, resid=None):
        ops = _ext.require()
        H = h.shape[-1]
        h2 = h.reshape(-1, H)
        u = F.linear(h2, w_up)
        m, mt = ops.swiglu_fwd_t(u)
        if resid is not None:  # residual stream as the down GEMM's C input (ops.linear.add_gemm)
            y = add_gemm(m, w_down, resid.reshape(-1, w_down.shape[0]))
        elif tp_group is None:
            y = F.linear(m, w_down)
        else:
            # tensor parallel (gate|up column-, down row-parallel): the down GEMM runs in token
            # chunks, each chunk's all-reduce launched async behind the next chunk's GEMM
            import torch.distributed as dist

            from ..parallel.tensor_parallel import _chunk_bounds

            y = torch.empty((m.shape[0], w_down.shape[0]), dtype=m.dtype, device=m.device)
            works = []
            for a, b in _chunk_bounds(m.shape[0], chunks):
                torch.mm(m[a:b], w_down.t(), out=y[a:b])
                works.append(coll.all_reduce(y[a:b], group=tp_group, async_op=True))
            for w in works:
                w.wait()
        # (weights on ctx: see ops.linear._LinearMainGradFn)
        ctx.save_for_backward(h2, u, mt)
        ctx.w_up, ctx.w_down = w_up, w_down
        ctx.hshape = h.shape
        ctx.tp_group = tp_group
        ctx.has_resid = resid is not None
        return y.view(*h.shape[:-1], w_down.shape[0])

    @staticmethod
    def backward(ctx, dy):
        h2, u, mt = ctx.saved_tensors
        w_up, w_down = ctx.w_up, ctx.w_down
        ops = _ext.require()
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dm = input_grad(dy2, w_down)
        accumulate_weight_grad(w_down, dy2, mt.t(), xt=mt)
        del mt
        du, dut = ops.swiglu_bwd_t(u, dm)
        del dm
        dh = input_grad(du, w_up) if ctx.needs_input_grad[0] else None
        work = None
        if dh is not None and ctx.tp_group is not None:
            # column-parallel input grad: all-reduce in flight during the gate|up weight grad
            import torch.distributed as dist

            dh = dh.contiguous()
            work = coll.all_reduce(dh, group=ctx.tp_group, async_op=True)
        accumulate_weight_grad(w_up, du, h2, dyt=dut)
        if work is not None:
            work.wait()
        return ((dh.view(ctx.hshape) if dh is not None else None), None, None, None, None,
                (dy if ctx.has_resid else None))


def swiglu_mlp_ok(h: torch.Tensor, w_up: torch.Tensor, w_down: torch.Tensor) -> bool:
    return (FUSED_MLP and _ext.use_native(h) and h.dtype == torch.bfloat16 and uses_main_grad(w_up)
            and uses_main_grad(w_down) and w_up.shape[0] == 2 * w_down.shape[1]
            and w_down.shape[1] % 64 == 0 and h.numel() // h.shape[-1] % 8 == 0)


def swiglu_mlp(h: torch.Tensor, w_up: torch.Tensor, w_down: torch.Tensor, tp_group=None,
               chunks: int = 1, resid: torch.Tensor = None) -> torch.Tensor:
    """Bias-free SwiGLU MLP with main_grad weight accumulation (see _SwiGLUMLPFn); callers check
    `swiglu_mlp_ok` first. With `tp_group` the node is the whole Megatron TP MLP (input
    replicated, output all-reduced) with its collectives overlapped. With `resid` (no TP) the
    result is resid + MLP(h), the add inside the down GEMM."""
    assert resid is None or tp_group is None
    return _SwiGLUMLPFn.apply(h, w_up, w_down, tp_group, chunks, resid)


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
