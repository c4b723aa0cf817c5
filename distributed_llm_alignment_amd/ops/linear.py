"""Linear layer whose weight gradient is accumulated straight into the flat fp32/bf16 grad
buffer by the GEMM itself (C = A^T B + C, beta = 1; bf16 operands, bf16 or fp32 C).

Eager autograd computes each weight gradient into a fresh tensor and then launches a separate
elementwise add into `.grad` on every micro-batch (≈1.5 % of a Llama-3-8B DPO step on MI355X,
measured: profiles/r1_baseline_kernel_stats.md). When the training engine has attached
`param.main_grad` (a view of its flat gradient buffer) this op instead issues
`main_grad.addmm_(dY^T, X)` — hipBLASLt folds the accumulation into the GEMM epilogue, no
temporary, one rounding — and notifies the engine's bucket scheduler itself.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _ext

# dX = dY @ W in the NN layout runs at 1.22-1.36 PF/s on gfx950 for Llama-3-8B shapes, the TN
# layout of the forward at 1.43-1.52 (tools/gemm_layout_probe.py, MI355X). The engine marks its
# 2-D weights `_dla_wt_ok`; the backward then keeps a transposed copy W^T (HIP tiled transpose,
# refreshed lazily when the weight's version counter or the engine's weight epoch moved, i.e.
# once per optimizer step) and
# computes dX = linear(dY, W^T). 16 GB of HBM for an 8B policy buys ~8 % of the step.
TRANSPOSED_DGRAD = os.environ.get("DLA_TRANSPOSED_DGRAD", "1") != "0"


def transposed_weight(weight: torch.Tensor) -> torch.Tensor:
    wt = getattr(weight, "_dla_wt", None)
    ep = getattr(weight, "_dla_epoch", None)
    key = (weight._version, ep[0] if ep is not None else 0)
    if wt is None or getattr(weight, "_dla_wt_ver", None) != key:
        with torch.no_grad():
            if wt is None:
                wt = torch.empty((weight.shape[1], weight.shape[0]), dtype=weight.dtype, device=weight.device)
            _ext.require().transpose_bf16(weight.detach(), wt)
        weight._dla_wt = wt
        weight._dla_wt_ver = key
    return wt


def input_grad(dy2: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """dX = dy2 @ weight ([M, N] x [N, K]); TN layout through the cached W^T when enabled."""
    if (TRANSPOSED_DGRAD and getattr(weight, "_dla_wt_ok", False) and weight.dtype == torch.bfloat16
            and _ext.use_native(weight) and weight.shape[0] % 8 == 0 and weight.shape[1] % 8 == 0):
        return F.linear(dy2, transposed_weight(weight))
    return dy2 @ weight


# Weight gradient dW += dY^T X reduces over the token dim, which is the slow dim of both
# operands (NT layout). For the large FFN weights it is faster to transpose both activations
# with the HIP tiled transpose and run the TN GEMM: Llama-3-8B up 1.66 -> 1.22 + 0.24 ms,
# down 0.95 -> 0.68 + 0.14 ms; no gain for qkv / o (one-off layout probe, MI355X).
TN_WGRAD = os.environ.get("DLA_TN_WGRAD", "1") != "0"
# lower bound: a small weight (the MoE router, [E, H]) is not worth transposing its [tokens, H]
# input for (Mixtral EP shape: 15 ms per step of [4096, 4096] transposes for an [8, 4096] gradient)
TN_WGRAD_MIN_ELEMS = int(float(os.environ.get("DLA_TN_WGRAD_MIN", str(1 << 20))))
# upper bound (A/B knob): the LM head's dY is the [tokens, vocab] logit gradient, whose transpose
# alone moves 2 x 2.1 GB per micro-batch at Llama-3 vocab
TN_WGRAD_MAX_ELEMS = int(os.environ.get("DLA_TN_WGRAD_MAX", str(1 << 62)))


def _tn_ok(mg: torch.Tensor, M: int) -> bool:
    N, K = mg.shape
    return (TN_WGRAD and TN_WGRAD_MIN_ELEMS <= N * K <= TN_WGRAD_MAX_ELEMS and mg.dtype in (torch.bfloat16, torch.float32)
            and _ext.use_native(mg) and M % 8 == 0 and N % 8 == 0 and K % 8 == 0)


_F32_ADDMM = {"ok": None}


def addmm_into(mg: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> None:
    """mg += a @ b with one rounding. bf16 operands into an fp32 main-grad buffer run as ONE
    hipBLASLt GEMM with a bf16 x bf16 -> fp32 C (beta = 1) epilogue: the accumulation over
    micro-batches happens in fp32 and no bf16 temporary exists."""
    if mg.dtype == a.dtype:
        mg.addmm_(a, b)
        return
    if mg.is_cuda and _F32_ADDMM["ok"] is not False:
        try:
            torch.addmm(mg, a, b, out_dtype=mg.dtype, out=mg)
            _F32_ADDMM["ok"] = True
            return
        except (RuntimeError, TypeError):
            _F32_ADDMM["ok"] = False
    mg.add_(a.to(mg.dtype) @ b.to(mg.dtype))


def _wgrad_accumulate(mg: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor,
                      dyt: torch.Tensor = None, xt: torch.Tensor = None) -> None:
    """mg += dy2^T x2. `dyt` / `xt` are optional already-transposed operands ([N, M] / [K, M]),
    e.g. written by a producer kernel as a second output (ops.activations.swiglu_mlp)."""
    N, K = mg.shape
    M = dy2.shape[0]
    if _tn_ok(mg, M) and (dyt is not None or dy2.is_contiguous()) and (xt is not None or x2.is_contiguous()):
        tr = _ext.require().transpose_bf16
        if dyt is None:
            dyt = torch.empty((N, M), dtype=dy2.dtype, device=dy2.device)
            tr(dy2, dyt)
        if xt is None:
            xt = torch.empty((K, M), dtype=x2.dtype, device=x2.device)
            tr(x2, xt)
        addmm_into(mg, dyt, xt.t())
        return
    addmm_into(mg, dy2.t(), x2)


def accumulate_weight_grad(weight: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor,
                           dyt: torch.Tensor = None, xt: torch.Tensor = None) -> bool:
    """main_grad += dy2^T @ x2 if the engine attached a main_grad; returns True if handled."""
    mg = getattr(weight, "main_grad", None)
    if mg is None or getattr(weight, "_dla_shared", False):
        return False
    _wgrad_accumulate(mg, dy2, x2, dyt, xt)
    hook = getattr(weight, "_dla_grad_hook", None)
    if hook is not None:
        hook(weight)
    return True


def uses_main_grad(weight: torch.Tensor) -> bool:
    return (weight.requires_grad and torch.is_grad_enabled() and getattr(weight, "main_grad", None) is not None
            and not getattr(weight, "_dla_shared", False))


class _LinearMainGradFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        # weights ride on ctx, not save_for_backward: under activation recompute
        # (torch.utils.checkpoint) saved tensors come back as detached aliases without the
        # engine's attributes (main_grad, the cached W^T), and the grads would be lost
        ctx.save_for_backward(x)
        ctx.weight = weight
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        weight = ctx.weight
        K, N = x.shape[-1], dy.shape[-1]
        dy2 = dy.reshape(-1, N)
        dx = input_grad(dy2, weight).view(x.shape) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, K)
            if not accumulate_weight_grad(weight, dy2, x2):
                dw = dy2.t() @ x2
        db = dy2.sum(0) if (ctx.has_bias and ctx.needs_input_grad[2]) else None
        return dx, dw, db


# ---------------------------------------------------------------------------------------------
# fp8 inference GEMMs for a FROZEN model (opt-in, `enable_fp8_inference`): e4m3 weights with
# per-output-row scales (quantised once: the cache key is the weight's version) and e4m3
# activations with per-row scales (one fused HIP pass, ops.moe.quant_fp8_rows), on hipBLASLt's fp8
# MFMA path (torch._scaled_mm): 2.3-2.8 PF/s vs 1.2-1.6 bf16 at the Llama-3-8B DPO shapes
# (round-5 one-off probe, since removed). Only without autograd and for >= 256 rows; the LM head, embeddings
# and norms stay bf16. Use: the DPO reference model (`dpo.reference_fp8`, `bench.py --ref-fp8`).
def fp8_inference_ok(x: torch.Tensor, weight: torch.Tensor, bias) -> bool:
    return (bias is None and getattr(weight, "_dla_fp8_infer", False) and not torch.is_grad_enabled()
            and x.is_cuda and x.dtype == torch.bfloat16 and weight.dim() == 2
            and x.numel() // max(x.shape[-1], 1) >= 256 and x.shape[-1] % 16 == 0 and weight.shape[0] % 16 == 0)


def fp8_linear_frozen(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    from .moe import fp8_mm, fp8_weight, quant_fp8_rows

    x2 = x.reshape(-1, x.shape[-1])
    xq, sx = quant_fp8_rows(x2)
    wq, sw = fp8_weight(weight)
    return fp8_mm(xq, sx, wq, sw).view(*x.shape[:-1], weight.shape[0])


def enable_fp8_inference(model, enabled: bool = True) -> int:
    """Mark the transformer-layer projection weights (qkv, o, gate|up, down) of a frozen model for
    the fp8 inference GEMMs; returns the number of weights marked. MoE experts keep their own fp8
    path (`moe.fp8`)."""
    n = 0
    for layer in getattr(model, "layers", []):
        at, mlp = getattr(layer, "attn", None), getattr(layer, "mlp", None)
        for w in (getattr(at, "qkv_proj", None), getattr(at, "o_proj", None),
                  getattr(mlp, "up_proj", None), getattr(mlp, "down_proj", None)):
            if isinstance(w, torch.Tensor) and w.dim() == 2:
                w._dla_fp8_infer = bool(enabled)
                if not enabled:
                    w.__dict__.pop("_dla_fp8", None)
                n += 1
    return n


class fp8_inference_scope:
    """Context manager: the layer projections of `model` run the fp8 inference GEMMs inside the
    block (no-grad calls of >= 256 rows only, as `enable_fp8_inference`), then the previous
    marking is restored. For a trainable policy's rollout prefill under fp8 rollouts
    (models.generation.generate(weight_dtype="fp8")): sampling-only, the update recomputes every
    log-prob in bf16."""

    def __init__(self, model, enabled: bool = True):
        self.model, self.enabled, self.prev = model, bool(enabled), []

    def __enter__(self):
        if self.enabled:
            for layer in getattr(self.model, "layers", []):
                at, mlp = getattr(layer, "attn", None), getattr(layer, "mlp", None)
                for w in (getattr(at, "qkv_proj", None), getattr(at, "o_proj", None),
                          getattr(mlp, "up_proj", None), getattr(mlp, "down_proj", None)):
                    if isinstance(w, torch.Tensor) and w.dim() == 2:
                        self.prev.append((w, getattr(w, "_dla_fp8_infer", None)))
                        w._dla_fp8_infer = True
        return self

    def __exit__(self, *exc):
        for w, v in self.prev:
            if v is None:
                w.__dict__.pop("_dla_fp8_infer", None)
            else:
                w._dla_fp8_infer = v
            if not v:
                # the e4m3 copy quantised for this scope (ops.moe.fp8_weight) would otherwise stay
                # resident on a trainable policy between rollouts (and be re-quantised after every
                # optimizer step anyway); a frozen model marked by enable_fp8_inference keeps it
                w.__dict__.pop("_dla_fp8", None)
        self.prev = []
        return False


def add_gemm(x2: torch.Tensor, weight: torch.Tensor, c2: torch.Tensor) -> torch.Tensor:
    """c2 + x2 @ weight^T ([M, K], [N, K], [M, N]) as ONE GEMM that reads c2 as its C input and
    writes a fresh D: hipBLASLt with C != D on the GPU (csrc/gemm_lt.cpp; torch.addmm would copy
    c2 into the output first), torch.addmm elsewhere."""
    if (x2.is_cuda and x2.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and c2.dtype == torch.bfloat16
            and x2.stride(-1) == 1 and weight.stride(-1) == 1 and c2.stride(-1) == 1):
        from ..utils.tuning import hipblaslt_solution

        sol = hipblaslt_solution(weight.shape[0], x2.shape[0], x2.shape[1], weight.stride(0), x2.stride(0),
                                 weight.shape[0])
        return _ext.require().linear_add_lt(x2, weight, c2, sol)
    return torch.addmm(c2, x2, weight.t())


class _LinearAddFn(torch.autograd.Function):
    """resid + x @ W^T as ONE hipBLASLt GEMM (the residual is the C input, beta = 1, C != D): the
    decoder's o / down projections add their output onto the residual stream in the epilogue,
    so the following RMSNorm reads one tensor and writes one instead of reading two and writing
    two. Backward: d(resid) = dy, the rest as _LinearMainGradFn (main_grad accumulation when the
    engine attached one, a plain .grad otherwise: the custom op has no autograd kernel of its
    own, so every differentiable call must come through here)."""

    @staticmethod
    def forward(ctx, x, weight, resid):
        ctx.save_for_backward(x)
        ctx.weight = weight  # (on ctx: see _LinearMainGradFn)
        N = weight.shape[0]
        y = add_gemm(x.reshape(-1, x.shape[-1]), weight, resid.reshape(-1, N))
        return y.view(resid.shape)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        weight = ctx.weight
        K, N = x.shape[-1], dy.shape[-1]
        dy2 = dy.reshape(-1, N)
        dx = input_grad(dy2, weight).view(x.shape) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, K)
            if not accumulate_weight_grad(weight, dy2, x2):
                dw = dy2.t() @ x2
        return dx, dw, (dy if ctx.needs_input_grad[2] else None)


def linear_add(x: torch.Tensor, weight: torch.Tensor, resid: torch.Tensor) -> torch.Tensor:
    """resid + linear(x, weight), the add inside the GEMM (bias-free projections)."""
    if fp8_inference_ok(x, weight, None):
        return fp8_linear_frozen(x, weight).add_(resid)
    if torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad or resid.requires_grad):
        return _LinearAddFn.apply(x, weight, resid)
    N = weight.shape[0]
    return add_gemm(x.reshape(-1, x.shape[-1]), weight, resid.reshape(-1, N)).view(resid.shape)


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None) -> torch.Tensor:
    # (fp8 inference first: it needs grad disabled, so a training forward never takes it; a
    # trainable policy's no-grad rollout prefill inside fp8_inference_scope does)
    if fp8_inference_ok(x, weight, bias):
        return fp8_linear_frozen(x, weight)
    if uses_main_grad(weight):
        return _LinearMainGradFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)
