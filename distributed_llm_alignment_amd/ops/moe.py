"""Mixture-of-experts ops: top-k router, token dispatch/combine and the grouped expert SwiGLU
(north-star "Mixtral 8x7B DPO with expert-parallel all-to-all").

HF Mixtral's sparse block (transformers/models/mixtral/modeling_mixtral.py) loops over experts
with boolean masks, `index_add_` and a fresh weight-gradient tensor per expert. Here:
  * router: `moe_topk_fwd` (renormalised top-k softmax == softmax over the k selected logits)
    and its analytic backward touching only k logits per token;
  * dispatch / combine: gather kernels over a token-slot -> expert-sorted-row map `pos`
    (deterministic, no atomics); combine's backward also returns the routing-weight grads;
  * experts: the device-driven grouped GEMM (csrc/grouped_gemm.hip): ONE launch per projection
    covers every expert, the per-expert row ranges come from a device offsets array (no host
    sync, no per-expert launch loop, hipGraph-capturable), SwiGLU is fused into the gate|up
    epilogue and the SwiGLU backward into the down projection's input-gradient epilogue, and
    weight gradients accumulate straight into the engine's grad buffer (`main_grad`, bf16 or
    fp32). `DLA_MOE_GEMM=loop|grouped` forces the per-expert hipBLASLt loop (host counts) or the
    grouped GEMM; the default `auto` takes the grouped GEMM everywhere since its counted 4-phase
    K step (round 5): Mixtral expert block fwd+bwd 18.6 vs 20.5 ms on the loop; Mixtral 2-layer
    DPO 60.8-60.9 vs 60.4-60.5 pairs/s (4 x 4 pairs), 67.8 vs 66.4 (16 pairs per micro-batch), fp8
    expert forward with the grouped backward 69.3 vs 67.6-68.0 with the loop backward (same box;
    `profiles/r5_grouped_gemm.md`). `DLA_MOE_GEMM=auto` + `DLA_MOE_BWD=loop` keeps the old fp8
    hybrid (grouped fp8 forward, per-expert loop backward);
  * optional fp8 (e4m3, row-wise scales) forward GEMMs (`fp8=True`) on the block-scaled
    16x16x128 MFMA, bf16 backward.
CPU (and non-bf16) inputs use the PyTorch reference path with identical semantics.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Union

import torch
import torch.nn.functional as F

from . import _ext
from .activations import swiglu
from .linear import _wgrad_accumulate, addmm_into


# ------------------------------------------------------------------------------ router
class _TopKFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, k):
        topv, topi = _ext.require().moe_topk_fwd(logits, int(k))
        ctx.save_for_backward(topv, topi)
        ctx.E = logits.shape[-1]
        ctx.mark_non_differentiable(topi)
        return topv, topi

    @staticmethod
    def backward(ctx, gv, _gi):
        topv, topi = ctx.saved_tensors
        dl = _ext.require().moe_topk_bwd(topv, topi, gv.float().contiguous(), ctx.E)
        return dl, None


def route_topk(logits: torch.Tensor, k: int):
    """logits [N, E] -> (weights fp32 [N, k], expert ids int32 [N, k]); weights are the softmax
    renormalised over the selected experts (Mixtral), descending."""
    if _ext.use_native(logits) and logits.dtype == torch.bfloat16:
        return _TopKFn.apply(logits.contiguous(), k)
    v, i = torch.topk(logits.float(), k, dim=-1)
    return torch.softmax(v, dim=-1), i.to(torch.int32)


def expert_positions(topi: torch.Tensor, num_experts: int):
    """Stable expert-major order of the N*k token slots.
    Returns pos [N, k] int32 (row of slot (t, j) in the expert-sorted matrix) and per-expert
    counts [E] (device)."""
    flat = topi.reshape(-1).long()
    order = torch.argsort(flat, stable=True)
    pos = torch.empty_like(order)
    pos[order] = torch.arange(order.numel(), device=order.device)
    # scatter_add histogram: unlike torch.bincount it never reads the max id on the host
    counts = torch.zeros(num_experts, dtype=torch.long, device=flat.device)
    counts.scatter_add_(0, flat, torch.ones_like(flat))
    return pos.view(topi.shape).to(torch.int32), counts


def expert_offsets(counts: torch.Tensor) -> torch.Tensor:
    """Per-expert counts [E] (device) -> exclusive row offsets [E + 1] int32 (device, no sync)."""
    offs = torch.zeros(counts.numel() + 1, dtype=torch.int32, device=counts.device)
    offs[1:] = torch.cumsum(counts, 0).to(torch.int32)
    return offs


# ------------------------------------------------------------------------------ dispatch
def _ref_dispatch(x, pos):
    k = pos.shape[1]
    xs = x.new_empty((x.shape[0] * k, x.shape[1]))
    return xs.index_copy(0, pos.reshape(-1).long(), x.repeat_interleave(k, dim=0))


def _ref_combine(ys, pos, w):
    g = ys.index_select(0, pos.reshape(-1).long()).view(pos.shape[0], pos.shape[1], -1)
    if w is not None:
        g = g * w.to(g.dtype).unsqueeze(-1)
    return g.sum(1)


class _DispatchFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pos):
        ctx.save_for_backward(pos)
        return _ext.require().moe_dispatch(x, pos)

    @staticmethod
    def backward(ctx, dxs):
        (pos,) = ctx.saved_tensors
        return _ext.require().moe_combine(dxs.contiguous(), pos, None), None


class _CombineFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ys, pos, w, permutation):
        ctx.save_for_backward(ys, pos, w)
        ctx.permutation = permutation
        return _ext.require().moe_combine(ys, pos, w)

    @staticmethod
    def backward(ctx, dout):
        ys, pos, w = ctx.saved_tensors
        dys, dw = _ext.require().moe_combine_bwd(dout.contiguous(), ys, pos, w, ctx.permutation)
        return dys, None, dw, None


def dispatch(x: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
    """x [N, H] -> xs [N*k, H] with xs[pos[t, j]] = x[t]."""
    if _ext.use_native(x) and x.dtype == torch.bfloat16:
        return _DispatchFn.apply(x.contiguous(), pos.contiguous())
    return _ref_dispatch(x, pos)


def combine(ys: torch.Tensor, pos: torch.Tensor, w: Optional[torch.Tensor],
            permutation: bool = False) -> torch.Tensor:
    """out[t] = sum_j w[t, j] * ys[pos[t, j]]. `permutation`: pos maps the N*k slots one-to-one
    onto the rows of ys (dropless dispatch), so the backward need not zero-fill ys' gradient;
    leave it False for capacity buffers (holes, dropped slots)."""
    if _ext.use_native(ys) and ys.dtype == torch.bfloat16:
        return _CombineFn.apply(ys.contiguous(), pos.contiguous(),
                                w.float().contiguous() if w is not None else None, bool(permutation))
    return _ref_combine(ys, pos, w)


# ------------------------------------------------------------------------------ fp8 GEMM
_FP8 = getattr(torch, "float8_e4m3fn", None)
_FP8_MAX = 448.0


def quant_fp8_rows(t: torch.Tensor):
    """Row-wise e4m3: (q [M, K] float8_e4m3fn, inv_scale [M, 1] fp32). Fused HIP kernel on GPU."""
    t = t.contiguous()
    if _ext.use_native(t) and t.dtype == torch.bfloat16 and t.shape[-1] % 8 == 0:
        return _ext.require().quant_fp8_rows(t)
    amax = t.abs().amax(dim=1, keepdim=True).float().clamp(min=1e-12)
    sc = _FP8_MAX / amax
    return (t.float() * sc).clamp(-_FP8_MAX, _FP8_MAX).to(_FP8), 1.0 / sc


def fp8_weight(w: torch.Tensor):
    """Cached row-wise e4m3 copy of a weight [..., N, K] (re-quantised when the weight's version
    counter or its engine's weight epoch moved, i.e. once per optimizer step)."""
    ep = getattr(w, "_dla_epoch", None)
    key = (w._version, ep[0] if ep is not None else 0)
    c = getattr(w, "_dla_fp8", None)
    if c is None or c[0] != key:
        with torch.no_grad():
            q, inv = quant_fp8_rows(w.detach().reshape(-1, w.shape[-1]))
        c = (key, q.view(w.shape), inv.view(*w.shape[:-1], 1))
        w._dla_fp8 = c
    return c[1], c[2]


def fp8_mm(xq, sx, wq, sw) -> torch.Tensor:
    """[M, K] x [N, K]^T with row-wise scales on the gfx950 fp8 MFMA path (hipBLASLt)."""
    return torch._scaled_mm(xq, wq.t(), scale_a=sx, scale_b=sw.t(), out_dtype=torch.bfloat16)


def fp8_linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y = x @ w^T with e4m3 operands and row-wise scales, bf16 output. Forward only."""
    xq, sx = quant_fp8_rows(x)
    wq, sw = quant_fp8_rows(w)
    return fp8_mm(xq, sx, wq, sw)


# ------------------------------------------------------------------------------ experts
class _ExpertsFn(torch.autograd.Function):
    """Grouped SwiGLU experts over the expert-sorted rows. counts is a host list."""

    @staticmethod
    def forward(ctx, xs, w_up, w_down, counts: List[int], fp8: bool):
        M, H = xs.shape
        F2 = w_up.shape[1]
        gu = xs.new_empty((M, F2))
        ys = xs.new_empty((M, H))
        if fp8:
            # e4m3 forward: activations quantised once per GEMM by the fused row-wise kernel,
            # expert weights cached quantised per optimizer step; fp32 accumulate, bf16 out
            wu_q, wu_s = fp8_weight(w_up)
            wd_q, wd_s = fp8_weight(w_down)
            xq, xsc = quant_fp8_rows(xs)
            s = 0
            for e, c in enumerate(counts):
                if c:
                    gu[s:s + c] = fp8_mm(xq[s:s + c], xsc[s:s + c], wu_q[e], wu_s[e])
                s += c
            aq, asc = quant_fp8_rows(swiglu(gu))
            s = 0
            for e, c in enumerate(counts):
                if c:
                    ys[s:s + c] = fp8_mm(aq[s:s + c], asc[s:s + c], wd_q[e], wd_s[e])
                s += c
        else:
            s = 0
            for e, c in enumerate(counts):
                if c:
                    torch.mm(xs[s:s + c], w_up[e].t(), out=gu[s:s + c])
                    torch.mm(swiglu(gu[s:s + c]), w_down[e].t(), out=ys[s:s + c])
                s += c
        ctx.save_for_backward(xs, gu)
        ctx.w_up, ctx.w_down = w_up, w_down  # (on ctx: see ops.linear._LinearMainGradFn)
        ctx.counts = list(counts)
        return ys

    @staticmethod
    def backward(ctx, dys):
        xs, gu = ctx.saved_tensors
        return _loop_experts_backward(dys, xs, gu, ctx.w_up, ctx.w_down, ctx.counts,
                                      ctx.needs_input_grad) + (None, None)


# The per-expert input-gradient GEMMs dA = dY W are NN-layout; hipBLASLt's default heuristic
# (used for these routing-dependent row counts, which no TunableOp table can list) picks a
# depth-32 tile for them. They can run in the forward's TN layout through a transposed expert-weight
# copy made once per optimizer step by the HIP tiled transpose. Mixtral 2-layer DPO, same box, two
# rounds: bf16 60.2-60.6 vs 59.6-59.8 pairs/s, fp8 forward 67.3-67.7 vs 66.9-67.0 (~1 %). The copy
# costs one more copy of the local expert weights (~90 GB per rank for Mixtral-8x7B without EP), so
# it is budgeted: DLA_MOE_TRANSPOSED_DGRAD=auto (default) makes copies only while the total stays
# within the budget below, =1 always, =0 never. `free_transposed_experts` drops the copies.
MOE_TRANSPOSED_DGRAD = os.environ.get("DLA_MOE_TRANSPOSED_DGRAD", "auto").lower()
# Default budget: 8 % of the device's memory (~23 GB on a 288 GB MI355X): the local expert stacks
# of Mixtral-8x7B under EP=8 (~11 GB) or a debug-depth model fit, the 90 GB of all experts on one
# rank do not. DLA_MOE_TDGRAD_BUDGET_GB overrides it.
_TDG_BUDGET_ENV = os.environ.get("DLA_MOE_TDGRAD_BUDGET_GB")
_TDG_FRACTION = 0.08
_TDG_BYTES = [0]  # bytes currently held by transposed copies in this process


def _tdgrad_budget(w: torch.Tensor) -> int:
    if _TDG_BUDGET_ENV is not None:
        return int(float(_TDG_BUDGET_ENV) * 2 ** 30)
    if w.device.type != "cuda":
        return 0
    return int(_TDG_FRACTION * torch.cuda.get_device_properties(w.device).total_memory)


def _tdgrad_allowed(*ws: torch.Tensor) -> bool:
    if MOE_TRANSPOSED_DGRAD in ("0", "off", "false"):
        return False
    if MOE_TRANSPOSED_DGRAD in ("1", "on", "true"):
        return True
    need = sum(w.numel() * w.element_size() for w in ws if getattr(w, "_dla_wT", None) is None)
    return bool(ws) and _TDG_BYTES[0] + need <= _tdgrad_budget(ws[0])


def free_transposed_experts(module) -> int:
    """Drop the cached transposed expert copies of every parameter of `module` (engine teardown,
    re-sharding). Returns the bytes released."""
    freed = 0
    for p in module.parameters():
        c = p.__dict__.pop("_dla_wT", None)
        if c is not None:
            freed += c[1].numel() * c[1].element_size()
    _TDG_BYTES[0] = max(0, _TDG_BYTES[0] - freed)
    return freed


def transposed_experts(w: torch.Tensor) -> torch.Tensor:
    """Cached [E, K, N] copy of expert weights [E, N, K], re-made when the weight's version
    counter or its engine's weight epoch moved (once per optimizer step)."""
    ep = getattr(w, "_dla_epoch", None)
    key = (w._version, ep[0] if ep is not None else 0)
    c = getattr(w, "_dla_wT", None)
    if c is None or c[0] != key:
        with torch.no_grad():
            if c is not None:
                t = c[1]
            else:
                t = torch.empty((w.shape[0], w.shape[2], w.shape[1]), dtype=w.dtype, device=w.device)
                _TDG_BYTES[0] += t.numel() * t.element_size()
            tr = _ext.require().transpose_bf16
            for e in range(w.shape[0]):
                tr(w.detach()[e], t[e])
        c = (key, t)
        w._dla_wT = c
    return c[1]


def _loop_experts_backward(dys, xs, gu, w_up, w_down, counts, needs):
    """Per-expert hipBLASLt backward of the SwiGLU experts (host counts): (dxs, d_up, d_down),
    weight grads accumulated into main_grad where the engine attached one."""
    dys = dys.contiguous()
    # only for weights whose updates the flat-buffer engine announces through its weight epoch
    # (in-place kernel updates move no version counter; FSDP re-gathers storage): as ops.linear
    tdg = (_ext.use_native(dys) and w_up.dtype == torch.bfloat16
           and getattr(w_up, "_dla_epoch", None) is not None
           and getattr(w_down, "_dla_epoch", None) is not None
           and w_up.shape[1] % 8 == 0 and w_up.shape[2] % 8 == 0
           and _tdgrad_allowed(w_down, *((w_up,) if needs[0] else ())))
    wdT = transposed_experts(w_down) if tdg else None  # [E, F, H]
    wuT = transposed_experts(w_up) if tdg and needs[0] else None  # [E, H, 2F]
    need_x = needs[0]
    dxs = torch.zeros_like(xs) if need_x else None
    mg_up = getattr(w_up, "main_grad", None)
    mg_down = getattr(w_down, "main_grad", None)
    g_up = mg_up if mg_up is not None else (torch.zeros_like(w_up) if needs[1] else None)
    g_down = mg_down if mg_down is not None else (torch.zeros_like(w_down) if needs[2] else None)
    s = 0
    for e, c in enumerate(counts):
        if c:
            dy = dys[s:s + c]
            g = gu[s:s + c]
            a = swiglu(g)
            da = F.linear(dy, wdT[e]) if tdg else dy @ w_down[e]
            if g_down is not None:
                addmm_into(g_down[e], dy.t(), a)
            dg = _swiglu_bwd(g, da)
            if need_x:
                torch.mm(dg, wuT[e].t() if tdg else w_up[e], out=dxs[s:s + c])
            if g_up is not None:
                addmm_into(g_up[e], dg.t(), xs[s:s + c])
        s += c
    outs = []
    for w, g, mg in ((w_up, g_up, mg_up), (w_down, g_down, mg_down)):
        if mg is not None:
            hook = getattr(w, "_dla_grad_hook", None)
            if hook is not None:
                hook(w)
            outs.append(None)
        else:
            outs.append(g)
    return dxs, outs[0], outs[1]


# One local expert (EP with E / ep = 1, e.g. Mixtral at ep 8): the group is the whole padded
# capacity buffer, so the down projection forward and the gate|up input gradient run as plain
# hipBLASLt GEMMs over its static row count (row-independent: the unwritten padding rows only
# produce output rows nobody reads, and the input gradient's are zeroed below). Measured in the
# Mixtral --ep-shape 8 step: the grouped kernel ran those two at 670 / 534 TFLOP/s at 4096 rows
# per call (one 256-row tile per CU over a 14336- / 28672-deep K). DLA_MOE_SINGLE_LIB=0: grouped.
MOE_SINGLE_LIB = os.environ.get("DLA_MOE_SINGLE_LIB", "1") != "0"


def _expert0_t(w: torch.Tensor) -> torch.Tensor:
    """Cached transposed copy of expert 0's weight w[0] ([N, K] -> [K, N]), refreshed when the
    weight's version counter or its engine's weight epoch moved."""
    ep = getattr(w, "_dla_epoch", None)
    key = (w._version, ep[0] if ep is not None else 0)
    c = getattr(w, "_dla_wt0", None)
    if c is None or c[0] != key:
        with torch.no_grad():
            t = c[1] if c is not None else torch.empty((w.shape[2], w.shape[1]), dtype=w.dtype, device=w.device)
            _ext.require().transpose_bf16(w.detach()[0], t)
        c = (key, t)
        w._dla_wt0 = c
    return c[1]


def _single_lib(offs: torch.Tensor, w: torch.Tensor, rows: int) -> bool:
    return (MOE_SINGLE_LIB and offs.numel() == 2 and w.shape[0] == 1 and w.dtype == torch.bfloat16
            and rows >= 256)


# Single local expert, main + overflow rows: the capacity buffer holds ep * C = cf * n * k rows, of
# which a balanced routing fills the first n * k (the expected load). The library GEMMs run over
# those `main` rows only; the rows past them (filled only when this rank's expert draws more than
# its share) run on the device-driven grouped kernels with offsets shifted by `main`, which exit
# at once when that overflow is empty. No host sync either way. DLA_MOE_MAIN_ROWS=0: the library
# GEMMs cover the whole buffer (every padding row computed).
MOE_MAIN_ROWS = os.environ.get("DLA_MOE_MAIN_ROWS", "1") != "0"


def _row_pieces(main: int, base: int):
    """Row ranges of the library GEMMs over [0, main): the expected rows [0, base) as one GEMM
    (the tuned shape) and any load-adaptive extension [base, main) as a second one -- one GEMM over
    an untuned row count (4608 at capacity 1.125) drew a hipBLASLt heuristic kernel 3x slower per
    row than the tuned 4096-row one (profiles/r6_mixtral.md)."""
    if 0 < base < main:
        return [(0, base), (base, main)]
    return [(0, main)]


def _tail_offs(offs: torch.Tensor, main: int) -> torch.Tensor:
    """Offsets of the rows past `main` (single group): [0, max(offs[-1] - main, 0)], on device."""
    return torch.clamp(offs - main, min=0).to(torch.int32)


# Capacity-buffer padding rows (past offs[-1]) zeroed in place on the node's own outputs instead of
# by out-of-place masked_fills (a clone + fill of the [rows, H] buffer each way; Mixtral EP shape:
# ~70 ms per step). DLA_MOE_TAIL_INPLACE=0 restores the masked_fills for A/B.
_TAIL_INPLACE = os.environ.get("DLA_MOE_TAIL_INPLACE", "1") != "0"


class _GroupedExpertsFn(torch.autograd.Function):
    """Grouped SwiGLU experts on the device-driven grouped GEMM; offs [E+1] int32 on device.
    `sync_free`: the backward also stays on the grouped kernels (never reads offs on the host)."""

    @staticmethod
    def forward(ctx, xs, w_up, w_down, offs, fp8: bool, sync_free: bool = False, main_rows: int = 0,
                base_rows: int = 0):
        C = _ext.require()
        rows = xs.shape[0]
        main = main_rows if (MOE_MAIN_ROWS and 0 < main_rows < rows) else rows
        base = base_rows if MOE_MAIN_ROWS else 0
        if fp8:
            wu_q, wu_s = fp8_weight(w_up)
            wd_q, wd_s = fp8_weight(w_down)
            xq, xsc = quant_fp8_rows(xs)
            gu, a = C.gg_fwd_swiglu(xq, wu_q, offs, xsc, wu_s)
            aq, asc = quant_fp8_rows(a)
            ys = C.gg_fwd(aq, wd_q, offs, asc, wd_s)
        else:
            gu, a = C.gg_fwd_swiglu(xs, w_up, offs, None, None)
            if _single_lib(offs, w_down, a.shape[0]) and (main < rows or 0 < base < main):
                ys = torch.empty((rows, w_down.shape[1]), dtype=a.dtype, device=a.device)
                for lo, hi in _row_pieces(main, base):
                    torch.matmul(a[lo:hi], w_down.detach()[0].t(), out=ys[lo:hi])
                if main < rows:
                    ys[main:].copy_(C.gg_fwd(a[main:], w_down, _tail_offs(offs, main), None, None))
            elif _single_lib(offs, w_down, a.shape[0]):
                ys = F.linear(a, w_down.detach()[0])
            else:
                ys = C.gg_fwd(a, w_down, offs, None, None)
        if sync_free and ys.shape[0] > 0 and _TAIL_INPLACE:
            # capacity buffer (experts_swiglu_offsets): rows past offs[-1] are zero, in place on
            # the fresh output (an out-of-place masked_fill cost a clone + fill per call)
            C.zero_rows_from(ys, offs[-1:])
        ctx.save_for_backward(xs, gu, offs)
        ctx.w_up, ctx.w_down = w_up, w_down  # (on ctx: see ops.linear._LinearMainGradFn)
        ctx.sync_free = sync_free
        ctx.main, ctx.base = main, base
        return ys

    @staticmethod
    def backward(ctx, dys):
        xs, gu, offs = ctx.saved_tensors
        w_up, w_down = ctx.w_up, ctx.w_down
        if not ctx.sync_free and _loop_backward_ok():
            # fp8 forward on the grouped kernel, bf16 backward on the per-expert hipBLASLt loop
            # (faster there; one host read of the offsets, outside any capture)
            o = offs.tolist()
            counts = [o[e + 1] - o[e] for e in range(len(o) - 1)]
            return _loop_experts_backward(dys, xs, gu, w_up, w_down, counts,
                                          ctx.needs_input_grad) + (None, None)
        C = _ext.require()
        dys = dys.contiguous()
        # da = dy . W_down fused with the SwiGLU backward -> dgu, plus the recomputed a
        dgu, a = C.gg_dgrad_swiglu(dys, w_down, offs, gu)
        single = _single_lib(offs, w_up, dgu.shape[0])
        if single:
            # the weight gradients reduce over the rows: the padding rows the grouped kernel left
            # unwritten must be zero (xs's and dys's already are)
            C.zero_rows_from(dgu, offs[1:])
            C.zero_rows_from(a, offs[1:])
        rows, main = dgu.shape[0], min(ctx.main, dgu.shape[0])
        offs_t = _tail_offs(offs, main) if single and main < rows else None
        outs = []
        for w, dy, x, need in ((w_up, dgu, xs, ctx.needs_input_grad[1]),
                               (w_down, dys, a, ctx.needs_input_grad[2])):
            mg = getattr(w, "main_grad", None)
            if single and mg is not None and mg.is_contiguous() and mg.dtype in (torch.bfloat16, torch.float32):
                if offs_t is not None:  # main rows on the library, overflow rows on the grouped kernel
                    _wgrad_accumulate(mg[0], dy[:main], x[:main])
                    C.gg_wgrad(dy[main:].contiguous(), x[main:].contiguous(), offs_t, mg, True)
                else:
                    _wgrad_accumulate(mg[0], dy, x)
                hook = getattr(w, "_dla_grad_hook", None)
                if hook is not None:
                    hook(w)
                outs.append(None)
            elif mg is not None and mg.is_contiguous() and mg.dtype in (torch.bfloat16, torch.float32):
                C.gg_wgrad(dy, x, offs, mg, True)
                hook = getattr(w, "_dla_grad_hook", None)
                if hook is not None:
                    hook(w)
                outs.append(None)
            elif need:
                gw = torch.empty_like(w)
                C.gg_wgrad(dy, x, offs, gw, False)
                outs.append(gw)
            else:
                outs.append(None)
        dxs = None
        if ctx.needs_input_grad[0]:
            if _single_lib(offs, w_up, dgu.shape[0]) and (offs_t is not None or 0 < ctx.base < main):
                dxs = torch.empty((rows, w_up.shape[2]), dtype=dgu.dtype, device=dgu.device)
                wt = _expert0_t(w_up)
                for lo, hi in _row_pieces(main, ctx.base):
                    torch.matmul(dgu[lo:hi], wt.t(), out=dxs[lo:hi])  # as F.linear below
                if offs_t is not None:
                    tail = C.gg_dgrad(dgu[main:], w_up, offs_t)
                    C.zero_rows_from(tail, offs_t[-1:])  # overflow rows the grouped kernel left unwritten
                    dxs[main:].copy_(tail)
            elif _single_lib(offs, w_up, dgu.shape[0]):
                dxs = F.linear(dgu, _expert0_t(w_up))  # dgu [M, 2F] . W_up[0] [2F, H], TN layout
            else:
                dxs = C.gg_dgrad(dgu, w_up, offs)
        if dxs is not None and dxs.shape[0] > 0 and not _TAIL_INPLACE:
            tail = torch.arange(dxs.shape[0], device=dxs.device) >= offs[-1].long()
            dxs = dxs.masked_fill(tail.unsqueeze(-1), 0)
        elif dxs is not None and dxs.shape[0] > 0 and not single:
            # rows past offs[-1] (padding of a capacity buffer) are never written by the grouped
            # kernel (single: dgu's padding rows are zero, so dxs's are too)
            C.zero_rows_from(dxs, offs[-1:])
        return dxs, outs[0], outs[1], None, None, None, None, None


def grouped_gemm_enabled() -> bool:
    """The grouped GEMM may be used (the condition for a host-sync-free, capturable MoE layer)."""
    return os.environ.get("DLA_MOE_GEMM", "auto") != "loop"


def _loop_backward_ok() -> bool:
    """DLA_MOE_BWD=loop (with DLA_MOE_GEMM=auto): the grouped node's backward runs the
    per-expert hipBLASLt loop instead of the grouped dgrad / wgrad kernels (the default)."""
    return (os.environ.get("DLA_MOE_GEMM", "auto") == "auto" and os.environ.get("DLA_MOE_BWD", "auto") == "loop"
            and not torch.cuda.is_current_stream_capturing())


def _use_grouped(fp8: bool, rows: int = 0) -> bool:
    """auto and grouped: the grouped GEMM (faster than the per-expert loop at every measured
    size since the counted 4-phase schedule, and host-sync free); loop: the per-expert loop."""
    return os.environ.get("DLA_MOE_GEMM", "auto") != "loop"


def _grouped_ok(xs, w_up, w_down) -> bool:
    F2, H = w_up.shape[1], w_up.shape[2]
    return (_ext.use_native(xs) and xs.dtype == torch.bfloat16
            and w_up.dtype == torch.bfloat16 and (F2 // 2) % 128 == 0 and H % 16 == 0
            and w_down.shape[1] == H and w_down.shape[2] == F2 // 2)


def _swiglu_bwd(gu, dout):
    if _ext.use_native(gu) and gu.dtype == torch.bfloat16:
        return _ext.require().swiglu_bwd(gu.contiguous(), dout.contiguous())
    with torch.enable_grad():
        g = gu.detach().requires_grad_(True)
        y = swiglu(g)
        (dg,) = torch.autograd.grad(y, g, dout)
    return dg


def experts_swiglu(xs: torch.Tensor, w_up: torch.Tensor, w_down: torch.Tensor,
                   counts: Union[torch.Tensor, Sequence[int]], fp8: bool = False) -> torch.Tensor:
    """xs [M, H] expert-sorted rows, w_up [E, 2F, H] ([gate; up]), w_down [E, H, F].
    counts: per-expert row counts, a device tensor (grouped GEMM path: never read on the host)
    or a host sequence."""
    if fp8 and not (xs.is_cuda and _FP8 is not None):
        fp8 = False
    xs = xs.contiguous()
    if _grouped_ok(xs, w_up, w_down) and _use_grouped(fp8, xs.shape[0]):
        if isinstance(counts, torch.Tensor):
            offs = expert_offsets(counts.to(xs.device))
        else:
            offs = expert_offsets(torch.tensor(list(counts), device=xs.device))
        return _GroupedExpertsFn.apply(xs, w_up, w_down, offs, bool(fp8))
    if isinstance(counts, torch.Tensor):
        counts = counts.tolist()  # host sync: per-expert loop path only
    return _ExpertsFn.apply(xs, w_up, w_down, [int(c) for c in counts], bool(fp8))


def _ref_grouped_experts(xs, w_up, w_down, offs):
    """Static-shape reference of the grouped experts for a device offsets array (no host read):
    every expert runs over all rows and keeps its [offs[e], offs[e+1]) range; rows past offs[-1]
    are zero. CPU / non-native path of `experts_swiglu_offsets`."""
    rows = torch.arange(xs.shape[0], device=xs.device).view(-1, 1)
    o = offs.to(xs.device).long()
    out = xs.new_zeros((xs.shape[0], w_down.shape[1]))
    for e in range(w_up.shape[0]):
        y = F.linear(swiglu(F.linear(xs, w_up[e])), w_down[e])
        out = torch.where((rows >= o[e]) & (rows < o[e + 1]), y, out)
    return out


def experts_swiglu_offsets(xs: torch.Tensor, w_up: torch.Tensor, w_down: torch.Tensor,
                           offs: torch.Tensor, fp8: bool = False, main_rows: int = 0,
                           base_rows: int = 0) -> torch.Tensor:
    """Grouped experts over rows whose per-expert ranges are given ONLY as a device offsets array
    offs [E+1] (rows past offs[-1] are padding: ignored, zero output and gradient). Never reads
    the offsets on the host, forward or backward: the sync-free expert-parallel path.
    `main_rows`: the library rows of a single local expert's buffer (see MOE_MAIN_ROWS); `base_rows`
    (<= main_rows) its expected fill, run as a GEMM of its own when main_rows extends past it."""
    xs = xs.contiguous()
    if _grouped_ok(xs, w_up, w_down):
        if fp8 and _FP8 is None:
            fp8 = False
        # rows past offs[-1] come back zero (zeroed in place inside the node)
        ys = _GroupedExpertsFn.apply(xs, w_up, w_down, offs.to(torch.int32), bool(fp8), True, int(main_rows),
                                     int(base_rows))
        if not _TAIL_INPLACE:
            tail = torch.arange(ys.shape[0], device=ys.device) >= offs[-1].long()
            ys = ys.masked_fill(tail.unsqueeze(-1), 0)
        return ys
    return _ref_grouped_experts(xs, w_up, w_down, offs)


def ref_moe(h2, router, w_up, w_down, k):
    """Plain PyTorch fp32 Mixtral block (HF semantics: the router GEMM runs in the model dtype,
    softmax / top-k / expert math in fp32) for tests."""
    logits = F.linear(h2, router).float()
    probs = torch.softmax(logits, dim=-1)
    topv, topi = torch.topk(probs, k, dim=-1)
    topv = topv / topv.sum(-1, keepdim=True)
    out = torch.zeros_like(h2, dtype=torch.float32)
    for j in range(k):
        for e in range(w_up.shape[0]):
            m = topi[:, j] == e
            if m.any():
                x = h2[m].float()
                gu = x @ w_up[e].float().t()
                Fd = gu.shape[-1] // 2
                a = F.silu(gu[:, :Fd]) * gu[:, Fd:]
                out[m] += topv[m, j:j + 1] * (a @ w_down[e].float().t())
    return out
