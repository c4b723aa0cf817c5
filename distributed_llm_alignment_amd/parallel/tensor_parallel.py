"""Tensor parallelism (Megatron-style) over an RCCL TP group.

Sharding applied in place to a built `CausalLM` (identical seeded init on every rank, so each
rank just keeps its slice — no broadcast):
  * attention: heads split across ranks; fused qkv_proj rows -> [q_r; k_r; v_r] (column
    parallel), o_proj columns (row parallel; bias added once after the all-reduce);
  * MLP: fused gate|up rows -> [gate_r; up_r] (column parallel), down_proj columns (row parallel);
  * embedding + LM head: vocabulary-parallel (rows [r*V/tp, (r+1)*V/tp)); the log-prob is the
    fused HIP logprob kernel per shard + an all-reduce of (max-lse, sum-exp, target logit) —
    full [N, V] logits never exist on any rank; the backward uses the global lse;
  * norms / residual stream replicated, or (sequence_parallel=True, Megatron-SP) sharded over
    the flattened token dim between the TP regions.
Communication per layer: forward 2 all-reduces of [B*T, H] (after o_proj and down_proj),
backward 2 (input grads of the column-parallel GEMMs). On 8 x MI355X the TP group is all-to-all
connected by xGMI, so RCCL's all-reduce uses every link.

Sequence parallel (hardware.tp_sequence_parallel): every all-reduce becomes a reduce-scatter
(after the row-parallel GEMM, into this rank's 1/tp of the tokens) plus an all-gather (before
the next column-parallel GEMM) — the same bytes on the ring, but the norms, residual adds and the
activations kept for backward are 1/tp per rank (70B at T=8k, TP=8: 8x less residual-stream
memory and norm work), and the gather/scatter pair is split so the layer's norm runs between
them. Weights applied to the sharded stream (norm weights, post-reduce biases, wpe) get partial
grads per rank; `tp_grad_sum` all-reduces those over the TP group in backward.
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F

from ..ops import _ext
from . import collectives as coll


# ------------------------------------------------------------------------------ primitives
class _CopyToTP(torch.autograd.Function):
    """identity forward; all-reduce of the input gradient backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        coll.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromTP(torch.autograd.Function):
    """all-reduce forward (sum of partial products); identity backward."""

    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous()
        coll.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


def tp_copy(x, group):
    return _CopyToTP.apply(x, group)


# ------------------------------------------------------------ Megatron sequence parallelism
class TPSeq:
    """Sequence-parallel state of one TP group: the residual stream between the TP regions is
    [N/tp, H] (rows r*N/tp .. of the flattened B*T tokens)."""

    def __init__(self, group):
        self.group = group
        self.tp = coll.world_size(group)
        self.rank = coll.rank(group)

    def local(self, full: torch.Tensor) -> torch.Tensor:
        n = full.shape[0] // self.tp
        return full[self.rank * n:(self.rank + 1) * n]


class _SPGather(torch.autograd.Function):
    """[n, H] local tokens -> [N, H] all tokens; backward: reduce-scatter (partial input grads of
    the column-parallel GEMM summed over TP, this rank's tokens kept)."""

    @staticmethod
    def forward(ctx, x, seq):
        ctx.seq = seq
        out = x.new_empty((x.shape[0] * seq.tp,) + tuple(x.shape[1:]))
        coll.all_gather_into_tensor(out, x.contiguous(), group=seq.group)
        return out

    @staticmethod
    def backward(ctx, g):
        seq = ctx.seq
        out = g.new_empty((g.shape[0] // seq.tp,) + tuple(g.shape[1:]))
        coll.reduce_scatter_tensor(out, g.contiguous(), group=seq.group)
        return out, None


class _SPReduceScatter(torch.autograd.Function):
    """[N, H] partial sums (row-parallel GEMM output) -> [n, H] summed local tokens; backward:
    all-gather."""

    @staticmethod
    def forward(ctx, x, seq):
        ctx.seq = seq
        out = x.new_empty((x.shape[0] // seq.tp,) + tuple(x.shape[1:]))
        coll.reduce_scatter_tensor(out, x.contiguous(), group=seq.group)
        return out

    @staticmethod
    def backward(ctx, g):
        seq = ctx.seq
        out = g.new_empty((g.shape[0] * seq.tp,) + tuple(g.shape[1:]))
        coll.all_gather_into_tensor(out, g.contiguous(), group=seq.group)
        return out, None


class _SPGatherReplicatedGrad(torch.autograd.Function):
    """all-gather whose incoming gradient is already complete and identical on every TP rank
    (the vocab-parallel log-prob all-reduces dh): backward keeps this rank's rows."""

    @staticmethod
    def forward(ctx, x, seq):
        ctx.seq = seq
        out = x.new_empty((x.shape[0] * seq.tp,) + tuple(x.shape[1:]))
        coll.all_gather_into_tensor(out, x.contiguous(), group=seq.group)
        return out

    @staticmethod
    def backward(ctx, g):
        return ctx.seq.local(g).contiguous(), None


class _TPGradSum(torch.autograd.Function):
    """identity forward; backward all-reduces the (partial, token-slice) gradient over TP."""

    @staticmethod
    def forward(ctx, w, group):
        ctx.group = group
        return w.view_as(w)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        coll.all_reduce(g, group=ctx.group)
        return g, None


# ------------------------------------------ Megatron-SP collectives overlapped with the GEMMs
# With DLA_TP_OVERLAP, the sequence-parallel gather -> column-parallel GEMM and row-parallel GEMM
# -> reduce-scatter pairs run chunk-pipelined instead of as one blocking collective each. The
# local rows [n, H] are cut into C chunks of m rows; chunk c of EVERY rank is gathered by one
# async all-gather into a [tp*m, H] block (rows (r, j) = token r*n + c*m + j), so the gathered
# tensor is "chunk-major" [C][tp][m]. The GEMM of block c runs while block c+1 is in flight; on
# the way out, the row-parallel GEMM of block c is reduce-scattered (async) straight into this
# rank's local rows [c*m, (c+1)*m) while block c+1 is multiplied. Per-token ops (the MLP) stay
# in chunk-major order end to end; attention needs token order, so its qkv output and O input are
# permuted (one copy of the small per-rank [N, q_l + 2 kv_l] / [N, q_l] tensors). The backward
# mirrors it: the adjoint all-gathers of dY are issued async up front and consumed chunk by chunk,
# the adjoint reduce-scatters are launched per chunk and overlap the weight-gradient GEMM.
def _sp_chunks(n: int, chunks: int) -> int:
    c = max(1, int(chunks))
    while c > 1 and (n % c or (n // c) % 8):
        c -= 1
    return c


def _sp_gather_async(x_local: torch.Tensor, seq: TPSeq, C: int):
    """x_local [n, K] -> (chunk-major [C*tp*m, K] buffer, per-chunk async all-gather works)."""
    n, K = x_local.shape
    m = n // C
    out = x_local.new_empty((n * seq.tp, K))
    works = []
    for c in range(C):
        works.append(coll.all_gather_into_tensor(out[c * seq.tp * m:(c + 1) * seq.tp * m],
                                                 x_local[c * m:(c + 1) * m].contiguous(),
                                                 group=seq.group, async_op=True))
    return out, works


def _to_token_order(t: torch.Tensor, tp: int, C: int) -> torch.Tensor:
    """chunk-major rows (c, r, j) -> token order (r, c, j)."""
    M, K = t.shape
    return t.view(C, tp, M // (C * tp), K).transpose(0, 1).reshape(M, K)


def _to_chunk_major(t: torch.Tensor, tp: int, C: int) -> torch.Tensor:
    M, K = t.shape
    return t.view(tp, C, M // (C * tp), K).transpose(0, 1).reshape(M, K)


def _dgrad_into(dy: torch.Tensor, weight: torch.Tensor, out: torch.Tensor) -> None:
    """out = dy @ weight through the cached W^T (TN layout) when the engine allows it."""
    from ..ops.linear import TRANSPOSED_DGRAD, transposed_weight

    if (TRANSPOSED_DGRAD and getattr(weight, "_dla_wt_ok", False) and weight.dtype == torch.bfloat16
            and _ext.use_native(weight) and weight.shape[0] % 8 == 0 and weight.shape[1] % 8 == 0):
        torch.mm(dy, transposed_weight(weight).t(), out=out)
    else:
        torch.mm(dy, weight, out=out)


def _wgrad(ctx_needs: bool, weight: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor):
    from ..ops.linear import accumulate_weight_grad

    if not ctx_needs or accumulate_weight_grad(weight, dy2, x2):
        return None
    return dy2.t() @ x2


class _SPGatherLinearFn(torch.autograd.Function):
    """y = gather_SP(x) W^T with the all-gather chunk-pipelined under the GEMM; `token_order`
    False keeps y chunk-major (per-token consumers)."""

    @staticmethod
    def forward(ctx, x, weight, seq, chunks, token_order):
        x2 = x.reshape(-1, x.shape[-1])
        n = x2.shape[0]
        C = _sp_chunks(n, chunks)
        xg, works = _sp_gather_async(x2, seq, C)
        blk = seq.tp * (n // C)
        y = x2.new_empty((n * seq.tp, weight.shape[0]))
        for c, w in enumerate(works):
            w.wait()
            torch.mm(xg[c * blk:(c + 1) * blk], weight.t(), out=y[c * blk:(c + 1) * blk])
        ctx.save_for_backward(xg)
        ctx.weight, ctx.seq, ctx.C, ctx.token_order, ctx.n = weight, seq, C, token_order, n
        return _to_token_order(y, seq.tp, C) if token_order else y

    @staticmethod
    def backward(ctx, dy):
        (xg,) = ctx.saved_tensors
        seq, C, n, weight = ctx.seq, ctx.C, ctx.n, ctx.weight
        dy2 = dy.reshape(-1, dy.shape[-1])
        dy2 = _to_chunk_major(dy2, seq.tp, C) if ctx.token_order else dy2.contiguous()
        m, blk = n // C, seq.tp * (n // C)
        dx, works, parts = None, [], []
        if ctx.needs_input_grad[0]:
            dx = dy2.new_empty((n, xg.shape[1]))
            for c in range(C):
                part = dy2.new_empty((blk, xg.shape[1]))
                _dgrad_into(dy2[c * blk:(c + 1) * blk], weight, part)
                parts.append(part)
                works.append(coll.reduce_scatter_tensor(dx[c * m:(c + 1) * m], part, group=seq.group,
                                                        async_op=True))
        dw = _wgrad(ctx.needs_input_grad[1], weight, dy2, xg)  # overlaps the reduce-scatters
        for w in works:
            w.wait()
        return dx, dw, None, None, None


class _SPLinearReduceScatterFn(torch.autograd.Function):
    """reduce_scatter_SP(a W^T) -> this rank's [n, N] rows, the reduce-scatter of token chunk c
    launched as soon as its GEMM finished; `token_order` False: `a` is already chunk-major."""

    @staticmethod
    def forward(ctx, a, weight, seq, chunks, token_order):
        a2 = a.reshape(-1, a.shape[-1])
        M = a2.shape[0]
        n = M // seq.tp
        C = _sp_chunks(n, chunks)
        a_cm = _to_chunk_major(a2, seq.tp, C) if token_order else a2.contiguous()
        m, blk = n // C, seq.tp * (n // C)
        y = a2.new_empty((n, weight.shape[0]))
        works, parts = [], []
        for c in range(C):
            part = torch.mm(a_cm[c * blk:(c + 1) * blk], weight.t())
            parts.append(part)
            works.append(coll.reduce_scatter_tensor(y[c * m:(c + 1) * m], part, group=seq.group,
                                                    async_op=True))
        for w in works:
            w.wait()
        ctx.save_for_backward(a_cm)
        ctx.weight, ctx.seq, ctx.C, ctx.token_order, ctx.ashape = weight, seq, C, token_order, a.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        (a_cm,) = ctx.saved_tensors
        seq, C, weight = ctx.seq, ctx.C, ctx.weight
        dyg, works = _sp_gather_async(dy.reshape(-1, dy.shape[-1]).contiguous(), seq, C)
        blk = dyg.shape[0] // C
        da = None
        if ctx.needs_input_grad[0]:
            da = a_cm.new_empty(a_cm.shape)
            for c, w in enumerate(works):
                w.wait()
                _dgrad_into(dyg[c * blk:(c + 1) * blk], weight, da[c * blk:(c + 1) * blk])
            if ctx.token_order:
                da = _to_token_order(da, seq.tp, C)
            da = da.view(ctx.ashape)
        else:
            for w in works:
                w.wait()
        dw = _wgrad(ctx.needs_input_grad[1], weight, dyg, a_cm)
        return da, dw, None, None, None


def sp_gather_linear(x, weight, seq: TPSeq, chunks: Optional[int] = None, token_order: bool = True):
    """Column-parallel GEMM on the SP-gathered input, gather chunk-pipelined (see above)."""
    return _SPGatherLinearFn.apply(x, weight, seq, chunks or tp_chunks("qkv"), token_order)


def sp_linear_reduce_scatter(a, weight, seq: TPSeq, chunks: Optional[int] = None, token_order: bool = True):
    """Row-parallel GEMM reduce-scattered over SP, chunk-pipelined (see above)."""
    return _SPLinearReduceScatterFn.apply(a, weight, seq, chunks or tp_chunks("o"), token_order)


def sp_gather(x, seq: TPSeq):
    return _SPGather.apply(x, seq)


def sp_reduce_scatter(x, seq: TPSeq):
    return _SPReduceScatter.apply(x, seq)


def sp_gather_replicated_grad(x, seq: TPSeq):
    return _SPGatherReplicatedGrad.apply(x, seq)


def tp_grad_sum(w, seq: Optional[TPSeq]):
    """Weight used on the token-sharded stream: its gradient is summed over the TP group."""
    if w is None or seq is None or not (torch.is_grad_enabled() and w.requires_grad):
        return w
    return _TPGradSum.apply(w, seq.group)


def tp_reduce(x, group):
    return _ReduceFromTP.apply(x, group)


# ------------------------------------------------------------ overlapped TP linear layers
# The plain TP layer issues every collective synchronously on the critical path: per layer and
# micro-batch, 2 forward all-reduces of the [B*T, H] row-parallel outputs and 2 backward
# all-reduces of the column-parallel input grads (Llama-3-70B at TP 8: 64 MB each at 4k tokens,
# about as long as the layer's GEMMs on one rank). With DLA_TP_OVERLAP (default on):
#   * row-parallel (o_proj, down_proj) forward: the GEMM runs in DLA_TP_CHUNKS token chunks and
#     chunk c's all-reduce is launched async (RCCL's stream) as soon as its rows exist, so it
#     overlaps the GEMM of chunk c+1; the layer waits once, before the residual add;
#   * column-parallel (qkv, gate|up) backward: dX = dY W is computed first, its all-reduce
#     launched async, THEN the weight-gradient GEMM runs (independent of it) while the
#     collective is in flight.
TP_OVERLAP = os.environ.get("DLA_TP_OVERLAP", "1") != "0"
TP_CHUNKS = max(1, int(os.environ.get("DLA_TP_CHUNKS", "4")))
# Token chunks per TP GEMM kind, instead of one global count: "qkv" (SP gather-linear), "o"
# (row-parallel / SP reduce-scatter of the attention output) and "mlp" (gate|up AND down: in
# the chunk-major Megatron-SP MLP both must use the same count). The 70B TP = 8 per-rank probe
# (profiles/r4_70b_tpshape.md) prices the split: C = 2 costs qkv +27 %, o +12 %, gate|up +1 %,
# down +4 % of the GEMM, C = 4 +68 / +45 / +25 / +29 % -- so 2 everywhere by default, each
# hiding half of its collective. DLA_TP_CHUNKS_<KIND> overrides one kind, DLA_TP_CHUNKS all.
TP_CHUNK_DEFAULTS = {"qkv": 2, "o": 2, "mlp": 2}


def tp_chunks(kind: str) -> int:
    env = os.environ.get(f"DLA_TP_CHUNKS_{kind.upper()}")
    if env:
        return max(1, int(env))
    env = os.environ.get("DLA_TP_CHUNKS")
    if env:
        return max(1, int(env))
    return TP_CHUNK_DEFAULTS[kind]


def _chunk_bounds(M: int, chunks: int):
    """Row ranges of `chunks` near-equal pieces, each a multiple of 8 rows (GEMM-friendly)."""
    step = max(8, ((M + chunks - 1) // chunks + 7) // 8 * 8)
    return [(a, min(M, a + step)) for a in range(0, M, step)]


def _linear_backward(ctx, dy2, x2, weight, async_group=None):
    """dX (optionally all-reduced async over `async_group`, overlapped with the weight grad), dW."""
    from ..ops.linear import accumulate_weight_grad, input_grad

    dx, work = None, None
    if ctx.needs_input_grad[0]:
        dx = input_grad(dy2, weight)
        if async_group is not None:
            dx = dx.contiguous()
            work = coll.all_reduce(dx, group=async_group, async_op=True)
    dw = None
    if ctx.needs_input_grad[1] and not accumulate_weight_grad(weight, dy2, x2):
        dw = dy2.t() @ x2
    if work is not None:
        work.wait()
    return dx, dw


class _ColParallelLinearFn(torch.autograd.Function):
    """y = x W^T (+ b), x replicated over the TP group (Megatron's f operator folded in): the
    backward all-reduces dX asynchronously behind the weight-gradient GEMM."""

    @staticmethod
    def forward(ctx, x, weight, bias, group):
        ctx.save_for_backward(x)
        ctx.weight, ctx.group, ctx.has_bias = weight, group, bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx, dw = _linear_backward(ctx, dy2, x.reshape(-1, x.shape[-1]), ctx.weight, ctx.group)
        db = dy2.sum(0) if (ctx.has_bias and ctx.needs_input_grad[2]) else None
        return (dx.view(x.shape) if dx is not None else None), dw, db, None


class _RowParallelLinearFn(torch.autograd.Function):
    """y = all_reduce(x W^T) over the TP group (Megatron's g operator folded in), the forward
    GEMM + all-reduce pipelined over token chunks; backward = the plain linear backward."""

    @staticmethod
    def forward(ctx, x, weight, group, chunks):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        M, N = x2.shape[0], weight.shape[0]
        y = torch.empty((M, N), dtype=x.dtype, device=x.device)
        works = []
        for a, b in _chunk_bounds(M, chunks):
            torch.mm(x2[a:b], weight.t(), out=y[a:b])
            works.append(coll.all_reduce(y[a:b], group=group, async_op=True))
        for w in works:
            w.wait()
        ctx.save_for_backward(x)
        ctx.weight = weight
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx, dw = _linear_backward(ctx, dy2, x.reshape(-1, x.shape[-1]), ctx.weight)
        return (dx.view(x.shape) if dx is not None else None), dw, None, None


def col_parallel_linear(x, weight, bias, group):
    """Column-parallel linear on a TP-replicated input (tp_copy + linear, overlapped backward)."""
    if not TP_OVERLAP:
        from ..ops.linear import linear

        return linear(tp_copy(x, group), weight, bias)
    return _ColParallelLinearFn.apply(x, weight, bias, group)


def row_parallel_linear(x, weight, group, chunks: Optional[int] = None):
    """Row-parallel linear summed over TP (linear + tp_reduce, chunk-pipelined forward)."""
    if not TP_OVERLAP:
        from ..ops.linear import linear

        return tp_reduce(linear(x, weight, None), group)
    return _RowParallelLinearFn.apply(x, weight, group, chunks or tp_chunks("o"))


def tp_all_gather_last(x: torch.Tensor, group) -> torch.Tensor:
    """Concatenate per-rank shards along the last dim (inference only, e.g. full logits)."""
    ws = coll.world_size(group)
    parts = [torch.empty_like(x) for _ in range(ws)]
    coll.all_gather(parts, x.contiguous(), group=group)
    return torch.cat(parts, dim=-1)


# ------------------------------------------------------------- vocabulary-parallel embedding
def vocab_parallel_embedding(ids: torch.Tensor, weight_l: torch.Tensor, off: int, group) -> torch.Tensor:
    V_l = weight_l.shape[0]
    local = ids - off
    own = (local >= 0) & (local < V_l)
    x = F.embedding(local.clamp(0, V_l - 1), weight_l) * own.unsqueeze(-1).to(weight_l.dtype)
    return tp_reduce(x, group)


# ------------------------------------------------------------- vocabulary-parallel log-prob
def _local_fwd(logits_l, targets, off):
    if _ext.use_native(logits_l):
        return _ext.require().logprob_fwd(logits_l, targets, int(off))
    lf = logits_l.float()
    lse = torch.logsumexp(lf, -1)
    t = targets - off
    own = (targets >= 0) & (t >= 0) & (t < lf.shape[-1])
    tl = lf.gather(-1, t.clamp(0, lf.shape[-1] - 1).unsqueeze(-1)).squeeze(-1)
    return torch.where(own, tl - lse, torch.zeros_like(tl)), lse


def _local_bwd(logits_l, targets, lse, g, off):
    if _ext.use_native(logits_l):
        _ext.require().logprob_bwd(logits_l, targets, lse, g.float().contiguous(), int(off))
        return logits_l
    lf = logits_l.float()
    p = torch.exp(lf - lse.unsqueeze(-1))
    t = targets - off
    own = (targets >= 0) & (t >= 0) & (t < lf.shape[-1])
    onehot = torch.zeros_like(p)
    onehot.scatter_(-1, t.clamp(0, lf.shape[-1] - 1).unsqueeze(-1), own.unsqueeze(-1).float())
    gr = torch.where(targets >= 0, g.float(), torch.zeros_like(g.float())).unsqueeze(-1)
    return (gr * (onehot - p)).to(logits_l.dtype)


class _VPLogprobFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hidden, weight_l, targets, off, group):
        logits_l = F.linear(hidden, weight_l)
        logp_l, lse_l = _local_fwd(logits_l, targets, off)
        V_l = weight_l.shape[0]
        t = targets - off
        own = (targets >= 0) & (t >= 0) & (t < V_l)
        tl_l = torch.where(own, logp_l + lse_l, torch.zeros_like(logp_l))
        # ONE latency-bound collective instead of three (max, sum-exp, target logit all-reduces):
        # every rank gathers all shards' (lse_r, target logit_r) and reduces them locally in a
        # fixed rank order (identical result on every rank)
        tp = coll.world_size(group)
        pair = torch.stack([lse_l.float(), tl_l.float()])
        allp = pair.new_empty((tp * 2,) + tuple(pair.shape[1:]))
        coll.all_gather_into_tensor(allp, pair.contiguous(), group=group)
        allp = allp.view((tp,) + tuple(pair.shape))
        lse = torch.logsumexp(allp[:, 0], dim=0)
        tl = allp[:, 1].sum(0)
        logp = torch.where(targets >= 0, tl - lse, torch.zeros_like(tl))
        ctx.save_for_backward(hidden, targets, lse, logits_l)
        ctx.weight_l = weight_l  # (on ctx: see ops.linear._LinearMainGradFn)
        ctx.off, ctx.group = off, group
        return logp

    @staticmethod
    def backward(ctx, g):
        hidden, targets, lse, logits_l = ctx.saved_tensors
        weight_l = ctx.weight_l
        dlog = _local_bwd(logits_l, targets, lse, g, ctx.off)
        dh, work = None, None
        if ctx.needs_input_grad[0]:
            from ..ops.linear import input_grad

            dh = input_grad(dlog, weight_l).contiguous()
            # in flight on RCCL's stream while the (vocab-shard) weight-gradient GEMM runs
            work = coll.all_reduce(dh, group=ctx.group, async_op=True)
        dw = None
        if ctx.needs_input_grad[1]:
            from ..ops.linear import accumulate_weight_grad

            if not accumulate_weight_grad(weight_l, dlog, hidden):
                dw = dlog.t() @ hidden
        if work is not None:
            work.wait()
        return dh, dw, None, None, None


def vocab_parallel_logprob(hidden, weight_l, targets, off: int, group) -> torch.Tensor:
    return _VPLogprobFn.apply(hidden.contiguous(), weight_l, targets.contiguous(), off, group)


# ------------------------------------------------------------------------- model sharding
# A sharded parameter carries `_dla_tp_spec = (dim, segments)`: along `dim` the full tensor is the
# concatenation of `segments` (e.g. [q, k, v] rows of the fused qkv projection); rank r keeps the
# r-th 1/tp slice of EVERY segment, concatenated. One rule drives sharding, gathering for
# checkpoints/HF export and re-sharding on load.
def shard_tensor(full: torch.Tensor, spec, r: int, tp: int) -> torch.Tensor:
    dim, segs = spec
    parts, o = [], 0
    for n in segs:
        c = n // tp
        parts.append(full.narrow(dim, o + r * c, c))
        o += n
    return torch.cat(parts, dim).contiguous()


def gather_tensor(local: torch.Tensor, spec, group) -> torch.Tensor:
    dim, segs = spec
    tp = coll.world_size(group)
    pieces = [torch.empty_like(local) for _ in range(tp)]
    coll.all_gather(pieces, local.contiguous(), group=group)
    loc = [n // tp for n in segs]
    per_rank = [torch.split(pc, loc, dim) for pc in pieces]
    return torch.cat([per_rank[rk][i] for i in range(len(segs)) for rk in range(tp)], dim)


def _tp_specs(cfg, tp: int):
    D = cfg.head_dim
    qkv = (0, [cfg.num_heads * D, cfg.num_kv_heads * D, cfg.num_kv_heads * D])
    Fd = cfg.intermediate_size
    up = (0, [Fd, Fd] if cfg.activation == "swiglu" else [Fd])
    specs = {"qkv_proj": qkv, "qkv_bias": qkv, "o_proj": (1, [cfg.num_heads * D]),
             "up_proj": up, "up_bias": up, "down_proj": (1, [Fd])}
    vocab = (0, [cfg.vocab_size]) if cfg.vocab_size % tp == 0 else None
    return specs, vocab


@torch.no_grad()
def apply_tensor_parallel(model, group, tp_rank: Optional[int] = None, tp_size: Optional[int] = None,
                          sequence_parallel: bool = False, force: bool = False):
    """Shard a CausalLM (or RewardModel backbone) in place for this TP rank; `sequence_parallel`
    additionally shards the residual stream over tokens (Megatron-SP: reduce-scatter / all-gather
    instead of all-reduce). `force` with a ONE-rank group: install the TP layers anyway (identity
    shards), so the column / row-parallel GEMMs, the SP gather-linear / reduce-scatter pipeline and
    the vocab-parallel log-prob issue their collectives on the communicator, on one GPU."""
    base = getattr(model, "backbone", model)
    cfg = base.cfg
    tp = tp_size or coll.world_size(group)
    r = coll.rank(group) if tp_rank is None else tp_rank
    if tp == 1 and not (force and group is not None):
        return model
    if cfg.is_moe:
        raise NotImplementedError("MoE layers use expert parallelism (parallel.expert), not TP")
    if cfg.num_heads % tp or cfg.num_kv_heads % tp or cfg.intermediate_size % tp:
        raise ValueError(f"heads ({cfg.num_heads}/{cfg.num_kv_heads}) and FFN ({cfg.intermediate_size}) "
                         f"must divide tp={tp}")
    specs, vocab = _tp_specs(cfg, tp)
    owners = None

    def shard(p, spec):
        nonlocal owners
        if p.is_meta:  # memory-bounded construction: local shape now, values later
            from ..models.materialize import _owners, reshape_meta

            owners = owners if owners is not None else _owners(model)
            dim, segs = spec
            shape = list(p.shape)
            shape[dim] = sum(n // tp for n in segs)
            reshape_meta(model, p, shape, owners, _dla_tp_spec=spec)
            return
        p.data = shard_tensor(p.data, spec, r, tp)
        p._dla_tp_spec = spec

    for layer in base.layers:
        at, mlp = layer.attn, layer.mlp
        for mod in (at, mlp):
            for name, spec in specs.items():
                p = getattr(mod, name, None)
                if isinstance(p, torch.nn.Parameter):
                    shard(p, spec)
        at.tp, at.h_local, at.kv_local = group, cfg.num_heads // tp, cfg.num_kv_heads // tp
        mlp.tp = group
        for p in (layer.ln1_w, getattr(layer, "ln1_b", None), getattr(layer, "ln2_w", None),
                  getattr(layer, "ln2_b", None), at.o_bias, mlp.down_bias):
            if p is not None:
                p._dla_tp_replicated = True
    for p in (base.norm_w, base.norm_b, base.wpe):
        if p is not None:
            p._dla_tp_replicated = True
    vocab_params = [p for p in (base.embed, base.lm_head, base.lm_head_bias) if p is not None]
    if vocab is not None:
        for p in vocab_params:
            shard(p, vocab)
        Vl = cfg.vocab_size // tp
        base.vocab_parallel = (r * Vl, Vl)
    else:
        for p in vocab_params:
            p._dla_tp_replicated = True
    for head in ("scorer", "v_head"):  # reward / value heads are replicated across TP ranks
        if hasattr(model, head):
            for p in getattr(model, head).parameters():
                p._dla_tp_replicated = True
    base.tp = group
    base.tp_size = tp
    base.tp_rank = r
    if sequence_parallel:
        seq = TPSeq(group)
        base.tp_seq = seq
        for layer in base.layers:
            layer.tp_seq = layer.attn.tp_seq = layer.mlp.tp_seq = seq
    return model


def is_tensor_parallel(model) -> bool:
    return getattr(getattr(model, "backbone", model), "tp_size", 1) > 1


@contextmanager
def tp_unsharded(model, writeback: bool = False):
    """Temporarily give every TP-sharded parameter its FULL tensor (collective over the TP group).

    Used around HF/state-dict export (read) and checkpoint load (`writeback=True`: the loaded full
    values are re-sliced into the rank's shard, which stays the same storage — e.g. the
    data-parallel engine's flat buffer view)."""
    base = getattr(model, "backbone", model)
    if getattr(base, "tp_size", 1) <= 1:
        yield model
        return
    group, tp, r = base.tp, base.tp_size, base.tp_rank
    saved = []
    with torch.no_grad():
        for p in model.parameters():
            spec = getattr(p, "_dla_tp_spec", None)
            if spec is not None:
                saved.append((p, p.data, spec))
                p.data = gather_tensor(p.data, spec, group)
    try:
        yield model
    finally:
        with torch.no_grad():
            for p, local, spec in saved:
                if writeback:
                    local.copy_(shard_tensor(p.data, spec, r, tp))
                p.data = local
