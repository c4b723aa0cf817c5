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
        dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromTP(torch.autograd.Function):
    """all-reduce forward (sum of partial products); identity backward."""

    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous()
        dist.all_reduce(x, group=group)
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
        self.tp = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

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
        dist.all_gather_into_tensor(out, x.contiguous(), group=seq.group)
        return out

    @staticmethod
    def backward(ctx, g):
        seq = ctx.seq
        out = g.new_empty((g.shape[0] // seq.tp,) + tuple(g.shape[1:]))
        dist.reduce_scatter_tensor(out, g.contiguous(), group=seq.group)
        return out, None


class _SPReduceScatter(torch.autograd.Function):
    """[N, H] partial sums (row-parallel GEMM output) -> [n, H] summed local tokens; backward:
    all-gather."""

    @staticmethod
    def forward(ctx, x, seq):
        ctx.seq = seq
        out = x.new_empty((x.shape[0] // seq.tp,) + tuple(x.shape[1:]))
        dist.reduce_scatter_tensor(out, x.contiguous(), group=seq.group)
        return out

    @staticmethod
    def backward(ctx, g):
        seq = ctx.seq
        out = g.new_empty((g.shape[0] * seq.tp,) + tuple(g.shape[1:]))
        dist.all_gather_into_tensor(out, g.contiguous(), group=seq.group)
        return out, None


class _SPGatherReplicatedGrad(torch.autograd.Function):
    """all-gather whose incoming gradient is already complete and identical on every TP rank
    (the vocab-parallel log-prob all-reduces dh): backward keeps this rank's rows."""

    @staticmethod
    def forward(ctx, x, seq):
        ctx.seq = seq
        out = x.new_empty((x.shape[0] * seq.tp,) + tuple(x.shape[1:]))
        dist.all_gather_into_tensor(out, x.contiguous(), group=seq.group)
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
        dist.all_reduce(g, group=ctx.group)
        return g, None


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
            work = dist.all_reduce(dx, group=async_group, async_op=True)
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
            works.append(dist.all_reduce(y[a:b], group=group, async_op=True))
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
    return _RowParallelLinearFn.apply(x, weight, group, chunks or TP_CHUNKS)


def tp_all_gather_last(x: torch.Tensor, group) -> torch.Tensor:
    """Concatenate per-rank shards along the last dim (inference only, e.g. full logits)."""
    ws = dist.get_world_size(group)
    parts = [torch.empty_like(x) for _ in range(ws)]
    dist.all_gather(parts, x.contiguous(), group=group)
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
        m = lse_l.clone()
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
        se = torch.exp(lse_l - m)
        dist.all_reduce(se, group=group)
        lse = m + torch.log(se)
        V_l = weight_l.shape[0]
        t = targets - off
        own = (targets >= 0) & (t >= 0) & (t < V_l)
        tl = torch.where(own, logp_l + lse_l, torch.zeros_like(logp_l))
        dist.all_reduce(tl, group=group)
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
        dh = None
        if ctx.needs_input_grad[0]:
            from ..ops.linear import input_grad

            dh = input_grad(dlog, weight_l).contiguous()
            dist.all_reduce(dh, group=ctx.group)
        dw = None
        if ctx.needs_input_grad[1]:
            from ..ops.linear import accumulate_weight_grad

            if not accumulate_weight_grad(weight_l, dlog, hidden):
                dw = dlog.t() @ hidden
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
    tp = dist.get_world_size(group)
    pieces = [torch.empty_like(local) for _ in range(tp)]
    dist.all_gather(pieces, local.contiguous(), group=group)
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
                          sequence_parallel: bool = False):
    """Shard a CausalLM (or RewardModel backbone) in place for this TP rank; `sequence_parallel`
    additionally shards the residual stream over tokens (Megatron-SP: reduce-scatter / all-gather
    instead of all-reduce)."""
    base = getattr(model, "backbone", model)
    cfg = base.cfg
    tp = tp_size or dist.get_world_size(group)
    r = dist.get_rank(group) if tp_rank is None else tp_rank
    if tp == 1:
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
