"""Expert parallelism for Mixtral-style MoE layers over an RCCL all-to-all group
(north-star "Mixtral 8x7B DPO with expert-parallel all-to-all").

Each rank of an EP group of size ep owns E/ep consecutive experts (`expert_up/down` sliced in
place, identical seeded init everywhere -> no broadcast). Two dispatch modes:

* `capacity` (`hardware.ep_capacity_factor` > 0, e.g. 2.0; `bench.py --ep-capacity`): NO host
  synchronisation anywhere in
  the layer, forward or backward. Every (source, destination) pair exchanges a fixed block of
  C = capacity_factor * N * k / ep rows (multiple of 8), so the all-to-all split sizes are known
  on the host without reading the routing: token slots are ordered expert-major on the device,
  each destination's slots beyond C are dropped (their combine weight becomes 0, the GShard /
  Switch convention; `dropped_slots()` reports the count lazily and the trainers log it as
  `moe/dropped_slots`, warning when nonzero), the per-(destination, local
  expert) counts travel in one small device-side all-to-all, and the receiver builds the
  expert-major row order and the grouped-GEMM offsets on the device. The grouped expert GEMM
  (csrc/grouped_gemm.hip) then runs over the padded [ep*C] buffer, touching only the valid rows.
  The tokens are processed in `chunks` (default 2) pipelined pieces: chunk c+1's dispatch
  all-to-all is in flight on RCCL's stream while chunk c's expert GEMMs run, and chunk c's
  return all-to-all overlaps chunk c+1's experts. With a capacity large enough that nothing is
  dropped the result equals the exact path (the MoE layer is per-token).
* `exact` (capacity factor 0, the trainers' default: HF Mixtral, which the reference runs, is
  dropless): dropless with host-known splits: the per-(rank, expert) counts
  are read on the host once per layer and `all_to_all_single` moves exactly the routed rows.

Expert weights are marked `_dla_expert`: the data-parallel engine reduces their grads over the
expert-data-parallel group (replicas holding the same experts) instead of the full DP group.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import ops


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, out_splits: List[int], in_splits: List[int], group):
        ctx.splits = (out_splits, in_splits)
        ctx.group = group
        out = x.new_empty((sum(out_splits),) + tuple(x.shape[1:]))
        dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        out_splits, in_splits = ctx.splits
        dx = g.new_empty((sum(in_splits),) + tuple(g.shape[1:]))
        dist.all_to_all_single(dx, g.contiguous(), in_splits, out_splits, group=ctx.group)
        return dx, None, None, None


def all_to_all(x, out_splits, in_splits, group):
    return _AllToAll.apply(x, list(out_splits), list(in_splits), group)


class _A2AStart(torch.autograd.Function):
    """Equal-split all-to-all launched asynchronously; `_A2AWait` completes it. The backward is
    split the same way: `_A2AWait.backward` (which autograd reaches first) launches the adjoint
    all-to-all asynchronously and `_A2AStart.backward` waits for it, so with several chunks the
    gradient exchange of one chunk overlaps the expert backward of another. `group=None` is the
    one-process shape mode (ExpertParallel(shape_ep=N)): the exchange is the identity."""

    @staticmethod
    def forward(ctx, x, group, holder):
        ctx.link = link = {"group": group}
        x = x.contiguous()
        if group is None:
            holder.append((None, link))
            return x.view_as(x)
        out = torch.empty_like(x)
        holder.append((dist.all_to_all_single(out, x, group=group, async_op=True), link))
        return out

    @staticmethod
    def backward(ctx, g):
        link = ctx.link
        if link.get("h") is not None:
            link.pop("h").wait()
        dx = link.pop("dx", None)
        if dx is None:  # the wait node's backward did not run first: exchange here
            if link["group"] is None:
                return g, None, None
            dx = torch.empty_like(g)
            dist.all_to_all_single(dx, g.contiguous(), group=link["group"])
        return dx, None, None


class _A2AWait(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out, holder):
        h, link = holder.pop(0)
        if h is not None:
            h.wait()
        ctx.link = link
        return out.view_as(out)

    @staticmethod
    def backward(ctx, g):
        link = ctx.link
        g = g.contiguous()
        if link["group"] is None:
            link["dx"] = g
        else:
            dx = torch.empty_like(g)
            link["h"] = dist.all_to_all_single(dx, g, group=link["group"], async_op=True)
            link["dx"] = dx
        return g, None


# the capacity routing's slot placement and receiver order as one HIP launch each
# (csrc/moe.hip ep_route / ep_expert_order) instead of ~20 torch ops; DLA_EP_NATIVE_ROUTE=0: torch
_NATIVE_ROUTE = os.environ.get("DLA_EP_NATIVE_ROUTE", "1") != "0"


# The token -> slot gather's backward as a per-token gather-sum through the slot positions (the
# combine kernel with unit weights) instead of an fp32 index_add + bf16 cast (Mixtral EP shape:
# 41 + 11 ms/step); DLA_EP_GATHER_BWD_COMBINE=0 keeps the index_add for A/B.
GATHER_BWD_COMBINE = os.environ.get("DLA_EP_GATHER_BWD_COMBINE", "1") != "0"
# Load-adaptive library rows for a single local expert: the hipBLASLt GEMMs cover the expected
# n * k rows of the capacity buffer, the rows past them run on the grouped kernels (ops.moe
# MOE_MAIN_ROWS). Under imbalanced routing those overflow launches are small-M grids (<= 160
# workgroups for 256 CUs over K = 14336 / 28672) at ~400 TF/s, so the rank of a hot expert paid
# 3x the library's cost for its extra rows (profiles/r6_mixtral.md). Each (layer, chunk) keeps
# the row count its expert actually received in a pinned host word, copied asynchronously after
# the routing (no sync); the next call widens the library's share to that count. The split point
# is only a performance hint -- every split gives the same rows -- so a value one call stale is
# harmless. DLA_EP_ADAPTIVE_MAIN=0: the static expected-rows split.
ADAPTIVE_MAIN = os.environ.get("DLA_EP_ADAPTIVE_MAIN", "1") != "0"


def _native_route(topi: torch.Tensor, E: int, ep: int, slots: int) -> bool:
    return _NATIVE_ROUTE and topi.is_cuda and E <= 64 and slots <= 16384 and topi.dtype in (torch.int32, torch.int64)


class _GatherRowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, idx, injective, inv):
        ctx.save_for_backward(idx, inv)
        ctx.R, ctx.injective = x.shape[0], injective
        return ops._ext.require().gather_rows(x, idx)

    @staticmethod
    def backward(ctx, g):
        idx, inv = ctx.saved_tensors
        if ctx.injective:  # one HIP scatter, no accumulation needed
            return ops._ext.require().scatter_rows(g.contiguous(), idx, ctx.R), None, None, None
        if inv is not None:
            # the inverse map given (row r of x read by entries inv[r, :], >= len(g) = none): a
            # gather-sum per row, fp32 in j order -- the MoE combine kernel with unit weights
            return ops._ext.require().moe_combine(g.contiguous(), inv, None), None, None, None
        # a row read by several slots (a token's k choices): accumulate, in fp32
        valid = (idx >= 0).unsqueeze(-1)
        dx = torch.zeros((ctx.R, g.shape[1]), dtype=torch.float32, device=g.device)
        dx.index_add_(0, idx.clamp(min=0), torch.where(valid, g.float(), torch.zeros((), device=g.device)))
        return dx.to(g.dtype), None, None, None


def _gather_rows(x: torch.Tensor, idx: torch.Tensor, injective: bool = True,
                 inv: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[i] = x[idx[i]] (idx < 0 -> zero row). Static shapes, no host sync; the backward is the
    matching scatter, or (`injective` False: a row read by several entries, e.g. a token's k
    slots) a scatter-add -- with `inv` ([rows of x, k] int32: the entries that read each row,
    values >= len(idx) for none) a gather-sum instead. On the GPU the forward and both backward
    forms are one HIP launch each (csrc/moe.hip gather_rows / scatter_rows / moe_combine)."""
    if (_NATIVE_ROUTE and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and x.shape[1] % 8 == 0
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and idx.dtype == torch.int64):
        if inv is not None and not (GATHER_BWD_COMBINE and inv.shape[0] == x.shape[0] and inv.shape[1] <= 8):
            inv = None
        return _GatherRowsFn.apply(x, idx.contiguous(), injective,
                                   inv.to(torch.int32).contiguous() if inv is not None else None)
    valid = (idx >= 0).unsqueeze(-1)
    return torch.where(valid, x.index_select(0, idx.clamp(min=0)), torch.zeros((), dtype=x.dtype, device=x.device))


class ExpertParallel:
    def __init__(self, group, num_experts: int, capacity_factor: float = 2.0, chunks: int = 2,
                 shape_ep: int = 1, shape_hot: bool = False):
        """`shape_ep` > 1 (one process, no group; bench.py --ep-shape): rank 0 of an EP group of
        that size. It keeps E/shape_ep experts and runs the capacity-padded, sync-free dispatch with
        every all-to-all replaced by the identity: the rows this rank would send to destination r
        stand in for the rows it would receive from source r. Under balanced routing that is the
        per-rank expert load of the real job (k x N slots into E/ep experts), so the timing is one
        EP rank's compute; the numerics are not the full model's (every slot meets the local
        experts). `shape_hot` (bench.py --ep-hot, one local expert): the rank of a HOT expert under
        imbalanced routing -- every source sends its full capacity C (the padding rows of each
        source block are zero rows that no slot reads back), so the expert runs capacity_factor x
        the balanced rows and everything past the expected n * k runs on the overflow path."""
        self.shape = int(shape_ep) > 1
        self.group = None if self.shape else group
        self.ep = int(shape_ep) if self.shape else dist.get_world_size(group)
        self.rank = 0 if self.shape else dist.get_rank(group)
        if num_experts % self.ep:
            raise ValueError(f"num_experts {num_experts} not divisible by ep {self.ep}")
        self.E = num_experts
        self.El = num_experts // self.ep
        self.capacity_factor = float(capacity_factor)
        self.chunks = max(1, int(chunks))
        self.shape_hot = bool(shape_hot) and self.shape
        if self.shape_hot and self.El != 1:
            raise ValueError("shape_hot needs one local expert per rank (--ep-shape = num_experts)")
        self._dropped = None  # device int64 counter of dropped token slots (capacity mode)
        self._seen_rows: dict = {}  # (id(moe), chunk) -> pinned int32 [1]: rows received last call

    def dropped_slots(self, reset: bool = True) -> int:
        """Token slots dropped by the capacity limit since the last call (one host read)."""
        if self._dropped is None:
            return 0
        n = int(self._dropped.item())
        if reset:
            self._dropped.zero_()
        return n

    def dispatch_combine(self, moe, h2: torch.Tensor, topv: torch.Tensor, topi: torch.Tensor):
        if self.capacity_factor > 0:
            return self._capacity(moe, h2, topv, topi)
        if self.shape:
            raise ValueError("the EP shape mode runs the capacity dispatch (capacity_factor > 0)")
        return self._exact(moe, h2, topv, topi)

    # ------------------------------------------------------------------ capacity (sync-free)
    def capacity(self, n_tokens: int, k: int) -> int:
        c = int(self.capacity_factor * n_tokens * k / self.ep + 0.999999)
        return max(8, (c + 7) // 8 * 8)

    def _route_chunk(self, topi: torch.Tensor, C: int):
        """Device-side slot placement for one token chunk: (send_src [ep*C] token index or -1,
        slot_pos [n, k] row of each slot in the send buffer or ep*C when dropped, send counts
        [ep, El] int32, dropped count)."""
        ep, El, E = self.ep, self.El, self.E
        n, k = topi.shape
        dev = topi.device
        if _native_route(topi, E, ep, n * k):
            if self._dropped is None:
                self._dropped = torch.zeros((), dtype=torch.long, device=dev)
            send_src, pos, sent = ops._ext.require().ep_route(topi.contiguous(), E, ep, C, self._dropped.view(1))
            return send_src, pos, sent, None  # (dropped slots counted by the kernel)
        flat = topi.reshape(-1).long()
        order = torch.argsort(flat, stable=True)
        rank_sorted = torch.empty_like(order)
        rank_sorted[order] = torch.arange(order.numel(), device=dev)
        counts = torch.zeros(E, dtype=torch.long, device=dev).scatter_add_(0, flat, torch.ones_like(flat))
        cum = torch.cumsum(counts, 0)
        dstart = (cum - counts).view(ep, El)[:, 0]  # first expert-major slot of each destination
        dest = flat // El
        off = rank_sorted - dstart[dest]  # slot's rank inside its destination block
        keep = off < C
        pos = torch.where(keep, dest * C + off, torch.full_like(off, ep * C))
        send_src = torch.full((ep * C + 1,), -1, dtype=torch.long, device=dev)
        send_src.scatter_(0, pos, torch.where(keep, torch.arange(n * k, device=dev) // k, -1))
        # per (destination, local expert) rows actually sent: the first C of the block in order
        cnt = counts.view(ep, El)
        before = torch.cumsum(cnt, 1) - cnt
        sent = torch.clamp(torch.clamp(C - before, min=0), max=cnt)
        return send_src[:ep * C], pos.view(n, k), sent.to(torch.int32), (~keep).sum()

    def _expert_order(self, rc: torch.Tensor, C: int):
        """Receiver side: rows [src s][j < sum_e rc[s, e]] (local-expert sorted per source) ->
        expert-major order. Returns (xe_src [ep*C] recv row or -1, inv [ep*C] expert-major position
        of every recv row or -1, grouped-GEMM offsets [El+1] int32)."""
        ep, El = self.ep, self.El
        dev = rc.device
        if rc.is_cuda and ep <= 64 and El <= 64 and _NATIVE_ROUTE:
            return ops._ext.require().ep_expert_order(rc.to(torch.int32).contiguous(), C)
        rc = rc.long()
        tot_s = rc.sum(1)  # rows received from each source
        cum_s = torch.cumsum(rc, 1)  # [ep, El] inclusive, per source
        r = torch.arange(C, device=dev).view(1, C).expand(ep, C)  # row within the source block
        e = (r.unsqueeze(-1) >= cum_s.unsqueeze(1)).sum(-1)  # local expert of the row (El: padding)
        valid = r < tot_s.view(ep, 1)
        e_c = e.clamp(max=El - 1)
        j = r - torch.gather(cum_s - rc, 1, e_c)  # index inside its (source, expert) run
        per_e = rc.sum(0)  # [El] rows per local expert
        starts_es = (torch.cumsum(rc.t().reshape(-1), 0) - rc.t().reshape(-1)).view(El, ep)  # (e, s)
        q = starts_es[e_c, torch.arange(ep, device=dev).view(ep, 1).expand(ep, C)] + j
        inv = torch.where(valid, q, torch.full_like(q, -1)).reshape(-1)
        xe_src = torch.full((ep * C + 1,), -1, dtype=torch.long, device=dev)
        xe_src.scatter_(0, torch.where(valid.reshape(-1), inv, torch.full_like(inv, ep * C)),
                        torch.arange(ep * C, device=dev))
        offs = torch.zeros(El + 1, dtype=torch.int32, device=dev)
        offs[1:] = torch.cumsum(per_e, 0).to(torch.int32)
        return xe_src[:ep * C], inv, offs

    def _capacity(self, moe, h2: torch.Tensor, topv: torch.Tensor, topi: torch.Tensor):
        N, H = h2.shape
        k = topi.shape[1]
        nch = self.chunks if N >= 8 * self.chunks else 1
        bounds = [(N * c // nch, N * (c + 1) // nch) for c in range(nch)]
        holder: list = []
        stage = []
        # chunk views by one split (its backward is one cat; per-chunk slices each build a zero
        # [N, H] gradient and add it)
        h2c = torch.split(h2, [b - a for a, b in bounds])
        topvc = torch.split(topv, [b - a for a, b in bounds])
        # 1) route every chunk and launch its dispatch all-to-alls (rows + counts) async
        for ci, (a, b) in enumerate(bounds):
            C = self.capacity(b - a, k)
            send_src, pos, sent, ndrop = self._route_chunk(topi[a:b], C)
            if ndrop is not None:
                if self._dropped is None:
                    self._dropped = torch.zeros((), dtype=torch.long, device=h2.device)
                self._dropped += ndrop
            if self.shape:
                rc, w = (torch.full_like(sent, C) if self.shape_hot else sent), None
            else:
                rc = torch.empty_like(sent)
                w = dist.all_to_all_single(rc, sent.contiguous(), group=self.group, async_op=True)
            # a token fills up to k slots: its gradient is the sum of theirs, gathered through pos
            xs = _gather_rows(h2c[ci], send_src, injective=False, inv=pos)
            xr = _A2AStart.apply(xs, self.group, holder)
            stage.append((C, pos, w, rc, xr, (b - a) * k))
        # 2) per chunk: wait for its rows, experts on the device-built order, return all-to-all
        back = []
        for ci, (C, pos, w, rc, xr, nk) in enumerate(stage):
            if w is not None:
                w.wait()
            xr = _A2AWait.apply(xr, holder)
            xe_src, inv, offs = self._expert_order(rc, C)
            xe = _gather_rows(xr, xe_src)
            # a single local expert's expected rows under balanced routing: the chunk's n * k slots
            # (its buffer holds cf * n * k), as a multiple of the 256-row GEMM tile; widened to
            # the rows this (layer, chunk) received last time (ADAPTIVE_MAIN)
            base = main = min(xe.shape[0], (nk + 255) // 256 * 256) if self.El == 1 else 0
            if main and ADAPTIVE_MAIN and xe.is_cuda:
                main = self._adaptive_main(moe, ci, main, xe.shape[0], offs)
            ye = ops.moe.experts_swiglu_offsets(xe, moe.expert_up, moe.expert_down, offs, fp8=moe.fp8,
                                                main_rows=main, base_rows=base)
            yr = _gather_rows(ye, inv)
            back.append((pos, _A2AStart.apply(yr, self.group, holder)))
        # 3) combine each chunk (dropped slots point one past the buffer: the native combine reads
        # them as zero; the CPU reference gets an appended zero row)
        outs = []
        for ci, (pos, ys) in enumerate(back):
            ys = _A2AWait.apply(ys, holder)
            if not ys.is_cuda:
                ys = torch.cat([ys, ys.new_zeros(1, H)], 0)
            outs.append(ops.moe.combine(ys, pos.to(torch.int32), topvc[ci]))
        return outs[0] if len(outs) == 1 else torch.cat(outs, 0)

    def _adaptive_main(self, moe, ci: int, main: int, rows: int, offs: torch.Tensor) -> int:
        """Library rows for this call from the count the same (layer, chunk) received last call;
        queues the copy of this call's count for the next one (never under graph capture)."""
        key = (id(moe), ci)
        seen = self._seen_rows.get(key)
        if seen is not None:
            got = int(seen[0])  # host read of a pinned word: no device sync
            main = min(rows, max(main, (got + 255) // 256 * 256))
        if not torch.cuda.is_current_stream_capturing():
            if seen is None:
                seen = torch.zeros(1, dtype=torch.int32, pin_memory=True)
                self._seen_rows[key] = seen
            seen.copy_(offs[-1:], non_blocking=True)
        return main

    # ------------------------------------------------------------------ exact (host splits)
    def _exact(self, moe, h2: torch.Tensor, topv: torch.Tensor, topi: torch.Tensor):
        ep, El = self.ep, self.El
        pos, counts = ops.moe.expert_positions(topi, self.E)
        recv = torch.empty_like(counts)
        dist.all_to_all_single(recv, counts.contiguous(), group=self.group)  # [ep*El] src-major
        both = torch.cat([counts, recv]).tolist()  # the one host sync of the layer
        sc, rc = both[:self.E], both[self.E:]
        send_splits = [sum(sc[d * El:(d + 1) * El]) for d in range(ep)]
        recv_splits = [sum(rc[s * El:(s + 1) * El]) for s in range(ep)]
        xs = ops.moe.dispatch(h2, pos)
        xr = all_to_all(xs, recv_splits, send_splits, self.group)
        # src-major [(s, e)] -> expert-major [(e, s)] rows
        dev = h2.device
        lens = torch.tensor(rc, device=dev)
        seg = torch.repeat_interleave(torch.arange(ep * El, device=dev), lens, output_size=len(xr))
        key = (seg % El) * ep + seg // El
        perm = torch.argsort(key, stable=True)
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(perm.numel(), device=dev)
        xe = xr.index_select(0, perm)
        # per-local-expert row counts from the host copy this layer already synced (the expert
        # GEMM, grouped or per-expert loop, then needs no further host round trip)
        counts_local = [sum(rc[s * El + e] for s in range(ep)) for e in range(El)]
        ye = ops.moe.experts_swiglu(xe, moe.expert_up, moe.expert_down, counts_local, fp8=moe.fp8)
        yr = ye.index_select(0, inv)
        ys = all_to_all(yr, send_splits, recv_splits, self.group)
        return ops.moe.combine(ys, pos, topv, permutation=True)  # dropless: N*k rows, one per slot


@torch.no_grad()
def apply_expert_parallel(model, mesh, capacity_factor: float = 2.0, chunks: int = 2,
                          shape_ep: int = 1, force: bool = False, shape_hot: bool = False):
    """Keep this rank's E/ep experts of every MoE layer and attach the all-to-all router
    (`capacity_factor` 0: exact dropless dispatch with one host read per layer). `shape_ep` > 1
    with `mesh=None`: the one-process shape mode of ExpertParallel (bench.py --ep-shape).
    `force`: attach the router even for a ONE-rank `mesh.ep_group` (init_distributed(force_pg)):
    every all-to-all of the dispatch then runs on the communicator, on one GPU."""
    base = getattr(model, "backbone", model)
    cfg = base.cfg
    if shape_ep > 1:
        if mesh is not None and mesh.ep > 1:
            raise ValueError("shape_ep is a one-process mode; it does not combine with a real EP group")
        if not cfg.is_moe:
            return model
        ep = ExpertParallel(None, cfg.num_experts, capacity_factor=capacity_factor, chunks=chunks,
                            shape_ep=shape_ep, shape_hot=shape_hot)
        for layer in base.layers:
            m = layer.mlp
            for nm in ("expert_up", "expert_down"):
                w = getattr(m, nm)
                w.data = w.data[:ep.El].contiguous()
                w._dla_expert = True  # its optimizer state is not sharded over the DP ranks
            m.ep = ep
        base.ep_size = ep.ep
        return model
    if (mesh.ep <= 1 and not (force and mesh.ep_group is not None)) or not cfg.is_moe:
        return model
    ep = ExpertParallel(mesh.ep_group, cfg.num_experts, capacity_factor=capacity_factor, chunks=chunks)
    lo, hi = ep.rank * ep.El, (ep.rank + 1) * ep.El
    owners = None
    for layer in base.layers:
        m = layer.mlp
        for nm in ("expert_up", "expert_down"):
            w = getattr(m, nm)
            if w.is_meta:  # memory-bounded construction: local rows now, values later
                from ..models.materialize import _owners, reshape_meta

                owners = owners if owners is not None else _owners(model)
                reshape_meta(model, w, (hi - lo,) + tuple(w.shape[1:]), owners, _dla_ep_rows=(lo, hi))
            else:
                w.data = w.data[lo:hi].contiguous()
        for w in (m.expert_up, m.expert_down):
            w._dla_expert = True
            w._dla_ep = (mesh.ep_group, ep.rank, ep.ep)  # dim-0 slice rank/size (checkpoint I/O)
        m.ep = ep
    base.ep_size = ep.ep
    base.ep_rank = ep.rank
    base.ep_group = mesh.ep_group
    return model
