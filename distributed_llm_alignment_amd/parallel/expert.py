"""Expert parallelism for Mixtral-style MoE layers over an RCCL all-to-all group
(north-star "Mixtral 8x7B DPO with expert-parallel all-to-all").

Each rank of an EP group of size ep owns E/ep consecutive experts (`expert_up/down` sliced in
place, identical seeded init everywhere -> no broadcast). Per MoE layer:
  1. route locally (HIP top-k kernel), order token slots expert-major (experts of one destination
     rank are contiguous), `moe_dispatch` gathers the rows;
  2. exchange the per-(rank, expert) counts with one tiny all-to-all, one host sync for the split
     sizes (the same sync the dropless local path needs for its GEMM loop);
  3. `all_to_all_single` of the token rows (xGMI is a full mesh on one MI355X node: every pair of
     ranks has its own link, so all-to-all runs at full per-link bandwidth);
  4. regroup source-major -> expert-major rows, grouped expert SwiGLU;
  5. the inverse all-to-all and the weighted `moe_combine`.
Backward mirrors it (all-to-all is its own adjoint with the splits swapped). Expert weights are
marked `_dla_expert`: the data-parallel engine reduces their grads over the expert-data-parallel
group (replicas holding the same experts) instead of the full DP group.
"""
from __future__ import annotations

from typing import List

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


class ExpertParallel:
    def __init__(self, group, num_experts: int):
        self.group = group
        self.ep = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if num_experts % self.ep:
            raise ValueError(f"num_experts {num_experts} not divisible by ep {self.ep}")
        self.E = num_experts
        self.El = num_experts // self.ep

    def dispatch_combine(self, moe, h2: torch.Tensor, topv: torch.Tensor, topi: torch.Tensor):
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
        return ops.moe.combine(ys, pos, topv)


@torch.no_grad()
def apply_expert_parallel(model, mesh):
    """Keep this rank's E/ep experts of every MoE layer and attach the all-to-all router."""
    base = getattr(model, "backbone", model)
    cfg = base.cfg
    if mesh.ep <= 1 or not cfg.is_moe:
        return model
    ep = ExpertParallel(mesh.ep_group, cfg.num_experts)
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
