"""Device mesh over the world: data-parallel x tensor-parallel x expert-parallel groups.

Rank layout (single node, 8 x MI355X, every pair of GPUs on its own xGMI link): TP groups are
contiguous rank blocks ([0..tp-1], ...), DP groups stride across them (ranks with the same TP
rank). On a fully connected xGMI mesh every placement has a dedicated link, so contiguous TP
blocks are chosen for multi-node extension (TP stays intra-node). EP groups are carved from the
DP dimension (experts sharded across data-parallel replicas, Switch/GShard style).

Sequence parallelism (Ulysses, `parallel.sequence`) sits between DP and TP:
rank = (dp_rank * sp + sp_rank) * tp + tp_rank. SP ranks share a batch (sequence slices of the
same rows), so `dp` / `dp_rank` / `dp_group` still index *batch* replicas (what the sampler
shards over), while gradients are reduced over `grad_group` = DP x SP (summed over SP, averaged
over DP: `DataParallelEngine(sp_size=sp)`).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch.distributed as dist

from .dist import new_group, state as dist_state


@dataclass
class Mesh:
    world: int
    rank: int
    tp: int
    dp: int
    ep: int
    tp_rank: int
    dp_rank: int
    ep_rank: int
    tp_group: Optional[object] = None
    dp_group: Optional[object] = None
    ep_group: Optional[object] = None        # ranks sharing one set of experts' tokens
    edp_group: Optional[object] = None       # ranks holding the SAME experts (grad reduction)
    world_group: Optional[object] = None
    sp: int = 1
    sp_rank: int = 0
    sp_group: Optional[object] = None        # ranks holding slices of the same sequences
    dpsp_group: Optional[object] = None      # DP x SP: gradient reduction when sp > 1

    @property
    def is_tp(self) -> bool:
        return self.tp > 1

    @property
    def grad_group(self):
        """Group over which dense gradients are reduced (DP, or DP x SP under sequence parallel)."""
        return self.dpsp_group if self.sp > 1 else self.dp_group


_MESH: Optional[Mesh] = None


def build_mesh(tp: int = 1, ep: int = 1, sp: int = 1) -> Mesh:
    """Create process groups (collective: every rank must call with the same arguments)."""
    global _MESH
    st = dist_state()
    world = st.world_size if st.initialized else 1
    rank = st.rank if st.initialized else 0
    if world % (tp * sp):
        raise ValueError(f"world {world} not divisible by tp {tp} x sp {sp}")
    if sp > 1 and (tp > 1 or ep > 1):
        raise ValueError("sequence parallel composes with data parallel only (tp = ep = 1)")
    if sp > 1:
        dp = world // sp
        mesh = Mesh(world=world, rank=rank, tp=1, dp=dp, ep=1, tp_rank=0, dp_rank=rank // sp,
                    ep_rank=0, sp=sp, sp_rank=rank % sp)
        mesh.world_group = dist.group.WORLD
        mesh.dpsp_group = dist.group.WORLD
        for d in range(dp):  # SP groups: contiguous blocks (one xGMI hop between any two)
            ranks = [d * sp + s for s in range(sp)]
            g = new_group(ranks)
            if rank in ranks:
                mesh.sp_group = g
        for s in range(sp):  # DP groups (batch replicas): same sp rank
            ranks = [d * sp + s for d in range(dp)]
            g = new_group(ranks) if dp > 1 else None
            if rank in ranks:
                mesh.dp_group = g
        _MESH = mesh
        return mesh
    dp = world // tp
    if dp % ep:
        raise ValueError(f"dp {dp} not divisible by ep {ep}")
    tp_rank, dp_rank = rank % tp, rank // tp
    mesh = Mesh(world=world, rank=rank, tp=tp, dp=dp, ep=ep, tp_rank=tp_rank, dp_rank=dp_rank,
                ep_rank=dp_rank % ep)
    if world == 1:
        if st.forced:  # one-rank process group (init_distributed(force_pg=True)): every group
            # is the one-rank WORLD group, so the engines issue their collectives on RCCL
            w = dist.group.WORLD
            mesh.world_group = mesh.tp_group = mesh.dp_group = mesh.ep_group = mesh.edp_group = w
        _MESH = mesh
        return mesh
    mesh.world_group = dist.group.WORLD
    for d in range(dp):  # TP groups
        ranks = [d * tp + t for t in range(tp)]
        g = new_group(ranks) if tp > 1 else None
        if rank in ranks:
            mesh.tp_group = g
    for t in range(tp):  # DP groups
        ranks = [d * tp + t for d in range(dp)]
        g = new_group(ranks) if dp > 1 else None
        if rank in ranks:
            mesh.dp_group = g
    if ep > 1:
        for t in range(tp):
            for blk in range(dp // ep):  # EP groups: ep consecutive DP replicas
                ranks = [(blk * ep + e) * tp + t for e in range(ep)]
                g = new_group(ranks)
                if rank in ranks:
                    mesh.ep_group = g
            for e in range(ep):  # replicas of the same expert shard
                ranks = [(blk * ep + e) * tp + t for blk in range(dp // ep)]
                g = new_group(ranks) if len(ranks) > 1 else None
                if rank in ranks:
                    mesh.edp_group = g
    _MESH = mesh
    return mesh


def current_mesh() -> Optional[Mesh]:
    """The mesh built by `build_mesh` (None if none was built: plain data parallel)."""
    return _MESH


def reset_mesh() -> None:
    global _MESH
    _MESH = None


def get_mesh() -> Mesh:
    global _MESH
    if _MESH is None:
        _MESH = build_mesh()
    return _MESH
