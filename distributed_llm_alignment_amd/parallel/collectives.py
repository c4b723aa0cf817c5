"""The collectives the engines issue, routed through one place so that a process group can be a
real RCCL / gloo group OR a `ShapeGroup`: a stand-in for N ranks inside ONE process.

A `ShapeGroup(N)` makes this process rank 0 of an N-rank group that does not exist. Every engine
then lays itself out exactly as that rank of the N-GPU job -- its parameter / optimizer shards,
its TP-sharded weights, its 1/N token slice under sequence parallel, its chunked GEMMs -- and the
collectives become local stand-ins that move the same bytes this rank writes:

  * all-gather: the local part is copied into every one of the N output slots;
  * reduce-scatter: this rank's output is slot 0 of the input (copied, not summed: the values
    stay at one rank's scale, so a stand-in chain of layers does not overflow);
  * all-reduce: the identity (in place);
  * all-to-all: the identity (the rows for destination r stand in for the rows from source r).

That is what `bench.py --tp-shape / --fsdp-shape / --edp-shape` time: one rank's compute,
memory and chunk-split costs at full model width and depth on one GPU, without the wire time
(the collective bytes each mesh must hide are reported beside it). The numerics are not the
full model's (every shard sees rank 0's slice), so shape groups are for timing only.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


class ShapeGroup:
    """N-rank stand-in group (this process is `rank`, default 0). See the module docstring."""

    def __init__(self, size: int, rank: int = 0):
        if size < 1 or not 0 <= rank < size:
            raise ValueError(f"ShapeGroup(size={size}, rank={rank})")
        self.size_, self.rank_ = int(size), int(rank)

    def size(self) -> int:
        return self.size_

    def rank(self) -> int:
        return self.rank_

    def __repr__(self):
        return f"ShapeGroup({self.size_})"


class _Done:
    """A completed async work (shape groups run their stand-ins synchronously)."""

    def wait(self, *a, **k):
        return True

    def is_completed(self):
        return True


def is_shape(group) -> bool:
    return isinstance(group, ShapeGroup)


def world_size(group=None) -> int:
    if isinstance(group, ShapeGroup):
        return group.size_
    return dist.get_world_size(group)


def rank(group=None) -> int:
    if isinstance(group, ShapeGroup):
        return group.rank_
    return dist.get_rank(group)


def all_gather_into_tensor(out: torch.Tensor, x: torch.Tensor, group=None, async_op: bool = False):
    if isinstance(group, ShapeGroup):
        out.view(group.size_, -1).copy_(x.reshape(1, -1).expand(group.size_, -1))
        return _Done() if async_op else None
    return dist.all_gather_into_tensor(out, x, group=group, async_op=async_op)


def reduce_scatter_tensor(out: torch.Tensor, x: torch.Tensor, op=dist.ReduceOp.SUM, group=None,
                          async_op: bool = False):
    if isinstance(group, ShapeGroup):
        out.copy_(x.reshape(group.size_, -1)[group.rank_].view_as(out))
        return _Done() if async_op else None
    return dist.reduce_scatter_tensor(out, x, op=op, group=group, async_op=async_op)


def all_reduce(x: torch.Tensor, op=dist.ReduceOp.SUM, group=None, async_op: bool = False):
    if isinstance(group, ShapeGroup):
        return _Done() if async_op else None
    return dist.all_reduce(x, op=op, group=group, async_op=async_op)


def all_gather(parts: List[torch.Tensor], x: torch.Tensor, group=None):
    if isinstance(group, ShapeGroup):
        for p in parts:
            p.copy_(x)
        return None
    return dist.all_gather(parts, x, group=group)


def all_to_all_single(out: torch.Tensor, x: torch.Tensor, out_splits: Optional[list] = None,
                      in_splits: Optional[list] = None, group=None, async_op: bool = False):
    if isinstance(group, ShapeGroup):
        out.copy_(x)
        return _Done() if async_op else None
    return dist.all_to_all_single(out, x, out_splits, in_splits, group=group, async_op=async_op)


def broadcast(x: torch.Tensor, src: int, group=None):
    if isinstance(group, ShapeGroup):
        return None
    return dist.broadcast(x, src=src, group=group)


def get_global_rank(group, r: int) -> int:
    if isinstance(group, ShapeGroup):
        return r
    return dist.get_global_rank(group, r)
