"""Sequence (context) parallelism, DeepSpeed-Ulysses style, over an RCCL SP group.

The reference has no long-context mechanism (inputs are truncated to 1024/2048 tokens,
src/data/datasets.py:57-63,108-114); SURVEY §5.7 lists Ulysses as the optional long-context path
on the same RCCL primitives. This module makes it a first-class mesh dimension:

  * every rank of an SP group holds a contiguous 1/P slice of each sequence (tokens
    [r*T/P, (r+1)*T/P)); embeddings, norms, MLP / MoE, the LM head and the fused log-prob kernels
    are token-local and run on the slice unchanged;
  * attention is the only token-mixing op. Around it two all-to-alls swap the sharded dimension:
    the fused QKV [B, T/P, (Hq+2Hkv)*D] becomes [B, T, (Hq+2Hkv)/P * D] (all tokens, 1/P of the
    q and kv heads), the HIP flash-attention kernel runs on full sequences with global positions
    and global padding / packing bounds, and the output goes back to [B, T/P, Hq*D];
  * sequence-level reductions (masked log-prob sums, token counts) are all-reduced over the SP
    group. The resulting loss is *replicated* on the SP ranks, so those reductions are identity
    in the backward, and each rank's parameter gradient is the partial sum over its own tokens.
    The gradient reducer therefore sums over SP and averages over DP
    (`DataParallelEngine(sp_size=P)`, group = the DP x SP "grad group" of `parallel.mesh`).

Per layer and direction the traffic is two all-to-alls of (Hq+2Hkv)*D and Hq*D per token, each
moving (P-1)/P of a rank's slice. On the fully connected xGMI mesh of an MI355X node an all-to-all
uses every point-to-point link at once (unlike a ring), which is why Ulysses, not ring attention,
is the CP scheme picked here. Requires Hkv % P == 0 (Llama-3-8B / 70B: P <= 8).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn.functional as F


# ------------------------------------------------------------------------------ primitives
class _AllToAll(torch.autograd.Function):
    """all_to_all_single over dim 0 (equal splits). Its own inverse, so backward is the same op."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        x = x.contiguous()
        out = torch.empty_like(x)
        dist.all_to_all_single(out, x, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        out = torch.empty_like(g)
        dist.all_to_all_single(out, g, group=ctx.group)
        return out, None


class _ReduceReplicated(torch.autograd.Function):
    """all-reduce (sum) forward; identity backward (the consumer is replicated on every SP rank)."""

    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous().clone()
        dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherReplicated(torch.autograd.Function):
    """all-gather along `dim` forward; backward keeps this rank's slice of the (replicated) grad."""

    @staticmethod
    def forward(ctx, x, group, dim):
        ctx.group, ctx.dim = group, dim
        P, r = dist.get_world_size(group), dist.get_rank(group)
        ctx.P, ctx.r, ctx.n = P, r, x.shape[dim]
        parts = [torch.empty_like(x.contiguous()) for _ in range(P)]
        dist.all_gather(parts, x.contiguous(), group=group)
        return torch.cat(parts, dim)

    @staticmethod
    def backward(ctx, g):
        return g.narrow(ctx.dim, ctx.r * ctx.n, ctx.n).contiguous(), None, None


# ------------------------------------------------------------------------------ SP context
class SequenceParallel:
    """Handle attached to a model (`CausalLM.sp`) and its attention modules."""

    def __init__(self, group):
        self.group = group
        self.size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    # --- layout helpers: full [B, T, ...] tensors (identical on all SP ranks) -> local slices
    def padded_len(self, T: int) -> int:
        return -(-T // self.size) * self.size

    def pad(self, x: Optional[torch.Tensor], value=0) -> Optional[torch.Tensor]:
        """Right-pad dim 1 to a multiple of P (the padding is masked everywhere)."""
        if x is None:
            return None
        extra = self.padded_len(x.shape[1]) - x.shape[1]
        if not extra:
            return x
        pad = [0, 0] * (x.dim() - 2) + [0, extra]
        return F.pad(x, pad, value=value)

    def local(self, x: Optional[torch.Tensor], dim: int = 1) -> Optional[torch.Tensor]:
        """This rank's contiguous chunk of an (already padded) full tensor along `dim`."""
        if x is None:
            return None
        n = x.shape[dim] // self.size
        return x.narrow(dim, self.rank * n, n)

    # --- collectives with replicated-consumer autograd semantics
    def reduce(self, x: torch.Tensor) -> torch.Tensor:
        return _ReduceReplicated.apply(x, self.group)

    def gather(self, x: torch.Tensor, dim: int = 1) -> torch.Tensor:
        return _GatherReplicated.apply(x, self.group, dim)

    # --- Ulysses attention
    def attention(self, qkv: torch.Tensor, Hq: int, Hkv: int, D: int, attn_fn):
        """qkv [B, T/P, (Hq+2Hkv)*D] (local tokens, all heads) -> [B, T/P, Hq*D].
        `attn_fn(qkv_full, hq_local, hkv_local)` runs attention on [B, T, (hq+2hkv)*D]."""
        P = self.size
        if Hq % P or Hkv % P:
            raise ValueError(f"sequence parallel degree {P} must divide the q ({Hq}) and kv ({Hkv}) heads")
        B, Tl, _ = qkv.shape
        hq, hkv = Hq // P, Hkv // P
        q, k, v = qkv.split([Hq * D, Hkv * D, Hkv * D], dim=-1)
        # per destination rank r: [q heads of group r | k heads of r | v heads of r]
        x = torch.cat([q.reshape(B, Tl, P, hq * D), k.reshape(B, Tl, P, hkv * D),
                       v.reshape(B, Tl, P, hkv * D)], dim=-1)
        x = _AllToAll.apply(x.permute(2, 0, 1, 3), self.group)       # [P(seq chunk), B, Tl, c]
        full = x.permute(1, 0, 2, 3).reshape(B, P * Tl, (hq + 2 * hkv) * D)
        a = attn_fn(full, hq, hkv)                                   # [B, T, hq*D]
        a = a.reshape(B, P, Tl, hq * D).permute(1, 0, 2, 3)
        a = _AllToAll.apply(a, self.group)                           # [P(head group), B, Tl, hq*D]
        return a.permute(1, 2, 0, 3).reshape(B, Tl, Hq * D)


def apply_sequence_parallel(model, group, force: bool = False) -> Optional[SequenceParallel]:
    """Attach Ulysses SP over `group` to a CausalLM (or a wrapper with `.backbone`). Weights are
    unchanged (replicated on the SP ranks); returns the handle (None for a 1-rank group unless
    `force`: then the head/sequence all-to-alls run on the one-rank communicator)."""
    if group is None or (dist.get_world_size(group) == 1 and not force):
        return None
    base = getattr(model, "backbone", model)
    sp = SequenceParallel(group)
    cfg = base.cfg
    if cfg.num_heads % sp.size or cfg.num_kv_heads % sp.size:
        raise ValueError(f"sp={sp.size} must divide num_heads={cfg.num_heads} and "
                         f"num_kv_heads={cfg.num_kv_heads}")
    if base.tp is not None:
        raise NotImplementedError("sequence parallel x tensor parallel is not supported")
    base.sp = sp
    for layer in base.layers:
        layer.attn.sp = sp
    return sp


def sp_of(model) -> Optional[SequenceParallel]:
    base = getattr(model, "backbone", model)
    return getattr(base, "sp", None)


def sp_full_hidden(model, h: torch.Tensor, T: int) -> torch.Tensor:
    """Local hidden [B, T/P, H] -> full [B, T, H] (replicated consumer, e.g. a pooled reward head)."""
    sp = sp_of(model)
    if sp is None:
        return h
    return sp.gather(h, dim=1)[:, :T]


def sp_shard_inputs(sp: SequenceParallel, input_ids, attention_mask, segment_ids=None
                    ) -> Tuple[torch.Tensor, Optional[torch.Tensor], Optional[torch.Tensor]]:
    """Pad full inputs to a multiple of P (mask 0 / segment 0 on the padding)."""
    if attention_mask is None and input_ids.shape[1] % sp.size:
        attention_mask = torch.ones_like(input_ids)
    return sp.pad(input_ids), sp.pad(attention_mask), sp.pad(segment_ids)
