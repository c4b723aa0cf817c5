"""Collective bytes one rank sends per optimizer step of the DPO job, per mesh (analytic).

The one-GPU shape benches (`bench.py --tp-shape / --fsdp-shape / --ep-shape / --edp-shape`) time a
rank's compute with local stand-ins for the collectives; this prices what those stand-ins skip:
the bytes each rank puts on xGMI per step, split by collective, so a mesh's per-rank step time
can be read against the link time it must hide (7 links x ~153 GB/s per MI355X; a ring collective
is bound by one link per hop).

Ring costs per rank (bf16 payloads): all-reduce 2 (n-1)/n x bytes, all-gather / reduce-scatter
(n-1)/n x (full) bytes, all-to-all (n-1)/n x bytes. One DPO micro-batch = policy forward +
backward on chosen and rejected, plus the frozen reference forward (the reference is sharded
like the policy: TP-split, or ZeRO-3 units gathered for its forward).
"""
from __future__ import annotations

from typing import Dict


def _ring(n: int) -> float:
    return (n - 1) / n if n > 1 else 0.0


def dpo_comm_bytes(cfg, seq_len: int, micro_pairs: int, accum: int, tp: int = 1, fsdp: int = 1,
                   dp: int = 1, ep: int = 1, edp: int = 1, ep_capacity: float = 1.25,
                   tp_seq: bool = False) -> Dict[str, float]:
    """Bytes sent per rank per optimizer step, by collective. `dp` = data-parallel replicas the
    ZeRO-1 gradient reduce spans (the FSDP group is `fsdp`); MoE: `ep` x `edp` ranks."""
    B2 = 2  # bf16
    H, L, V = cfg.hidden_size, cfg.num_layers, cfg.vocab_size
    T = 2 * micro_pairs * seq_len  # tokens of one micro-batch (chosen + rejected)
    n_params = cfg.num_params()
    out: Dict[str, float] = {}
    # ---- tensor parallel: per layer 2 forward all-reduces (o, down) for the policy AND the
    # reference, 2 backward all-reduces of the column-parallel input grads; the vocab-parallel
    # embedding all-reduce (policy + ref) and the log-prob dh all-reduce. Megatron-SP sends the
    # same ring bytes as reduce-scatter + all-gather pairs.
    if tp > 1:
        act = T * H * B2
        n_ar = 6 * L + 3
        out["tp_allreduce"] = accum * n_ar * 2 * _ring(tp) * act
    local_params = n_params / tp
    if cfg.is_moe and ep > 1:
        # expert weights split over ep, dense weights replicated
        E = cfg.num_experts
        exp_params = L * E * 3 * cfg.intermediate_size * H
        local_params = (n_params - exp_params) + exp_params / ep
        k = cfg.num_experts_per_tok
        C = ep_capacity * T * k / ep  # rows per (source, destination) block
        a2a = ep * C * H * B2
        # dispatch + return, forward (policy + ref) and backward (policy)
        out["ep_all_to_all"] = accum * L * 6 * _ring(ep) * a2a
        out["edp_grad_reduce"] = 2 * _ring(edp) * exp_params / ep * B2  # RS + AG over replicas
        dense = n_params - exp_params
        out["dp_grad_reduce"] = 2 * _ring(ep * edp) * dense * B2
        return out
    if fsdp > 1:
        # ZeRO-3: per micro-batch the policy units are gathered for the forward and again for the
        # backward, their grads reduce-scattered, and the reference units gathered once
        out["fsdp_allgather"] = accum * 3 * _ring(fsdp) * local_params * B2
        out["fsdp_reduce_scatter"] = accum * _ring(fsdp) * local_params * B2
    if dp > 1:
        out["dp_grad_reduce"] = 2 * _ring(dp) * local_params * B2  # ZeRO-1 RS + AG once per step
    return out
