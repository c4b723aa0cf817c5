"""Training objectives (SURVEY layer L5), each a pure function of (models, batch) so trainers,
benchmarks and tests share one implementation.

  dpo_step_loss    reference train_dpo.py:106-121 (length-normalised seq log-probs, DPO loss)
  sft_loss         reference train_sft.py:145-146 (HF causal-LM CE, ignore -100)
  reward_loss      reference train_reward.py:139-148 (Bradley-Terry pairwise)
  rlhf_loss        reference train_rlhf.py:127-153 (REINFORCE with KL-shaped reward)
  distill_loss     reference train_distill.py:125-147 (CE on rollouts or ensemble forward KL)
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from .. import ops


def concat_pair(batch: Dict[str, Dict[str, torch.Tensor]], pad_id: int = 0):
    """Stack chosen and rejected into one [2B, T] batch (one forward instead of two; the math is
    per-sequence so this is identical to the reference's separate forwards)."""
    c, r = batch["chosen"], batch["rejected"]
    T = max(c["input_ids"].shape[1], r["input_ids"].shape[1])

    def pad(x, v):
        return F.pad(x, (0, T - x.shape[1]), value=v)

    ids = torch.cat([pad(c["input_ids"], pad_id), pad(r["input_ids"], pad_id)])
    mask = torch.cat([pad(c["attention_mask"], 0), pad(r["attention_mask"], 0)])
    loss_mask = None
    if "loss_mask" in c:
        loss_mask = torch.cat([pad(c["loss_mask"], 0), pad(r["loss_mask"], 0)])
    return ids, mask, loss_mask


def sequence_logps(model, ids, mask, reduction: str = "mean", loss_mask=None):
    """Per-sequence log-prob; `loss_mask` (optional) restricts scoring to response tokens."""
    if loss_mask is None:
        return model.sequence_logprob(ids, mask, reduction)
    h = model(ids, mask)
    tgt, m = ops.shifted_targets(ids, loss_mask)
    S, T, H = h.shape
    lp = ops.linear_logprob(h.reshape(S * T, H), model.head_weight, tgt.reshape(-1)).view(S, T)
    return ops.seq_reduce(lp, m, mean=(reduction == "mean"))


def dpo_step_loss(policy, ref, batch, beta: float = 0.1, label_smoothing: float = 0.0,
                  reduction: str = "mean", ref_logps: Optional[torch.Tensor] = None, pad_id: int = 0):
    ids, mask, lm = concat_pair(batch, pad_id)
    B = ids.shape[0] // 2
    pol = sequence_logps(policy, ids, mask, reduction, lm)
    if ref_logps is None:
        with torch.no_grad():
            ref_logps = sequence_logps(ref, ids, mask, reduction, lm)
    loss, metrics = ops.dpo_loss(pol[:B], pol[B:], ref_logps[:B], ref_logps[B:], beta, label_smoothing)
    metrics["policy_chosen_logps"] = pol[:B].detach()
    metrics["policy_rejected_logps"] = pol[B:].detach()
    return loss, metrics


def sft_loss(model, batch) -> torch.Tensor:
    return model.causal_lm_loss(batch["input_ids"], batch["labels"], batch.get("attention_mask"))


def reward_loss(rm, batch, pad_id: int = 0):
    ids, mask, _ = concat_pair(batch, pad_id)
    B = ids.shape[0] // 2
    scores = rm(ids, mask)
    loss, acc = ops.pairwise_loss(scores[:B], scores[B:], return_accuracy=True)
    return loss, {"accuracy": acc, "chosen_scores": scores[:B].detach(), "rejected_scores": scores[B:].detach()}


def rlhf_loss(policy, ref, seqs, mask, rewards, kl_coef: float = 0.1):
    pol = policy.sequence_logprob(seqs, mask, "mean")
    with torch.no_grad():
        ref_lp = ref.sequence_logprob(seqs, mask, "mean")
    loss, kl_mean, adv = ops.kl_penalty_pg(pol, ref_lp, rewards, kl_coef)
    return loss, {"kl": kl_mean, "advantages": adv, "policy_logps": pol.detach()}


def distill_loss(student, teachers: Sequence, batch, use_kl: bool):
    """CE on teacher rollouts (labels = input_ids) or token-masked ensemble forward-KL. KL mode
    compares every position (unshifted), as the reference does (train_distill.py:140-144)."""
    if not (use_kl and teachers):
        return student.causal_lm_loss(batch["input_ids"], batch["labels"], batch.get("attention_mask"))
    ids, mask = batch["input_ids"], batch["attention_mask"]
    for t in teachers:
        if t.cfg.vocab_size != student.cfg.vocab_size:
            raise ValueError("KL distillation requires teacher and student to share a vocabulary "
                             "(SURVEY Appendix A #15)")
    hs = student(ids, mask)
    s_logits = student.logits(hs)
    with torch.no_grad():
        t_logits = torch.stack([t.logits(t(ids, mask)) for t in teachers])
    S, T, V = s_logits.shape
    kl = ops.ensemble_kl(s_logits.reshape(S * T, V), t_logits.reshape(len(teachers), S * T, V)).view(S, T)
    m = mask.float()
    return (kl * m).sum() / m.sum()
