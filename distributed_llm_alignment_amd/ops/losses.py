"""Sequence-level alignment objectives as fused HIP epilogue kernels.

Each GPU path is one launch computing loss, gradient coefficients and metrics together (no
host sync); CPU paths are the literal reference formulas:
  * dpo_loss        src/training/train_dpo.py:42-44
  * pairwise_loss   src/models/reward_model.py:67-68
  * kl_penalty_pg   src/training/train_rlhf.py:149-153
  * ensemble_kl     src/training/train_distill.py:127-144
  * gae / ppo_policy_loss / ppo_value_loss: token-level actor-critic PPO (north-star config; the
    reference's REINFORCE above stays the default RLHF algorithm)
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn.functional as F

from . import _ext


# ------------------------------------------------------------------------------------- DPO
class _DPOFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pol, ref, beta, label_smoothing):
        loss, dpol, rewards, metrics = _ext.require().dpo_loss(pol, ref, beta, label_smoothing)
        ctx.save_for_backward(dpol)
        ctx.mark_non_differentiable(rewards, metrics)
        return loss, rewards, metrics

    @staticmethod
    def backward(ctx, gloss, _gr, _gm):
        (dpol,) = ctx.saved_tensors
        return dpol * gloss, None, None, None


def dpo_loss(policy_chosen: torch.Tensor, policy_rejected: torch.Tensor, ref_chosen: torch.Tensor,
             ref_rejected: torch.Tensor, beta: float = 0.1, label_smoothing: float = 0.0
             ) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """-logsigmoid(beta*((pc-pr)-(rc-rr))).mean() (+ optional conservative label smoothing).

    Returns (loss, metrics) where metrics holds device tensors: chosen/rejected implicit
    rewards, reward accuracy and margin (no host sync)."""
    pol = torch.cat([policy_chosen, policy_rejected]).float().contiguous()
    ref = torch.cat([ref_chosen, ref_rejected]).float().detach().contiguous()
    B = policy_chosen.shape[0]
    if _ext.use_native(pol):
        loss, rewards, m = _DPOFn.apply(pol, ref, float(beta), float(label_smoothing))
        metrics = {"rewards/chosen": m[0], "rewards/rejected": m[1], "rewards/accuracy": m[2],
                   "rewards/margin": m[3], "rewards_per_seq": rewards}
        return loss, metrics
    z = beta * ((pol[:B] - pol[B:]) - (ref[:B] - ref[B:]))
    loss = (-(1 - label_smoothing) * F.logsigmoid(z) - label_smoothing * F.logsigmoid(-z)).mean()
    rc = (beta * (pol[:B] - ref[:B])).detach()
    rr = (beta * (pol[B:] - ref[B:])).detach()
    metrics = {"rewards/chosen": rc.mean(), "rewards/rejected": rr.mean(),
               "rewards/accuracy": (rc > rr).float().mean(), "rewards/margin": z.detach().mean(),
               "rewards_per_seq": torch.cat([rc, rr])}
    return loss, metrics


# ------------------------------------------------------------------------------ pairwise RM
class _PairwiseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sc, sr):
        loss, dsc, dsr, acc = _ext.require().pairwise_loss(sc, sr)
        ctx.save_for_backward(dsc, dsr)
        ctx.mark_non_differentiable(acc)
        return loss, acc

    @staticmethod
    def backward(ctx, gloss, _gacc):
        dsc, dsr = ctx.saved_tensors
        return dsc * gloss, dsr * gloss


def pairwise_loss(chosen_scores: torch.Tensor, rejected_scores: torch.Tensor,
                  return_accuracy: bool = False):
    """Bradley-Terry: -logsigmoid(s_c - s_r).mean()."""
    sc = chosen_scores.float().contiguous()
    sr = rejected_scores.float().contiguous()
    if _ext.use_native(sc):
        loss, acc = _PairwiseFn.apply(sc, sr)
    else:
        loss = -F.logsigmoid(sc - sr).mean()
        acc = (sc > sr).float().mean().detach()
    return (loss, acc) if return_accuracy else loss


# ------------------------------------------------------------------- REINFORCE + KL penalty
class _KLPGFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lp, lr, reward, kl_coef):
        loss, klm, dlp, adv = _ext.require().kl_penalty_pg(lp, lr, reward, kl_coef)
        ctx.save_for_backward(dlp)
        ctx.mark_non_differentiable(klm, adv)
        return loss, klm, adv

    @staticmethod
    def backward(ctx, gloss, _gk, _ga):
        (dlp,) = ctx.saved_tensors
        return dlp * gloss, None, None, None


def kl_penalty_pg(policy_logp: torch.Tensor, ref_logp: torch.Tensor, reward: torch.Tensor,
                  kl_coef: float = 0.1):
    """kl = lp - lr; r' = r - c*kl; A = r' - mean(r'); loss = -mean(stopgrad(A) * lp).

    Returns (loss, kl_mean, advantages)."""
    lp = policy_logp.float().contiguous()
    lr = ref_logp.float().detach().contiguous()
    r = reward.float().detach().contiguous()
    if _ext.use_native(lp):
        return _KLPGFn.apply(lp, lr, r, float(kl_coef))
    kl = lp.detach() - lr
    shaped = r - kl_coef * kl
    adv = shaped - shaped.mean()
    loss = -(adv * lp).mean()
    return loss, kl.mean(), adv


# ----------------------------------------------------------------- ensemble-KL distillation
class _EnsembleKLFn(torch.autograd.Function):
    """KL(p_bar || q) per row from student logits [N, V] and K teacher logits [K, N, V]."""

    @staticmethod
    def forward(ctx, s_logits, t_logits):
        ops = _ext.require()
        s_lse = ops.row_lse(s_logits)
        K, N, V = t_logits.shape
        t_lse = ops.row_lse(t_logits.view(K * N, V)).view(K, N)
        kl = ops.ensemble_kl(s_logits, t_logits, s_lse, t_lse, None, False)  # read-only here
        ctx.save_for_backward(s_logits, t_logits, s_lse, t_lse)
        return kl

    @staticmethod
    def backward(ctx, g):
        ops = _ext.require()
        s_logits, t_logits, s_lse, t_lse = ctx.saved_tensors
        ds = s_logits.clone()
        ops.ensemble_kl(ds, t_logits, s_lse, t_lse, g.float().contiguous(), True)
        return ds, None


def ensemble_kl(student_logits: torch.Tensor, teacher_logits: torch.Tensor) -> torch.Tensor:
    """student [N, V], teachers [K, N, V] (same vocab) -> per-row KL(mean_k p_k || q) [N]."""
    if _ext.use_native(student_logits):
        return _EnsembleKLFn.apply(student_logits.contiguous(), teacher_logits.contiguous().detach())
    logq = F.log_softmax(student_logits.float(), dim=-1)
    pbar = torch.softmax(teacher_logits.float(), dim=-1).mean(0)
    return F.kl_div(logq, pbar, reduction="none").sum(-1)


# ------------------------------------------------------------- PPO (actor-critic) objectives
# Token-level PPO for the north-star "PPO RLHF (actor + critic + reward)" configuration; the
# reference's sequence-level REINFORCE (train_rlhf.py:149-153, `kl_penalty_pg` above) stays the
# default algorithm. [S, T] fp32 grids; `mask` selects action tokens.
def gae(rewards: torch.Tensor, values: torch.Tensor, mask: torch.Tensor, gamma: float = 1.0,
        lam: float = 0.95):
    """Generalised advantage estimation (no gradient):
    A_t = m_t (delta_t + gamma lam m_{t+1} A_{t+1}), delta_t = r_t + gamma m_{t+1} V_{t+1} - V_t.
    Returns (advantages, returns = A + V)."""
    r = rewards.detach().float().contiguous()
    v = values.detach().float().contiguous()
    m = mask.detach().float().contiguous()
    if _ext.use_native(r):
        return _ext.require().gae(r, v, m, float(gamma), float(lam))
    S, T = r.shape
    adv = torch.zeros_like(r)
    nxt = torch.zeros(S, dtype=r.dtype, device=r.device)
    zero = torch.zeros_like(nxt)
    for t in range(T - 1, -1, -1):
        mn = m[:, t + 1] if t + 1 < T else zero
        vn = v[:, t + 1] if t + 1 < T else zero
        delta = r[:, t] + gamma * mn * vn - v[:, t]
        nxt = m[:, t] * (delta + gamma * lam * mn * nxt)
        adv[:, t] = nxt
    return adv, adv + v


class _PPOPolicyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lp, old, adv, mask, eps):
        loss, dlp, metrics = _ext.require().ppo_policy_loss(lp, old, adv, mask, eps)
        ctx.save_for_backward(dlp)
        ctx.mark_non_differentiable(metrics)
        return loss, metrics

    @staticmethod
    def backward(ctx, gloss, _gm):
        (dlp,) = ctx.saved_tensors
        return dlp * gloss, None, None, None, None


def ppo_policy_loss(logp: torch.Tensor, old_logp: torch.Tensor, advantages: torch.Tensor,
                    mask: torch.Tensor, clip_eps: float = 0.2):
    """Clipped surrogate, mean over masked tokens of max(-A rho, -A clip(rho, 1 +- eps)),
    rho = exp(logp - old_logp). Returns (loss, {clipfrac, approx_kl}) (device tensors)."""
    lp = logp.float().contiguous()
    old = old_logp.detach().float().contiguous()
    a = advantages.detach().float().contiguous()
    m = mask.detach().float().contiguous()
    if _ext.use_native(lp):
        loss, met = _PPOPolicyFn.apply(lp, old, a, m, float(clip_eps))
        return loss, {"clipfrac": met[0], "approx_kl": met[1]}
    n = m.sum().clamp(min=1)
    rho = torch.exp(lp - old)
    per = torch.maximum(-a * rho, -a * rho.clamp(1 - clip_eps, 1 + clip_eps))
    loss = (per * m).sum() / n
    with torch.no_grad():
        clipfrac = (((rho - 1).abs() > clip_eps).float() * m).sum() / n
        akl = (((rho - 1) - (lp - old)) * m).sum() / n
    return loss, {"clipfrac": clipfrac, "approx_kl": akl}


class _PPOValueFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, val, old, ret, mask, clip):
        loss, dval = _ext.require().ppo_value_loss(val, old, ret, mask, clip)
        ctx.save_for_backward(dval)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dval,) = ctx.saved_tensors
        return dval * g, None, None, None, None


def ppo_value_loss(values: torch.Tensor, old_values: torch.Tensor, returns: torch.Tensor,
                   mask: torch.Tensor, clip: float = 0.2) -> torch.Tensor:
    """0.5 * masked mean of max((V - R)^2, (V_clip - R)^2), V_clip = V_old + clamp(V - V_old, +-c)."""
    v = values.float().contiguous()
    old = old_values.detach().float().contiguous()
    R = returns.detach().float().contiguous()
    m = mask.detach().float().contiguous()
    if _ext.use_native(v):
        return _PPOValueFn.apply(v, old, R, m, float(clip))
    n = m.sum().clamp(min=1)
    vc = old + (v - old).clamp(-clip, clip)
    return 0.5 * (torch.maximum((v - R) ** 2, (vc - R) ** 2) * m).sum() / n
