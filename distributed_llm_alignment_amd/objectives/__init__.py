"""Training objectives (SURVEY layer L5), each a pure function of (models, batch) so trainers,
benchmarks and tests share one implementation.

  dpo_step_loss    reference train_dpo.py:106-121 (length-normalised seq log-probs, DPO loss)
  sft_loss         reference train_sft.py:145-146 (HF causal-LM CE, ignore -100)
  reward_loss      reference train_reward.py:139-148 (Bradley-Terry pairwise)
  rlhf_loss        reference train_rlhf.py:127-153 (REINFORCE with KL-shaped reward)
  ppo_rollout_stats / ppo_loss  token-level actor-critic PPO (GAE, clipped surrogate + value
                   loss) for `ppo.algorithm: ppo` (north-star config; not in the reference)
  distill_loss     reference train_distill.py:125-147 (CE on rollouts or ensemble forward KL)
"""
from __future__ import annotations

import os
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
    from ..models.transformer import sp_seq_reduce

    h = model(ids, mask)
    tgt, m = model._sp_targets(*ops.shifted_targets(ids, loss_mask))
    lp = model._masked_token_logprob(h, tgt)
    return sp_seq_reduce(model.sp, lp, m, reduction == "mean")


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


def ref_sequence_logps(ref, batch, reduction: str = "mean", pad_id: int = 0):
    """The frozen reference's per-sequence log-probs for a preference batch ([2B]: chosen, rejected)."""
    ids, mask, lm = concat_pair(batch, pad_id)
    with torch.no_grad():
        return sequence_logps(ref, ids, mask, reduction, lm)


class RefLogpsStream:
    """Runs the frozen reference forward on a second HIP stream so it overlaps the policy's
    forward/backward on the main stream (the two are independent until the DPO loss). The ref
    pass is GEMM-light relative to its memory-bound phases (attention, norms, SwiGLU) and the
    policy's are the same: interleaving the two streams fills the gaps each leaves on the CUs.
    `submit(batch)` returns a handle; `result(handle)` makes the main stream wait for it.
    On CPU (or with enabled=False) it simply computes inline."""

    def __init__(self, ref, reduction: str = "mean", pad_id: int = 0, enabled: bool = True):
        self.ref, self.reduction, self.pad_id = ref, reduction, pad_id
        dev = next(ref.parameters()).device
        self.stream = torch.cuda.Stream(device=dev) if (enabled and dev.type == "cuda") else None

    def submit(self, batch):
        if self.stream is None:
            return ref_sequence_logps(self.ref, batch, self.reduction, self.pad_id), None
        main = torch.cuda.current_stream(self.stream.device)
        self.stream.wait_stream(main)  # batch tensors were produced on the main stream
        with torch.cuda.stream(self.stream):
            lp = ref_sequence_logps(self.ref, batch, self.reduction, self.pad_id)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return lp, ev

    def result(self, handle):
        lp, ev = handle
        if ev is not None:
            main = torch.cuda.current_stream(lp.device)
            main.wait_event(ev)
            lp.record_stream(main)
        return lp


def sft_loss(model, batch) -> torch.Tensor:
    return model.causal_lm_loss(batch["input_ids"], batch["labels"], batch.get("attention_mask"),
                                batch.get("segment_ids"))


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


def action_mask(mask: torch.Tensor, prompt_len: int) -> torch.Tensor:
    """[S, T] fp32: 1 at grid positions t whose action (token t + 1) is a generated, valid token
    (prompt tokens and padding after EOS are not actions)."""
    S, T = mask.shape
    act = torch.zeros((S, T), dtype=torch.float32, device=mask.device)
    gen = (torch.arange(1, T, device=mask.device) >= prompt_len).float()
    act[:, :-1] = mask[:, 1:].float() * gen
    return act


@torch.no_grad()
def ppo_rollout_stats(policy, ref, critic, seqs, mask, prompt_len: int, scores, kl_coef: float = 0.1,
                      gamma: float = 1.0, lam: float = 0.95, whiten: bool = True):
    """Token-level PPO targets for one batch of rollouts (actor-critic; the north-star
    "PPO RLHF (actor + critic + reward)" config). Per-token reward = -kl_coef * (logp - logp_ref)
    on every action, plus the reward-model score on the last action; GAE(gamma, lam) over the
    critic's values; advantages whitened over the action tokens."""
    old_lp = policy.token_logprobs(seqs, mask)
    ref_lp = ref.token_logprobs(seqs, mask)
    values = critic(seqs, mask)
    act = action_mask(mask, prompt_len)
    kl = (old_lp - ref_lp) * act
    rewards = -kl_coef * kl
    S, T = act.shape
    last = (act * torch.arange(T, device=act.device, dtype=act.dtype)).argmax(1)
    has = act.sum(1) > 0
    rewards[torch.arange(S, device=act.device), last] += torch.where(has, scores.float(), torch.zeros_like(scores.float()))
    adv, ret = ops.gae(rewards, values, act, gamma, lam)
    if whiten:
        n = act.sum().clamp(min=1)
        mu = (adv * act).sum() / n
        var = (((adv - mu) ** 2) * act).sum() / n
        adv = (adv - mu) * torch.rsqrt(var + 1e-8) * act
    return {"old_logp": old_lp, "values": values, "advantages": adv, "returns": ret, "act": act,
            "kl": kl.sum(1) / act.sum(1).clamp(min=1), "scores": scores.float()}


# The actor and the critic of a PPO minibatch are independent until the summed loss: the critic's
# forward (and, through autograd's per-node streams, its backward) runs on a side stream so the two
# models' kernels share the chip. At the PPO shapes (4 rollouts x 768 tokens per minibatch) the
# o / down projections are [3072, 4096] outputs = 192 256x256 tiles for 256 CUs, so one model alone
# leaves a quarter of the CUs idle in every such GEMM. DLA_PPO_CRITIC_STREAM=0: one stream.
PPO_CRITIC_STREAM = os.environ.get("DLA_PPO_CRITIC_STREAM", "1") != "0"
_CRITIC_STREAMS: Dict[int, "torch.cuda.Stream"] = {}


def ppo_critic_stream(device: torch.device):
    """The side stream the critic runs on (None off the GPU or when disabled)."""
    if not (PPO_CRITIC_STREAM and device.type == "cuda"):
        return None
    i = device.index if device.index is not None else torch.cuda.current_device()
    if i not in _CRITIC_STREAMS:
        _CRITIC_STREAMS[i] = torch.cuda.Stream(device=i)
    return _CRITIC_STREAMS[i]


def ppo_loss(policy, critic, seqs, mask, stats: Dict[str, torch.Tensor], clip_eps: float = 0.2,
             value_clip: float = 0.2, vf_coef: float = 0.1):
    """Clipped surrogate (HIP fused fwd+bwd) + vf_coef * clipped value loss on one minibatch.
    Run its backward through `ppo_backward` (joins the critic's stream afterwards)."""
    cs = ppo_critic_stream(seqs.device)
    main = torch.cuda.current_stream(seqs.device) if cs is not None else None
    if cs is not None:
        cs.wait_stream(main)  # the critic's weights (last optimizer step) and this minibatch
        with torch.cuda.stream(cs):
            v = critic(seqs, mask)
            vl = ops.ppo_value_loss(v, stats["values"], stats["returns"], stats["act"], value_clip)
    lp = policy.token_logprobs(seqs, mask)
    pl, pm = ops.ppo_policy_loss(lp, stats["old_logp"], stats["advantages"], stats["act"], clip_eps)
    if cs is None:
        v = critic(seqs, mask)
        vl = ops.ppo_value_loss(v, stats["values"], stats["returns"], stats["act"], value_clip)
    else:
        main.wait_stream(cs)
        vl.record_stream(main)
    return pl + vf_coef * vl, {"policy_loss": pl.detach(), "value_loss": vl.detach(), **pm}


def ppo_backward(loss: torch.Tensor) -> None:
    """loss.backward() for `ppo_loss`: the critic's backward nodes run on its side stream and its
    weight gradients are accumulated there (GEMM-epilogue main_grad writes that autograd does not
    order against the caller's stream), so the caller's stream waits for that stream before the
    optimizer steps read the gradient buffers."""
    loss.backward()
    cs = ppo_critic_stream(loss.device)
    if cs is not None:
        torch.cuda.current_stream(loss.device).wait_stream(cs)


# Tokens per ensemble-KL chunk: (teachers + 1) x chunk x V bf16 logits exist at a time
# (V = 51200, 2 teachers, 1024 tokens: 315 MB) instead of [K, S, T, V] for the whole batch.
KL_CHUNK_TOKENS = int(os.environ.get("DLA_KL_CHUNK_TOKENS", "1024"))


def _kl_chunk(student, teachers, hs_c, ths_c):
    s_logits = student.logits(hs_c)
    with torch.no_grad():
        t_logits = torch.stack([t.logits(h) for t, h in zip(teachers, ths_c)])
    return ops.ensemble_kl(s_logits, t_logits)


def chunked_ensemble_kl(student, teachers: Sequence, hs: torch.Tensor, ths: Sequence[torch.Tensor],
                        chunk: Optional[int] = None) -> torch.Tensor:
    """Per-token forward KL(mean_k softmax(teacher_k) || softmax(student)) from final hidden rows
    (student hs [N, H] with grad, teacher hidden [N, H] each), token-chunked: each chunk's
    student and teacher logits are produced by the LM-head GEMMs, reduced by the fused HIP
    ensemble-KL kernel and dropped; the backward recomputes the chunk (activation checkpoint), so
    neither [K, N, V] teacher logits nor [N, V] student logits are ever materialised whole
    (reference: src/training/train_distill.py:130-144 stacks all teacher logits)."""
    from torch.utils.checkpoint import checkpoint

    chunk = int(chunk or KL_CHUNK_TOKENS)
    N = hs.shape[0]
    outs = []
    for i in range(0, N, chunk):
        hs_c = hs[i:i + chunk]
        ths_c = [h[i:i + chunk] for h in ths]
        if torch.is_grad_enabled() and hs.requires_grad and N > chunk:
            outs.append(checkpoint(_kl_chunk, student, teachers, hs_c, ths_c, use_reentrant=False))
        else:
            outs.append(_kl_chunk(student, teachers, hs_c, ths_c))
    return outs[0] if len(outs) == 1 else torch.cat(outs)


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
    with torch.no_grad():
        ths = [t(ids, mask) for t in teachers]  # teacher hidden states only: [S, T, H] each
    S, T = hs.shape[0], hs.shape[1]
    kl = chunked_ensemble_kl(student, teachers, hs.reshape(S * T, -1),
                             [h.reshape(S * T, -1) for h in ths]).view(S, T)
    sp = student.sp
    if sp is None:
        m = mask.float()
        return (kl * m).sum() / m.sum()
    m = sp.local(sp.pad(mask.float(), 0))  # sequence parallel: this rank's token slice
    return sp.reduce((kl * m).sum()) / sp.reduce(m.sum())
