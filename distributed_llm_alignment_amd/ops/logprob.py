"""Fused LM-head log-probabilities (SURVEY K9 + K10 + K11 + K16).

`linear_logprob(hidden, weight, targets)` = log_softmax(hidden @ W^T)[targets] per row without
ever materialising fp32 [N, V] tensors:
  * forward: one hipBLASLt GEMM -> bf16 logits; the HIP row kernel streams each logits row once
    (online max/sum) and emits logp + lse (fp32, per row).
  * backward: the HIP kernel rewrites the SAVED bf16 logits in place into dlogits
    (g * (onehot - softmax)), which feed the two grad GEMMs directly (dH = dL W, dW = dL^T H);
    with a main_grad on the LM head the same kernel also writes dL^T, the TN weight-gradient
    operand, so no separate transpose pass re-reads the [N, V] gradient.
    With grads off (frozen reference / reward scoring) logits are produced chunk by chunk and
    dropped, so the no-grad footprint is one chunk.
Semantics mirror the reference `compute_logprobs` (src/training/train_dpo.py:31-39): logits in
the model dtype (bf16), log-softmax in fp32, targets < 0 ignored (logp 0, no gradient).

`sequence_logprob(...)` adds the masked per-sequence reduction (length-normalised mean by default,
exactly the reference's `/ mask.sum(1).clamp(min=1)`, or sum) as a HIP kernel pair.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import _ext
from .linear import input_grad

# no-grad (frozen reference) logits are produced and dropped per chunk of rows: 8192 rows x the
# Llama-3 vocabulary is a 2.1 GB bf16 transient, one GEMM per DPO micro-batch (two 4096-row
# chunks ran 2 x 2.93 ms vs 5.5 ms for the one 8192-row GEMM in the step, profiles/r6_*)
_NO_GRAD_CHUNK = 8192
# dlogits^T from the logprob backward kernel (A/B switch, read once)
LOGPROB_T = os.environ.get("DLA_LOGPROB_T", "1") != "0"


def _ref_linear_logprob(hidden, weight, targets):
    logits = F.linear(hidden, weight).float()
    lse = torch.logsumexp(logits, dim=-1)
    safe = targets.clamp(min=0)
    lp = logits.gather(-1, safe.unsqueeze(-1)).squeeze(-1) - lse
    return torch.where(targets >= 0, lp, torch.zeros_like(lp))


class _LinearLogprobFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hidden, weight, targets):
        ops = _ext.require()
        need_grad = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        N = hidden.shape[0]
        if need_grad:
            logits = F.linear(hidden, weight)
            logp, lse = ops.logprob_fwd(logits, targets)
            ctx.save_for_backward(hidden, targets, lse, logits)
            ctx.weight = weight  # (on ctx: see ops.linear._LinearMainGradFn)
            return logp
        logp = torch.empty(N, dtype=torch.float32, device=hidden.device)
        for s in range(0, N, _NO_GRAD_CHUNK):
            e = min(N, s + _NO_GRAD_CHUNK)
            lg = F.linear(hidden[s:e], weight)
            lp, _ = ops.logprob_fwd(lg, targets[s:e])
            logp[s:e] = lp
        return logp

    @staticmethod
    def backward(ctx, g):
        ops = _ext.require()
        hidden, targets, lse, logits = ctx.saved_tensors
        weight = ctx.weight
        from .linear import _tn_ok, accumulate_weight_grad

        g = g.float().contiguous()
        dlt = None
        mg = getattr(weight, "main_grad", None)
        if (LOGPROB_T and ctx.needs_input_grad[1] and mg is not None and not getattr(weight, "_dla_shared", False)
                and _tn_ok(mg, logits.shape[0])):
            # the LM head's weight gradient runs as a TN GEMM on dlogits^T: write it from the
            # same pass that turns the logits into dlogits (undefined when the shape is outside
            # the kernel -> in-place kernel + transpose inside accumulate_weight_grad)
            dlt = ops.logprob_bwd_t(logits, targets, lse, g)
            if not dlt.numel():
                dlt = None
        if dlt is None:
            ops.logprob_bwd(logits, targets, lse, g)
        dlogits = logits  # rewritten in place
        dh = input_grad(dlogits, weight) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            if not accumulate_weight_grad(weight, dlogits, hidden, dyt=dlt):
                dw = dlogits.t() @ hidden
        return dh, dw, None


def linear_logprob(hidden: torch.Tensor, weight: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
    """hidden [N, H], weight [V, H], targets [N] (int64, <0 = ignore) -> logp [N] fp32."""
    if _ext.use_native(hidden):
        return _LinearLogprobFn.apply(hidden.contiguous(), weight, targets.contiguous())
    return _ref_linear_logprob(hidden, weight, targets)


class _SeqReduceFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lp, mask, mean):
        ops = _ext.require()
        s, cnt = ops.seq_reduce(lp, mask)
        ctx.save_for_backward(mask, cnt)
        ctx.mean = mean
        return s / cnt.clamp(min=1.0) if mean else s

    @staticmethod
    def backward(ctx, g):
        mask, cnt = ctx.saved_tensors
        return _ext.require().seq_expand_grad(g.float().contiguous(), mask, cnt, ctx.mean), None, None


def seq_reduce(token_lp: torch.Tensor, mask: torch.Tensor, mean: bool = True) -> torch.Tensor:
    """token_lp [S, T] fp32, mask [S, T] -> masked mean (or sum) over T."""
    mask = mask.float().contiguous()
    if _ext.use_native(token_lp):
        return _SeqReduceFn.apply(token_lp.contiguous(), mask, mean)
    s = (token_lp * mask).sum(dim=1)
    return s / mask.sum(dim=1).clamp(min=1) if mean else s


def shifted_targets(input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor],
                    ignore_index: int = -100):
    """targets[t] = input_ids[t+1]; last position ignored. mask[t] = am[t] * am[t+1].

    For right padding this equals the reference's `attention_mask[:, 1:]`; for left padding it
    also drops the pad -> first-token "prediction" the reference would score (its query row
    sees no valid keys)."""
    S, T = input_ids.shape
    tgt = torch.full_like(input_ids, ignore_index)
    tgt[:, :-1] = input_ids[:, 1:]
    mask = torch.zeros((S, T), dtype=torch.float32, device=input_ids.device)
    if attention_mask is None:
        mask[:, :-1] = 1.0
    else:
        am = attention_mask.float()
        mask[:, :-1] = am[:, 1:] * am[:, :-1]
    tgt = torch.where(mask > 0, tgt, torch.full_like(tgt, ignore_index))
    return tgt, mask


def sequence_logprob(hidden: torch.Tensor, weight: torch.Tensor, input_ids: torch.Tensor,
                     attention_mask: Optional[torch.Tensor] = None,
                     reduction: str = "mean") -> torch.Tensor:
    """Per-sequence log p(x_{t+1} | x_<=t) reduced over valid positions.

    hidden [S, T, H] final hidden states (after the final norm), weight [V, H] LM head.
    reduction 'mean' reproduces the reference's length-normalised `compute_logprobs`.
    """
    S, T, H = hidden.shape
    tgt, mask = shifted_targets(input_ids, attention_mask)
    lp = linear_logprob(hidden.reshape(S * T, H), weight, tgt.reshape(-1)).view(S, T)
    return seq_reduce(lp, mask, mean=(reduction == "mean"))


def token_nll(hidden: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """HF ForCausalLMLoss: mean over labels != -100 of -log p(labels[t+1] | x_<=t)."""
    S, T, H = hidden.shape
    tgt = torch.full_like(labels, -100)
    tgt[:, :-1] = labels[:, 1:]
    tgt = tgt.reshape(-1)
    lp = linear_logprob(hidden.reshape(S * T, H), weight, tgt)
    n = (tgt >= 0).sum().clamp(min=1)
    return -(lp.sum() / n)
