"""`ppo.update_micro_batch` (training/train_rlhf.py reinforce_update): the micro-batched update is
the gradient of per-micro-batch baselines weighted by their share of the rollouts -- what the
reference's multi-process run computes (per-process `rewards.mean()`, DDP average) -- and with
micro = 0 it is the plain full-batch `rlhf_loss` backward."""
import contextlib

import torch

from distributed_llm_alignment_amd.models import build_model, get_config
from distributed_llm_alignment_amd.objectives import rlhf_loss
from distributed_llm_alignment_amd.training.train_rlhf import reinforce_update


class _Eng:
    def no_sync(self):
        return contextlib.nullcontext()


def _grads(m):
    out = [p.grad.detach().clone() for p in m.parameters() if p.grad is not None]
    m.zero_grad(set_to_none=True)
    return out


def _close(a, b):
    return all(torch.allclose(x, y, rtol=1e-4, atol=1e-6) for x, y in zip(a, b))


def test_micro_batched_reinforce_update_matches_per_rank_baselines():
    cfg = get_config("tiny-llama")
    pol = build_model(cfg, device="cpu", seed=0)
    ref = build_model(cfg, device="cpu", seed=1).requires_grad_(False)
    g = torch.Generator().manual_seed(0)
    seqs = torch.randint(3, cfg.vocab_size, (4, 24), generator=g)
    mask = torch.ones_like(seqs)
    mask[1, :5] = 0
    scores = torch.randn(4, generator=g)

    # micro = 2: two "ranks" of 2 rollouts, each with its own baseline, averaged
    loss, m = reinforce_update(pol, ref, _Eng(), seqs, mask, scores, 0.1, 2)
    g_micro = _grads(pol)
    parts = []
    for sl in (slice(0, 2), slice(2, 4)):
        l, mm = rlhf_loss(pol, ref, seqs[sl], mask[sl], scores[sl], 0.1)
        (0.5 * l).backward()
        parts.append((l.detach(), mm["kl"]))
    assert _close(g_micro, _grads(pol))
    assert torch.allclose(loss, 0.5 * (parts[0][0] + parts[1][0]))
    assert torch.allclose(m["kl"], 0.5 * (parts[0][1] + parts[1][1]))

    # ragged split (3 + 1): the 1-rollout tail would have a zero advantage on its own, so it is
    # folded into the previous micro-batch -> one micro-batch of 4 (= the full-batch loss)
    reinforce_update(pol, ref, _Eng(), seqs, mask, scores, 0.1, 3)
    g_uneven = _grads(pol)
    rlhf_loss(pol, ref, seqs, mask, scores, 0.1)[0].backward()
    assert _close(g_uneven, _grads(pol))

    # micro = 0 (and micro >= batch): the full-batch loss with one baseline
    reinforce_update(pol, ref, _Eng(), seqs, mask, scores, 0.1, 0)
    g_full = _grads(pol)
    rlhf_loss(pol, ref, seqs, mask, scores, 0.1)[0].backward()
    assert _close(g_full, _grads(pol))
    reinforce_update(pol, ref, _Eng(), seqs, mask, scores, 0.1, 4)
    assert _close(g_full, _grads(pol))
    # the baselines differ, so the gradients do
    assert not _close(g_micro, g_full)
