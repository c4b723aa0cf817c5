"""CPU tier, multi-process (gloo): Ulysses sequence parallelism (parallel.sequence).

  * SP=2 per-sequence log-probs / SFT loss / PPO token log-probs equal the dense model's, with
    padding (left and right), an odd length (SP pads to a multiple of P), GQA, sliding window,
    learned positions (GPT-2), the parallel block + LM-head bias (phi-2) and packed sequences;
  * the per-rank parameter gradients sum to the dense gradient;
  * a DP=2 x SP=2 mesh (world 4) gives the same DPO update as plain DP=2.
"""
import pytest
import torch

from test_distributed_cpu import _tp_dpo_step, run_ranks


def _batch(cfg, S=4, T=37, seed=5):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(3, cfg.vocab_size, (S, T), generator=g)
    mask = torch.ones(S, T, dtype=torch.long)
    mask[1, 30:] = 0          # right padding
    mask[2, :6] = 0           # left padding
    mask[3, 33:] = 0
    return ids, mask


def _sp_vs_dense(rank, world, name, what):
    import torch

    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.parallel.mesh import build_mesh
    from distributed_llm_alignment_amd.parallel.sequence import apply_sequence_parallel

    mesh = build_mesh(sp=world)
    cfg = get_config(name)
    dense = build_model(cfg, device="cpu", seed=0)
    spm = build_model(cfg, device="cpu", seed=0)
    apply_sequence_parallel(spm, mesh.sp_group)
    ids, mask = _batch(cfg)
    with torch.no_grad():  # this rank really holds half of the (padded 37 -> 38) tokens
        assert spm(ids, mask).shape[1] == 19 and dense(ids, mask).shape[1] == 37

    def run(m):
        if what == "seq_logprob":
            return m.sequence_logprob(ids, mask, "mean")
        if what == "seq_logprob_sum":
            return m.sequence_logprob(ids, mask, "sum")
        if what == "token_logprobs":
            return m.token_logprobs(ids, mask)
        if what == "sft_packed":
            seg = torch.zeros_like(ids)
            seg[:, :12], seg[:, 12:30], seg[:, 30:35] = 1, 2, 3
            labels = ids.clone()
            labels[:, [0, 12, 30]] = -100
            labels[seg == 0] = -100
            return m.causal_lm_loss(ids, labels, None, segment_ids=seg)
        labels = torch.where(mask > 0, ids, torch.full_like(ids, -100))
        return m.causal_lm_loss(ids, labels, mask)

    a, b = run(dense), run(spm)
    w = torch.linspace(0.5, 1.5, a.numel()).view_as(a)
    (a * w).sum().backward()
    (b * w).sum().backward()
    grads_sp = {n: p.grad.detach().clone() for n, p in spm.named_parameters()}
    torch.distributed.barrier()
    for n in sorted(grads_sp):
        torch.distributed.all_reduce(grads_sp[n], group=mesh.sp_group)
    err = max(float((p.grad - grads_sp[n]).abs().max() / (p.grad.abs().max() + 1e-12))
              for n, p in dense.named_parameters())
    return a.detach(), b.detach(), err


@pytest.mark.parametrize("name,what", [
    ("tiny-llama", "seq_logprob"),
    ("tiny-llama", "seq_logprob_sum"),
    ("tiny-llama", "token_logprobs"),
    ("tiny-llama", "sft"),
    ("tiny-llama", "sft_packed"),
    ("tiny-mistral", "seq_logprob"),
    ("tiny-gpt2", "seq_logprob"),
    ("tiny-phi", "sft"),
])
def test_sp2_matches_dense(name, what):
    res = run_ranks(_sp_vs_dense, 2, (name, what))
    for r in (0, 1):
        a, b, err = res[r]
        assert a.shape == b.shape
        assert torch.allclose(a, b, atol=2e-5, rtol=1e-5), (a, b)
        assert err < 1e-4, err


def _sp_dpo_step(rank, world, sp):
    import torch

    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.objectives import dpo_step_loss
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine
    from distributed_llm_alignment_amd.parallel.mesh import build_mesh
    from distributed_llm_alignment_amd.parallel.sequence import apply_sequence_parallel

    mesh = build_mesh(sp=sp)
    cfg = get_config("tiny-llama")
    pol = build_model(cfg, device="cpu", seed=0)
    ref = build_model(cfg, device="cpu", seed=0).requires_grad_(False)
    apply_sequence_parallel(pol, mesh.sp_group)
    apply_sequence_parallel(ref, mesh.sp_group)
    eng = DataParallelEngine(pol, lr=1e-2, weight_decay=0.01, max_grad_norm=0.05, group=mesh.grad_group,
                             bucket_mb=0.05, sp_size=mesh.sp)
    g = torch.Generator().manual_seed(11)
    b = synthetic_preference_batch(4, 16, cfg.vocab_size, generator=g)
    per = 4 // mesh.dp
    mine = {s: {k: v[mesh.dp_rank * per:(mesh.dp_rank + 1) * per] for k, v in b[s].items()} for s in b}
    loss, _ = dpo_step_loss(pol, ref, mine)
    loss.backward()
    eng.step()
    eng.wait_params()
    loss2, _ = dpo_step_loss(pol, ref, mine)
    return float(eng.last_grad_norm), loss2


def test_dp2_sp2_mesh_matches_dp2():
    """World 4 as DP=2 x SP=2 (ZeRO-1 over the DP x SP grad group) == plain DP=2, same batch."""
    dp = run_ranks(_tp_dpo_step, 2, (1,))
    sp = run_ranks(_sp_dpo_step, 4, (2,))
    assert sp[0][0] == pytest.approx(dp[0][0], rel=1e-4)  # global grad norm (clip active)
    # ranks (0, 1) hold DP replica 0, ranks (2, 3) replica 1; SP ranks agree on the loss
    assert float(sp[0][1]) == pytest.approx(float(sp[1][1]), abs=1e-6)
    assert float(sp[0][1]) == pytest.approx(float(dp[0][1]), abs=1e-5)
    assert float(sp[2][1]) == pytest.approx(float(dp[1][1]), abs=1e-5)


def test_trainers_with_sequence_parallel(tmp_path):
    """SFT (gradient checkpointing: the all-to-alls re-run in the recompute) then DPO with
    hardware.sp_size=2 on 2 gloo ranks, incl. resume; the DPO loss starts at ln 2."""
    from test_distributed_cpu import _tp_trainers

    from distributed_llm_alignment_amd.data import write_jsonl
    from distributed_llm_alignment_amd.data.synthetic import (synthetic_instruction_records,
                                                              synthetic_preference_records)

    write_jsonl(tmp_path / "sft.jsonl", synthetic_instruction_records(16, seed=1))
    write_jsonl(tmp_path / "pref.jsonl", synthetic_preference_records(16, seed=3))
    res = run_ranks(_tp_trainers, 2, (str(tmp_path), {"sp_size": 2, "gradient_accumulation_steps": 1}))
    losses = res[0]
    assert losses and abs(losses[0] - 0.6931) < 0.02
