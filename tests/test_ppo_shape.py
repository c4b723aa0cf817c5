"""PPO actor-critic step on engines laid out as one rank of an N-rank ZeRO-1 job
(`DataParallelEngine(shape_world=N)`, tools/bench_rlhf.py --algorithm ppo --zero-shape N):
optimizer state exists for 1/N of each model, only that chunk of every bucket is updated, and a
2-layer PPO step gives finite, nonzero policy and critic gradients that move both models."""
import pytest
import torch


def _ppo_step(dev, shape_world):
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.models.reward import ValueModel
    from distributed_llm_alignment_amd.objectives import ppo_backward, ppo_loss, ppo_rollout_stats
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine

    dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
    cfg = get_config("tiny-llama-d128", num_layers=2)
    pol = build_model(cfg, device=dev, dtype=dt, seed=0)
    ref = build_model(cfg, device=dev, dtype=dt, seed=0).requires_grad_(False).eval()
    critic = ValueModel(build_model(cfg, device=dev, dtype=dt, seed=1, headless=True))
    kw = dict(lr=1e-3, betas=(0.9, 0.95), weight_decay=0.01, max_grad_norm=1.0, shape_world=shape_world)
    eng, ceng = DataParallelEngine(pol, **kw), DataParallelEngine(critic, **kw)
    g = torch.Generator().manual_seed(0)
    P, R, S = 16, 16, 4
    seqs = torch.randint(3, cfg.vocab_size, (S, P + R), generator=g).to(dev)
    mask = torch.ones_like(seqs)
    mask[0, P + 10:] = 0  # one rollout ended early
    scores = torch.randn(S, generator=g).to(dev)
    p0, c0 = eng.param_buf.detach().float().clone(), ceng.param_buf.detach().float().clone()
    stats = ppo_rollout_stats(pol, ref, critic, seqs, mask, P, scores, 0.05, 1.0, 0.95)
    for lo, hi in ((0, 2), (2, 4)):
        mb = {k: v[lo:hi] for k, v in stats.items() if k in ("old_logp", "values", "advantages", "returns", "act")}
        loss, _ = ppo_loss(pol, critic, seqs[lo:hi], mask[lo:hi], mb, 0.2, 0.2, 0.1)
        ppo_backward(loss)
        pn, cn = float(eng.step()), float(ceng.step())
        assert torch.isfinite(loss).item() and 0 < pn < float("inf") and 0 < cn < float("inf"), (loss, pn, cn)
    return eng, ceng, p0, c0


def _check_shape(eng, p0, N):
    assert eng.shape_only and eng.world == N and not eng._comm
    assert eng.master.numel() == eng.numel // N == eng.exp_avg.numel()
    moved = (eng.param_buf.detach().float() - p0).abs() > 0
    for b in eng.buckets:  # only this rank's chunk of every bucket was updated
        c = b.size // N
        assert moved[b.start:b.start + c].any()
        assert not moved[b.start + c:b.end].any()


def test_ppo_step_zero_shape_cpu():
    eng, ceng, p0, c0 = _ppo_step(torch.device("cpu"), 4)
    _check_shape(eng, p0, 4)
    _check_shape(ceng, c0, 4)
    with pytest.raises(RuntimeError):
        eng.optimizer_state()


@pytest.mark.gpu
def test_ppo_step_zero_shape_gpu():
    from distributed_llm_alignment_amd.ops import _ext

    _ext.require()
    eng, ceng, p0, c0 = _ppo_step(torch.device("cuda", 0), 8)
    _check_shape(eng, p0, 8)
    _check_shape(ceng, c0, 8)


def _ppo_grads(dev):
    """Policy and critic gradient buffers after one PPO minibatch backward (no optimizer step)."""
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.models.reward import ValueModel
    from distributed_llm_alignment_amd.objectives import ppo_backward, ppo_loss, ppo_rollout_stats
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine

    cfg = get_config("tiny-llama-d128", num_layers=2)
    torch.manual_seed(0)  # the value head's init draws from the global generator
    pol = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    ref = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0).requires_grad_(False).eval()
    critic = ValueModel(build_model(cfg, device=dev, dtype=torch.bfloat16, seed=1, headless=True))
    eng, ceng = DataParallelEngine(pol, lr=1e-3), DataParallelEngine(critic, lr=1e-3)
    g = torch.Generator().manual_seed(0)
    P, R, S = 16, 16, 4
    seqs = torch.randint(3, cfg.vocab_size, (S, P + R), generator=g).to(dev)
    mask = torch.ones_like(seqs)
    scores = torch.randn(S, generator=g).to(dev)
    stats = ppo_rollout_stats(pol, ref, critic, seqs, mask, P, scores, 0.05, 1.0, 0.95)
    mb = {k: v for k, v in stats.items() if k in ("old_logp", "values", "advantages", "returns", "act")}
    # advantages are whitened over the batch: perturb old_logp so the ratio is not exactly 1
    mb["old_logp"] = mb["old_logp"] - 0.05
    loss, _ = ppo_loss(pol, critic, seqs, mask, mb, 0.2, 0.2, 0.1)
    ppo_backward(loss)
    torch.cuda.synchronize()
    return eng.grad_buf.float().clone(), ceng.grad_buf.float().clone()


@pytest.mark.gpu
def test_ppo_critic_side_stream_matches_one_stream():
    """The critic's forward / backward on its side stream (objectives.PPO_CRITIC_STREAM) gives the
    policy and critic gradients of the single-stream backward (compared before any optimizer
    step: AdamW's first update is lr x sign(g), which turns rounding-level noise into lr-sized
    weight differences)."""
    import distributed_llm_alignment_amd.objectives as obj
    from distributed_llm_alignment_amd.ops import _ext

    _ext.require()
    prev = obj.PPO_CRITIC_STREAM
    out = {}
    try:
        for on in (True, False):
            obj.PPO_CRITIC_STREAM = on
            out[on] = _ppo_grads(torch.device("cuda", 0))
    finally:
        obj.PPO_CRITIC_STREAM = prev
    for a, b in zip(out[True], out[False]):
        assert a.abs().sum() > 0
        assert ((a - b).norm() / b.norm()).item() < 1e-2
