"""MoE (Mixtral) op and layer semantics on CPU: the dispatch/grouped-expert/combine pipeline
matches a plain PyTorch fp32 HF-style sparse block (forward and gradients)."""
import pytest
import torch

from distributed_llm_alignment_amd import ops
from distributed_llm_alignment_amd.models import build_model, get_config


def test_route_topk_matches_renormalised_softmax():
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(37, 8, generator=g)
    v, i = ops.moe.route_topk(logits, 2)
    p = torch.softmax(logits, -1)
    rv, ri = torch.topk(p, 2, -1)
    assert torch.equal(i.long(), ri)
    assert torch.allclose(v, rv / rv.sum(-1, keepdim=True), atol=1e-6)


def test_dispatch_combine_roundtrip():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(11, 16, generator=g)
    topi = torch.randint(0, 4, (11, 2), generator=g, dtype=torch.int32)
    pos, counts = ops.moe.expert_positions(topi, 4)
    assert sorted(pos.reshape(-1).tolist()) == list(range(22))
    assert counts.sum() == 22
    xs = ops.moe.dispatch(x, pos)
    # rows are grouped by expert
    e_of_row = torch.empty(22, dtype=torch.long)
    e_of_row[pos.reshape(-1).long()] = topi.reshape(-1).long()
    assert torch.all(e_of_row[1:] >= e_of_row[:-1])
    w = torch.rand(11, 2, generator=g)
    out = ops.moe.combine(xs, pos, w)
    assert torch.allclose(out, x * w.sum(-1, keepdim=True), atol=1e-6)


def test_moe_layer_matches_reference_fwd_bwd():
    cfg = get_config("tiny-mixtral")
    m = build_model(cfg, device="cpu", seed=3)
    moe = m.layers[0].mlp
    g = torch.Generator().manual_seed(4)
    h = torch.randn(2, 9, cfg.hidden_size, generator=g, requires_grad=True)
    out = moe(h)
    ref = ops.moe.ref_moe(h.reshape(-1, cfg.hidden_size), moe.router, moe.expert_up, moe.expert_down,
                          cfg.num_experts_per_tok).view_as(h)
    assert torch.allclose(out, ref, atol=1e-5)
    go = torch.randn(out.shape, generator=g)
    grads = torch.autograd.grad(out, [h, moe.router, moe.expert_up, moe.expert_down], go)
    h2 = h.detach().clone().requires_grad_(True)
    params = [p.detach().clone().requires_grad_(True) for p in (moe.router, moe.expert_up, moe.expert_down)]
    ref = ops.moe.ref_moe(h2.reshape(-1, cfg.hidden_size), *params, cfg.num_experts_per_tok).view_as(h2)
    rgrads = torch.autograd.grad(ref, [h2, *params], go)
    for a, b in zip(grads, rgrads):
        assert torch.allclose(a, b, atol=1e-4), (a - b).abs().max()


def test_mixtral_dpo_step_runs_with_engine():
    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.objectives import dpo_step_loss
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine

    cfg = get_config("tiny-mixtral")
    pol = build_model(cfg, device="cpu", seed=0)
    ref = build_model(cfg, device="cpu", seed=0).requires_grad_(False)
    eng = DataParallelEngine(pol, lr=1e-2)
    b = synthetic_preference_batch(2, 16, cfg.vocab_size, generator=torch.Generator().manual_seed(0))
    l0, _ = dpo_step_loss(pol, ref, b)
    l0.backward()
    assert float(eng.step()) > 0
    assert pol.layers[0].mlp.expert_up.grad.abs().sum() == 0  # grads zeroed after step


def test_expert_parallel_shape_mode_one_rank():
    """bench.py --ep-shape: one EP rank's experts (E / N per layer) behind the capacity dispatch
    with identity all-to-alls; expert buckets keep unsharded optimizer state while the dense ones
    are laid out as 1 of N ZeRO-1 ranks, and a DPO step trains the local experts."""
    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.objectives import dpo_step_loss
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine
    from distributed_llm_alignment_amd.parallel.expert import apply_expert_parallel

    cfg = get_config("tiny-mixtral")
    N = cfg.num_experts // 2
    pol = build_model(cfg, device="cpu", seed=0)
    ref = build_model(cfg, device="cpu", seed=0).requires_grad_(False)
    for m in (pol, ref):
        apply_expert_parallel(m, None, capacity_factor=2.0, shape_ep=N)
    mlp = pol.layers[0].mlp
    assert mlp.expert_up.shape[0] == 2 and mlp.ep.shape and mlp.ep.ep == N
    eng = DataParallelEngine(pol, lr=1e-2, shape_world=N)
    assert any(b.expert and b.world == 1 for b in eng.buckets)
    assert any(not b.expert and b.world == N for b in eng.buckets)
    w0 = mlp.expert_up.detach().clone()
    b = synthetic_preference_batch(2, 16, cfg.vocab_size, generator=torch.Generator().manual_seed(0))
    loss, _ = dpo_step_loss(pol, ref, b)
    loss.backward()
    assert torch.isfinite(loss) and float(eng.step()) > 0
    assert not torch.equal(w0, mlp.expert_up.detach())


def test_expert_parallel_shape_hot_expert(monkeypatch):
    """bench.py --ep-hot: in the EP shape mode with one local expert, every source sends its full
    capacity, so the expert GEMM runs capacity x the balanced rows (the overflow path past the
    expected n * k); the padding rows are zeros no slot reads back, so the layer output equals
    the balanced shape mode's."""
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.parallel.expert import apply_expert_parallel

    cfg = get_config("tiny-mixtral")
    E = cfg.num_experts
    seen = []
    real = ops.moe.experts_swiglu_offsets

    def spy(xe, w_up, w_down, offs, **kw):
        seen.append((xe.shape[0], int(offs[-1]), kw.get("main_rows", 0)))
        return real(xe, w_up, w_down, offs, **kw)

    monkeypatch.setattr(ops.moe, "experts_swiglu_offsets", spy)
    outs = []
    h = torch.randn(2, 512, cfg.hidden_size, generator=torch.Generator().manual_seed(1))
    for hot in (False, True):
        m = build_model(cfg, device="cpu", seed=0)
        apply_expert_parallel(m, None, capacity_factor=1.5, shape_ep=E, shape_hot=hot)
        seen.clear()
        with torch.no_grad():
            outs.append(m.layers[0].mlp(h))
        rows, used, main = seen[0]
        if hot:
            assert used == rows > main  # every capacity row computed, past the expected rows
        else:
            assert used <= main
    torch.testing.assert_close(outs[1], outs[0], rtol=1e-5, atol=1e-6)
    with pytest.raises(ValueError):
        apply_expert_parallel(build_model(cfg, device="cpu", seed=0), None, shape_ep=E // 2, shape_hot=True)
