"""Memory-bounded model construction (models/materialize.py; VERDICT r2 next-round #3a): a
model built on the meta device and materialised after tensor-parallel / FSDP / expert-parallel
sharding holds exactly the weights of the build-then-shard path, and the construction peak is
this rank's share of the model plus ONE full parameter (TP) or one FSDP unit — never the whole
model (the reference's ZeRO-3 zero.Init route: config/deepspeed_zero3.json:5-15,
src/training/utils.py:62-63). gloo, world 2."""
import torch

from test_distributed_cpu import run_ranks


def _model_bytes(m):
    return sum(p.numel() * p.element_size() for p in m.parameters())


def _tp_meta(rank, world):
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.models import materialize as mt
    from distributed_llm_alignment_amd.parallel.mesh import build_mesh
    from distributed_llm_alignment_amd.parallel.tensor_parallel import apply_tensor_parallel

    mesh = build_mesh(tp=world)
    cfg = get_config("tiny-llama")
    full = build_model(cfg, device="cpu", seed=3)
    total = _model_bytes(full)
    max_param = max(p.numel() * p.element_size() for p in full.parameters())
    apply_tensor_parallel(full, mesh.tp_group)
    mt.reset_stats()
    meta = build_model(cfg, device="cpu", seed=3, meta=True)
    assert mt.has_meta_params(meta)
    apply_tensor_parallel(meta, mesh.tp_group)
    assert all(p.is_meta for p in meta.parameters())
    mt.materialize(meta, "cpu")
    same = all(torch.equal(a, b) for a, b in zip(full.parameters(), meta.parameters()))
    specs = all(getattr(a, "_dla_tp_spec", None) == getattr(b, "_dla_tp_spec", None)
                for a, b in zip(full.parameters(), meta.parameters()))
    ids = torch.randint(3, cfg.vocab_size, (2, 9), generator=torch.Generator().manual_seed(1))
    lp_a = full.sequence_logprob(ids, torch.ones_like(ids)).detach()
    lp_b = meta.sequence_logprob(ids, torch.ones_like(ids)).detach()
    return same, specs, torch.equal(lp_a, lp_b), mt.STATS["peak_bytes"], total, max_param


def test_tp_meta_construction_equals_build_then_shard_and_is_bounded():
    res = run_ranks(_tp_meta, 2)
    for r in (0, 1):
        same, specs, lp_same, peak, total, max_param = res[r]
        assert same and specs and lp_same
        assert peak <= total // 2 + max_param, (peak, total, max_param)


def _fsdp_meta(rank, world):
    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.models import materialize as mt
    from distributed_llm_alignment_amd.objectives import dpo_step_loss
    from distributed_llm_alignment_amd.parallel.fsdp import FullyShardedEngine, ShardedInference

    cfg = get_config("tiny-llama")
    b = synthetic_preference_batch(2, 16, cfg.vocab_size, generator=torch.Generator().manual_seed(rank))
    out = []
    for use_meta in (False, True):
        mt.reset_stats()
        pol = build_model(cfg, device="cpu", seed=0, meta=use_meta)
        ref = build_model(cfg, device="cpu", seed=0, meta=use_meta).requires_grad_(False)
        total = sum(p.numel() * 4 for p in pol.parameters())
        layer = max(sum(p.numel() * 4 for p in l.parameters()) for l in pol.layers)
        # the root unit (embeddings, final norm, LM head) stays gathered on every rank
        root = sum(p.numel() * 4 for n, p in pol.named_parameters() if not n.startswith("layers."))
        eng = FullyShardedEngine(pol, lr=1e-2)
        ShardedInference(ref)
        peak = mt.STATS["peak_bytes"]
        assert not mt.has_meta_params(pol) and not mt.has_meta_params(ref)
        loss, _ = dpo_step_loss(pol, ref, b)
        loss.backward()
        eng.step()
        loss2 = float(dpo_step_loss(pol, ref, b)[0])
        out.append((float(loss), loss2, peak, total, layer + root, eng.param_shard.clone()))
    return out


def test_fsdp_meta_construction_unit_by_unit():
    res = run_ranks(_fsdp_meta, 2)
    for r in (0, 1):
        (l0, l0b, _, _, _, sh0), (l1, l1b, peak, total, layer, sh1) = res[r]
        assert l0 == l1 and l0b == l1b
        assert torch.equal(torch.as_tensor(sh0), torch.as_tensor(sh1))
        # two models (policy + frozen ref) each at 1/2 (+ their resident root units), plus one
        # full unit being assembled (`layer` = one layer + root bytes)
        assert peak <= total + 2 * layer, (peak, total, layer)
        assert peak < 2 * total  # the replicated build would hold both models whole


def _ep_meta(rank, world):
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.models import materialize as mt
    from distributed_llm_alignment_amd.parallel.expert import apply_expert_parallel
    from distributed_llm_alignment_amd.parallel.mesh import build_mesh

    mesh = build_mesh(ep=world)
    cfg = get_config("tiny-mixtral")
    full = build_model(cfg, device="cpu", seed=2)
    apply_expert_parallel(full, mesh)
    meta = build_model(cfg, device="cpu", seed=2, meta=True)
    apply_expert_parallel(meta, mesh)
    mt.materialize(meta, "cpu")
    return all(torch.equal(a, b) for a, b in zip(full.parameters(), meta.parameters()))


def test_ep_meta_construction_equals_build_then_shard():
    res = run_ranks(_ep_meta, 2)
    assert res[0] and res[1]


def test_meta_from_checkpoint_equals_loaded(tmp_path):
    """Values can come from a lazily read HF checkpoint instead of the seeded init."""
    from distributed_llm_alignment_amd.models import build_model, get_config, load_causal_lm
    from distributed_llm_alignment_amd.models import materialize as mt
    from distributed_llm_alignment_amd.utils.checkpoint import save_state

    cfg = get_config("tiny-llama")
    m = build_model(cfg, device="cpu", seed=11)
    save_state(tmp_path / "ck", [m], None, step=1)
    eager = load_causal_lm(str(tmp_path / "ck" / "hf"), gradient_checkpointing=False, device="cpu").model
    lazy = load_causal_lm(str(tmp_path / "ck" / "hf"), gradient_checkpointing=False, device="cpu",
                          meta_init=True).model
    assert mt.has_meta_params(lazy)
    mt.materialize(lazy, "cpu")
    assert all(torch.equal(a, b) for a, b in zip(eager.parameters(), lazy.parameters()))
    assert all(torch.equal(a, b) for a, b in zip(m.parameters(), lazy.parameters()))
