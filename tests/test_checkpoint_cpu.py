"""Memory-bounded, sharded checkpoints (utils/sharded_io.py), gloo.

  * FSDP save streams one unit at a time (never more than one non-root unit full) and the
    streamed `model.safetensors` is byte-identical to the one the whole-model gather writes;
  * per-rank weight shards (FSDP flat shards, TP slices, EP expert stacks) resume exactly, and
    tools/consolidate_checkpoint.py --weights rebuilds the HF-named file from them offline;
  * large models go to HF index shards (`model-0000k-of-0000n` + index) that load back;
  * TP=2 and EP=2 checkpoints load into an unsharded model (cross-layout resume).
"""
import importlib.util
import os
from pathlib import Path

import pytest
import torch

from test_distributed_cpu import run_ranks

ROOT = Path(__file__).resolve().parents[1]


def _tool():
    spec = importlib.util.spec_from_file_location("cons", ROOT / "tools" / "consolidate_checkpoint.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _files_equal(a, b):
    from safetensors.torch import load_file

    x, y = load_file(str(a)), load_file(str(b))
    return sorted(x) == sorted(y) and all(torch.equal(x[k], y[k]) for k in x)


def _fsdp_save(rank, world, root):
    from safetensors.torch import save_file

    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.objectives import dpo_step_loss
    from distributed_llm_alignment_amd.parallel.fsdp import (FullyShardedEngine, ShardedInference,
                                                             fsdp_full_params)
    from distributed_llm_alignment_amd.utils import sharded_io
    from distributed_llm_alignment_amd.utils.checkpoint import load_state, save_state

    cfg = get_config("tiny-llama")
    pol = build_model(cfg, device="cpu", seed=0)
    ref = build_model(cfg, device="cpu", seed=0).requires_grad_(False)
    eng = FullyShardedEngine(pol, lr=1e-2)
    ShardedInference(ref)
    b = synthetic_preference_batch(2, 16, cfg.vocab_size, generator=torch.Generator().manual_seed(rank))
    dpo_step_loss(pol, ref, b)[0].backward()
    eng.step()
    sharded_io.STATS["max_full_units"] = 0
    save_state(f"{root}/ck", [pol, ref], eng, step=1, weights="both")
    peak = sharded_io.STATS["max_full_units"]
    with fsdp_full_params(pol):  # the old whole-model gather path, for comparison
        if rank == 0:
            sd = {k: v.detach().clone() for k, v in pol.hf_state_dict().items()}
            save_file(sd, f"{root}/gathered.safetensors", metadata={"format": "pt"})
    want = float(dpo_step_loss(pol, ref, b)[0])
    # resume from the per-rank shards into a differently initialised model
    pol2 = build_model(cfg, device="cpu", seed=5)
    ref2 = build_model(cfg, device="cpu", seed=5).requires_grad_(False)
    eng2 = FullyShardedEngine(pol2, lr=1e-2)
    ShardedInference(ref2)
    load_state(f"{root}/ck", [pol2, ref2], eng2)
    got = float(dpo_step_loss(pol2, ref2, b)[0])
    return peak, len(eng.units), want, got


def test_fsdp_streamed_save_is_bounded_and_identical(tmp_path):
    res = run_ranks(_fsdp_save, 2, (str(tmp_path),))
    for r in (0, 1):
        peak, units, want, got = res[r]
        assert units > 2 and peak <= 1, (peak, units)
        assert want == pytest.approx(got, abs=1e-6)
    ck = tmp_path / "ck"
    a, b = ck / "model.safetensors", tmp_path / "gathered.safetensors"
    assert a.read_bytes() == b.read_bytes()  # streamed == whole-model gather, byte for byte
    assert (ck / "model.fsdp0-tp0-ep0.safetensors").exists() and (ck / "model.fsdp1-tp0-ep0.safetensors").exists()
    assert (ck / "hf" / "model.safetensors").exists() and (ck / "hf" / "config.json").exists()
    out = _tool().consolidate_weights(ck, "model", tmp_path / "offline")
    assert out == ["model.safetensors"]
    assert (tmp_path / "offline" / "model.safetensors").read_bytes() == a.read_bytes()
    out1 = _tool().consolidate_weights(ck, "model_1", tmp_path / "offline")
    assert _files_equal(tmp_path / "offline" / "model_1.safetensors", ck / "model_1.safetensors")


def _tp_save(rank, world, root, kind):
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.parallel.mesh import build_mesh
    from distributed_llm_alignment_amd.utils.checkpoint import save_state

    mesh = build_mesh(**{kind: 2})
    name = "tiny-mixtral" if kind == "ep" else "tiny-llama"
    cfg = get_config(name)
    m = build_model(cfg, device="cpu", seed=0)
    if kind == "tp":
        from distributed_llm_alignment_amd.parallel.tensor_parallel import apply_tensor_parallel

        apply_tensor_parallel(m, mesh.tp_group)
    else:
        from distributed_llm_alignment_amd.parallel.expert import apply_expert_parallel

        apply_expert_parallel(m, mesh)
    with torch.no_grad():  # make every element distinct so a mis-merge cannot pass
        for i, p in enumerate(m.parameters()):
            p.add_(0.001 * (i + 1))
    save_state(f"{root}/ck", [m], None, step=3, weights="both")
    ids = torch.randint(3, cfg.vocab_size, (2, 11), generator=torch.Generator().manual_seed(1))
    return m.sequence_logprob(ids, torch.ones_like(ids)).detach()


@pytest.mark.parametrize("kind", ["tp", "ep"])
def test_tp_ep_shards_consolidate_and_load_unsharded(tmp_path, kind):
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.utils.checkpoint import load_model_weights

    res = run_ranks(_tp_save, 2, (str(tmp_path), kind))
    ck = tmp_path / "ck"
    assert (ck / "model.fsdp0-tp0-ep0.safetensors").exists()
    other = "model.fsdp0-tp1-ep0.safetensors" if kind == "tp" else "model.fsdp0-tp0-ep1.safetensors"
    assert (ck / other).exists()
    out = _tool().consolidate_weights(ck, "model", tmp_path / "offline")
    assert _files_equal(tmp_path / "offline" / out[0], ck / "model.safetensors")
    cfg = get_config("tiny-mixtral" if kind == "ep" else "tiny-llama")
    dense = build_model(cfg, device="cpu", seed=9)
    load_model_weights(dense, ck, 0)
    ids = torch.randint(3, cfg.vocab_size, (2, 11), generator=torch.Generator().manual_seed(1))
    lp = dense.sequence_logprob(ids, torch.ones_like(ids)).detach()
    assert torch.allclose(lp, torch.as_tensor(res[0]), atol=1e-5)


def test_large_model_writes_hf_index_shards(tmp_path, monkeypatch):
    from distributed_llm_alignment_amd.models import build_model, get_config, load_causal_lm
    from distributed_llm_alignment_amd.utils import sharded_io
    from distributed_llm_alignment_amd.utils.checkpoint import load_model_weights, save_state

    monkeypatch.setattr(sharded_io, "SINGLE_FILE_MAX_BYTES", 1 << 16)
    monkeypatch.setattr(sharded_io, "SHARD_BYTES", 1 << 17)
    cfg = get_config("tiny-llama")
    m = build_model(cfg, device="cpu", seed=0)
    save_state(tmp_path / "ck", [m], None, step=1)
    ck = tmp_path / "ck"
    assert not (ck / "model.safetensors").exists()
    shards = sorted(ck.glob("model-*-of-*.safetensors"))
    assert len(shards) > 1 and (ck / "model.safetensors.index.json").exists()
    m2 = build_model(cfg, device="cpu", seed=3)
    load_model_weights(m2, ck, 0)
    assert all(torch.equal(a, b) for a, b in zip(m.parameters(), m2.parameters()))
    b = load_causal_lm(str(ck / "hf"), device="cpu", gradient_checkpointing=False)
    assert all(torch.equal(a, c) for a, c in zip(m.parameters(), b.model.parameters()))


def test_rng_state_is_weights_only_loadable(tmp_path):
    import random

    import numpy as np

    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.utils.checkpoint import load_state, save_state

    m = build_model(get_config("tiny-llama"), device="cpu", seed=0)
    random.seed(4)
    np.random.seed(4)
    torch.manual_seed(4)
    save_state(tmp_path / "ck", [m], None, step=7)
    want = (random.random(), float(np.random.rand()), float(torch.rand(1)))
    torch.load(str(tmp_path / "ck" / "random_states_0.pkl"), weights_only=True)  # no pickle code
    random.seed(0)
    np.random.seed(0)
    torch.manual_seed(0)
    assert load_state(tmp_path / "ck", [m]) == 7
    assert (random.random(), float(np.random.rand()), float(torch.rand(1))) == want


def _fsdp_regroup(rank, world, root):
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.parallel.fsdp import FullyShardedEngine, fsdp_full_params
    from distributed_llm_alignment_amd.utils import sharded_io
    from distributed_llm_alignment_amd.utils.checkpoint import load_model_weights, save_state

    cfg = get_config("tiny-llama")
    pol = build_model(cfg, device="cpu", seed=0)
    with torch.no_grad():
        for i, p in enumerate(pol.parameters()):
            p.add_(0.001 * (i + 1))
    eng = FullyShardedEngine(pol, lr=1e-2)
    save_state(f"{root}/ck", [pol], eng, step=1, weights="both")
    with fsdp_full_params(pol):
        want = [p.detach().clone() for p in pol.parameters()]
    # same world, different unit grouping (fsdp_min_num_params): the flat shards must be refused
    pol2 = build_model(cfg, device="cpu", seed=5)
    eng2 = FullyShardedEngine(pol2, lr=1e-2, min_num_params=10 ** 9)
    regrouped = len(eng2.units) != len(eng.units)
    took_shards = sharded_io.load_rank_shards(pol2, f"{root}/ck", "model")
    load_model_weights(pol2, f"{root}/ck", 0)  # falls back to the HF-named files
    with fsdp_full_params(pol2):
        same = all(torch.equal(a, b) for a, b in zip(want, pol2.parameters()))
    return regrouped, took_shards, same


def test_fsdp_shards_refused_when_unit_grouping_changes(tmp_path):
    """a flat FSDP shard saved under one unit grouping must not be loaded under
    another even when the total length matches; the HF-named weights load instead, exactly."""
    res = run_ranks(_fsdp_regroup, 2, (str(tmp_path),))
    for r in (0, 1):
        regrouped, took, same = res[r]
        assert regrouped and not took and same


def test_fsdp_weight_epoch_moves_with_the_shards():
    """Gathers preserve the params' version counters, so weight-derived caches (the decode
    kernels' folded / tiled copies, keyed by ops.decode._wkey) key on the engine's weight epoch:
    it must move on every optimizer step and state writeback, and refresh_folded_weights must
    leave a sharded model alone (its weights are not resident)."""
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.parallel.fsdp import FullyShardedEngine

    cfg = get_config("tiny-llama")
    pol = build_model(cfg, device="cpu", seed=0)
    eng = FullyShardedEngine(pol, lr=1e-2)
    w = pol.layers[0].attn.qkv_proj
    k0 = ops.decode._wkey(w)
    ids = torch.randint(3, cfg.vocab_size, (2, 16), generator=torch.Generator().manual_seed(0))
    pol(ids).float().pow(2).mean().backward()
    eng.step()
    k1 = ops.decode._wkey(w)
    assert k1[2] != k0[2]
    with eng.summon_full_params(writeback=True):
        pass
    assert ops.decode._wkey(w)[2] != k1[2]
    assert pol.layers_sharded()
    ops.decode.refresh_folded_weights(pol)  # no-op while sharded
    assert getattr(w, "_dla_fold", None) is None
