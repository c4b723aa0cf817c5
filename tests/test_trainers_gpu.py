"""GPU tier for the trainer CLIs (SURVEY §4 items 5-6 on MI355X): SFT then DPO on a tiny
random-init Llama (head_dim 128: native HIP attention) through the engine's main-grad GEMM path,
with activation recompute off, full, and selective. Every trainable weight must move (no
gradient silently dropped — the failure mode of main-grad autograd nodes under recompute) and
the DPO loss must fall from ln 2."""
import json
from pathlib import Path

import pytest
import torch
import yaml

from distributed_llm_alignment_amd.data import write_jsonl
from distributed_llm_alignment_amd.data.synthetic import synthetic_instruction_records, synthetic_preference_records

pytestmark = pytest.mark.gpu


def _cfg(tmp, name, body):
    p = Path(tmp) / f"{name}.yaml"
    p.write_text(yaml.safe_dump(body))
    return str(p)


def _metrics(log_dir):
    return [json.loads(l) for l in (Path(log_dir) / "metrics.jsonl").read_text().splitlines()]


def _logs(tmp, stage):
    return {"logging": {"output_dir": str(Path(tmp) / "ck" / stage), "log_dir": str(Path(tmp) / "logs" / stage),
                        "log_every_steps": 1, "eval_every_steps": 100, "save_every_steps": 100}}


@pytest.mark.parametrize("ckpt", [False, True, "mlp", "attention"])
def test_sft_then_dpo_gpu_every_weight_trains(tmp_path, ckpt):
    from distributed_llm_alignment_amd.models import load_causal_lm
    from distributed_llm_alignment_amd.ops import _ext
    from distributed_llm_alignment_amd.training import train_dpo, train_sft

    _ext.require()
    d = tmp_path
    write_jsonl(d / "sft.jsonl", synthetic_instruction_records(32, seed=1))
    write_jsonl(d / "pref.jsonl", synthetic_preference_records(32, seed=3))
    sft = {"seed": 42, "model": {"model_name_or_path": "tiny-llama-d128", "max_seq_length": 128,
                                 "gradient_checkpointing": ckpt},
           "data": {"source": "local", "train_path": str(d / "sft.jsonl"), "num_workers": 0},
           # 8 rows per micro-batch: B*T stays a multiple of 8 whatever the padded length, so
           # every step takes the fused SwiGLU-MLP main-grad node; weight decay 0 (the SFT
           # default): a weight whose gradient was dropped would not move at all
           "optimization": {"micro_batch_size": 8, "learning_rate": 3e-3, "warmup_steps": 0,
                            "max_train_steps": 4, "weight_decay": 0.0},
           **_logs(d, "sft")}
    assert train_sft.main(["--config", _cfg(d, "sft", sft)]) == 0
    latest = d / "ck" / "sft" / "latest"
    # the trainer's own init: same seed, same device (the CUDA generator's stream), same dtype
    init = load_causal_lm("tiny-llama-d128", gradient_checkpointing=False, device="cuda", seed=42).model
    trained = load_causal_lm(str(latest), gradient_checkpointing=False, device="cpu").model
    for (n, a), (_, b) in zip(init.named_parameters(), trained.named_parameters()):
        # 4 Adam steps at lr 3e-3 move a weight by ~1e-2: a snapshot from another RNG stream
        # would differ by the weights' own magnitude
        assert (a.float().cpu() - b.float()).abs().max() < 0.5 * a.float().abs().max() + 0.05, n
    frozen = [n for (n, a), (_, b) in zip(init.named_parameters(), trained.named_parameters())
              if torch.equal(a.float().cpu(), b.float())]
    assert not frozen, f"weights that never received a gradient: {frozen}"

    dpo = {"seed": 7, "model": {"policy_model_name_or_path": str(latest), "reference_model_name_or_path": str(latest),
                                "beta": 0.1, "max_seq_length": 128, "gradient_checkpointing": ckpt},
           "data": {"preference_path": str(d / "pref.jsonl"), "num_workers": 0},
           "optimization": {"micro_batch_size": 4, "learning_rate": 2e-3, "max_train_steps": 10},
           **_logs(d, "dpo")}
    assert train_dpo.main(["--config", _cfg(d, "dpo", dpo)]) == 0
    m = [r["train/loss"] for r in _metrics(d / "logs" / "dpo") if "train/loss" in r]
    assert m[0] == pytest.approx(0.6931, abs=0.02)
    assert min(m[-3:]) < m[0] - 0.02, m
