"""CPU tier end-to-end: every CLI on a tiny random-init model with
synthetic / local JSONL data — loss finite (and decreasing where meaningful), metrics JSONL
written with the reference metric names, accelerate-layout checkpoints present, stages chain
through `latest` exports, and `--resume` continues."""
import json
import os
from pathlib import Path

import pytest
import yaml

from distributed_llm_alignment_amd.data import write_jsonl
from distributed_llm_alignment_amd.data.synthetic import (synthetic_instruction_records,
                                                          synthetic_preference_records,
                                                          synthetic_prompt_records)


def _cfg(tmp, name, body):
    p = Path(tmp) / f"{name}.yaml"
    p.write_text(yaml.safe_dump(body))
    return str(p)


def _metrics(log_dir):
    p = Path(log_dir) / "metrics.jsonl"
    return [json.loads(l) for l in p.read_text().splitlines()]


def _common(tmp, stage, steps=6, accum=1):
    return {"logging": {"output_dir": str(Path(tmp) / "ck" / stage), "log_dir": str(Path(tmp) / "logs" / stage),
                        "log_every_steps": 2, "eval_every_steps": 3, "save_every_steps": 4},
            "hardware": {"gradient_accumulation_steps": accum}}


def test_sft_reward_dpo_distill_rlhf_pipeline(tmp_path):
    from distributed_llm_alignment_amd.training import (generate_teacher_data, train_distill, train_dpo,
                                                        train_reward, train_rlhf, train_sft)

    d = tmp_path
    write_jsonl(d / "sft.jsonl", synthetic_instruction_records(24, seed=1))
    write_jsonl(d / "sft_eval.jsonl", synthetic_instruction_records(6, seed=2))
    write_jsonl(d / "pref.jsonl", synthetic_preference_records(24, seed=3))
    write_jsonl(d / "prompts.jsonl", synthetic_prompt_records(8, seed=4))

    # ---- SFT (cosine schedule, eval loss, grad accumulation)
    sft = {"seed": 42, "model": {"model_name_or_path": "tiny-llama", "max_seq_length": 96,
                                 "gradient_checkpointing": True},
           "data": {"source": "local", "train_path": str(d / "sft.jsonl"), "eval_path": str(d / "sft_eval.jsonl"),
                    "num_workers": 0},
           "optimization": {"micro_batch_size": 2, "learning_rate": 3e-3, "warmup_steps": 1,
                            "max_train_steps": 8, "lr_scheduler": "cosine"},
           **_common(d, "sft", accum=2)}
    assert train_sft.main(["--config", _cfg(d, "sft", sft)]) == 0
    m = _metrics(d / "logs" / "sft")
    assert any("train/loss" in r for r in m) and any("eval/loss" in r for r in m)
    final = d / "ck" / "sft" / "final"
    for f in ("model.safetensors", "optimizer.bin", "scheduler.bin", "random_states_0.pkl"):
        assert (final / f).exists(), f
    latest = d / "ck" / "sft" / "latest"
    assert (latest / "config.json").exists()

    # ---- resume SFT from step_4 for 2 more steps
    sft2 = dict(sft)
    sft2["optimization"] = dict(sft["optimization"], max_train_steps=10)
    assert train_sft.main(["--config", _cfg(d, "sft2", sft2), "--resume", str(d / "ck" / "sft" / "final")]) == 0

    # ---- reward model on preference pairs
    rw = {"model": {"base_model_name_or_path": str(latest), "pooling": "last_token", "dropout": 0.1,
                    "max_seq_length": 96},
          "data": {"source": "local", "train_path": str(d / "pref.jsonl"), "eval_path": str(d / "pref.jsonl"),
                   "num_workers": 0},
          "optimization": {"micro_batch_size": 2, "learning_rate": 1e-3, "max_train_steps": 6},
          **_common(d, "reward")}
    assert train_reward.main(["--config", _cfg(d, "rw", rw)]) == 0
    m = _metrics(d / "logs" / "reward")
    assert any("eval/acc" in r for r in m)
    rfinal = d / "ck" / "reward" / "final"
    assert (rfinal / "model.safetensors").exists()

    # ---- DPO from the SFT export; loss starts at ln 2 and decreases
    dpo = {"seed": 7, "model": {"policy_model_name_or_path": str(latest), "reference_model_name_or_path": str(latest),
                                "beta": 0.1, "max_seq_length": 96, "gradient_checkpointing": False},
           "data": {"preference_path": str(d / "pref.jsonl"), "num_workers": 0},
           "optimization": {"micro_batch_size": 4, "learning_rate": 2e-3, "max_train_steps": 12},
           **_common(d, "dpo")}
    assert train_dpo.main(["--config", _cfg(d, "dpo", dpo)]) == 0
    m = [r for r in _metrics(d / "logs" / "dpo") if "train/loss" in r]
    assert m[0]["train/loss"] == pytest.approx(0.6931, abs=0.02)
    assert m[-1]["train/loss"] < m[0]["train/loss"]
    assert any("train/preference_rate" in r for r in _metrics(d / "logs" / "dpo"))
    dfinal = d / "ck" / "dpo" / "final"
    assert (dfinal / "model.safetensors").exists() and (dfinal / "model_1.safetensors").exists()

    # ---- teacher rollouts with reward scores
    out = d / "rollouts.jsonl"
    assert generate_teacher_data.main(["--teacher", str(d / "ck" / "dpo" / "latest"), "--prompts", str(d / "prompts.jsonl"),
                                       "--output", str(out), "--reward_model", str(rfinal), "--batch_size", "3",
                                       "--max_new_tokens", "8"]) == 0
    recs = [json.loads(l) for l in out.read_text().splitlines()]
    assert len(recs) == 8 and all({"prompt", "teacher_response", "reward"} <= set(r) for r in recs)

    # ---- distillation: CE mode, then 2-teacher ensemble KL mode
    for mode in ("ce", "kl"):
        dist = {"model": {"student_model_name_or_path": "tiny-llama", "max_seq_length": 96},
                "distill": {"use_kl": mode == "kl", "on_policy": mode == "kl",
                            "teacher_model_names_or_paths": [str(d / "ck" / "dpo" / "latest"), str(latest)]},
                "data": {"teacher_samples_path": str(out), "num_workers": 0},
                "optimization": {"micro_batch_size": 2, "learning_rate": 1e-3, "max_train_steps": 4},
                **_common(d, f"distill_{mode}")}
        assert train_distill.main(["--config", _cfg(d, f"dist_{mode}", dist)]) == 0
        assert any("train/reward_mean" in r for r in _metrics(d / "logs" / f"distill_{mode}"))
    assert (d / "ck" / "distill_kl" / "final" / "model_2.safetensors").exists()

    # ---- RLHF with the trained reward model
    rl = {"seed": 21, "model": {"policy_model_name_or_path": str(latest), "reference_model_name_or_path": str(latest),
                                "max_seq_length": 64},
          "reward_model": {"path": str(rfinal), "base_model_name_or_path": str(latest)},
          "ppo": {"batch_size": 4, "learning_rate": 1e-4, "kl_coef": 0.1, "steps": 4,
                  "generation_params": {"max_new_tokens": 6, "temperature": 0.7, "top_p": 0.9}},
          "sampling": {"source": "local", "prompt_path": str(d / "prompts.jsonl")},
          "logging": {"output_dir": str(d / "ck" / "rlhf"), "log_dir": str(d / "logs" / "rlhf"), "log_every_steps": 2}}
    assert train_rlhf.main(["--config", _cfg(d, "rl", rl)]) == 0
    m = _metrics(d / "logs" / "rlhf")
    assert all(k in m[-1] for k in ("train/loss", "train/kl"))
    for f in ("model.safetensors", "model_1.safetensors", "model_2.safetensors"):
        assert (d / "ck" / "rlhf" / f).exists()


def test_eval_clis(tmp_path):
    from distributed_llm_alignment_amd.eval import eval_alignment, eval_latency

    write_jsonl(tmp_path / "ev.jsonl", [{"question": "why?"}, {"prompt": "how?"}, {"instruction": "do"}])
    cfg = {"seed": 0, "models": {"tiny": "tiny-llama"},
           "benchmarks": {"local": {"type": "local", "prompts_path": str(tmp_path / "ev.jsonl"), "max_samples": 2}},
           "latency": {"batch_sizes": [1, 2], "seq_lengths": [16], "warmup_steps": 1, "measure_steps": 2},
           "generation": {"max_new_tokens": 4},
           "logging": {"output_path": str(tmp_path / "out" / "results.json"), "table_path": str(tmp_path / "out" / "summary.md")}}
    p = _cfg(tmp_path, "eval", cfg)
    assert eval_alignment.main(["--config", p]) == 0
    res = json.loads((tmp_path / "out" / "results.json").read_text())
    assert set(res["tiny"]["local"]) == {"avg_length", "refusal_rate", "toxicity_proxy"}
    assert "| Model |" in (tmp_path / "out" / "summary.md").read_text()
    assert eval_latency.main(["--config", p, "--decode_tokens", "3"]) == 0
    lat = json.loads((tmp_path / "out" / "latency.json").read_text())
    assert {"batch_size", "seq_length", "tokens_per_second", "latency_ms"} <= set(lat["tiny"][0])


def test_summarize_responses_keywords():
    from distributed_llm_alignment_amd.eval.eval_alignment import summarize_responses

    m = summarize_responses(["Sorry, I cannot", "a bomb here", "fine answer"])
    assert m["refusal_rate"] == pytest.approx(1 / 3) and m["toxicity_proxy"] == pytest.approx(1 / 3)
    assert m["avg_length"] == pytest.approx((3 + 3 + 2) / 3)


@pytest.mark.parametrize("packing", [False, True])
def test_gpt2_cpu_plumbing_config(tmp_path, monkeypatch, packing):
    """BASELINE.json config 1 (GPT-2-small SFT, CPU, world_size=1, synthetic pairs); also with
    `data.packing: true` (packed rows, block-diagonal attention)."""
    from distributed_llm_alignment_amd.training import train_sft

    monkeypatch.chdir(tmp_path)
    root = Path(__file__).resolve().parent.parent
    rc = train_sft.main(["--config", str(root / "config" / "sft_gpt2_cpu.yaml"),
                         "--override", "optimization.max_train_steps=4", "--override", "logging.save_every_steps=0",
                         "--override", "model.max_seq_length=64",
                         "--override", f"data.packing={str(packing).lower()}"])
    assert rc == 0
    m = _metrics(tmp_path / "logs" / "sft_gpt2_cpu")
    assert len(m) == 2 and all(r["train/loss"] == r["train/loss"] for r in m)
    assert (tmp_path / "checkpoints" / "sft_gpt2_cpu" / "final" / "model.safetensors").exists()


def test_fault_injection_and_resume_reproduces_trajectory(tmp_path, monkeypatch):
    """kill the run at step 5 (after the step-4 checkpoint), restart with --resume
    from `latest`, and the losses of steps 5..8 equal an uninterrupted run's."""
    from distributed_llm_alignment_amd.training import train_sft
    from distributed_llm_alignment_amd.utils.debug import FaultInjected

    d = tmp_path
    write_jsonl(d / "sft.jsonl", synthetic_instruction_records(32, seed=1))

    def cfg(name, out):
        body = {"seed": 5, "model": {"model_name_or_path": "tiny-llama", "max_seq_length": 160,
                                     "gradient_checkpointing": False},
                "data": {"source": "local", "train_path": str(d / "sft.jsonl"), "num_workers": 0},
                "optimization": {"micro_batch_size": 2, "learning_rate": 3e-3, "max_train_steps": 8,
                                 "warmup_steps": 2, "lr_scheduler": "cosine"},
                "logging": {"output_dir": str(d / out), "log_dir": str(d / f"logs_{out}"),
                            "log_every_steps": 1, "save_every_steps": 4},
                "debug": {"check_sync_every": 1}}
        return _cfg(d, name, body)

    assert train_sft.main(["--config", cfg("a", "full")]) == 0
    ref = {r["step"]: r["train/loss"] for r in _metrics(d / "logs_full") if "train/loss" in r}
    monkeypatch.setenv("DLA_FAULT_STEP", "5")
    with pytest.raises(FaultInjected):
        train_sft.main(["--config", cfg("b", "crash")])
    monkeypatch.delenv("DLA_FAULT_STEP")
    assert train_sft.main(["--config", cfg("b", "crash"), "--resume", str(d / "crash" / "latest")]) == 0
    got = {r["step"]: r["train/loss"] for r in _metrics(d / "logs_crash") if "train/loss" in r}
    for s in range(5, 9):
        assert got[s] == pytest.approx(ref[s], rel=1e-5, abs=1e-6), (s, got[s], ref[s])
    rec = [r for r in _metrics(d / "logs_full") if "perf/samples_per_s" in r]
    assert rec and "time/fwd_bwd_s" in rec[-1]


def test_tracing_and_profile_window(tmp_path):
    from distributed_llm_alignment_amd.utils.tracing import PHASES, ProfileWindow, trace_range

    with trace_range("unit"):
        sum(range(1000))
    assert "time/unit_s" in PHASES.pop()
    pw = ProfileWindow([1, 2], str(tmp_path / "prof"))
    pw.step(1)
    import torch

    torch.ones(4).sum()
    pw.step(2)
    assert (tmp_path / "prof" / "trace.json").exists() and (tmp_path / "prof" / "kernels.txt").exists()


@pytest.mark.parametrize("cfg_name,ov", [
    ("dpo_llama3_70b", ["model.policy_model_name_or_path=tiny-llama", "model.reference_model_name_or_path=tiny-llama",
                        "hardware.tp_size=1", "hardware.gradient_accumulation_steps=1"]),
    ("dpo_mixtral_8x7b", ["model.policy_model_name_or_path=tiny-mixtral",
                          "model.reference_model_name_or_path=tiny-mixtral", "hardware.ep_size=1",
                          "hardware.gradient_accumulation_steps=1"]),
    ("dpo_llama3_8b", ["model.policy_model_name_or_path=tiny-llama", "model.reference_model_name_or_path=tiny-llama",
                       "hardware.gradient_accumulation_steps=1"]),
])
def test_north_star_configs_run_scaled_down(tmp_path, cfg_name, ov):
    """The shipped north-star configs parse and drive the DPO trainer (architecture overridden to
    the tiny preset of the same family, world 1)."""
    from distributed_llm_alignment_amd.training import train_dpo

    root = Path(__file__).resolve().parents[1]
    args = ["--config", str(root / "config" / f"{cfg_name}.yaml"),
            "--override", "optimization.max_train_steps=2", "--override", "optimization.micro_batch_size=2",
            "--override", "model.max_seq_length=64", "--override", "data.num_samples=8",
            "--override", "data.num_workers=0", "--override", f"logging.output_dir={tmp_path / 'ck'}",
            "--override", f"logging.log_dir={tmp_path / 'logs'}", "--override", "logging.save_every_steps=0"]
    for o in ov:
        args += ["--override", o]
    assert train_dpo.main(args) == 0
    assert (tmp_path / "ck" / "final" / "model.safetensors").exists()


def test_rlhf_ppo_actor_critic(tmp_path):
    """`ppo.algorithm: ppo`: critic + GAE + clipped surrogate/value losses, 2 minibatches x
    2 epochs, critic checkpoint as the 4th model."""
    from distributed_llm_alignment_amd.training import train_rlhf

    d = tmp_path
    write_jsonl(d / "prompts.jsonl", synthetic_prompt_records(8, seed=4))
    rl = {"seed": 5, "model": {"policy_model_name_or_path": "tiny-llama",
                               "reference_model_name_or_path": "tiny-llama", "max_seq_length": 64},
          "reward_model": {"base_model_name_or_path": "tiny-llama"},
          "ppo": {"algorithm": "ppo", "batch_size": 4, "learning_rate": 1e-4, "kl_coef": 0.05,
                  "steps": 3, "ppo_epochs": 2, "num_minibatches": 2, "gamma": 1.0, "lam": 0.95,
                  "vf_coef": 0.1, "generation_params": {"max_new_tokens": 6, "temperature": 0.7,
                                                        "top_p": 0.9}},
          "sampling": {"source": "local", "prompt_path": str(d / "prompts.jsonl")},
          "logging": {"output_dir": str(d / "ck" / "ppo"), "log_dir": str(d / "logs" / "ppo"),
                      "log_every_steps": 1}}
    assert train_rlhf.main(["--config", _cfg(d, "ppo", rl)]) == 0
    m = _metrics(d / "logs" / "ppo")
    for k in ("train/loss", "train/kl", "train/value_loss", "train/clipfrac", "train/approx_kl"):
        assert k in m[-1], k
    assert all(abs(r["train/loss"]) < 1e4 for r in m)
    for f in ("model.safetensors", "model_3.safetensors", "critic_optimizer_shard_0.safetensors"):
        assert (d / "ck" / "ppo" / f).exists(), f


@pytest.mark.parametrize("cfg_name", ["rlhf_llama3_8b", "rlhf_ppo_llama3_8b"])
def test_rlhf_north_star_configs_run_scaled_down(tmp_path, cfg_name):
    """The shipped RLHF north-star configs (REINFORCE and actor-critic PPO) drive the trainer
    with the architecture overridden to the tiny preset, world 1."""
    from distributed_llm_alignment_amd.training import train_rlhf

    root = Path(__file__).resolve().parents[1]
    args = ["--config", str(root / "config" / f"{cfg_name}.yaml")]
    for o in ["model.policy_model_name_or_path=tiny-llama", "model.reference_model_name_or_path=tiny-llama",
              "reward_model.base_model_name_or_path=tiny-llama", "critic.base_model_name_or_path=tiny-llama",
              "model.max_seq_length=48", "sampling.num_samples=8", "ppo.batch_size=4", "ppo.steps=2",
              "ppo.generation_params.max_new_tokens=4", f"logging.output_dir={tmp_path / 'ck'}",
              f"logging.log_dir={tmp_path / 'logs'}", "logging.log_every_steps=1"]:
        args += ["--override", o]
    assert train_rlhf.main(args) == 0
    assert (tmp_path / "ck" / "model_2.safetensors").exists()
