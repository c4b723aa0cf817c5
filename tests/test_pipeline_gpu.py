"""GPU tier for the rest of the pipeline CLIs (SURVEY §4 item 5 on MI355X): the reward, teacher
rollout, distillation (CE and ensemble-KL), RLHF (REINFORCE-KL and actor-critic PPO) and eval
CLIs on a tiny random-init Llama with head_dim 128, so every stage runs the native HIP path
(flash attention, fused reward head, hipGraph decode + fused sampler, KL-penalty / GAE / PPO
kernels, chunked ensemble KL). Stages chain through the `latest` exports exactly as the CPU
pipeline test does (tests/test_trainers_cpu.py); here the point is that they run on the card."""
import json
from pathlib import Path

import pytest
import yaml

from distributed_llm_alignment_amd.data import write_jsonl
from distributed_llm_alignment_amd.data.synthetic import (synthetic_instruction_records,
                                                          synthetic_preference_records,
                                                          synthetic_prompt_records)

pytestmark = pytest.mark.gpu

MODEL = "tiny-llama-d128"


def _cfg(tmp, name, body):
    p = Path(tmp) / f"{name}.yaml"
    p.write_text(yaml.safe_dump(body))
    return str(p)


def _metrics(log_dir):
    return [json.loads(l) for l in (Path(log_dir) / "metrics.jsonl").read_text().splitlines()]


def _logs(tmp, stage, every=1, eval_every=100):
    return {"logging": {"output_dir": str(Path(tmp) / "ck" / stage), "log_dir": str(Path(tmp) / "logs" / stage),
                        "log_every_steps": every, "eval_every_steps": eval_every, "save_every_steps": 100}}


@pytest.fixture(scope="module")
def stages(tmp_path_factory):
    """SFT export + reward model: the inputs of every later stage."""
    from distributed_llm_alignment_amd.ops import _ext
    from distributed_llm_alignment_amd.training import train_reward, train_sft

    _ext.require()
    d = tmp_path_factory.mktemp("pipeline")
    write_jsonl(d / "sft.jsonl", synthetic_instruction_records(16, seed=1))
    write_jsonl(d / "pref.jsonl", synthetic_preference_records(16, seed=3))
    write_jsonl(d / "prompts.jsonl", synthetic_prompt_records(8, seed=4))
    sft = {"seed": 42, "model": {"model_name_or_path": MODEL, "max_seq_length": 96},
           "data": {"source": "local", "train_path": str(d / "sft.jsonl"), "num_workers": 0},
           "optimization": {"micro_batch_size": 4, "learning_rate": 1e-3, "max_train_steps": 3},
           **_logs(d, "sft")}
    assert train_sft.main(["--config", _cfg(d, "sft", sft)]) == 0
    latest = d / "ck" / "sft" / "latest"
    rw = {"model": {"base_model_name_or_path": str(latest), "pooling": "last_token", "dropout": 0.1,
                    "max_seq_length": 96},
          "data": {"source": "local", "train_path": str(d / "pref.jsonl"), "eval_path": str(d / "pref.jsonl"),
                   "num_workers": 0},
          "optimization": {"micro_batch_size": 4, "learning_rate": 1e-3, "max_train_steps": 4},
          **_logs(d, "reward", eval_every=2)}
    assert train_reward.main(["--config", _cfg(d, "rw", rw)]) == 0
    m = _metrics(d / "logs" / "reward")
    assert any("eval/acc" in r for r in m)
    assert all(r["train/loss"] == r["train/loss"] for r in m if "train/loss" in r)  # finite (no NaN)
    return d, latest, d / "ck" / "reward" / "final"


def test_teacher_rollouts_and_distillation_gpu(stages):
    from distributed_llm_alignment_amd.training import generate_teacher_data, train_distill

    d, latest, rfinal = stages
    out = d / "rollouts.jsonl"
    assert generate_teacher_data.main(["--teacher", str(latest), "--prompts", str(d / "prompts.jsonl"),
                                       "--output", str(out), "--reward_model", str(rfinal),
                                       "--batch_size", "4", "--max_new_tokens", "8"]) == 0
    recs = [json.loads(l) for l in out.read_text().splitlines()]
    assert len(recs) == 8 and all({"prompt", "teacher_response", "reward"} <= set(r) for r in recs)
    for mode in ("ce", "kl"):
        dist = {"model": {"student_model_name_or_path": MODEL, "max_seq_length": 96},
                "distill": {"use_kl": mode == "kl", "on_policy": mode == "kl",
                            "teacher_model_names_or_paths": [str(latest), str(latest)]},
                "data": {"teacher_samples_path": str(out), "num_workers": 0},
                "optimization": {"micro_batch_size": 2, "learning_rate": 1e-3, "max_train_steps": 3},
                **_logs(d, f"distill_{mode}")}
        assert train_distill.main(["--config", _cfg(d, f"dist_{mode}", dist)]) == 0
        m = [r for r in _metrics(d / "logs" / f"distill_{mode}") if "train/loss" in r]
        assert m and all(abs(r["train/loss"]) < 1e4 for r in m)
    assert (d / "ck" / "distill_kl" / "final" / "model_2.safetensors").exists()


@pytest.mark.parametrize("algo", ["reinforce", "ppo"])
def test_rlhf_gpu(stages, algo):
    from distributed_llm_alignment_amd.training import train_rlhf

    d, latest, rfinal = stages
    ppo = {"batch_size": 4, "learning_rate": 1e-4, "kl_coef": 0.1, "steps": 3,
           "generation_params": {"max_new_tokens": 8, "temperature": 0.7, "top_p": 0.9}}
    if algo == "ppo":
        ppo.update({"algorithm": "ppo", "ppo_epochs": 2, "num_minibatches": 2, "vf_coef": 0.1})
    rl = {"seed": 21, "model": {"policy_model_name_or_path": str(latest), "reference_model_name_or_path": str(latest),
                                "max_seq_length": 64},
          "reward_model": {"path": str(rfinal), "base_model_name_or_path": str(latest)},
          "ppo": ppo,
          "sampling": {"source": "local", "prompt_path": str(d / "prompts.jsonl")},
          "logging": {"output_dir": str(d / "ck" / f"rl_{algo}"), "log_dir": str(d / "logs" / f"rl_{algo}"),
                      "log_every_steps": 1}}
    assert train_rlhf.main(["--config", _cfg(d, f"rl_{algo}", rl)]) == 0
    m = _metrics(d / "logs" / f"rl_{algo}")
    keys = ("train/loss", "train/kl") + (("train/value_loss", "train/clipfrac") if algo == "ppo" else ())
    assert all(k in m[-1] for k in keys), m[-1]
    assert all(abs(r["train/loss"]) < 1e4 for r in m)
    assert (d / "ck" / f"rl_{algo}" / "model_2.safetensors").exists()


def test_eval_clis_gpu(stages, tmp_path):
    from distributed_llm_alignment_amd.eval import eval_alignment, eval_latency

    d, latest, _ = stages
    write_jsonl(tmp_path / "ev.jsonl", [{"question": "why?"}, {"prompt": "how?"}, {"instruction": "do"}])
    cfg = {"seed": 0, "models": {"sft": str(latest)},
           "benchmarks": {"local": {"type": "local", "prompts_path": str(tmp_path / "ev.jsonl"), "max_samples": 3}},
           "latency": {"batch_sizes": [1, 4], "seq_lengths": [64], "warmup_steps": 1, "measure_steps": 2},
           "generation": {"max_new_tokens": 6},
           "logging": {"output_path": str(tmp_path / "out" / "results.json"),
                       "table_path": str(tmp_path / "out" / "summary.md")}}
    p = _cfg(tmp_path, "eval", cfg)
    assert eval_alignment.main(["--config", p]) == 0
    res = json.loads((tmp_path / "out" / "results.json").read_text())
    assert set(res["sft"]["local"]) == {"avg_length", "refusal_rate", "toxicity_proxy"}
    assert eval_latency.main(["--config", p, "--decode_tokens", "3"]) == 0
    lat = json.loads((tmp_path / "out" / "latency.json").read_text())
    assert len(lat["sft"]) == 2 and all(r["tokens_per_second"] > 0 for r in lat["sft"])
