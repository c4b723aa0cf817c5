"""Reference config / launcher parity: every config file the reference ships exists
here under the same name, and each stage config runs through its trainer's real config path
(`--config <reference name>` + overrides that swap in a tiny model, local synthetic data and
a tmp output dir — no network). FSDP plugin keys are honoured or rejected loudly."""
import glob
import os
from pathlib import Path

import pytest
import yaml

from distributed_llm_alignment_amd.data import write_jsonl
from distributed_llm_alignment_amd.data.synthetic import (synthetic_instruction_records,
                                                          synthetic_preference_records,
                                                          synthetic_prompt_records)

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference/distributed-llm-alignment/config")

REFERENCE_CONFIGS = [
    "accelerate_config.yaml", "deepspeed_zero3.json", "distill_config.yaml", "dpo_config.yaml",
    "dpo_hh.yaml", "eval_config.yaml", "fsdp_config.yaml", "reward_config.yaml", "reward_hh.yaml",
    "rlhf_config.yaml", "sft_alpaca.yaml", "sft_config.yaml", "sft_ultrachat.yaml",
    "ablations/clip_grad_0_5.yaml", "ablations/high_beta_dpo.yaml", "ablations/low_lr.yaml",
    "data_sources/pref_hh_rlhf.yaml", "data_sources/pref_shp.yaml",
    "data_sources/rlhf_prompts_hh.yaml", "data_sources/sft_alpaca.yaml",
    "data_sources/sft_ultrachat.yaml",
]


def test_every_reference_config_name_exists():
    for name in REFERENCE_CONFIGS:
        assert (ROOT / "config" / name).exists(), name
    if REF.exists():  # and nothing the reference ships is missing from the list above
        theirs = {str(Path(p).relative_to(REF)) for p in glob.glob(str(REF / "**" / "*.*"), recursive=True)}
        assert theirs <= set(REFERENCE_CONFIGS), theirs - set(REFERENCE_CONFIGS)


def test_launch_script_defaults_are_reference_names():
    want = {"launch_sft.sh": "config/sft_config.yaml", "launch_reward.sh": "config/reward_config.yaml",
            "launch_dpo.sh": "config/dpo_config.yaml", "launch_rlhf.sh": "config/rlhf_config.yaml",
            "launch_distill.sh": "config/distill_config.yaml",
            "launch_distill_multi.sh": "config/distill_config.yaml",
            "launch_eval.sh": "config/eval_config.yaml"}
    for script, cfg in want.items():
        assert cfg in (ROOT / "scripts" / script).read_text(), script


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("cfgdata")
    write_jsonl(d / "sft.jsonl", synthetic_instruction_records(12, seed=1))
    write_jsonl(d / "pref.jsonl", synthetic_preference_records(12, seed=3))
    write_jsonl(d / "prompts.jsonl", synthetic_prompt_records(6, seed=4))
    rollouts = [{"prompt": r["prompt"], "teacher_response": r["response"], "reward": 0.5}
                for r in synthetic_instruction_records(8, seed=5)]
    write_jsonl(d / "rollouts.jsonl", rollouts)
    return d


def _ov(tmp, stage, extra):
    base = ["optimization.max_train_steps=2", f"logging.output_dir={tmp / 'ck' / stage}",
            f"logging.log_dir={tmp / 'logs' / stage}", "logging.save_every_steps=0",
            "logging.use_wandb=false", "data.num_workers=0", "hardware.gradient_accumulation_steps=1"]
    out = []
    for o in base + extra:
        out += ["--override", o]
    return out


SFT_LOCAL = lambda d: ["data.source=local", f"data.train_path={d / 'sft.jsonl'}",  # noqa: E731
                       f"data.eval_path={d / 'sft.jsonl'}", "data.template=null",
                       "model.model_name_or_path=tiny-llama", "model.max_seq_length=64",
                       "optimization.micro_batch_size=2"]
PREF_LOCAL = lambda d: ["data.source=local", f"data.train_path={d / 'pref.jsonl'}",  # noqa: E731
                        f"data.eval_path={d / 'pref.jsonl'}", f"data.preference_path={d / 'pref.jsonl'}",
                        "model.max_seq_length=64", "optimization.micro_batch_size=2"]


@pytest.mark.parametrize("name", ["sft_config.yaml", "sft_alpaca.yaml", "sft_ultrachat.yaml"])
def test_sft_reference_configs_run(tmp_path, data, name):
    from distributed_llm_alignment_amd.training import train_sft

    assert train_sft.main(["--config", str(ROOT / "config" / name), *_ov(tmp_path, "sft", SFT_LOCAL(data))]) == 0


@pytest.mark.parametrize("name", ["reward_config.yaml", "reward_hh.yaml"])
def test_reward_reference_configs_run(tmp_path, data, name):
    from distributed_llm_alignment_amd.training import train_reward

    ov = PREF_LOCAL(data) + ["model.base_model_name_or_path=tiny-llama"]
    assert train_reward.main(["--config", str(ROOT / "config" / name), *_ov(tmp_path, "rw", ov)]) == 0


@pytest.mark.parametrize("name,overlay", [("dpo_config.yaml", None), ("dpo_hh.yaml", None),
                                          ("dpo_config.yaml", "ablations/high_beta_dpo.yaml"),
                                          ("dpo_config.yaml", "ablations/low_lr.yaml"),
                                          ("dpo_config.yaml", "ablations/clip_grad_0_5.yaml")])
def test_dpo_reference_configs_run(tmp_path, data, name, overlay):
    from distributed_llm_alignment_amd.training import train_dpo

    ov = PREF_LOCAL(data) + ["model.policy_model_name_or_path=tiny-llama",
                             "model.reference_model_name_or_path=tiny-llama"]
    args = ["--config", str(ROOT / "config" / name)]
    if overlay:
        args += ["--overlay", str(ROOT / "config" / overlay)]
    assert train_dpo.main(args + _ov(tmp_path, "dpo", ov)) == 0


def test_rlhf_reference_config_runs(tmp_path, data):
    from distributed_llm_alignment_amd.training import train_rlhf

    ov = ["model.policy_model_name_or_path=tiny-llama", "model.reference_model_name_or_path=tiny-llama",
          "model.max_seq_length=48", "reward_model.path=null", "reward_model.base_model_name_or_path=tiny-llama",
          "ppo.batch_size=2", "ppo.steps=2", "ppo.generation_params.max_new_tokens=4",
          "sampling.source=local", f"sampling.prompt_path={data / 'prompts.jsonl'}"]
    assert train_rlhf.main(["--config", str(ROOT / "config" / "rlhf_config.yaml"), *_ov(tmp_path, "rl", ov)]) == 0


def test_distill_reference_config_runs(tmp_path, data):
    from distributed_llm_alignment_amd.training import train_distill

    ov = ["model.student_model_name_or_path=tiny-llama", "model.teacher_path=tiny-llama",
          "distill.teacher_model_name_or_path=tiny-llama", "model.max_seq_length=64",
          f"data.teacher_samples_path={data / 'rollouts.jsonl'}", "optimization.micro_batch_size=2"]
    assert train_distill.main(["--config", str(ROOT / "config" / "distill_config.yaml"),
                               *_ov(tmp_path, "dist", ov)]) == 0


def test_eval_reference_config_runs(tmp_path, data):
    from distributed_llm_alignment_amd.eval import eval_alignment

    cfg = yaml.safe_load((ROOT / "config" / "eval_config.yaml").read_text())
    assert set(cfg["models"]) >= {"base", "sft", "dpo", "distill"}
    args = ["--config", str(ROOT / "config" / "eval_config.yaml"), "--max_prompts", "2"]
    for o in ["models={tiny: tiny-llama}", "generation.max_new_tokens=3",
              f"benchmarks={{local: {{type: local, prompts_path: {data / 'prompts.jsonl'}, max_samples: 2}}}}",
              f"logging.output_path={tmp_path / 'res.json'}", f"logging.table_path={tmp_path / 'sum.md'}"]:
        args += ["--override", o]
    assert eval_alignment.main(args) == 0
    assert (tmp_path / "res.json").exists()


def test_flat_data_source_fragments_overlay():
    from distributed_llm_alignment_amd.utils.config import load_config

    cfg = load_config(ROOT / "config" / "sft_config.yaml",
                      overlays=[ROOT / "config" / "data_sources" / "sft_alpaca.yaml"])
    assert cfg["data"]["hf_path"] == "yahma/alpaca-cleaned" and cfg["data"]["mask_prompt"] is True
    cfg = load_config(ROOT / "config" / "rlhf_config.yaml",
                      overlays=[ROOT / "config" / "data_sources" / "rlhf_prompts_hh.yaml"])
    assert cfg["sampling"]["limit"] == 20000 and cfg["sampling"]["prompt_key"] == "prompt"
    if REF.exists():  # the reference's own fragments work the same way
        cfg = load_config(ROOT / "config" / "dpo_config.yaml", overlays=[REF / "data_sources" / "pref_shp.yaml"])
        assert cfg["data"]["hf_path"] == "stanfordnlp/SHP"


def test_fsdp_keys_honoured_or_rejected(tmp_path):
    import torch

    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.parallel.fsdp import FullyShardedEngine, default_units
    from distributed_llm_alignment_amd.utils.config import hardware_parallel, load_config

    hp = hardware_parallel(load_config(ROOT / "config" / "fsdp_config.yaml"))
    assert hp["fsdp"] and hp["zero_stage"] == 3 and hp["fsdp_min_num_params"] == 1_000_000
    assert hp["cpu_offload"] is False
    m = build_model(get_config("tiny-llama"), device="cpu", seed=0)
    per_layer = sum(p.numel() for p in m.layers[0].parameters())
    assert [len(u) for u in default_units(m, 0)] == [1, 1]
    assert [len(u) for u in default_units(m, per_layer + 1)] == [2]  # size-based wrap merges layers
    eng = FullyShardedEngine(m, lr=1e-3, min_num_params=per_layer + 1)
    assert len(eng.units) == 2  # one merged layer unit + the root
    with pytest.raises(ValueError, match="offload"):
        FullyShardedEngine(build_model(get_config("tiny-llama"), device="cpu", seed=0), cpu_offload=True)
    bad = tmp_path / "ds.json"
    bad.write_text('{"zero_optimization": {"stage": 3, "offload_param": {"device": "cpu"}}}')
    with pytest.raises(ValueError, match="offload"):
        hardware_parallel({"hardware": {"deepspeed_config": str(bad)}})
    x = torch.randint(3, 500, (2, 9))
    assert torch.isfinite(m.sequence_logprob(x, torch.ones_like(x))).all()
