"""CPU tier: data schemas, templating, masking, padding, loaders."""
import json

import pytest
import torch

from distributed_llm_alignment_amd.data import (InstructionDataset, PreferenceDataset, TeacherRolloutDataset,
                                                build_instruction_dataset, build_preference_dataset,
                                                load_preference_records, pad_batch, read_jsonl, write_jsonl)
from distributed_llm_alignment_amd.models import ByteTokenizer


@pytest.fixture
def tok():
    return ByteTokenizer()


def test_sft_template_and_prompt_mask(tok):
    ds = InstructionDataset(tok, 64, mask_prompt=True, records=[{"prompt": " Hi? ", "response": "Yo."}])
    item = ds[0]
    text_ids = tok("Hi?\n\nYo.</s>")["input_ids"]
    assert item["input_ids"].tolist() == text_ids
    n_prompt = len(tok("Hi?\n\n")["input_ids"])
    assert (item["labels"][:n_prompt] == -100).all()
    assert item["labels"][n_prompt:].tolist() == text_ids[n_prompt:]
    assert text_ids[-1] == tok.eos_token_id


def test_truncation(tok):
    ds = InstructionDataset(tok, 5, mask_prompt=False, records=[{"prompt": "abcdefgh", "response": "x"}])
    assert len(ds[0]["input_ids"]) == 5


def test_pad_batch_values():
    b = [{"input_ids": torch.tensor([5, 6, 7]), "attention_mask": torch.tensor([1, 1, 1]), "labels": torch.tensor([5, 6, 7])},
         {"input_ids": torch.tensor([8]), "attention_mask": torch.tensor([1]), "labels": torch.tensor([8])}]
    out = pad_batch(b, pad_token_id=2)
    assert out["input_ids"][1].tolist() == [8, 2, 2]
    assert out["attention_mask"][1].tolist() == [1, 0, 0]
    assert out["labels"][1].tolist() == [8, -100, -100]


def test_preference_collate_layout(tok):
    ds = PreferenceDataset(tok, 64, records=[{"prompt": "p", "chosen": "good answer", "rejected": "bad"},
                                             {"prompt": "q", "chosen": "a", "rejected": "bb"}])
    batch = ds.collate([ds[0], ds[1]])
    assert set(batch) == {"chosen", "rejected"}
    assert batch["chosen"]["input_ids"].shape[0] == 2
    assert batch["rejected"]["attention_mask"][1].sum() == len(tok("q\n\nbb</s>")["input_ids"])


def test_teacher_rollout_collate_stacks_rewards(tok, tmp_path):
    """Reference crashes here (pad_sequence on 0-d tensors)."""
    p = tmp_path / "r.jsonl"
    write_jsonl(p, [{"prompt": "a", "teacher_response": "b", "reward": 0.5}, {"prompt": "c", "teacher_response": "dd"}])
    ds = TeacherRolloutDataset(p, tok, 32)
    batch = ds.collate([ds[0], ds[1]])
    assert batch["reward"].tolist() == [0.5, 1.0]
    assert batch["labels"].shape == batch["input_ids"].shape


def test_local_loaders_limit_and_paths(tok, tmp_path):
    p = tmp_path / "pref.jsonl"
    write_jsonl(p, [{"prompt": f"p{i}", "chosen": "c", "rejected": "r"} for i in range(10)])
    recs = load_preference_records({"source": "local", "preference_path": str(p), "limit": 4})
    assert len(recs) == 4
    ds = build_preference_dataset({"source": "local", "train_path": str(p), "max_seq_length": 16}, tok)
    assert len(ds) == 10 and ds.max_length == 16
    sft = build_instruction_dataset({"source": "synthetic", "num_samples": 7}, tok)
    assert len(sft) == 7 and sft.max_length == 2048


def test_hh_rlhf_common_prefix_adapter(monkeypatch):
    rows = [{"chosen": "\n\nHuman: hi\n\nAssistant: hello there", "rejected": "\n\nHuman: hi\n\nAssistant: go away"}]

    class FakeDS(list):
        pass

    import distributed_llm_alignment_amd.data.datasets as dmod

    monkeypatch.setattr(dmod, "_load_hf", lambda cfg, split: FakeDS(rows))
    recs = load_preference_records({"source": "hf", "hf_path": "x", "columns": {"chosen": "chosen", "rejected": "rejected"}})
    assert recs[0]["prompt"].endswith("Assistant:")
    assert recs[0]["chosen"] == " hello there" and recs[0]["rejected"] == " go away"


def test_reference_configs_load_with_our_schema():
    """The reference's own YAML files parse and map onto this framework's settings."""
    import glob
    import os

    from distributed_llm_alignment_amd.utils.config import hardware_parallel, load_config

    root = "/root/reference/distributed-llm-alignment/config"
    files = sorted(glob.glob(os.path.join(root, "*.yaml")))
    if not files:
        pytest.skip("reference configs not mounted")
    for f in files:
        cfg = load_config(f)
        hp = hardware_parallel({**cfg, "hardware": {**(cfg.get("hardware") or {}),
                                                    "deepspeed_config": None}})
        assert hp["grad_accum"] >= 1
    fsdp = load_config(os.path.join(root, "fsdp_config.yaml"))
    hp = hardware_parallel(fsdp)
    assert hp["fsdp"] is True and hp["zero_stage"] == 3
