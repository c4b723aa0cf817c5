"""Datasets, collation and record loaders with the reference's data semantics
(src/data/datasets.py):

  SFT        {"prompt","response"}          text = f"{prompt}\\n\\n{response}{eos}", labels = ids,
                                            prompt tokens -> -100 when mask_prompt
  Preference {"prompt","chosen","rejected"}  two sequences, no prompt masking (reference default;
                                            `mask_prompt=True` available as an option)
  Teacher    {"prompt","teacher_response","reward"?}  reward defaults to 1.0
  pad_batch  right padding; labels -> -100, input_ids -> pad id, attention_mask -> 0, other -> 0

Deviations (documented fixes of SURVEY Appendix A):
  #2  0-d tensors (teacher `reward`) are stacked, not passed to pad_sequence (which crashes).
  #14 the SFT prompt mask length is measured with the SAME special-token setting as the full
      text, so BOS-adding tokenizers no longer mask one token short.
  #18 hh-rlhf-style rows without a `prompt` column get prompt = common prefix of chosen/rejected.
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, List, Optional

import torch
from torch.utils.data import Dataset


@dataclass
class Sample:
    prompt: str
    response: Optional[str] = None
    chosen: Optional[str] = None
    rejected: Optional[str] = None
    reward: Optional[float] = None


def read_jsonl(path) -> List[Dict[str, Any]]:
    with Path(path).open("r", encoding="utf-8") as fh:
        return [json.loads(line) for line in fh if line.strip()]


def write_jsonl(path, records) -> None:
    Path(path).parent.mkdir(parents=True, exist_ok=True)
    with Path(path).open("w", encoding="utf-8") as fh:
        for r in records:
            fh.write(json.dumps(r) + "\n")


def _ids(enc) -> torch.Tensor:
    x = enc["input_ids"]
    if isinstance(x, torch.Tensor):
        return x.reshape(-1).long()
    return torch.tensor(x, dtype=torch.long).reshape(-1)


def _eos(tokenizer) -> str:
    return getattr(tokenizer, "eos_token", None) or getattr(tokenizer, "pad_token", None) or "</s>"


def _pad_id(tokenizer) -> int:
    pid = getattr(tokenizer, "pad_token_id", None)
    return pid if pid is not None else 0


class InstructionDataset(Dataset):
    """Tokenised prompt/response pairs for SFT (reference datasets.py:30-83)."""

    def __init__(self, tokenizer, max_length: int, mask_prompt: bool = True, path=None,
                 records: Optional[List[Dict[str, Any]]] = None):
        if records is None and path is None:
            raise ValueError("Provide either records or path for InstructionDataset")
        self.records = records if records is not None else read_jsonl(path)
        self.tokenizer = tokenizer
        self.max_length = max_length
        self.mask_prompt = mask_prompt
        self.eos = _eos(tokenizer)

    def __len__(self) -> int:
        return len(self.records)

    def __getitem__(self, idx: int) -> Dict[str, torch.Tensor]:
        item = self.records[idx]
        prompt = str(item["prompt"]).strip()
        response = str(item["response"]).strip()
        enc = self.tokenizer(f"{prompt}\n\n{response}{self.eos}", truncation=True,
                             max_length=self.max_length, padding=False)
        input_ids = _ids(enc)
        labels = input_ids.clone()
        if self.mask_prompt:
            penc = self.tokenizer(f"{prompt}\n\n", truncation=True, max_length=self.max_length,
                                  padding=False)
            labels[: min(len(_ids(penc)), len(labels))] = -100
        return {"input_ids": input_ids, "attention_mask": torch.ones_like(input_ids),
                "labels": labels}

    def collate(self, batch):
        return pad_batch(batch, _pad_id(self.tokenizer))


class PackedDataset(Dataset):
    """`data.packing: true` (a dead key in the reference, sft_config.yaml:16): SFT
    examples concatenated into rows of at most `max_length` tokens, in order (greedy, a new row
    when the next example does not fit). Each row carries `segment_ids` (1, 2, ... per example),
    so the model runs block-diagonal causal attention with per-example positions
    (models.transformer.packed_layout) — numerically the same as the examples run one by one,
    without the padding FLOPs. Labels are -100 at each example's first token, so no example is
    trained to predict the next one's start."""

    def __init__(self, base: Dataset, max_length: int):
        self.base = base
        self.max_length = max_length
        self.tokenizer = getattr(base, "tokenizer", None)
        self.rows: List[List[int]] = []
        cur: List[int] = []
        used = 0
        for i in range(len(base)):
            n = min(int(base[i]["input_ids"].numel()), max_length)
            if cur and used + n > max_length:
                self.rows.append(cur)
                cur, used = [], 0
            cur.append(i)
            used += n
        if cur:
            self.rows.append(cur)

    def __len__(self) -> int:
        return len(self.rows)

    def __getitem__(self, idx: int) -> Dict[str, torch.Tensor]:
        ids, labels, segs = [], [], []
        for j, i in enumerate(self.rows[idx]):
            ex = self.base[i]
            x = ex["input_ids"][: self.max_length]
            lab = ex["labels"][: self.max_length].clone()
            lab[0] = -100
            ids.append(x)
            labels.append(lab)
            segs.append(torch.full_like(x, j + 1))
        input_ids = torch.cat(ids)
        return {"input_ids": input_ids, "attention_mask": torch.ones_like(input_ids),
                "labels": torch.cat(labels), "segment_ids": torch.cat(segs)}

    def collate(self, batch):
        return pad_batch(batch, _pad_id(self.tokenizer) if self.tokenizer is not None else 0)


class PreferenceDataset(Dataset):
    """(prompt, chosen, rejected) triples for RM / DPO (reference datasets.py:86-152)."""

    def __init__(self, tokenizer, max_length: int, path=None,
                 records: Optional[List[Dict[str, Any]]] = None, mask_prompt: bool = False):
        if records is None and path is None:
            raise ValueError("Provide either records or path for PreferenceDataset")
        self.records = records if records is not None else read_jsonl(path)
        self.tokenizer = tokenizer
        self.max_length = max_length
        self.eos = _eos(tokenizer)
        self.mask_prompt = mask_prompt

    def __len__(self) -> int:
        return len(self.records)

    def _tokenize(self, prompt: str, response: str) -> Dict[str, torch.Tensor]:
        enc = self.tokenizer(f"{prompt}\n\n{response}{self.eos}", truncation=True,
                             max_length=self.max_length, padding=False)
        ids = _ids(enc)
        out = {"input_ids": ids, "attention_mask": torch.ones_like(ids)}
        if self.mask_prompt:
            penc = self.tokenizer(f"{prompt}\n\n", truncation=True, max_length=self.max_length)
            lm = torch.ones_like(ids)
            lm[: min(len(_ids(penc)), len(ids))] = 0
            out["loss_mask"] = lm
        return out

    def __getitem__(self, idx: int) -> Dict[str, torch.Tensor]:
        item = self.records[idx]
        prompt = str(item["prompt"]).strip()
        c = self._tokenize(prompt, str(item["chosen"]).strip())
        r = self._tokenize(prompt, str(item["rejected"]).strip())
        out = {"chosen_input_ids": c["input_ids"], "chosen_attention_mask": c["attention_mask"],
               "rejected_input_ids": r["input_ids"], "rejected_attention_mask": r["attention_mask"]}
        if self.mask_prompt:
            out["chosen_loss_mask"] = c["loss_mask"]
            out["rejected_loss_mask"] = r["loss_mask"]
        return out

    def collate(self, batch):
        pid = _pad_id(self.tokenizer)
        out = {}
        for side in ("chosen", "rejected"):
            keys = [k for k in batch[0] if k.startswith(side + "_")]
            out[side] = pad_batch([{k[len(side) + 1:]: item[k] for k in keys} for item in batch], pid)
        return out


class TeacherRolloutDataset(Dataset):
    """Teacher rollouts for distillation (reference datasets.py:155-196)."""

    def __init__(self, path=None, tokenizer=None, max_length: int = 2048,
                 records: Optional[List[Dict[str, Any]]] = None):
        self.records = records if records is not None else read_jsonl(path)
        self.tokenizer = tokenizer
        self.max_length = max_length
        self.eos = _eos(tokenizer)

    def __len__(self) -> int:
        return len(self.records)

    def __getitem__(self, idx: int) -> Dict[str, torch.Tensor]:
        item = self.records[idx]
        prompt = str(item["prompt"]).strip()
        response = str(item["teacher_response"]).strip()
        reward = float(item.get("reward", 1.0))
        enc = self.tokenizer(f"{prompt}\n\n{response}{self.eos}", truncation=True,
                             max_length=self.max_length, padding=False)
        ids = _ids(enc)
        return {"input_ids": ids, "attention_mask": torch.ones_like(ids), "labels": ids.clone(),
                "reward": torch.tensor(reward, dtype=torch.float32)}

    def collate(self, batch):
        return pad_batch(batch, _pad_id(self.tokenizer))


class EvalPromptDataset(Dataset):
    def __init__(self, path):
        self.records = read_jsonl(path)

    def __len__(self):
        return len(self.records)

    def __getitem__(self, idx):
        return self.records[idx]


def pad_batch(batch: List[Dict[str, torch.Tensor]], pad_token_id: int) -> Dict[str, torch.Tensor]:
    """Right-pad each key; 0-d tensors are stacked (fix for Appendix A #2)."""
    out: Dict[str, torch.Tensor] = {}
    for key in batch[0].keys():
        tensors = [ex[key] for ex in batch]
        if tensors[0].dim() == 0:
            out[key] = torch.stack(tensors)
            continue
        if key == "labels":
            pad = -100
        elif key == "input_ids":
            pad = pad_token_id
        else:
            pad = 0
        out[key] = torch.nn.utils.rnn.pad_sequence(tensors, batch_first=True, padding_value=pad)
    return out


# ------------------------------------------------------------------------------ record loaders
def _load_hf(cfg: Dict[str, Any], split: str):
    from datasets import load_dataset

    split_name = cfg.get(f"{split}_split") or cfg.get("split", split)
    return load_dataset(cfg["hf_path"], cfg.get("hf_name"), split=split_name, streaming=False)


def _common_prefix(a: str, b: str) -> str:
    n = 0
    for x, y in zip(a, b):
        if x != y:
            break
        n += 1
    cut = a.rfind("Assistant:", 0, n)
    return a[: cut + len("Assistant:")] if cut >= 0 else a[:n]


def load_instruction_records(cfg: Dict[str, Any], split: str = "train") -> List[Dict[str, Any]]:
    source = cfg.get("source", "local")
    limit = cfg.get("limit")
    if source == "synthetic":
        from .synthetic import synthetic_instruction_records

        records = synthetic_instruction_records(int(cfg.get("num_samples", 256)), seed=int(cfg.get("seed", 0)))
    elif source == "hf":
        ds = _load_hf(cfg, split)
        cols = cfg.get("columns", {})
        pk, rk = cols.get("prompt", "prompt"), cols.get("response", "response")
        template = cfg.get("template")
        records = []
        for row in ds:
            prompt = template.format(**row) if template else row[pk]
            records.append({"prompt": prompt, "response": row[rk]})
    else:
        path = cfg.get(f"{split}_path") or cfg.get("path")
        if path is None:
            raise ValueError(f"data config has no {split}_path/path")
        records = read_jsonl(path)
    if limit:
        records = records[: int(limit)]
    return records


def load_preference_records(cfg: Dict[str, Any], split: str = "train") -> List[Dict[str, Any]]:
    source = cfg.get("source", "local")
    limit = cfg.get("limit")
    if source == "synthetic":
        from .synthetic import synthetic_preference_records

        records = synthetic_preference_records(int(cfg.get("num_samples", 256)), seed=int(cfg.get("seed", 0)))
    elif source == "hf":
        ds = _load_hf(cfg, split)
        cols = cfg.get("columns", {})
        pk, ck, rk = cols.get("prompt", "prompt"), cols.get("chosen", "chosen"), cols.get("rejected", "rejected")
        template = cfg.get("template")
        label_key = cfg.get("label_column")  # e.g. SHP "labels": 1 -> A preferred
        records = []
        for row in ds:
            chosen, rejected = row[ck], row[rk]
            if label_key is not None and not row[label_key]:
                chosen, rejected = rejected, chosen
            if template:
                prompt = template.format(**row)
            elif pk in row:
                prompt = row[pk]
            else:
                prompt = _common_prefix(chosen, rejected)
                chosen, rejected = chosen[len(prompt):], rejected[len(prompt):]
            records.append({"prompt": prompt, "chosen": chosen, "rejected": rejected})
    else:
        path = cfg.get(f"{split}_path") or cfg.get("path") or cfg.get("preference_path")
        if path is None:
            raise ValueError(f"data config has no {split}_path/path/preference_path")
        records = read_jsonl(path)
    if limit:
        records = records[: int(limit)]
    return records


def build_instruction_dataset(cfg: Dict[str, Any], tokenizer, split: str = "train"):
    max_length = cfg.get("max_length", cfg.get("max_seq_length", 2048))
    ds = InstructionDataset(tokenizer=tokenizer, max_length=max_length,
                            mask_prompt=cfg.get("mask_prompt", True),
                            records=load_instruction_records(cfg, split=split))
    return PackedDataset(ds, max_length) if cfg.get("packing", False) else ds


def build_preference_dataset(cfg: Dict[str, Any], tokenizer, split: str = "train") -> PreferenceDataset:
    return PreferenceDataset(tokenizer=tokenizer,
                             max_length=cfg.get("max_length", cfg.get("max_seq_length", 1024)),
                             records=load_preference_records(cfg, split=split),
                             mask_prompt=cfg.get("mask_prompt", False))
