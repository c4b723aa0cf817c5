"""Synthetic data (no network): text records in the reference JSONL schemas, and token-level
batches of exact shape for benchmarks (SURVEY §7.2 slices A/B: synthetic instruction pairs and
preference pairs with a controllable length distribution)."""
from __future__ import annotations

import random
from typing import Dict, List, Optional

import torch

_WORDS = ("the a model answer question explain why how what data train learn align reward "
          "policy value safe helpful honest step reason compute kernel wave memory cache token "
          "sequence batch gradient update loss optimize scale network parallel fast").split()


def _sentence(rng: random.Random, lo: int, hi: int) -> str:
    return " ".join(rng.choice(_WORDS) for _ in range(rng.randint(lo, hi)))


def synthetic_instruction_records(n: int, seed: int = 0, lo: int = 4, hi: int = 24) -> List[Dict[str, str]]:
    rng = random.Random(seed)
    return [{"prompt": _sentence(rng, lo, hi) + "?", "response": _sentence(rng, lo, 2 * hi) + "."}
            for _ in range(n)]


def synthetic_preference_records(n: int, seed: int = 0, lo: int = 4, hi: int = 24) -> List[Dict[str, str]]:
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        p = _sentence(rng, lo, hi) + "?"
        good = "Sure. " + _sentence(rng, lo, 2 * hi) + "."
        bad = "No. " + _sentence(rng, lo, hi)
        out.append({"prompt": p, "chosen": good, "rejected": bad})
    return out


def synthetic_prompt_records(n: int, seed: int = 0) -> List[Dict[str, str]]:
    rng = random.Random(seed)
    return [{"prompt": _sentence(rng, 4, 16) + "?"} for _ in range(n)]


def synthetic_preference_batch(pairs: int, seq_len: int, vocab_size: int, device=None,
                               generator: Optional[torch.Generator] = None,
                               min_len: Optional[int] = None, pad_id: int = 0) -> Dict[str, Dict[str, torch.Tensor]]:
    """Token-level DPO micro-batch in the PreferenceDataset.collate layout. With min_len, each
    sequence gets a random length in [min_len, seq_len] (right padded); else all full length."""
    def side():
        ids = torch.randint(3, vocab_size, (pairs, seq_len), generator=generator)
        mask = torch.ones(pairs, seq_len, dtype=torch.long)
        if min_len is not None and min_len < seq_len:
            lens = torch.randint(min_len, seq_len + 1, (pairs,), generator=generator)
            ar = torch.arange(seq_len).unsqueeze(0)
            mask = (ar < lens.unsqueeze(1)).long()
            ids = torch.where(mask.bool(), ids, torch.full_like(ids, pad_id))
        return {"input_ids": ids.to(device), "attention_mask": mask.to(device)}

    return {"chosen": side(), "rejected": side()}


def synthetic_lm_batch(batch: int, seq_len: int, vocab_size: int, device=None,
                       generator: Optional[torch.Generator] = None) -> Dict[str, torch.Tensor]:
    ids = torch.randint(3, vocab_size, (batch, seq_len), generator=generator)
    return {"input_ids": ids.to(device), "attention_mask": torch.ones_like(ids).to(device),
            "labels": ids.clone().to(device)}
