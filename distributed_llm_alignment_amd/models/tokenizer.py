"""Tokenizers: HF tokenizers from local directories, plus an offline byte-level fallback.

The reference calls `AutoTokenizer.from_pretrained(name, use_fast=True)` and sets
pad := eos when missing (src/models/base_model.py:23-25). Without network access a hub id cannot
be fetched, so for presets / random-init models the framework uses `ByteTokenizer`, which has
the same call surface the data pipeline needs (`__call__`, `decode`, `batch_decode`,
`pad_token_id`, `eos_token`, `model_max_length`, `padding_side`).
"""
from __future__ import annotations

from pathlib import Path
from typing import Dict, List, Optional, Sequence, Union

import torch


class ByteTokenizer:
    """UTF-8 bytes -> ids `byte + offset`; ids 0/1/2 = pad/bos/eos by default."""

    def __init__(self, vocab_size: int = 259, bos_token_id: int = 1, eos_token_id: int = 2,
                 pad_token_id: Optional[int] = None, offset: int = 3, model_max_length: int = 4096,
                 add_bos: bool = True):
        self.offset = offset
        self.vocab_size = max(vocab_size, 256 + offset)
        self.bos_token_id = bos_token_id
        self.eos_token_id = eos_token_id
        self.pad_token_id = pad_token_id if pad_token_id is not None else eos_token_id
        self.bos_token = "<s>"
        self.eos_token = "</s>"
        self.pad_token = self.eos_token if self.pad_token_id == eos_token_id else "<pad>"
        self.model_max_length = model_max_length
        self.padding_side = "right"
        self.add_bos = add_bos

    def _encode_one(self, text: str, add_special_tokens: bool = True) -> List[int]:
        ids: List[int] = []
        if add_special_tokens and self.add_bos:
            ids.append(self.bos_token_id)
        i = 0
        eos = self.eos_token
        while i < len(text):
            if text.startswith(eos, i):
                ids.append(self.eos_token_id)
                i += len(eos)
                continue
            j = text.find(eos, i)
            chunk = text[i:] if j < 0 else text[i:j]
            ids.extend(b + self.offset for b in chunk.encode("utf-8"))
            i += len(chunk)
        return ids

    def encode(self, text: str, add_special_tokens: bool = True) -> List[int]:
        return self._encode_one(text, add_special_tokens)

    def __call__(self, text: Union[str, Sequence[str]], truncation: bool = False,
                 max_length: Optional[int] = None, padding: Union[bool, str] = False,
                 return_tensors: Optional[str] = None, add_special_tokens: bool = True, **_):
        single = isinstance(text, str)
        texts = [text] if single else list(text)
        batch = [self._encode_one(t, add_special_tokens) for t in texts]
        if truncation and max_length:
            batch = [ids[:max_length] for ids in batch]
        masks = [[1] * len(ids) for ids in batch]
        if padding and len(batch) > 0:
            L = max(len(x) for x in batch)
            if padding == "max_length" and max_length:
                L = max_length
            for k in range(len(batch)):
                n = L - len(batch[k])
                if self.padding_side == "left":
                    batch[k] = [self.pad_token_id] * n + batch[k]
                    masks[k] = [0] * n + masks[k]
                else:
                    batch[k] = batch[k] + [self.pad_token_id] * n
                    masks[k] = masks[k] + [0] * n
        out: Dict[str, object] = {"input_ids": batch, "attention_mask": masks}
        if return_tensors == "pt":
            out = {k: torch.tensor(v, dtype=torch.long) for k, v in out.items()}
        elif single:
            out = {k: v[0] for k, v in out.items()}
        return _Encoding(out)

    def decode(self, ids, skip_special_tokens: bool = False) -> str:
        if isinstance(ids, torch.Tensor):
            ids = ids.tolist()
        bs = bytearray()
        parts: List[str] = []
        for t in ids:
            t = int(t)
            if t >= self.offset and t < self.offset + 256:
                bs.append(t - self.offset)
            else:
                if bs:
                    parts.append(bs.decode("utf-8", errors="replace"))
                    bs = bytearray()
                if not skip_special_tokens:
                    parts.append(self.eos_token if t == self.eos_token_id else
                                 self.bos_token if t == self.bos_token_id else "")
        if bs:
            parts.append(bs.decode("utf-8", errors="replace"))
        return "".join(parts)

    def batch_decode(self, seqs, skip_special_tokens: bool = False) -> List[str]:
        return [self.decode(s, skip_special_tokens) for s in seqs]

    def save_pretrained(self, path: Union[str, Path]):
        import json

        Path(path).mkdir(parents=True, exist_ok=True)
        (Path(path) / "dla_tokenizer.json").write_text(json.dumps({
            "type": "byte", "vocab_size": self.vocab_size, "bos_token_id": self.bos_token_id,
            "eos_token_id": self.eos_token_id, "pad_token_id": self.pad_token_id,
            "offset": self.offset, "model_max_length": self.model_max_length}))


class _Encoding(dict):
    """dict with attribute access and `.to(device)` like transformers.BatchEncoding."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def to(self, device):
        return _Encoding({k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in self.items()})


def load_tokenizer(name_or_path: str, cfg=None):
    """HF tokenizer from a local dir when present, else ByteTokenizer sized to the model."""
    p = Path(str(name_or_path))
    if p.is_dir() and (p / "dla_tokenizer.json").exists():
        import json

        d = json.loads((p / "dla_tokenizer.json").read_text())
        return ByteTokenizer(vocab_size=d["vocab_size"], bos_token_id=d["bos_token_id"],
                             eos_token_id=d["eos_token_id"], pad_token_id=d["pad_token_id"],
                             offset=d["offset"], model_max_length=d["model_max_length"])
    if p.is_dir() and any((p / f).exists() for f in ("tokenizer.json", "tokenizer_config.json", "tokenizer.model")):
        from transformers import AutoTokenizer

        tok = AutoTokenizer.from_pretrained(str(p), use_fast=True)
        if tok.pad_token is None:
            tok.pad_token = tok.eos_token
        return tok
    vocab = cfg.vocab_size if cfg is not None else 259
    bos = cfg.bos_token_id if cfg is not None and cfg.bos_token_id < 3 else 1
    eos = cfg.eos_token_id if cfg is not None and cfg.eos_token_id < 3 else 2
    return ByteTokenizer(vocab_size=vocab, bos_token_id=bos, eos_token_id=eos,
                         model_max_length=(cfg.max_position_embeddings if cfg is not None else 4096))
