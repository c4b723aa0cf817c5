"""Autoregressive generation with a preallocated KV cache.

Replaces HF `model.generate` used by the reference's RLHF rollouts (src/training/train_rlhf.py:123-124),
teacher data generation (generate_teacher_data.py:72-79) and alignment eval
(eval_alignment.py:68-79). Prompts are LEFT-padded (fixing Appendix A #10); positions start at
each row's first real token; finished rows emit `pad_token_id`. The cache is contiguous
[L, B, T_max, Hkv, D] per K/V sized once for prompt + max_new_tokens (HBM is plentiful), the
prefill runs the flash-attention kernel over the whole prompt and each decode step attends
to the cache through the same kernel with causal offset.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from .. import ops
from .transformer import CausalLM, attention_layout


class KVCache:
    def __init__(self, model: CausalLM, batch: int, max_len: int, kv_start: Optional[torch.Tensor]):
        cfg = model.cfg
        dev, dt = model.embed.device, model.embed.dtype
        L, Hkv, D = cfg.num_layers, model.layers[0].attn.kv_local, cfg.head_dim
        self.h_local, self.kv_local = model.layers[0].attn.h_local, Hkv
        self.cfg = cfg
        self.k = torch.empty((L, batch, max_len, Hkv, D), device=dev, dtype=dt)
        self.v = torch.empty((L, batch, max_len, Hkv, D), device=dev, dtype=dt)
        self.max_len = max_len
        self.len = 0
        self.batch = batch
        self.kv_start = kv_start.to(torch.int32) if kv_start is not None else None
        self._pos = None

    def positions_for(self, T: int) -> torch.Tensor:
        dev = self.k.device
        t = torch.arange(self.len, self.len + T, device=dev, dtype=torch.int32).unsqueeze(0)
        start = self.kv_start.unsqueeze(1) if self.kv_start is not None else 0
        self._pos = (t - start).clamp(min=0).expand(self.batch, T).contiguous()
        return self._pos

    def attend(self, layer: int, qkv: torch.Tensor, rope, window: int) -> torch.Tensor:
        cfg = self.cfg
        B, T, _ = qkv.shape
        if self.len + T > self.max_len:
            raise RuntimeError("KV cache overflow")
        q, k, v = ops.attention.rope_qk(qkv, rope, self.h_local, self.kv_local, cfg.head_dim,
                                        positions=self._pos)
        self.k[layer, :, self.len:self.len + T] = k
        self.v[layer, :, self.len:self.len + T] = v
        end = self.len + T
        o = ops.attention_core(q.contiguous(), self.k[layer, :, :end], self.v[layer, :, :end],
                               causal=True, causal_off=self.len, window=window,
                               kv_start=self.kv_start, kv_end=None)
        return o.reshape(B, T, self.h_local * cfg.head_dim)

    def advance(self, T: int):
        self.len += T


@dataclass
class GenerationConfig:
    max_new_tokens: int = 256
    do_sample: bool = True
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    eos_token_id: Optional[int] = None
    pad_token_id: Optional[int] = None


def sample_next(logits: torch.Tensor, do_sample: bool, temperature: float, top_p: float,
                top_k: int = 0, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """logits [B, V] fp32 -> token ids [B]. Temperature, top-k, nucleus (top-p) filtering."""
    if not do_sample or temperature <= 0:
        return logits.argmax(-1)
    logits = logits / temperature
    if top_k and top_k > 0:
        kth = torch.topk(logits, top_k, dim=-1).values[:, -1:]
        logits = logits.masked_fill(logits < kth, float("-inf"))
    if top_p < 1.0:
        sl, si = torch.sort(logits, descending=True, dim=-1)
        probs = torch.softmax(sl, dim=-1)
        cum = probs.cumsum(-1)
        remove = (cum - probs) > top_p
        sl = sl.masked_fill(remove, float("-inf"))
        logits = torch.full_like(logits, float("-inf")).scatter(-1, si, sl)
    probs = torch.softmax(logits, dim=-1)
    return torch.multinomial(probs, 1, generator=generator).squeeze(-1)


@torch.no_grad()
def generate(model: CausalLM, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
             max_new_tokens: int = 256, do_sample: bool = True, temperature: float = 1.0,
             top_p: float = 1.0, top_k: int = 0, eos_token_id: Optional[int] = None,
             pad_token_id: Optional[int] = None, generator: Optional[torch.Generator] = None,
             return_mask: bool = False):
    """Left-padded prompts [B, Tp] -> sequences [B, Tp + n] (n <= max_new_tokens).

    With `return_mask`, also returns the attention mask of the full sequence (prompt mask, then
    1 for every generated token up to and including EOS, 0 afterwards) — the correct mask for
    the RLHF log-prob pass (fixes Appendix A #10's `generated != pad` which drops real EOS)."""
    was_training = model.training
    model.eval()
    B, Tp = input_ids.shape
    eos = eos_token_id if eos_token_id is not None else model.cfg.eos_token_id
    pad = pad_token_id if pad_token_id is not None else eos
    kv_start = None
    if attention_mask is not None:
        kv_start, _, _ = attention_layout(attention_mask)
    cache = KVCache(model, B, Tp + max_new_tokens, kv_start)
    h = model(input_ids, cache=cache)
    out = [input_ids]
    gen_mask = []
    finished = torch.zeros(B, dtype=torch.bool, device=input_ids.device)
    last = h[:, -1]
    for step in range(max_new_tokens):
        logits = model.logits(last).float()
        nxt = sample_next(logits, do_sample, temperature, top_p, top_k, generator)
        if model.tp_size > 1:  # every TP rank must continue with the same token
            import torch.distributed as dist

            dist.broadcast(nxt, src=dist.get_global_rank(model.tp, 0), group=model.tp)
        nxt = torch.where(finished, torch.full_like(nxt, pad), nxt)
        gen_mask.append((~finished).long())
        out.append(nxt.unsqueeze(1))
        finished = finished | (nxt == eos)
        if step + 1 < max_new_tokens:
            if step % 16 == 15 and bool(finished.all()):
                break
            last = model(nxt.unsqueeze(1), cache=cache)[:, -1]
    if was_training:
        model.train()
    seqs = torch.cat(out, dim=1)
    if not return_mask:
        return seqs
    pm = attention_mask if attention_mask is not None else torch.ones_like(input_ids)
    return seqs, torch.cat([pm.long(), torch.stack(gen_mask, 1)], dim=1)
