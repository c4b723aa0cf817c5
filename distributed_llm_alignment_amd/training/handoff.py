"""Rollout -> reward-model hand-off without leaving the device.

The reference decodes every sampled response to text and re-tokenises `prompt + "\\n\\n" +
response` with the reward tokenizer (src/training/train_rlhf.py:131-147): a device->host copy,
Python string work per rollout, and a host->device copy, on the critical path of every RLHF
step. When the reward model uses the SAME tokenizer as the policy (same vocabulary and special
tokens: the default, the reward model is trained from the policy base), the reward input ids are
already on the device: `prompt ids ⊕ ids("\\n\\n") ⊕ response ids`, with the special tokens that
`batch_decode(skip_special_tokens=True)` would drop (EOS, padding, ...) removed and the result
right-padded and truncated to `max_length` like the tokenizer call. Built with a handful of
fused tensor ops: no host sync, no Python loop over rollouts.

Equality with the text path holds whenever re-tokenising the decoded text reproduces the ids
(always for byte-level text that is valid UTF-8 with the byte tokenizer; for BPE tokenizers
when the sampled ids are the canonical tokenization and no merge crosses the "\\n\\n"
boundary). Where it does not, the device path scores exactly the tokens the policy generated,
which is what the log-probs in the loss are computed over. `ppo.reward_handoff: text` keeps the
reference behaviour; `device` forces the device path. `auto` (default) takes the device path when
the tokenizers match, and for non-byte (BPE) tokenizers first checks it on the first batch: both
paths are built once, and if the ids differ (a merge across the boundary, a non-canonical sample)
the hand-off falls back to `text` for the rest of the run, so the default scores what the
reference scores.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch


def _special_ids(tok) -> Sequence[int]:
    ids = set()
    for k in ("all_special_ids",):
        v = getattr(tok, k, None)
        if v:
            ids.update(int(i) for i in v)
    for k in ("bos_token_id", "eos_token_id", "pad_token_id"):
        v = getattr(tok, k, None)
        if v is not None:
            ids.add(int(v))
    return sorted(ids)


def tokenizers_match(a, b) -> bool:
    """Same tokenizer for hand-off purposes: same class, vocabulary and special-token ids."""
    if a is b:
        return True
    if type(a) is not type(b):
        return False
    from ..models.tokenizer import ByteTokenizer

    if isinstance(a, ByteTokenizer):
        return all(getattr(a, k) == getattr(b, k) for k in
                   ("vocab_size", "offset", "bos_token_id", "eos_token_id", "pad_token_id", "add_bos"))
    if _special_ids(a) != _special_ids(b):
        return False
    try:
        return len(a) == len(b) and a.get_vocab() == b.get_vocab()
    except Exception:
        return False


def special_token_table(tok, vocab_size: int, device) -> torch.Tensor:
    """bool [V]: ids that `decode(..., skip_special_tokens=True)` drops (or that decode to
    nothing: ids outside the byte range of the byte tokenizer)."""
    from ..models.tokenizer import ByteTokenizer

    t = torch.zeros(vocab_size, dtype=torch.bool)
    if isinstance(tok, ByteTokenizer):
        t[:] = True
        t[tok.offset:min(vocab_size, tok.offset + 256)] = False
    else:
        for i in _special_ids(tok):
            if 0 <= i < vocab_size:
                t[i] = True
    return t.to(device)


def separator_ids(tok, text: str = "\n\n") -> torch.Tensor:
    enc = tok(text, add_special_tokens=False)
    ids = enc["input_ids"]
    return torch.tensor(list(ids), dtype=torch.long)


def device_reward_inputs(prompt_ids: torch.Tensor, prompt_mask: torch.Tensor, seqs: torch.Tensor,
                         sep: torch.Tensor, special: torch.Tensor, pad_id: int, max_length: int,
                         gen_mask: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """prompt_ids / prompt_mask [B, P] (left-padded, as tokenised for generation), seqs [B, P+R]
    (prompt + generated), sep [S] -> (ids [B, W], mask [B, W]) right-padded, W = min(P+S+R,
    max_length). gen_mask [B, P+R] (1 through the EOS) restricts the response to generated
    tokens; ids flagged in `special` are dropped like skip_special_tokens."""
    B, P = prompt_ids.shape
    dev = seqs.device
    resp = seqs[:, P:]
    R = resp.shape[1]
    sep = sep.to(dev)
    S = sep.numel()
    special = special.to(dev)
    keep_r = ~special[resp.clamp(0, special.numel() - 1)]
    if gen_mask is not None:
        keep_r = keep_r & gen_mask[:, P:].bool()
    tokens = torch.cat([prompt_ids.to(dev), sep.view(1, S).expand(B, S), resp], 1)
    keep = torch.cat([prompt_mask.to(dev).bool(), torch.ones(B, S, dtype=torch.bool, device=dev), keep_r], 1)
    W = min(P + S + R, int(max_length))
    pos = torch.cumsum(keep.to(torch.int32), 1) - 1
    valid = keep & (pos < W)
    dest = torch.where(valid, pos.to(torch.long), torch.full_like(pos, W, dtype=torch.long))
    out = torch.full((B, W + 1), int(pad_id), dtype=tokens.dtype, device=dev)
    out.scatter_(1, dest, torch.where(valid, tokens, torch.full_like(tokens, int(pad_id))))
    n = keep.sum(1).clamp(max=W)
    mask = (torch.arange(W, device=dev).view(1, W) < n.view(B, 1)).to(prompt_mask.dtype)
    return out[:, :W].contiguous(), mask


class RewardHandoff:
    """Chooses and runs the hand-off once per trainer (`ppo.reward_handoff: auto|device|text`)."""

    def __init__(self, policy_tok, reward_tok, vocab_size: int, device, max_length: int,
                 mode: str = "auto", validate_every: int = 16):
        mode = str(mode or "auto").lower()
        if mode not in ("auto", "device", "text"):
            raise ValueError(f"ppo.reward_handoff must be auto|device|text, got {mode!r}")
        match = tokenizers_match(policy_tok, reward_tok)
        if mode == "device" and not match:
            raise ValueError("ppo.reward_handoff=device needs the reward tokenizer to equal the policy's")
        self.device_path = match and mode != "text"
        self.ptok, self.rtok, self.max_length = policy_tok, reward_tok, int(max_length)
        from ..models.tokenizer import ByteTokenizer

        # auto + BPE: validate the device ids against the text round trip on the first batch and
        # then every `validate_every`-th batch (a later batch can hold a merge across the "\n\n"
        # boundary or a non-canonical sample); the verdict is agreed over all ranks (MIN), so every
        # DP rank stays on the same hand-off path
        self._validate = self.device_path and mode == "auto" and not isinstance(reward_tok, ByteTokenizer)
        self._validate_every = max(1, int(validate_every))
        self._calls = 0
        self.fallback_reason = None
        if self.device_path:
            self.special = special_token_table(reward_tok, vocab_size, device)
            self.sep = separator_ids(reward_tok).to(device)
            self.pad = int(reward_tok.pad_token_id if reward_tok.pad_token_id is not None else 0)

    def __call__(self, prompts, ids, am, seqs, gen_mask=None):
        if self.device_path:
            out = device_reward_inputs(ids, am, seqs, self.sep, self.special, self.pad,
                                       self.max_length, gen_mask)
            due = self._validate and self._calls % self._validate_every == 0
            self._calls += 1
            if not due:
                return out
            ref = self._text(prompts, ids, seqs)
            if self._agree(self._same(out, ref)):
                return out
            # the tokenizer does not round-trip these ids (on some rank): text from now on
            self.device_path = False
            self.fallback_reason = f"device ids differ from the text round trip at batch {self._calls}"
            import warnings

            warnings.warn(f"reward hand-off: {self.fallback_reason}; using the text path from now on")
            return ref
        return self._text(prompts, ids, seqs)

    @staticmethod
    def _agree(ok: bool) -> bool:
        """MIN of `ok` over every rank (identical decision everywhere); local value without a group."""
        from ..parallel.dist import state

        st = state()
        if not st.initialized:
            return ok
        import torch.distributed as dist

        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=st.device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    @staticmethod
    def _same(a, b) -> bool:
        (ia, ma), (ib, mb) = a, b
        n = max(ia.shape[1], ib.shape[1])
        pad = lambda t: torch.nn.functional.pad(t, (0, n - t.shape[1]))  # noqa: E731
        ma, mb = pad(ma.long()), pad(mb.long())
        return bool(torch.equal(ma, mb) and torch.equal(pad(ia) * ma, pad(ib) * mb))

    def _text(self, prompts, ids, seqs):
        responses = self.ptok.batch_decode(seqs[:, ids.shape[1]:], skip_special_tokens=True)
        fused = [f"{p}\n\n{r}" for p, r in zip(prompts, responses)]
        enc = self.rtok(fused, return_tensors="pt", padding=True, truncation=True, max_length=self.max_length)
        return enc["input_ids"].to(seqs.device), enc["attention_mask"].to(seqs.device)
