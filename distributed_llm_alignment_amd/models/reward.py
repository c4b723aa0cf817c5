"""Scalar reward model: native backbone + Dropout + Linear(H, 1) head.

Mirrors src/models/reward_model.py:38-64: `backbone` is the headless decoder (HF AutoModel
layout), `scorer = Sequential(Dropout(p), Linear(H, 1))`, pooling `last_token` (index
`mask.sum - 1` for right padding; generalised here to the last valid position for left padding
too) or `mean` (masked mean). Checkpoint keys: `backbone.*` + `scorer.1.weight` / `scorer.1.bias`.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn as nn

from ..ops import _ext
from .transformer import CausalLM, attention_layout


class _RewardHeadFn(torch.autograd.Function):
    """Fused pooling + dropout + Linear(H, 1) (csrc/reward_head.hip)."""

    @staticmethod
    def forward(ctx, hidden, w, b, last, mask, p: float, seed: int):
        C = _ext.require()
        score, pooled = C.reward_head_fwd(hidden, last, mask, w.reshape(-1), b, p, seed)
        ctx.save_for_backward(hidden, w, last, mask, pooled)
        ctx.p, ctx.seed, ctx.has_b = p, seed, b is not None
        return score

    @staticmethod
    def backward(ctx, ds):
        hidden, w, last, mask, pooled = ctx.saved_tensors
        ds = ds.float().contiguous()
        dh = None
        if ctx.needs_input_grad[0]:
            dh = _ext.require().reward_head_bwd(ds, hidden, last, mask, w.reshape(-1), ctx.p, ctx.seed)
        dw = (ds.unsqueeze(1) * pooled).sum(0).to(w.dtype).view_as(w) if ctx.needs_input_grad[1] else None
        db = ds.sum().to(w.dtype).reshape(1) if (ctx.has_b and ctx.needs_input_grad[2]) else None
        return dh, dw, db, None, None, None, None


class RewardModel(nn.Module):
    def __init__(self, backbone: CausalLM, pooling: str = "last_token", dropout: float = 0.1):
        super().__init__()
        if pooling not in ("last_token", "mean"):
            raise ValueError(f"pooling must be last_token|mean, got {pooling!r}")
        self.backbone = backbone
        self.pooling = pooling
        H = backbone.cfg.hidden_size
        dev, dt = backbone.embed.device, backbone.embed.dtype
        self.scorer = nn.Sequential(nn.Dropout(dropout), nn.Linear(H, 1, device=dev, dtype=dt))
        with torch.no_grad():
            nn.init.normal_(self.scorer[1].weight, std=1.0 / (H + 1) ** 0.5)
            self.scorer[1].bias.zero_()

    def pool(self, hidden: torch.Tensor, attention_mask: torch.Tensor) -> torch.Tensor:
        if attention_mask is None:
            return hidden[:, -1] if self.pooling == "last_token" else hidden.mean(1)
        if self.pooling == "last_token":
            _, end, _ = attention_layout(attention_mask)
            idx = (end.long() - 1).clamp(min=0)
            return hidden[torch.arange(hidden.shape[0], device=hidden.device), idx]
        m = attention_mask.to(hidden.dtype).unsqueeze(-1)
        return (hidden * m).sum(1) / attention_mask.sum(1, keepdim=True).clamp(min=1).to(hidden.dtype)

    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor = None) -> torch.Tensor:
        from ..parallel.sequence import sp_full_hidden

        h = sp_full_hidden(self.backbone, self.backbone(input_ids, attention_mask), input_ids.shape[1])
        lin = self.scorer[1]
        if (_ext.use_native(h) and h.dtype == torch.bfloat16 and lin.weight.dtype == torch.bfloat16
                and h.shape[-1] % 8 == 0 and h.stride(-1) == 1):
            return self._fused_head(h, attention_mask)
        return self.scorer(self.pool(h, attention_mask)).squeeze(-1).float()

    def _fused_head(self, h: torch.Tensor, attention_mask) -> torch.Tensor:
        B, T = h.shape[0], h.shape[1]
        last = mask = None
        if self.pooling == "last_token":
            if attention_mask is None:
                last = torch.full((B,), T - 1, dtype=torch.int32, device=h.device)
            else:
                _, end, _ = attention_layout(attention_mask)
                last = (end - 1).clamp(min=0).to(torch.int32).contiguous()
        else:
            mask = (torch.ones((B, T), device=h.device) if attention_mask is None
                    else attention_mask.float()).contiguous()
        drop = self.scorer[0]
        p = float(drop.p) if (self.training and drop.p > 0) else 0.0
        # dropout seed from torch's host generator (torch.manual_seed reproducible, no GPU sync)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0
        if h.stride(1) % 8 or h.stride(0) % 8 or h.data_ptr() % 16:
            h = h.contiguous()
        lin = self.scorer[1]
        return _RewardHeadFn.apply(h, lin.weight, lin.bias, last, mask, p, seed)

    def hf_state_dict(self, only=None) -> Dict[str, torch.Tensor]:
        from .hf_io import to_hf_state_dict

        bb_only = None if only is None else {n[len("backbone."):] for n in only if n.startswith("backbone.")}
        sd = {f"backbone.{k}": v for k, v in to_hf_state_dict(self.backbone, base=True, only=bb_only).items()}
        for name in ("weight", "bias"):
            if only is None or f"scorer.1.{name}" in only:
                sd[f"scorer.1.{name}"] = getattr(self.scorer[1], name).detach()
        return sd

    @torch.no_grad()
    def load_hf_state_dict(self, sd, strict: bool = True, only=None, used_out=None):
        from .hf_io import load_hf_state_dict, renamed

        sd = renamed(sd, lambda k: k[len("module."):] if k.startswith("module.") else k)
        bb = renamed(sd, lambda k: k[len("backbone."):] if k.startswith("backbone.") else None)
        bb_only = None if only is None else {n[len("backbone."):] for n in only if n.startswith("backbone.")}
        bb_used = set()
        missing, unexpected = load_hf_state_dict(self.backbone, bb, strict=False, base=True,
                                                 only=bb_only, used_out=bb_used)
        if used_out is not None:
            used_out.update("backbone." + k for k in bb_used)
        missing = [m for m in missing if not m.startswith("lm_head")]
        for name in ("weight", "bias"):
            key = f"scorer.1.{name}"
            if only is not None and key not in only:
                continue
            if used_out is not None and key in sd:
                used_out.add(key)
            if key in sd:
                getattr(self.scorer[1], name).copy_(sd[key].to(self.scorer[1].weight.dtype))
            else:
                missing.append(key)
        if strict and missing:
            raise KeyError(f"reward checkpoint missing keys: {missing[:8]}")
        return missing, unexpected


class ValueModel(nn.Module):
    """PPO critic: headless native decoder + per-token `Linear(H, 1)` value head. values[s, t]
    estimates the return from the state that ends at token t (the same grid as the token
    log-probs: position t scores the action that emits token t + 1). Checkpoint keys:
    `backbone.*` + `v_head.weight` / `v_head.bias`. Not part of the reference (its RLHF loop is
    critic-free REINFORCE); used by `ppo.algorithm: ppo`."""

    def __init__(self, backbone: CausalLM):
        super().__init__()
        self.backbone = backbone
        H = backbone.cfg.hidden_size
        dev, dt = backbone.embed.device, backbone.embed.dtype
        self.v_head = nn.Linear(H, 1, device=dev, dtype=dt)
        with torch.no_grad():
            nn.init.normal_(self.v_head.weight, std=1.0 / (H + 1) ** 0.5)
            self.v_head.bias.zero_()

    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor = None) -> torch.Tensor:
        v = self.v_head(self.backbone(input_ids, attention_mask)).squeeze(-1).float()
        sp = getattr(self.backbone, "sp", None)
        return v if sp is None else sp.gather(v, dim=1)[:, :input_ids.shape[1]]

    def hf_state_dict(self, only=None) -> Dict[str, torch.Tensor]:
        from .hf_io import to_hf_state_dict

        bb_only = None if only is None else {n[len("backbone."):] for n in only if n.startswith("backbone.")}
        sd = {f"backbone.{k}": v for k, v in to_hf_state_dict(self.backbone, base=True, only=bb_only).items()}
        for name in ("weight", "bias"):
            if only is None or f"v_head.{name}" in only:
                sd[f"v_head.{name}"] = getattr(self.v_head, name).detach()
        return sd

    @torch.no_grad()
    def load_hf_state_dict(self, sd, strict: bool = True, only=None, used_out=None):
        from .hf_io import load_hf_state_dict, renamed

        sd = renamed(sd, lambda k: k[len("module."):] if k.startswith("module.") else k)
        bb = renamed(sd, lambda k: k[len("backbone."):] if k.startswith("backbone.") else None)
        bb_only = None if only is None else {n[len("backbone."):] for n in only if n.startswith("backbone.")}
        bb_used = set()
        missing, unexpected = load_hf_state_dict(self.backbone, bb, strict=False, base=True,
                                                 only=bb_only, used_out=bb_used)
        if used_out is not None:
            used_out.update("backbone." + k for k in bb_used)
        missing = [m for m in missing if not m.startswith("lm_head")]
        for name in ("weight", "bias"):
            key = f"v_head.{name}"
            if only is not None and key not in only:
                continue
            if used_out is not None and key in sd:
                used_out.add(key)
            if key in sd:
                getattr(self.v_head, name).copy_(sd[key].to(self.v_head.weight.dtype))
            else:
                missing.append(key)
        if strict and missing:
            raise KeyError(f"value-model checkpoint missing keys: {missing[:8]}")
        return missing, unexpected
