"""HF state-dict key mapping for the native models (SURVEY §2.7 #5 key names).

Native parameters are fused (qkv_proj = [q; k; v], up_proj = [gate; up]); HF checkpoints keep
them separate. `to_hf_state_dict` splits (views, no copies), `load_hf_state_dict` fuses. Key
layouts follow the HF modeling files the reference relies on (LlamaForCausalLM /
MistralForCausalLM / MixtralForCausalLM / GPT2LMHeadModel / PhiForCausalLM); `base=True`
produces the headless `AutoModel` layout used under `backbone.` by the reward model
(src/models/reward_model.py:29-33, 38-44).
"""
from __future__ import annotations

from collections.abc import Mapping
from typing import Callable, Dict, Iterable, List, Optional, Set, Tuple

import torch

_LLAMA_LIKE = ("llama", "mistral", "mixtral")


def _layer_map(cfg, i: int) -> List[Tuple[str, str, tuple]]:
    """(native_name, hf_name, slice-spec) triples for layer i; slice-spec = (dim0 start, stop)."""
    q, kv, F = cfg.q_size, cfg.kv_size, cfg.intermediate_size
    n = f"layers.{i}."
    if cfg.arch in _LLAMA_LIKE:
        p = f"model.layers.{i}."
        m = [
            (n + "ln1_w", p + "input_layernorm.weight", None),
            (n + "ln2_w", p + "post_attention_layernorm.weight", None),
            (n + "attn.qkv_proj", p + "self_attn.q_proj.weight", (0, q)),
            (n + "attn.qkv_proj", p + "self_attn.k_proj.weight", (q, q + kv)),
            (n + "attn.qkv_proj", p + "self_attn.v_proj.weight", (q + kv, q + 2 * kv)),
            (n + "attn.o_proj", p + "self_attn.o_proj.weight", None),
        ]
        if cfg.attn_bias:
            m += [(n + "attn.qkv_bias", p + "self_attn.q_proj.bias", (0, q)),
                  (n + "attn.qkv_bias", p + "self_attn.k_proj.bias", (q, q + kv)),
                  (n + "attn.qkv_bias", p + "self_attn.v_proj.bias", (q + kv, q + 2 * kv))]
        if cfg.is_moe:
            m.append((n + "mlp.router", p + "block_sparse_moe.gate.weight", None))
            for e in range(cfg.num_experts):
                ep = p + f"block_sparse_moe.experts.{e}."
                m += [(n + "mlp.expert_up", ep + "w1.weight", ("expert", e, 0, F)),
                      (n + "mlp.expert_up", ep + "w3.weight", ("expert", e, F, 2 * F)),
                      (n + "mlp.expert_down", ep + "w2.weight", ("expert", e, None, None))]
        else:
            m += [(n + "mlp.up_proj", p + "mlp.gate_proj.weight", (0, F)),
                  (n + "mlp.up_proj", p + "mlp.up_proj.weight", (F, 2 * F)),
                  (n + "mlp.down_proj", p + "mlp.down_proj.weight", None)]
        return m
    if cfg.arch == "phi":
        p = f"model.layers.{i}."
        return [
            (n + "ln1_w", p + "input_layernorm.weight", None),
            (n + "ln1_b", p + "input_layernorm.bias", None),
            (n + "attn.qkv_proj", p + "self_attn.q_proj.weight", (0, q)),
            (n + "attn.qkv_proj", p + "self_attn.k_proj.weight", (q, q + kv)),
            (n + "attn.qkv_proj", p + "self_attn.v_proj.weight", (q + kv, q + 2 * kv)),
            (n + "attn.qkv_bias", p + "self_attn.q_proj.bias", (0, q)),
            (n + "attn.qkv_bias", p + "self_attn.k_proj.bias", (q, q + kv)),
            (n + "attn.qkv_bias", p + "self_attn.v_proj.bias", (q + kv, q + 2 * kv)),
            (n + "attn.o_proj", p + "self_attn.dense.weight", None),
            (n + "attn.o_bias", p + "self_attn.dense.bias", None),
            (n + "mlp.up_proj", p + "mlp.fc1.weight", None),
            (n + "mlp.up_bias", p + "mlp.fc1.bias", None),
            (n + "mlp.down_proj", p + "mlp.fc2.weight", None),
            (n + "mlp.down_bias", p + "mlp.fc2.bias", None),
        ]
    if cfg.arch == "gpt2":
        p = f"transformer.h.{i}."
        # HF GPT-2 Conv1D stores [in, out]: marked with "T" (transpose)
        return [
            (n + "ln1_w", p + "ln_1.weight", None), (n + "ln1_b", p + "ln_1.bias", None),
            (n + "ln2_w", p + "ln_2.weight", None), (n + "ln2_b", p + "ln_2.bias", None),
            (n + "attn.qkv_proj", p + "attn.c_attn.weight", "T"),
            (n + "attn.qkv_bias", p + "attn.c_attn.bias", None),
            (n + "attn.o_proj", p + "attn.c_proj.weight", "T"),
            (n + "attn.o_bias", p + "attn.c_proj.bias", None),
            (n + "mlp.up_proj", p + "mlp.c_fc.weight", "T"),
            (n + "mlp.up_bias", p + "mlp.c_fc.bias", None),
            (n + "mlp.down_proj", p + "mlp.c_proj.weight", "T"),
            (n + "mlp.down_bias", p + "mlp.c_proj.bias", None),
        ]
    raise ValueError(cfg.arch)


def _global_map(cfg) -> List[Tuple[str, str, tuple]]:
    if cfg.arch == "gpt2":
        m = [("embed", "transformer.wte.weight", None), ("wpe", "transformer.wpe.weight", None),
             ("norm_w", "transformer.ln_f.weight", None), ("norm_b", "transformer.ln_f.bias", None)]
    elif cfg.arch == "phi":
        m = [("embed", "model.embed_tokens.weight", None),
             ("norm_w", "model.final_layernorm.weight", None),
             ("norm_b", "model.final_layernorm.bias", None),
             ("lm_head", "lm_head.weight", None), ("lm_head_bias", "lm_head.bias", None)]
    else:
        m = [("embed", "model.embed_tokens.weight", None), ("norm_w", "model.norm.weight", None)]
        if not cfg.tie_word_embeddings:
            m.append(("lm_head", "lm_head.weight", None))
    return m


def key_map(cfg):
    m = _global_map(cfg)
    for i in range(cfg.num_layers):
        m += _layer_map(cfg, i)
    return m


def _strip_base(k: str) -> str:
    for pre in ("model.", "transformer."):
        if k.startswith(pre):
            return k[len(pre):]
    return k


def _slice(t: torch.Tensor, spec):
    if spec is None:
        return t
    if spec == "T":
        return t.t()
    if spec[0] == "expert":
        _, e, a, b = spec
        return t[e] if a is None else t[e, a:b]
    a, b = spec
    return t[a:b]


class LazyTensors(Mapping):
    """Read-on-access tensor mapping: keys are known up front, a tensor is materialised only when
    indexed (safetensors files of a 70B checkpoint never have to sit in host memory at once)."""

    def __init__(self, keys: Iterable[str], getter: Callable[[str], torch.Tensor]):
        self._keys = list(keys)
        self._set = set(self._keys)
        self._get = getter

    def __getitem__(self, k):
        if k not in self._set:
            raise KeyError(k)
        return self._get(k)

    def __iter__(self):
        return iter(self._keys)

    def __len__(self):
        return len(self._keys)

    def __contains__(self, k):
        return k in self._set


def renamed(sd: Mapping, fn: Callable[[str], Optional[str]]) -> LazyTensors:
    """Lazy view of `sd` with keys mapped through `fn` (None drops a key); no tensor is read."""
    m = {}
    for k in sd:
        nk = fn(k)
        if nk is not None:
            m[nk] = k
    return LazyTensors(m.keys(), lambda k: sd[m[k]])


def to_hf_state_dict(model, base: bool = False, only: Optional[Set[str]] = None) -> Dict[str, torch.Tensor]:
    """HF-named views of the native parameters; `only` restricts to a set of native names (the
    streamed checkpoint writer converts one FSDP unit / layer at a time)."""
    params = dict(model.named_parameters())
    out: Dict[str, torch.Tensor] = {}
    for native, hf, spec in key_map(model.cfg):
        if native not in params or (only is not None and native not in only):
            continue
        if base and hf.startswith("lm_head"):
            continue
        t = _slice(params[native].detach(), spec)
        if spec == "T":
            t = t.contiguous()
        out[_strip_base(hf) if base else hf] = t
    return out


@torch.no_grad()
def _unfuse_moe_experts(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Newer transformers keep Mixtral experts fused in memory (`mlp.gate.weight`,
    `mlp.experts.gate_up_proj` [E, 2F, H] = [w1; w3], `mlp.experts.down_proj` [E, H, F] = w2);
    checkpoints on disk use the per-expert `block_sparse_moe.experts.{e}.w1/w3/w2` names the key
    map speaks. Rewrite the fused form into the per-expert one."""
    if not any(k.endswith("mlp.experts.gate_up_proj") for k in sd):
        return sd
    out = {}
    for k, v in sd.items():
        if k.endswith("mlp.experts.gate_up_proj"):
            pre = k[: -len("mlp.experts.gate_up_proj")] + "block_sparse_moe.experts."
            F = v.shape[1] // 2
            for e in range(v.shape[0]):
                out[f"{pre}{e}.w1.weight"] = v[e, :F]
                out[f"{pre}{e}.w3.weight"] = v[e, F:]
        elif k.endswith("mlp.experts.down_proj"):
            pre = k[: -len("mlp.experts.down_proj")] + "block_sparse_moe.experts."
            for e in range(v.shape[0]):
                out[f"{pre}{e}.w2.weight"] = v[e]
        elif k.endswith("mlp.gate.weight") and ".layers." in k:
            out[k[: -len("mlp.gate.weight")] + "block_sparse_moe.gate.weight"] = v
        else:
            out[k] = v
    return out


def load_hf_state_dict(model, sd: Mapping, strict: bool = True, base: bool = False,
                       only: Optional[Set[str]] = None, used_out: Optional[set] = None):
    """Copy HF tensors into the fused native parameters. Accepts `module.` prefixes (DDP) and the
    fused in-memory Mixtral expert layout of newer transformers. `sd` may be lazy (LazyTensors):
    only the tensors of the parameters being loaded are read. With `only` (native names) the
    other parameters are skipped and neither missing nor unexpected keys are judged here; the
    keys consumed are added to `used_out`."""
    sd = renamed(sd, lambda k: k[len("module."):] if k.startswith("module.") else k)
    if model.cfg.is_moe and any(k.endswith("mlp.experts.gate_up_proj") for k in sd):
        sd = _unfuse_moe_experts({k: sd[k] for k in sd})
    params = dict(model.named_parameters())
    used = set()
    missing = []
    for native, hf, spec in key_map(model.cfg):
        if native not in params or (only is not None and native not in only):
            continue
        key = hf
        if key not in sd:
            alt = _strip_base(hf)
            if alt in sd:
                key = alt
            elif hf.startswith("lm_head") and model.cfg.tie_word_embeddings:
                continue
            else:
                missing.append(hf)
                continue
        src = sd[key]
        if spec == "T":  # HF Conv1D [in, out] -> native [out, in]
            dst, src = params[native].data, src.t()
        else:
            dst = _slice(params[native].data, spec)
        if tuple(dst.shape) != tuple(src.shape):
            raise ValueError(f"shape mismatch for {hf}: ckpt {tuple(src.shape)} vs model {tuple(dst.shape)}")
        dst.copy_(src.to(dst.dtype))
        used.add(key)
    if used_out is not None:
        used_out.update(used)
    if only is not None:
        return missing, []
    unexpected = [k for k in sd if k not in used and not k.endswith("rotary_emb.inv_freq")
                  and not k.startswith("lm_head") and ".attn.bias" not in k and ".attn.masked_bias" not in k]
    if strict and (missing or unexpected):
        raise KeyError(f"missing={missing[:8]} unexpected={unexpected[:8]}")
    return missing, unexpected
