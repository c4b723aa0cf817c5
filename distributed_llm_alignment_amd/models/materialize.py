"""Memory-bounded model construction for models that do not fit one GPU replicated
(north-star config 4, Llama-3-70B: 141 GB of bf16 weights per copy; DPO co-locates the policy
AND a frozen reference).

The reference reaches ZeRO-3 through accelerate's DeepSpeed plugin, which builds the model
already partitioned (`zero.Init`, config/deepspeed_zero3.json:5-15 via src/training/utils.py:
62-63). Here a model is first built on the `meta` device (shapes only, no memory), the
parallelism is applied to it structurally (tensor-parallel slices and expert-parallel stacks
change parameter SHAPES, still on meta), and only then are values produced — one parameter at a
time (`materialize`), or one FSDP unit at a time inside the sharded engines
(parallel/fsdp.py), each value generated in full on the device, sliced to this rank's shard and
the full copy dropped before the next. Peak device memory during construction is therefore the
rank's local shards plus ONE full parameter (or one FSDP unit), never the whole model.

Values come from the same per-parameter seeded init as `CausalLM.init_weights`
(models/transformer.py: every parameter has its own generator), or from a lazily read HF
checkpoint (the `key_map` pieces of that one parameter), so the result is bitwise identical to
building the whole model and sharding it afterwards.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

# accounting for the construction-peak test: bytes of materialised parameter values that are
# live right now / at most (local shards kept + the transient full value being sliced)
STATS = {"live_bytes": 0, "peak_bytes": 0, "max_full_bytes": 0}


def reset_stats() -> None:
    STATS.update(live_bytes=0, peak_bytes=0, max_full_bytes=0)


def _account(delta: int) -> None:
    STATS["live_bytes"] += delta
    STATS["peak_bytes"] = max(STATS["peak_bytes"], STATS["live_bytes"])


def build_meta(cfg, dtype, seed: int = 0, headless: bool = False, state_dict=None):
    """CausalLM on the meta device; every parameter remembers (name, index, full shape) and the
    model remembers where values come from (seed, or a lazy HF state dict)."""
    from .transformer import CausalLM

    model = CausalLM(cfg, device="meta", dtype=dtype, headless=headless)
    for idx, (name, p) in enumerate(model.named_parameters()):
        p._dla_src = (name, idx, tuple(p.shape))
    model._dla_meta = {"seed": int(seed), "dtype": dtype, "sd": state_dict}
    return model


def has_meta_params(model: nn.Module) -> bool:
    return any(p.is_meta for p in model.parameters())


def _owners(model: nn.Module) -> Dict[int, List[Tuple[nn.Module, str]]]:
    out: Dict[int, List[Tuple[nn.Module, str]]] = {}
    for mod in model.modules():
        for n, p in mod._parameters.items():
            if p is not None:
                out.setdefault(id(p), []).append((mod, n))
    return out


def replace_param(model: nn.Module, old: nn.Parameter, value: torch.Tensor, owners=None) -> nn.Parameter:
    """Swap `old` (e.g. a meta parameter) for a Parameter wrapping `value` everywhere it is
    registered (tied weights included), carrying over its `_dla_*` attributes."""
    owners = owners if owners is not None else _owners(model)
    # `.data =` on a fresh parameter (not Parameter(value)): the parameter keeps a version
    # counter of its own, as after the engines' usual `p.data = view`, so re-filling a shared
    # flat buffer (FSDP gathers) never trips autograd's saved-tensor version check
    new = nn.Parameter(torch.empty(0, dtype=value.dtype, device=value.device),
                       requires_grad=old.requires_grad)
    new.data = value
    new.__dict__.update(old.__dict__)
    for mod, n in owners.get(id(old), []):
        mod._parameters[n] = new
    return new


def reshape_meta(model: nn.Module, p: nn.Parameter, shape, owners=None, **attrs) -> nn.Parameter:
    """Structural sharding on meta: `p` gets the local `shape` (no values), plus attributes."""
    new = replace_param(model, p, torch.empty(shape, device="meta", dtype=p.dtype), owners)
    for k, v in attrs.items():
        setattr(new, k, v)
    return new


def _base(model):
    return getattr(model, "backbone", model)


def _meta_info(model):
    base = _base(model)
    info = getattr(base, "_dla_meta", None) or getattr(model, "_dla_meta", None)
    if info is None:
        raise RuntimeError("model has meta parameters but no construction info (build_meta)")
    return base, info


def full_value(model: nn.Module, p: nn.Parameter, device) -> torch.Tensor:
    """The FULL (unsharded) value of parameter `p` on `device`."""
    from .transformer import init_param_tensor

    base, info = _meta_info(model)
    name, idx, shape = p._dla_src
    dtype = info["dtype"]
    sd = info["sd"]
    if sd is None:
        return init_param_tensor(base.cfg, name, idx, shape, info["seed"], device, dtype)
    from .hf_io import _slice, _strip_base, key_map

    out = torch.zeros(shape, device=device, dtype=dtype)
    found = False
    for native, hf, spec in key_map(base.cfg):
        if native != name:
            continue
        key = hf if hf in sd else (_strip_base(hf) if _strip_base(hf) in sd else None)
        if key is None:
            continue
        src = sd[key]
        dst = out if spec == "T" else _slice(out, spec)
        dst.copy_((src.t() if spec == "T" else src).to(device=device, dtype=dtype))
        found = True
    if not found:  # a parameter the checkpoint lacks (e.g. a tied head): seeded init
        return init_param_tensor(base.cfg, name, idx, shape, info["seed"], device, dtype)
    return out


def local_value(model: nn.Module, p: nn.Parameter, device) -> torch.Tensor:
    """This rank's shard of `p`: the full value, then the expert-parallel row range and the
    tensor-parallel slice recorded by the structural sharding. The full copy is dropped."""
    full = full_value(model, p, device)
    fb = full.numel() * full.element_size()
    STATS["max_full_bytes"] = max(STATS["max_full_bytes"], fb)
    _account(fb)
    t = full
    ep = getattr(p, "_dla_ep_rows", None)
    if ep is not None:
        t = t[ep[0]:ep[1]]
    spec = getattr(p, "_dla_tp_spec", None)
    if spec is not None and tuple(t.shape) != tuple(p.shape):
        from ..parallel.tensor_parallel import shard_tensor

        base = _base(model)
        t = shard_tensor(t, spec, base.tp_rank, base.tp_size)  # a new tensor
    # a view into the full value would keep all of it alive: copy the slice out
    shares = t.untyped_storage().data_ptr() == full.untyped_storage().data_ptr()
    out = t.clone() if (shares and t.numel() != full.numel()) else t.contiguous()
    if tuple(out.shape) != tuple(p.shape):
        raise RuntimeError(f"{p._dla_src[0]}: materialised {tuple(out.shape)} != local {tuple(p.shape)}")
    _account(out.numel() * out.element_size() - fb)
    del full
    return out


@torch.no_grad()
def materialize(model: nn.Module, device) -> nn.Module:
    """Replace every meta parameter by its local value on `device`, one at a time."""
    owners = _owners(model)
    seen = set()
    for p in list(model.parameters()):
        if id(p) in seen or not p.is_meta:
            continue
        seen.add(id(p))
        replace_param(model, p, local_value(model, p, device), owners)
    return model
