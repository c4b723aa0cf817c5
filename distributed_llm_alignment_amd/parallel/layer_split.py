"""Single-process layer-split model parallelism: the reference's `device_map="auto"` (SURVEY §2.3
P7; src/models/base_model.py:33, reward_model.py:32, generate_teacher_data.py:43,
eval_alignment.py:63, eval_latency.py:32).

HF's big-model dispatch places consecutive decoder layers on consecutive GPUs and hops the
activations between them. On MI355X (288 GB of HBM3E per GPU) every model the reference or the
north-star configs name fits on ONE device, so the trainers and CLIs default to one device per
process (one process per GPU, data parallel over RCCL), which is strictly faster. This module
keeps the capability for models that do not fit — e.g. a >140 B-parameter bf16 checkpoint for
single-process inference — with the same semantics: contiguous layer ranges balanced by
parameter bytes, embedding / final norm / LM head on the first device (so targets, masks and
sampling stay where `input_ids` live), [B, T, H] activations hopped with peer copies over xGMI.
Autograd flows through the hops, so a layer-split model also trains (naive, un-pipelined MP).

`load_causal_lm(..., device_map="auto")` calls `dispatch_layers` when more than one device is
visible; `device_map` may also be an explicit device list.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import torch


def _layer_bytes(layer: torch.nn.Module) -> int:
    return sum(p.numel() * p.element_size() for p in layer.parameters())


def plan_layer_split(layer_bytes: Sequence[int], n_dev: int, first_extra: int = 0) -> List[int]:
    """Device index per layer: contiguous ranges, greedy fill to an even share of the total
    bytes (`first_extra` = bytes already on device 0: embedding, final norm, LM head)."""
    n_dev = max(1, min(n_dev, len(layer_bytes))) if layer_bytes else 1
    total = sum(layer_bytes) + first_extra
    share = total / n_dev
    out, dev, used = [], 0, first_extra
    for i, b in enumerate(layer_bytes):
        remaining_layers = len(layer_bytes) - i
        remaining_devs = n_dev - dev - 1
        # move on when this device is full, but never leave a later device without a layer
        if dev < n_dev - 1 and (used + b / 2 > share or remaining_layers <= remaining_devs) and used > 0:
            dev, used = dev + 1, 0
        out.append(dev)
        used += b
    return out


def resolve_devices(device_map: Union[str, Sequence, None]) -> Optional[List[torch.device]]:
    if device_map is None:
        return None
    if isinstance(device_map, str):
        if device_map != "auto":
            return [torch.device(device_map)]
        n = torch.cuda.device_count() if torch.cuda.is_available() else 0
        return [torch.device("cuda", i) for i in range(n)] if n > 1 else None
    return [torch.device(d) for d in device_map]


def dispatch_layers(model, devices: Sequence[Union[str, torch.device]]):
    """Move `model` (CausalLM, or a RewardModel / ValueModel wrapping one as `.backbone`) onto
    `devices` layer-wise and make its forward hop activations. Returns the per-layer devices."""
    lm = getattr(model, "backbone", model)
    devs = [torch.device(d) for d in devices]
    if getattr(lm, "tp_size", 1) > 1 or getattr(lm, "_dla_fsdp", None) is not None:
        raise ValueError("layer split is a single-process mode; it does not combine with TP / FSDP")
    first = devs[0]
    extra = sum(p.numel() * p.element_size() for n, p in lm.named_parameters() if not n.startswith("layers."))
    plan = plan_layer_split([_layer_bytes(l) for l in lm.layers], len(devs), extra)
    for name, p in list(lm.named_parameters(recurse=False)):
        p.data = p.data.to(first)
    for i, layer in enumerate(lm.layers):
        layer.to(devs[plan[i]])
    lm_mods = {id(m) for m in lm.modules()}
    for mod in model.modules():  # heads of RewardModel / ValueModel stay with the embedding
        if id(mod) not in lm_mods:
            for p in mod.parameters(recurse=False):
                p.data = p.data.to(first)
    lm.layer_devices = [devs[j] for j in plan]
    return lm.layer_devices
