"""Model/tokenizer loading API, mirroring the reference's `load_causal_lm` / `build_reward_model`
(src/models/base_model.py:11-59, src/models/reward_model.py:20-35) without HF modeling code.

Fixes relative to the reference: models are placed on ONE device
(this process's GPU) instead of `device_map="auto"`; reward checkpoints are actually reloaded
(`model.safetensors` / `model_N.safetensors` / `pytorch_model.bin`, `module.` stripped, strict).
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, Optional, Tuple

import torch

from .config import ModelConfig, get_config
from .reward import RewardModel, ValueModel
from .tokenizer import load_tokenizer
from .transformer import CausalLM, build_model, default_dtype


@dataclass
class ModelBundle:
    model: Any
    tokenizer: Any


def default_device() -> torch.device:
    if torch.cuda.is_available():
        import os

        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    return torch.device("cpu")


def _weight_files(path: Path):
    if (path / "model.safetensors").exists():
        return [path / "model.safetensors"]
    index = path / "model.safetensors.index.json"
    if index.exists():  # HF index shards (model-0000k-of-0000n), never model_1* files
        wm = json.loads(index.read_text())["weight_map"]
        return [path / f for f in sorted(set(wm.values()))]
    if (path / "pytorch_model.bin").exists():
        return [path / "pytorch_model.bin"]
    return []


def read_state_dict(path: Path):
    """HF weights of a model directory as a lazy mapping (tensors are read on access)."""
    from ..utils.sharded_io import open_consolidated
    from .hf_io import LazyTensors

    lazy = open_consolidated(path, "model")
    if lazy is not None:
        return lazy
    sd: Dict[str, torch.Tensor] = {}
    for f in _weight_files(Path(path)):
        sd.update(torch.load(str(f), map_location="cpu", weights_only=True))
    return LazyTensors(sd.keys(), sd.__getitem__)


def load_causal_lm(model_name_or_path: str, gradient_checkpointing: bool = True,
                   use_flash_attention: bool = False, torch_dtype: Optional[torch.dtype] = None,
                   device=None, seed: int = 0, headless: bool = False,
                   device_map=None, meta_init: bool = False) -> ModelBundle:
    """Preset name / HF hub alias -> random init (seeded, identical on all ranks);
    local dir (config.json + safetensors) -> loaded weights. `use_flash_attention` is accepted
    for config compatibility: the native model always runs the HIP flash-attention kernel.

    `device_map` ("auto" or a device list) splits the layers over several devices in ONE process
    (parallel.layer_split; the reference's device_map="auto", base_model.py:33). "auto" with a
    single visible GPU is the plain one-device placement."""
    from ..parallel.layer_split import dispatch_layers, resolve_devices

    split = resolve_devices(device_map)
    split = split if split is not None and len(split) > 1 else None
    if split is not None:
        dtype = torch_dtype or default_dtype(split[0])
        device = torch.device("cpu")  # materialise on the host, then place layer ranges
    else:
        device = torch.device(device) if device is not None else default_device()
        dtype = torch_dtype or default_dtype(device)
    cfg = get_config(model_name_or_path)
    p = Path(str(model_name_or_path))
    has_weights = p.is_dir() and bool(_weight_files(p))
    if meta_init and split is None:
        # memory-bounded construction: shapes only now; values (seeded init or the lazily read
        # checkpoint) are produced per parameter / FSDP unit after parallelize() has sharded the
        # shapes (models/materialize.py)
        from .materialize import build_meta

        model = build_meta(cfg, dtype, seed=seed, headless=headless,
                           state_dict=read_state_dict(p) if has_weights else None)
    else:
        model = build_model(cfg, device=device, dtype=dtype, seed=seed, init=not has_weights, headless=headless)
        if has_weights:
            sd = read_state_dict(p)
            model.load_hf_state_dict(sd, strict=False)
    if split is not None:
        dispatch_layers(model, split)
    if gradient_checkpointing:  # True / "full", or a selective policy ("mlp", "attention")
        model.gradient_checkpointing_enable(gradient_checkpointing)
    tok = load_tokenizer(model_name_or_path, cfg)
    return ModelBundle(model=model, tokenizer=tok)


def build_reward_model(base_model_name_or_path: str, pooling: str = "last_token", dropout: float = 0.1,
                       device=None, torch_dtype=None, seed: int = 0,
                       checkpoint: Optional[str] = None) -> Tuple[RewardModel, Any]:
    device = torch.device(device) if device is not None else default_device()
    bundle = load_causal_lm(base_model_name_or_path, gradient_checkpointing=False,
                            torch_dtype=torch_dtype, device=device, seed=seed, headless=True)
    rm = RewardModel(bundle.model, pooling=pooling, dropout=dropout)
    if checkpoint:
        load_reward_checkpoint(rm, checkpoint)
    return rm, bundle.tokenizer


def build_value_model(base_model_name_or_path: str, device=None, torch_dtype=None, seed: int = 0,
                      gradient_checkpointing: bool = False) -> Tuple[ValueModel, Any]:
    """PPO critic on the headless backbone of `base_model_name_or_path` (a preset, a local HF dir
    or a reward-model `hf/` export: its backbone weights initialise the critic)."""
    device = torch.device(device) if device is not None else default_device()
    bundle = load_causal_lm(base_model_name_or_path, gradient_checkpointing=gradient_checkpointing,
                            torch_dtype=torch_dtype, device=device, seed=seed, headless=True)
    return ValueModel(bundle.model), bundle.tokenizer


def load_reward_checkpoint(rm: RewardModel, path: str, model_index: Optional[int] = None):
    """Load a reward model from an accelerate-layout dir (`model.safetensors`, or
    `model_{i}.safetensors`), an `hf/` export, or `pytorch_model.bin`."""
    from ..utils.sharded_io import open_consolidated

    p = Path(path)
    if p.is_file():
        if p.suffix == ".safetensors":
            from safetensors.torch import load_file

            sd = load_file(str(p))
        else:
            sd = torch.load(str(p), map_location="cpu", weights_only=True)
        rm.load_hf_state_dict(sd, strict=True)
        return str(p)
    cand = ([(p, f"model_{model_index}")] if model_index else []) + [(p, "model"), (p / "hf", "model")]
    for d, stem in cand:
        sd = open_consolidated(d, stem)  # single file or HF index shards, read lazily
        if sd is not None:
            rm.load_hf_state_dict(sd, strict=True)
            return str(d / stem)
    if (p / "pytorch_model.bin").exists():
        rm.load_hf_state_dict(torch.load(str(p / "pytorch_model.bin"), map_location="cpu",
                                         weights_only=True), strict=True)
        return str(p / "pytorch_model.bin")
    raise FileNotFoundError(f"no reward weights under {path}")


def count_trainable_params(model) -> Dict[str, Any]:
    total = sum(p.numel() for p in model.parameters())
    trainable = sum(p.numel() for p in model.parameters() if p.requires_grad)
    return {"total_params": total, "trainable_params": trainable,
            "trainable_ratio": trainable / total if total else 0.0}


def freeze_except_lora(model, lora_layers: Optional[str] = None) -> None:
    for name, param in model.named_parameters():
        param.requires_grad = bool(lora_layers and lora_layers in name)


def save_hf_pretrained(model, tokenizer, path: str):
    """HF-style export (config.json + model.safetensors + tokenizer) so stages chain
    (fixes Appendix A #6)."""
    from safetensors.torch import save_file

    p = Path(path)
    save_hf_export_files(model, tokenizer, path)
    sd = {k: v.detach().contiguous().cpu() for k, v in model.hf_state_dict().items()}
    save_file(_dedupe(sd), str(p / "model.safetensors"))


def save_hf_export_files(model, tokenizer, path: str):
    """Everything of an HF export except the weights: config.json, dla_config.json, tokenizer."""
    p = Path(path)
    p.mkdir(parents=True, exist_ok=True)
    base = model.backbone if isinstance(model, (RewardModel, ValueModel)) else model
    (p / "config.json").write_text(json.dumps(base.cfg.to_hf(), indent=2))
    (p / "dla_config.json").write_text(json.dumps(base.cfg.to_dict(), indent=2))
    if tokenizer is not None and hasattr(tokenizer, "save_pretrained"):
        tokenizer.save_pretrained(str(p))


def _dedupe(sd):
    seen = {}
    out = {}
    for k, v in sd.items():
        key = (v.data_ptr(), v.shape, v.stride()) if v.numel() else None
        if key is not None and key in seen:
            out[k] = v.clone()
        else:
            out[k] = v
            seen[key] = k
    return out
