"""YAML config system compatible with the reference schema.

`load_config(path)` is the reference's plain `yaml.safe_load` (src/training/utils.py:18-21);
additionally overlays (deep-merged YAML fragments such as config/ablations/*.yaml and
config/data_sources/*.yaml, which the reference asks users to paste by hand, README.md:122-126)
and dotted `key.path=value` overrides (values parsed as YAML scalars) compose from the CLI.
"""
from __future__ import annotations

import argparse
import copy
import json
from pathlib import Path
from typing import Any, Dict, Iterable, List, Optional

import yaml


def deep_merge(base: Dict[str, Any], over: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = deep_merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def apply_override(cfg: Dict[str, Any], spec: str) -> Dict[str, Any]:
    if "=" not in spec:
        raise ValueError(f"override must look like key.path=value, got {spec!r}")
    key, raw = spec.split("=", 1)
    val = yaml.safe_load(raw) if raw != "" else None
    node = cfg
    parts = key.strip().split(".")
    for p in parts[:-1]:
        if not isinstance(node.get(p), dict):
            node[p] = {}
        node = node[p]
    node[parts[-1]] = val
    return cfg


def load_config(path, overlays: Optional[Iterable[str]] = None,
                overrides: Optional[Iterable[str]] = None) -> Dict[str, Any]:
    with open(path, "r", encoding="utf-8") as fh:
        cfg = yaml.safe_load(fh) or {}
    for ov in overlays or []:
        with open(ov, "r", encoding="utf-8") as fh:
            cfg = deep_merge(cfg, _as_overlay(yaml.safe_load(fh) or {}))
    for o in overrides or []:
        cfg = apply_override(cfg, o)
    return cfg


_TOP_LEVEL = {"model", "data", "optimization", "logging", "hardware", "distill", "ppo", "sampling",
              "reward_model", "models", "benchmarks", "generation", "latency", "seed"}


def _as_overlay(frag: Dict[str, Any]) -> Dict[str, Any]:
    """The reference's data-source presets (config/data_sources/*.yaml) are FLAT fragments meant to
    be pasted under `data:` (README.md:122-126) — or under `sampling:` for RLHF prompt sources
    (they carry `prompt_key`). Wrap such a fragment so it can be passed as an overlay."""
    if "source" in frag and not (set(frag) & _TOP_LEVEL):
        return {"sampling" if "prompt_key" in frag else "data": frag}
    return frag


def flatten_dict(config: Dict[str, Any], parent_key: str = "", sep: str = ".") -> Dict[str, Any]:
    items: Dict[str, Any] = {}
    for key, value in config.items():
        new_key = f"{parent_key}{sep}{key}" if parent_key else key
        if isinstance(value, dict):
            items.update(flatten_dict(value, new_key, sep=sep))
        else:
            items[new_key] = value
    return items


def save_json(obj: Dict[str, Any], path) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    with path.open("w", encoding="utf-8") as fh:
        json.dump(obj, fh, indent=2, default=str)


def add_config_args(parser: argparse.ArgumentParser) -> argparse.ArgumentParser:
    """The reference CLI contract (`--config PATH`, required) plus composable extras."""
    parser.add_argument("--config", required=True, type=str, help="Path to YAML config")
    parser.add_argument("--overlay", action="append", default=[],
                        help="YAML fragment deep-merged over the config (repeatable)")
    parser.add_argument("--override", action="append", default=[],
                        help="dotted key.path=value override (repeatable)")
    parser.add_argument("--resume", default=None,
                        help="checkpoint dir (or 'latest') to resume from")
    return parser


def config_from_args(args) -> Dict[str, Any]:
    return load_config(args.config, getattr(args, "overlay", None), getattr(args, "override", None))


def hardware_parallel(cfg: Dict[str, Any]) -> Dict[str, Any]:
    """Map the reference's hardware block (accelerate mixed_precision, DeepSpeed ZeRO-3 JSON,
    FSDP plugin dict incl. the invalid `offload_params` / `auto_wrap_policy: size` keys,
    SURVEY Appendix A #16) onto this framework's parallel settings."""
    hw = cfg.get("hardware", {}) or {}
    out = {
        "grad_accum": int(hw.get("gradient_accumulation_steps", 1) or 1),
        "mixed_precision": hw.get("mixed_precision", "bf16"),
        "zero_stage": hw.get("zero_stage"),
        "tp_size": int(hw.get("tp_size", 1) or 1),
        "ep_size": int(hw.get("ep_size", 1) or 1),
        "sp_size": int(hw.get("sp_size", 1) or 1),  # Ulysses sequence parallel (parallel.sequence)
        # expert parallel dispatch: fixed-capacity blocks (no host sync; 0 = exact, host splits)
        "ep_capacity_factor": float(hw.get("ep_capacity_factor", 0.0)),
        "ep_chunks": int(hw.get("ep_chunks", 2) or 1),
        # Megatron sequence parallel inside the TP group (reduce-scatter / all-gather, sharded norms)
        "tp_sequence_parallel": bool(hw.get("tp_sequence_parallel", False)),
        "bucket_mb": float(hw.get("bucket_mb", 256)),
        "master_weights": bool(hw.get("master_weights", True)),
        "grad_dtype": hw.get("grad_dtype", "auto"),      # fp32 main grads (auto: grad_accum >= 16)
        "reduce_dtype": hw.get("reduce_dtype"),          # bucket collective dtype (default: grad)
        # build on the meta device, materialise only this rank's shards (auto: TP or FSDP)
        "sharded_init": hw.get("sharded_init", "auto"),
        "fsdp": False,
    }
    ds = hw.get("deepspeed_config")
    if ds:
        try:
            with open(ds, "r", encoding="utf-8") as fh:
                ds_cfg = json.load(fh)
            zo = ds_cfg.get("zero_optimization", {}) or {}
            stage = int(zo.get("stage", 0))
            for k in ("offload_optimizer", "offload_param"):
                if str((zo.get(k) or {}).get("device", "none")).lower() not in ("none", "null"):
                    raise ValueError(f"{ds}: zero_optimization.{k} offload is not supported "
                                     f"(state stays in 288 GB HBM per MI355X)")
            if ds_cfg.get("gradient_clipping") is not None:
                out["ds_gradient_clipping"] = float(ds_cfg["gradient_clipping"])
        except (OSError, json.JSONDecodeError):
            stage = 3
        out["zero_stage"] = stage if out["zero_stage"] is None else out["zero_stage"]
        out["fsdp"] = stage >= 3
    fs = hw.get("fsdp")
    if fs:
        strategy = fs.get("sharding_strategy", 1)
        out["fsdp"] = str(strategy).upper() in ("1", "FULL_SHARD")
        out["fsdp_min_num_params"] = int(fs.get("min_num_params", 1e6))
        out["cpu_offload"] = bool(fs.get("offload_params", fs.get("cpu_offload", False)))
        if out["zero_stage"] is None:
            out["zero_stage"] = 3 if out["fsdp"] else 2
    return out
