#!/usr/bin/env python
"""Offline consolidation of a sharded checkpoint's optimizer state ("per-rank shard
files plus a consolidation tool that emits the flat layout").

Training writes `optimizer_shard_{rank}.safetensors` (each rank's ZeRO-1 / ZeRO-3 slice of the
fp32 Adam moments and master weights, streamed from the device) and `dla_optimizer_layout.json`;
`save_state` consolidates `optimizer.bin` itself up to DLA_OPTIMIZER_BIN_MAX_NUMEL parameters
(default 16B: Llama-3-8B yes, 70B no). This tool rebuilds that `optimizer.bin`
(torch.optim.AdamW state_dict, param index = module parameter order, as accelerate writes it)
offline for any size, with the shard files mapped read-only (host memory ~one parameter).
Tensor-parallel checkpoints (tp_size > 1) are refused: their shards are TP slices.

`--weights` rebuilds the HF-named model files (`model.safetensors`, or HF index shards for
large models) from the per-rank weight shards `{stem}.fsdp{r}-tp{t}-ep{e}.safetensors` +
`{stem}.shards.json` (utils/sharded_io.py): FSDP flat shards are re-assembled per unit, TP
slices merged segment-wise, expert stacks concatenated, then converted to HF names — one unit
at a time (safetensors slices are read lazily), so host memory stays bounded by one unit plus
one output shard.

    python tools/consolidate_checkpoint.py checkpoints/dpo/step_500 [--out optimizer.bin]
    python tools/consolidate_checkpoint.py checkpoints/dpo/step_500 --weights [--stem model_1] [--out-dir DIR]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def consolidate(ckpt: Path, out: Path | None = None) -> Path:
    """optimizer.bin from the per-rank shards (page-cache mapped, ~one parameter of host memory:
    distributed_llm_alignment_amd/utils/consolidate.py)."""
    from distributed_llm_alignment_amd.utils.consolidate import consolidate_optimizer

    try:
        return consolidate_optimizer(ckpt, out)
    except ValueError as e:
        raise SystemExit(str(e))


class _Native:
    """Stand-in for a model: `cfg` + `named_parameters()` over host tensors (for the key map)."""

    def __init__(self, cfg, tensors):
        self.cfg = cfg
        self._t = tensors

    def named_parameters(self):
        return iter(self._t.items())


def _merge_tp(pieces, spec):
    dim, segs = spec
    tp = len(pieces)
    loc = [n // tp for n in segs]
    per_rank = [torch.split(pc, loc, dim) for pc in pieces]
    return torch.cat([per_rank[rk][i] for i in range(len(segs)) for rk in range(tp)], dim)


def _to_hf(kind, cfg, tensors):
    from distributed_llm_alignment_amd.models.hf_io import to_hf_state_dict

    if kind in ("RewardModel", "ValueModel"):
        bb = {n[len("backbone."):]: t for n, t in tensors.items() if n.startswith("backbone.")}
        out = {f"backbone.{k}": v for k, v in to_hf_state_dict(_Native(cfg, bb), base=True).items()}
        out.update({n: t for n, t in tensors.items() if not n.startswith("backbone.")})
        return out
    if kind == "CausalLM":
        return to_hf_state_dict(_Native(cfg, tensors))
    return dict(tensors)


def consolidate_weights(ckpt: Path, stem: str = "model", out_dir: Path | None = None):
    """Per-rank weight shards -> HF-named `{stem}.safetensors` (or index shards) in out_dir."""
    from safetensors import safe_open

    from distributed_llm_alignment_amd.models.config import ModelConfig
    from distributed_llm_alignment_amd.utils.sharded_io import FSDP_KEY, ConsolidatedWriter

    lay = json.loads((ckpt / f"{stem}.shards.json").read_text())
    tp, ep, fw = int(lay["tp_size"]), int(lay["ep_size"]), int(lay["fsdp_world"])
    params = lay["params"]
    cfg = ModelConfig.from_dict(lay["cfg"]) if lay.get("cfg") else None
    handles = {}

    def h(r, t, e):
        key = (r, t, e)
        if key not in handles:
            f = ckpt / f"{stem}.fsdp{r}-tp{t}-ep{e}.safetensors"
            if not f.exists():
                raise SystemExit(f"missing weight shard {f}")
            handles[key] = safe_open(str(f), framework="pt")
        return handles[key]

    def numel(shape):
        n = 1
        for d in shape:
            n *= d
        return n

    def local(name, t, e, unit_flat=None, offset=None):
        if unit_flat is not None:
            return unit_flat[t][offset:offset + numel(params[name]["shape"])].view(params[name]["shape"])
        return h(0, t, e).get_tensor(name)

    def full(name, getter):
        info = params[name]
        if info["tp_spec"] is not None:
            return _merge_tp([getter(t, 0) for t in range(tp)], (info["tp_spec"][0], info["tp_spec"][1]))
        if int(info["ep"]) > 1:
            return torch.cat([getter(0, e) for e in range(int(info["ep"]))], 0)
        return getter(0, 0)

    groups = []  # [(unit or None, [names])]
    if lay.get("fsdp_units"):
        groups = [(u, [q["name"] for q in u["params"]]) for u in lay["fsdp_units"]]
        in_units = {n for _, ns in groups for n in ns}
        rest = [n for n in params if n not in in_units]
        if rest:
            groups.append((None, rest))
    else:
        by_layer, rest = {}, []
        for n in params:
            parts = n.split(".")
            i = parts.index("layers") if "layers" in parts else -1
            if i >= 0 and i + 1 < len(parts) and parts[i + 1].isdigit():
                by_layer.setdefault(int(parts[i + 1]), []).append(n)
            else:
                rest.append(n)
        groups = [(None, by_layer[k]) for k in sorted(by_layer)] + ([(None, rest)] if rest else [])
    total = sum(numel(v["shape"]) * (tp if v["tp_spec"] is not None else 1) * int(v["ep"]) * 2
                for v in params.values())
    out_dir = Path(out_dir or ckpt)
    out_dir.mkdir(parents=True, exist_ok=True)
    w = ConsolidatedWriter(out_dir, stem, total)
    for u, names in groups:
        flats = None
        if u is not None:  # re-assemble the unit's flat buffer per TP rank from the FSDP ranks
            c, so = int(u["chunk"]), int(u["shard_off"])
            flats = [torch.cat([h(r, t, 0).get_slice(FSDP_KEY)[so:so + c] for r in range(fw)])
                     for t in range(tp)]
        offs = {q["name"]: q["offset"] for q in u["params"]} if u is not None else {}
        tensors = {}
        for n in names:
            if n in offs:
                tensors[n] = full(n, lambda t, e, n=n: local(n, t, e, flats, offs[n]))
            else:
                tensors[n] = full(n, lambda t, e, n=n: local(n, t, e))
        hf = _to_hf(lay.get("kind"), cfg, tensors)
        w.add({k: v.contiguous().clone() for k, v in hf.items()})
    return w.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("checkpoint")
    ap.add_argument("--out", default=None)
    ap.add_argument("--weights", action="store_true", help="consolidate model weights instead")
    ap.add_argument("--stem", default="model")
    ap.add_argument("--out-dir", default=None)
    a = ap.parse_args(argv)
    if a.weights:
        print(consolidate_weights(Path(a.checkpoint), a.stem, Path(a.out_dir) if a.out_dir else None))
        return 0
    print(consolidate(Path(a.checkpoint), Path(a.out) if a.out else None))
    return 0


if __name__ == "__main__":
    sys.exit(main())
