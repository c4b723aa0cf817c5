"""Consolidation of per-rank optimizer shards into accelerate's `optimizer.bin` (torch.optim.AdamW
state_dict, param index = module parameter order) — reference `src/training/utils.py:99-102`
(`accelerator.save_state` always writes it).

Training writes `optimizer_shard_{rank}.safetensors` (utils/stream_st.py) and
`dla_optimizer_layout.json`. This module maps every shard file read-only (page cache, no
anonymous host memory), finds each parameter's `exp_avg` / `exp_avg_sq` in the rank pieces that
hold it, and hands `torch.save` either a zero-copy view of the mapping (the parameter lies in one
rank's piece: the common case) or a copy assembled from the pieces (a parameter that straddles
ranks: bounded by one parameter). Host memory therefore stays at ~one parameter however large the
model, which is what lets `save_state` write optimizer.bin at 7B/8B scale in-line (rank 0, after
the shard barrier) and `tools/consolidate_checkpoint.py` do it offline for anything. Legacy
`optimizer_shard_{rank}.pt` files are read with `torch.load(mmap=True, weights_only=True)`.
Tensor-parallel and expert-parallel checkpoints are refused: their shards are TP slices / per-EP-rank
experts, not one flat state.
"""
from __future__ import annotations

import bisect
import json
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import torch

_KEYS = ("exp_avg", "exp_avg_sq")


def _open_shard(ckpt: Path, r: int) -> Dict[str, object]:
    f = ckpt / f"optimizer_shard_{r}.safetensors"
    if f.exists():
        from .stream_st import mmap_tensor, read_header

        hdr = read_header(f)
        sd: Dict[str, object] = dict(hdr[2])
        sd.update({k: mmap_tensor(f, k, hdr) for k in hdr[0]})
        return sd
    f = ckpt / f"optimizer_shard_{r}.pt"
    if f.exists():
        return torch.load(str(f), map_location="cpu", weights_only=True, mmap=True)
    raise FileNotFoundError(f"missing optimizer shard {r} in {ckpt}")


def _segments(lay) -> List[Tuple[int, int, int, int]]:
    """(global start, global end, rank, offset in that rank's shard), sorted by start."""
    seg = []
    if lay["kind"] == "flat":
        for b in lay["buckets"]:
            size, bw = b["end"] - b["start"], int(b["world"])
            if lay["zero"]:
                c = size // bw
                for r in range(bw):
                    seg.append((b["start"] + r * c, b["start"] + (r + 1) * c, r, b["shard_off"]))
            else:
                seg.append((b["start"], b["end"], 0, b["start"]))
    else:  # fsdp units: global offset = running sum of unit numels
        base, world = 0, int(lay["world"])
        for u in lay["units"]:
            c = int(u["chunk"])
            for r in range(world):
                seg.append((base + r * c, base + (r + 1) * c, r, int(u["shard_off"])))
            base += int(u["numel"])
    seg.sort()
    return seg


def _param_offsets(lay) -> Dict[int, Tuple[int, List[int]]]:
    if lay["kind"] == "flat":
        return {p["index"]: (p["offset"], p["shape"]) for p in lay["params"]}
    out, base = {}, 0
    for u in lay["units"]:
        for p in u["params"]:
            out[p["index"]] = (base + p["offset"], p["shape"])
        base += int(u["numel"])
    return out


def _gather(shards, seg, starts, key: str, o: int, n: int) -> Optional[torch.Tensor]:
    i = bisect.bisect_right(starts, o) - 1
    s0, e0, r0, so0 = seg[i]
    src0 = shards[r0].get(key)
    if src0 is None:
        return None
    if o + n <= e0:  # wholly inside one rank's piece: a view of the mapping (no copy)
        return src0[so0 + (o - s0): so0 + (o - s0) + n]
    out = torch.empty(n, dtype=src0.dtype)
    pos = o
    while pos < o + n:
        s, e, r, so = seg[i]
        take = min(e, o + n) - pos
        out[pos - o: pos - o + take].copy_(shards[r][key][so + (pos - s): so + (pos - s) + take])
        pos += take
        i += 1
    return out


def consolidate_optimizer(ckpt, out=None) -> Path:
    """Write `optimizer.bin` (torch AdamW state_dict) for the checkpoint directory `ckpt`."""
    ckpt = Path(ckpt)
    lay = json.loads((ckpt / "dla_optimizer_layout.json").read_text())
    if int(lay.get("tp_size", 1)) > 1:
        raise ValueError("tensor-parallel optimizer shards are TP slices; consolidate per TP rank")
    if any(b.get("expert") for b in lay.get("buckets", [])):
        # expert buckets: world = expert-DP size, rank = expert-DP rank, indices local to one
        # EP rank's experts; the layout (written by rank 0) does not describe the other experts
        raise ValueError("expert-parallel optimizer shards hold per-EP-rank experts; a flat "
                         "optimizer.bin cannot be built from them (resume from the shards)")
    world = int(lay["world"])
    n_ranks = world if (lay["kind"] != "flat" or lay["zero"]) else 1
    shards = [_open_shard(ckpt, r) for r in range(n_ranks)]
    seg = _segments(lay)
    starts = [s[0] for s in seg]
    step = float(shards[0]["step"])
    state = {}
    for idx, (o, shape) in sorted(_param_offsets(lay).items()):
        n = 1
        for d in shape:
            n *= d
        ent = {"step": torch.tensor(step)}
        for k in _KEYS:
            t = _gather(shards, seg, starts, k, o, n)
            if t is not None:
                ent[k] = t.view(shape)
        state[idx] = ent
    sh0 = shards[0]
    group = {"lr": sh0["lr"], "betas": tuple(sh0["betas"]), "eps": sh0["eps"],
             "weight_decay": sh0["weight_decay"], "amsgrad": False, "foreach": None, "maximize": False,
             "capturable": False, "differentiable": False, "fused": None, "params": sorted(state)}
    out = Path(out) if out is not None else ckpt / "optimizer.bin"
    tmp = out.with_suffix(out.suffix + ".tmp")
    torch.save({"state": state, "param_groups": [group]}, tmp)
    tmp.replace(out)
    return out
