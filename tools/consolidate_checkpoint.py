#!/usr/bin/env python
"""Offline consolidation of a sharded checkpoint's optimizer state ("per-rank shard
files plus a consolidation tool that emits the flat layout").

Training writes `optimizer_shard_{rank}.pt` (each rank's ZeRO-1 / ZeRO-3 slice of the fp32 Adam
moments and master weights) and `dla_optimizer_layout.json`; above ~2B parameters the
in-training gather to a torch-format `optimizer.bin` is skipped (it would need the whole fp32
state on one rank). This tool rebuilds that `optimizer.bin` (torch.optim.AdamW state_dict, param
index = module parameter order, as accelerate writes it) on the CPU, streaming one shard at a
time. Tensor-parallel checkpoints (tp_size > 1) are refused: their shards are TP slices.

    python tools/consolidate_checkpoint.py checkpoints/dpo/step_500 [--out optimizer.bin]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch


def consolidate(ckpt: Path, out: Path | None = None, master: bool = False) -> Path:
    lay = json.loads((ckpt / "dla_optimizer_layout.json").read_text())
    if int(lay.get("tp_size", 1)) > 1:
        raise SystemExit("tensor-parallel optimizer shards are TP slices; consolidate per TP rank")
    world = int(lay["world"])
    shards = []
    for r in range(world):
        f = ckpt / f"optimizer_shard_{r}.pt"
        if not f.exists():
            raise SystemExit(f"missing {f}")
        shards.append(torch.load(str(f), map_location="cpu", weights_only=True))
    keys = ["exp_avg", "exp_avg_sq"] + (["master"] if master else [])
    full = {k: torch.zeros(int(lay["numel"]), dtype=torch.float32) for k in keys}
    if lay["kind"] == "flat":
        for b in lay["buckets"]:
            size, bw = b["end"] - b["start"], int(b["world"])
            c = size // bw
            for r in range(bw if lay["zero"] else 1):
                sh = shards[r]
                for k in keys:
                    if sh.get(k) is None:
                        continue
                    src = sh[k][b["shard_off"]:b["shard_off"] + c] if lay["zero"] else sh[k][b["start"]:b["end"]]
                    dst = full[k][b["start"] + r * c: b["start"] + (r + 1) * c] if lay["zero"] else full[k][b["start"]:b["end"]]
                    dst.copy_(src)
        params = lay["params"]
        locate = {p["index"]: p["offset"] for p in params}
    else:  # fsdp units: global offset = running sum of unit numels
        params, locate, base = [], {}, 0
        for u in lay["units"]:
            c = int(u["chunk"])
            for r in range(world):
                for k in keys:
                    if shards[r].get(k) is None:
                        continue
                    full[k][base + r * c: base + (r + 1) * c].copy_(shards[r][k][u["shard_off"]:u["shard_off"] + c])
            for p in u["params"]:
                params.append(p)
                locate[p["index"]] = base + p["offset"]
            base += int(u["numel"])
    step = float(shards[0]["step"])
    state = {}
    for p in sorted(params, key=lambda q: q["index"]):
        n = 1
        for d in p["shape"]:
            n *= d
        o = locate[p["index"]]
        state[p["index"]] = {"step": torch.tensor(step),
                             **{k: full[k][o:o + n].view(p["shape"]).clone() for k in ("exp_avg", "exp_avg_sq")}}
    sh0 = shards[0]
    group = {"lr": sh0["lr"], "betas": tuple(sh0["betas"]), "eps": sh0["eps"], "weight_decay": sh0["weight_decay"],
             "amsgrad": False, "foreach": None, "maximize": False, "capturable": False, "differentiable": False,
             "fused": None, "params": sorted(state)}
    out = out or ckpt / "optimizer.bin"
    torch.save({"state": state, "param_groups": [group]}, out)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("checkpoint")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    print(consolidate(Path(a.checkpoint), Path(a.out) if a.out else None))
    return 0


if __name__ == "__main__":
    sys.exit(main())
