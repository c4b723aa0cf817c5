"""Checkpoint / resume in the accelerate `save_state` layout.

`save_state(dir, models=[m0, m1, ...], engine, scheduler, step)` writes, like
`accelerator.save_state` for a single-process / DDP run:
  model.safetensors, model_1.safetensors, ...   HF key names, in `prepare` order
                                                 (DPO: policy, ref; RLHF: policy, ref, reward;
                                                 distill: student, teachers...)
  optimizer.bin                                  torch AdamW-format state dict (consolidated)
  scheduler.bin                                  only when a scheduler is given
  random_states_{rank}.pkl                       step + python / numpy / torch / cuda RNG
Extras the reference lacks (Appendix A #6, §5.4 gaps): `optimizer_shard_{rank}.safetensors`
(exact ZeRO-sharded state for fast resume, streamed from the device through one pinned buffer:
host RSS stays bounded however large the shard, utils/stream_st.py), `dla_state.json` (step, layout), an `hf/` export of model 0
(config.json + model.safetensors + tokenizer, `from_pretrained`-style so stages chain), a
`latest` pointer next to the step dirs, and keep-last-N rotation. `load_state` resumes; model
loading tolerates `module.` prefixes and `pytorch_model.bin`.
"""
from __future__ import annotations

import json
import os
import random
import shutil
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from ..parallel import dist as pdist

CONSOLIDATE_MAX_NUMEL = 2_000_000_000  # in-memory gather of optimizer.bin up to ~2B params
# Above that, optimizer.bin is consolidated by rank 0 from the page-cache mapped shard files
# (tools/consolidate_checkpoint.py; no host copy of the whole state) up to this many params
# (DLA_OPTIMIZER_BIN_MAX_NUMEL; 0 disables): Llama-3-8B is written by default, 70B is not (a
# 560 GB file from one rank) and stays consolidatable offline with the same tool.
STREAM_CONSOLIDATE_MAX_NUMEL = int(float(os.environ.get("DLA_OPTIMIZER_BIN_MAX_NUMEL", "1.6e10")))


def _rng_state() -> Dict[str, Any]:
    """Reference keys (accelerate random_states_{rank}.pkl), stored with tensors / tuples / ints
    only so resuming loads them with torch.load(weights_only=True) (no pickle execution)."""
    name, key, pos, has_gauss, cached = np.random.get_state()
    st = {"random_state": random.getstate(),
          "numpy_random_seed": (name, torch.from_numpy(key.astype(np.int64)), int(pos),
                                int(has_gauss), float(cached)),
          "torch_manual_seed": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["torch_cuda_manual_seed"] = torch.cuda.get_rng_state_all()
    return st


def _set_rng_state(st: Dict[str, Any]):
    v, internal, gauss = st["random_state"]
    random.setstate((v, tuple(internal), gauss))
    name, key, pos, has_gauss, cached = st["numpy_random_seed"]
    np.random.set_state((name, np.asarray(key, dtype=np.int64).astype(np.uint32), pos, has_gauss, cached))
    torch.set_rng_state(st["torch_manual_seed"])
    if torch.cuda.is_available() and "torch_cuda_manual_seed" in st:
        torch.cuda.set_rng_state_all(st["torch_cuda_manual_seed"])


def _is_sharded(model) -> bool:
    from ..parallel.tensor_parallel import is_tensor_parallel

    return (getattr(model, "_dla_fsdp", None) is not None or is_tensor_parallel(model)
            or any(getattr(p, "_dla_ep", None) is not None for p in model.parameters()))


def _stem(i: int) -> str:
    return "model" if i == 0 else f"model_{i}"


def save_state(output_dir, models: Sequence, engine=None, scheduler=None, step: int = 0,
               tokenizer=None, hf_export: bool = True, keep_last: Optional[int] = None,
               extra: Optional[Dict[str, Any]] = None, weights: Optional[str] = None) -> Path:
    """`weights`: "full" (HF-named, streamed one unit at a time), "sharded" (per-rank local
    files only, no collective), "both", or None = DLA_CKPT_WEIGHTS / auto ("both" when a model is
    sharded across ranks, else "full")."""
    from ..models.loader import save_hf_export_files
    from . import sharded_io

    out = Path(output_dir)
    st = pdist.state()
    if st.is_main:
        out.mkdir(parents=True, exist_ok=True)
    pdist.barrier()
    if engine is not None and hasattr(engine, "wait_params"):
        engine.wait_params()  # overlapped ZeRO-1 all-gathers must land before weights are read
    from ..parallel.tensor_parallel import is_tensor_parallel

    tp = any(is_tensor_parallel(m) for m in models)
    mode = weights or os.environ.get("DLA_CKPT_WEIGHTS") or "auto"
    for i, m in enumerate(models):
        m_mode = mode if mode != "auto" else ("both" if _is_sharded(m) else "full")
        if m_mode in ("sharded", "both"):
            sharded_io.save_rank_shards(m, out, _stem(i))
        if m_mode in ("full", "both"):
            files = sharded_io.save_consolidated(m, out, _stem(i), st.is_main)
            if i == 0 and hf_export and st.is_main:
                # the HF export shares the weight files (hard links: no second gather or copy)
                hf = out / "hf"
                hf.mkdir(parents=True, exist_ok=True)
                for f in files + ([f"{_stem(i)}.safetensors.index.json"] if len(files) > 1 else []):
                    _link_or_copy(out / f, hf / f)
                save_hf_export_files(m, tokenizer, str(hf))
    if st.is_main and scheduler is not None:
        torch.save(scheduler.state_dict(), out / "scheduler.bin")
    if engine is not None:
        from .stream_st import save_streamed

        osd_local = engine.optimizer_state()
        tens = {k: v for k, v in osd_local.items() if isinstance(v, torch.Tensor) or v is None}
        meta = {k: (list(v) if isinstance(v, tuple) else v) for k, v in osd_local.items() if k not in tens}
        save_streamed(out / f"optimizer_shard_{st.rank}.safetensors", tens, meta)
        if st.is_main and hasattr(engine, "layout"):
            (out / "dla_optimizer_layout.json").write_text(json.dumps(engine.layout()))
        # expert-parallel state: each EP rank holds different experts under local indices, and the
        # expert buckets are sharded over the expert-DP group, not the global ranks -- one flat
        # optimizer.bin cannot be assembled from rank-local layouts (the per-rank shards are the
        # checkpoint; like TP, consolidation is refused rather than written partially)
        ep = bool(getattr(engine, "has_experts", False))
        if engine.numel <= CONSOLIDATE_MAX_NUMEL and not tp and not ep:
            osd = engine.torch_optimizer_state_dict()  # collective under ZeRO (gathered per unit)
            if st.is_main:
                torch.save(osd, out / "optimizer.bin")
        elif (not tp and not ep and engine.numel <= STREAM_CONSOLIDATE_MAX_NUMEL
              and hasattr(engine, "layout")):
            pdist.barrier()  # every rank's shard is on disk
            if st.is_main:
                from .consolidate import consolidate_optimizer as consolidate

                consolidate(out, out / "optimizer.bin")
    torch.save({"step": step, **_rng_state()}, out / f"random_states_{st.rank}.pkl")
    if st.is_main:
        meta = {"step": step, "world_size": st.world_size, "num_models": len(models),
                "zero": getattr(engine, "zero", 0) if engine is not None else None,
                "weights": mode, **(extra or {})}
        (out / "dla_state.json").write_text(json.dumps(meta, indent=2))
        if models:
            # self-describing root: the model-0 architecture + tokenizer, so a checkpoint dir can be
            # passed wherever a model path is expected (e.g. --reward_model checkpoints/reward/final)
            base = getattr(models[0], "backbone", models[0])
            if hasattr(base, "cfg"):
                (out / "dla_config.json").write_text(json.dumps(base.cfg.to_dict(), indent=2))
            if tokenizer is not None and hasattr(tokenizer, "save_pretrained"):
                tokenizer.save_pretrained(str(out))
        _update_latest(out)
        if keep_last:
            _rotate(out.parent, keep_last)
    pdist.barrier()
    return out


def _link_or_copy(src: Path, dst: Path) -> None:
    if dst.exists():
        dst.unlink()
    try:
        os.link(src, dst)
    except OSError:
        shutil.copyfile(src, dst)


def _update_latest(ckpt: Path):
    """`<output_dir>/latest` -> the newest checkpoint's HF export (or dir) so downstream configs
    that point at `checkpoints/<stage>/latest` load."""
    link = ckpt.parent / "latest"
    target = ckpt / "hf" if (ckpt / "hf").exists() else ckpt
    try:
        if link.is_symlink() or link.is_file():
            link.unlink()
        elif link.is_dir():
            shutil.rmtree(link)
        os.symlink(os.path.relpath(target, ckpt.parent), link)
    except OSError:
        shutil.copytree(target, link)
    (ckpt.parent / "latest_checkpoint.txt").write_text(ckpt.name)


def _rotate(root: Path, keep: int):
    steps = sorted([p for p in root.glob("step_*") if p.is_dir()],
                   key=lambda p: int(p.name.split("_")[1]) if p.name.split("_")[1].isdigit() else 0)
    for p in steps[:-keep]:
        shutil.rmtree(p, ignore_errors=True)


def resolve_checkpoint(path) -> Optional[Path]:
    p = Path(path)
    if p.name == "latest" or (p / "latest_checkpoint.txt").exists():
        root = p.parent if p.name == "latest" else p
        marker = root / "latest_checkpoint.txt"
        if marker.exists():
            return root / marker.read_text().strip()
    return p if p.exists() else None


def _weights_present(d: Path, index: int) -> bool:
    stem = _stem(index)
    return ((d / f"{stem}.safetensors").exists() or (d / f"{stem}.safetensors.index.json").exists()
            or (d / f"{stem}.shards.json").exists())


def load_model_weights(model, ckpt_dir, index: int = 0, strict: bool = True):
    """Load model `index` of a checkpoint into a (possibly FSDP / TP / EP sharded) model.
    Per-rank shard files are used when their layout matches (exact, no collective on the
    weights); otherwise the HF-named files are streamed in one unit at a time."""
    from . import sharded_io
    from ..models.hf_io import LazyTensors

    d = Path(ckpt_dir)
    stem = _stem(index)
    if (d / f"{stem}.shards.json").exists() and sharded_io.load_rank_shards(model, d, stem):
        return [], []
    sd = sharded_io.open_consolidated(d, stem)
    if sd is None and (d / "pytorch_model.bin").exists() and index == 0:
        raw = torch.load(str(d / "pytorch_model.bin"), map_location="cpu", weights_only=True)
        sd = LazyTensors(raw.keys(), raw.__getitem__)
    if sd is None:
        raise FileNotFoundError(f"no weights for model {index} in {d}")
    return sharded_io.load_consolidated(model, sd, strict=strict)


def load_state(ckpt_dir, models: Sequence, engine=None, scheduler=None, load_models: bool = True) -> int:
    """Resume: weights, optimizer (exact sharded state when layouts match), scheduler, RNG.
    Returns the saved step."""
    d = resolve_checkpoint(ckpt_dir)
    if d is None:
        raise FileNotFoundError(ckpt_dir)
    st = pdist.state()
    if load_models:
        for i, m in enumerate(models):
            if _weights_present(d, i):
                load_model_weights(m, d, i, strict=True)
    if engine is not None:
        shard = d / f"optimizer_shard_{st.rank}.safetensors"
        legacy = d / f"optimizer_shard_{st.rank}.pt"
        if shard.exists():
            from .stream_st import mmap_tensor, read_header

            hdr = read_header(shard)
            sd = dict(hdr[2])
            sd.update({k: mmap_tensor(shard, k, hdr) for k in hdr[0]})  # copied chunk-free by .copy_
            sd.setdefault("master", None)
            engine.load_optimizer_state(sd)
        elif legacy.exists():
            sd = torch.load(str(legacy), map_location="cpu", weights_only=True)
            engine.load_optimizer_state({k: (v.to(engine.device) if isinstance(v, torch.Tensor) else v)
                                         for k, v in sd.items()})
        else:
            engine.sync_master_from_params()
        if engine.master is None:
            engine.sync_master_from_params()
    if scheduler is not None and (d / "scheduler.bin").exists():
        scheduler.load_state_dict(torch.load(str(d / "scheduler.bin"), weights_only=True))
    rs = d / f"random_states_{st.rank}.pkl"
    step = 0
    if rs.exists():
        try:
            rstate = torch.load(str(rs), weights_only=True)  # never unpickles code
        except Exception as e:  # e.g. a pre-r2 file holding numpy arrays: resume without RNG
            import warnings

            warnings.warn(f"RNG state {rs} not restored (not weights_only-loadable: {e})")
            rstate = None
        if rstate is not None:
            step = int(rstate.get("step", 0))
            _set_rng_state(rstate)
    meta = d / "dla_state.json"
    if meta.exists():
        step = int(json.loads(meta.read_text()).get("step", step))
    # weight-derived caches (W^T for the TN dgrad, fp8 / transposed expert copies) were keyed on
    # versions the in-place loads above did not move: drop them so nothing stale is read
    for m in models:
        invalidate_weight_caches(m)
    if engine is not None and hasattr(engine, "_wt_epoch"):
        engine._wt_epoch[0] += 1
    return step


def invalidate_weight_caches(model) -> None:
    """Drop every cache derived from a parameter's values (ops.linear `_dla_wt`, ops.moe
    `_dla_fp8` / `_dla_wT`): the next use rebuilds it from the current weights."""
    from ..ops.moe import free_transposed_experts

    free_transposed_experts(model)
    for p in model.parameters():
        for k in ("_dla_wt_ver", "_dla_fp8"):
            p.__dict__.pop(k, None)
        for k in ("_dla_fold", "_dla_fold_t", "_dla_fold_g", "_dla_tile"):  # ops.decode derived weights
            c = p.__dict__.get(k)
            if c is not None:  # keep the buffer (a captured decode graph reads it), mark stale
                setattr(p, k, (None, c[1]))
