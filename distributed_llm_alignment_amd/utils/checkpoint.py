"""Checkpoint / resume in the accelerate `save_state` layout.

`save_state(dir, models=[m0, m1, ...], engine, scheduler, step)` writes, like
`accelerator.save_state` for a single-process / DDP run:
  model.safetensors, model_1.safetensors, ...   HF key names, in `prepare` order
                                                 (DPO: policy, ref; RLHF: policy, ref, reward;
                                                 distill: student, teachers...)
  optimizer.bin                                  torch AdamW-format state dict (consolidated)
  scheduler.bin                                  only when a scheduler is given
  random_states_{rank}.pkl                       step + python / numpy / torch / cuda RNG
Extras the reference lacks (Appendix A #6, §5.4 gaps): `optimizer_shard_{rank}.pt` (exact
ZeRO-sharded state for fast resume), `dla_state.json` (step, layout), an `hf/` export of model 0
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

CONSOLIDATE_MAX_NUMEL = 2_000_000_000  # gather a torch-format optimizer.bin up to ~2B params


def _model_file(i: int) -> str:
    return "model.safetensors" if i == 0 else f"model_{i}.safetensors"


def _rng_state() -> Dict[str, Any]:
    st = {"random_state": random.getstate(),
          "numpy_random_seed": np.random.get_state(),
          "torch_manual_seed": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["torch_cuda_manual_seed"] = torch.cuda.get_rng_state_all()
    return st


def _set_rng_state(st: Dict[str, Any]):
    random.setstate(st["random_state"])
    np.random.set_state(st["numpy_random_seed"])
    torch.set_rng_state(st["torch_manual_seed"])
    if torch.cuda.is_available() and "torch_cuda_manual_seed" in st:
        torch.cuda.set_rng_state_all(st["torch_cuda_manual_seed"])


def _state_dict_of(model) -> Dict[str, torch.Tensor]:
    sd = model.hf_state_dict() if hasattr(model, "hf_state_dict") else model.state_dict()
    out, seen = {}, {}
    for k, v in sd.items():
        t = v.detach().contiguous().cpu()
        key = (v.data_ptr(), tuple(v.shape), tuple(v.stride()))
        out[k] = t.clone() if key in seen else t
        seen[key] = k
    return out


def save_state(output_dir, models: Sequence, engine=None, scheduler=None, step: int = 0,
               tokenizer=None, hf_export: bool = True, keep_last: Optional[int] = None,
               extra: Optional[Dict[str, Any]] = None) -> Path:
    from safetensors.torch import save_file

    out = Path(output_dir)
    st = pdist.state()
    if st.is_main:
        out.mkdir(parents=True, exist_ok=True)
    pdist.barrier()
    if engine is not None and hasattr(engine, "wait_params"):
        engine.wait_params()  # overlapped ZeRO-1 all-gathers must land before weights are read
    from contextlib import ExitStack

    from ..parallel.fsdp import fsdp_full_params
    from ..parallel.tensor_parallel import is_tensor_parallel, tp_unsharded

    tp = any(is_tensor_parallel(m) for m in models)
    with ExitStack() as stack:
        for m in models:  # sharded weights are gathered on every rank (collectives)
            stack.enter_context(fsdp_full_params(m))
            stack.enter_context(tp_unsharded(m))
        if st.is_main:
            for i, m in enumerate(models):
                save_file(_state_dict_of(m), str(out / _model_file(i)), metadata={"format": "pt"})
            if hf_export and models:
                from ..models.loader import save_hf_pretrained

                save_hf_pretrained(models[0], tokenizer, str(out / "hf"))
    if st.is_main and scheduler is not None:
        torch.save(scheduler.state_dict(), out / "scheduler.bin")
    if engine is not None:
        torch.save({k: (v.cpu() if isinstance(v, torch.Tensor) else v)
                    for k, v in engine.optimizer_state().items()}, out / f"optimizer_shard_{st.rank}.pt")
        if st.is_main and hasattr(engine, "layout"):
            (out / "dla_optimizer_layout.json").write_text(json.dumps(engine.layout()))
        if engine.numel <= CONSOLIDATE_MAX_NUMEL and not tp:
            osd = engine.torch_optimizer_state_dict()  # collective under ZeRO
            if st.is_main:
                torch.save(osd, out / "optimizer.bin")
    torch.save({"step": step, **_rng_state()}, out / f"random_states_{st.rank}.pkl")
    if st.is_main:
        meta = {"step": step, "world_size": st.world_size, "num_models": len(models),
                "zero": getattr(engine, "zero", 0) if engine is not None else None, **(extra or {})}
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


def load_model_weights(model, ckpt_dir, index: int = 0, strict: bool = True):
    from safetensors.torch import load_file

    d = Path(ckpt_dir)
    f = d / _model_file(index)
    if f.exists():
        sd = load_file(str(f))
    elif (d / "pytorch_model.bin").exists() and index == 0:
        sd = torch.load(str(d / "pytorch_model.bin"), map_location="cpu", weights_only=True)
    else:
        raise FileNotFoundError(f"no weights for model {index} in {d}")
    from ..parallel.fsdp import fsdp_full_params
    from ..parallel.tensor_parallel import tp_unsharded

    # full tensors in, re-sliced to this TP rank / FSDP shard
    with fsdp_full_params(model, writeback=True), tp_unsharded(model, writeback=True):
        if hasattr(model, "load_hf_state_dict"):
            return model.load_hf_state_dict(sd, strict=strict)
        sd = {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}
        return model.load_state_dict(sd, strict=strict)


def load_state(ckpt_dir, models: Sequence, engine=None, scheduler=None, load_models: bool = True) -> int:
    """Resume: weights, optimizer (exact sharded state when layouts match), scheduler, RNG.
    Returns the saved step."""
    d = resolve_checkpoint(ckpt_dir)
    if d is None:
        raise FileNotFoundError(ckpt_dir)
    st = pdist.state()
    if load_models:
        for i, m in enumerate(models):
            if (d / _model_file(i)).exists():
                load_model_weights(m, d, i, strict=True)
    if engine is not None:
        shard = d / f"optimizer_shard_{st.rank}.pt"
        if shard.exists():
            sd = torch.load(str(shard), map_location="cpu", weights_only=True)
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
        rstate = torch.load(str(rs), weights_only=False)  # written by this framework (own file)
        step = int(rstate.get("step", 0))
        _set_rng_state(rstate)
    meta = d / "dla_state.json"
    if meta.exists():
        step = int(json.loads(meta.read_text()).get("step", step))
    return step
