"""Shared trainer core ("all share one Trainer core").

Reference loop semantics kept (src/training/train_{sft,reward,dpo,distill}.py):
  * `global_step` counts MICRO-batches; log / eval / save / max_train_steps are in micro-steps
    (Appendix A #12);
  * gradients accumulate over `hardware.gradient_accumulation_steps` micro-batches, the loss is
    divided by that count (accelerator.backward), the optimizer + clipping run on sync steps and
    at the end of the dataloader (accelerate's `accumulate` semantics);
  * checkpoints at `step_{N}` every `save_every_steps` and at `final`.
What differs: no accelerate; one process per GPU with RCCL; the DataParallelEngine (flat buffers,
overlapped bucketed reduce-scatter, ZeRO-1, fused AdamW) replaces DDP/DeepSpeed/FSDP; metrics are
really logged (JSONL); `--resume` restores weights, optimizer, scheduler, RNG and step.
"""
from __future__ import annotations

import contextlib
import os
import random
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch

from ..optim.scheduler import LRSchedule
from ..parallel.data_parallel import DataParallelEngine
from ..parallel.dist import DistState, init_distributed
from ..utils.checkpoint import load_state, resolve_checkpoint, save_state
from ..utils.config import hardware_parallel
from ..utils.debug import FaultInjector, check_replicas_in_sync
from ..utils.logging import MetricsLogger, RunningLoss, log_rank_zero
from ..utils.tracing import PHASES, ProfileWindow, trace_range


def seed_everything(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


@dataclass
class TrainContext:
    cfg: Dict[str, Any]
    dist: DistState
    device: torch.device
    logger: MetricsLogger
    hw: Dict[str, Any]
    output_dir: str
    log_dir: str
    seed: int
    stage: str
    extras: Dict[str, Any] = field(default_factory=dict)
    mesh: Any = None

    @property
    def dp_size(self) -> int:
        return self.mesh.dp if self.mesh is not None else self.dist.world_size

    @property
    def is_main(self) -> bool:
        return self.dist.is_main

    def log(self, msg: str):
        log_rank_zero(msg, self.is_main)


def setup(cfg: Dict[str, Any], stage: str, default_seed: int = 0) -> TrainContext:
    hw_cfg = cfg.get("hardware", {}) or {}
    st = init_distributed(timeout_s=int(hw_cfg.get("collective_timeout_s", 1800)))
    if st.device.type == "cuda":
        from ..utils.tuning import enable_gemm_tuning

        enable_gemm_tuning(st.device.index)
    seed = int(cfg.get("seed", default_seed))
    seed_everything(seed)
    lg = cfg.get("logging", {}) or {}
    out = lg.get("output_dir", f"checkpoints/{stage}")
    log_dir = lg.get("log_dir", f"logs/{stage}")
    if st.is_main:
        Path(out).mkdir(parents=True, exist_ok=True)
        Path(log_dir).mkdir(parents=True, exist_ok=True)
    logger = MetricsLogger(log_dir, st.is_main, use_wandb=bool(lg.get("use_wandb", False)),
                           config=cfg, run_name=cfg.get("experiment_name"))
    hw = hardware_parallel(cfg)
    from ..parallel.mesh import build_mesh

    mesh = build_mesh(tp=hw["tp_size"], ep=hw["ep_size"], sp=hw.get("sp_size", 1))  # collective
    return TrainContext(cfg=cfg, dist=st, device=st.device, logger=logger, hw=hw,
                        output_dir=out, log_dir=log_dir, seed=seed, stage=stage, mesh=mesh)


def parallelize(ctx: TrainContext, model):
    """Apply the configured model parallelism (hardware.tp_size / ep_size) in place. Every rank
    built the same seeded (or loaded) weights, so sharding is a local slice — no broadcast."""
    m = ctx.mesh
    if m is None:
        return model
    base = getattr(model, "backbone", model)
    if m.tp > 1:
        from ..parallel.tensor_parallel import apply_tensor_parallel

        apply_tensor_parallel(model, m.tp_group,
                              sequence_parallel=bool(ctx.hw.get("tp_sequence_parallel", False)))
    if m.sp > 1:
        from ..parallel.sequence import apply_sequence_parallel

        apply_sequence_parallel(model, m.sp_group)
    if m.ep > 1 and base.cfg.is_moe:
        from ..parallel.expert import apply_expert_parallel

        apply_expert_parallel(model, m, capacity_factor=ctx.hw.get("ep_capacity_factor", 0.0),
                              chunks=ctx.hw.get("ep_chunks", 2))
    if base.cfg.is_moe and (ctx.cfg.get("model", {}) or {}).get("moe_fp8", False):
        for layer in base.layers:  # e4m3 expert GEMMs in the forward (bf16 backward)
            layer.mlp.fp8 = True
    trainable = any(p.requires_grad for p in model.parameters())
    if use_fsdp(ctx) and not trainable:
        # frozen reference / teachers are sharded too (C10): 1/dp of their weights resident
        from ..parallel.fsdp import ShardedInference

        ShardedInference(model, group=m.dp_group, min_num_params=ctx.hw.get("fsdp_min_num_params", 0))
    from ..models.materialize import has_meta_params, materialize

    if has_meta_params(model) and not (use_fsdp(ctx) and trainable):
        # memory-bounded construction (meta_init): this rank's TP / EP shards only, one parameter
        # at a time; a trainable FSDP model is materialised unit by unit by its engine instead
        materialize(model, ctx.device)
    return model


def meta_init(ctx: TrainContext) -> bool:
    """hardware.sharded_init: build models on the meta device and materialise only this rank's
    shards (auto: whenever tensor parallelism or ZeRO-3 / FSDP shards the weights)."""
    v = ctx.hw.get("sharded_init", "auto")
    if isinstance(v, str) and v.lower() == "auto":
        return (ctx.mesh is not None and ctx.mesh.tp > 1) or bool(use_fsdp(ctx))
    return bool(v)


def use_fsdp(ctx: TrainContext) -> bool:
    """ZeRO-3 / FSDP FULL_SHARD requested (hardware.zero_stage: 3, a DeepSpeed stage-3 JSON or an
    `fsdp` block) and there is more than one data-parallel rank to shard over."""
    z = ctx.hw.get("zero_stage")
    return (ctx.hw.get("fsdp") or (z is not None and int(z) >= 3)) and ctx.dp_size > 1


def make_engine(ctx: TrainContext, model, lr: float, betas=(0.9, 0.999), weight_decay: float = 0.0,
                max_grad_norm: float = 1.0):
    groups = dict(group=ctx.mesh.grad_group if ctx.mesh is not None else None,
                  tp_group=ctx.mesh.tp_group if ctx.mesh is not None else None)
    sp = ctx.mesh.sp if ctx.mesh is not None else 1
    if ctx.mesh is not None and ctx.mesh.ep > 1:
        groups["expert_group"] = ctx.mesh.edp_group
    if use_fsdp(ctx):
        if sp > 1:
            raise NotImplementedError("ZeRO-3 / FSDP with sequence parallel: use zero_stage <= 1")
        from ..parallel.fsdp import FullyShardedEngine

        return FullyShardedEngine(model, lr=lr, betas=betas, weight_decay=weight_decay,
                                  max_grad_norm=max_grad_norm, grad_dtype=grad_dtypes(ctx)[0],
                                  master_weights=ctx.hw.get("master_weights", True), sp_size=sp,
                                  min_num_params=ctx.hw.get("fsdp_min_num_params", 0),
                                  cpu_offload=ctx.hw.get("cpu_offload", False), **groups)
    if ctx.hw.get("cpu_offload"):
        raise ValueError("hardware.fsdp.offload_params / cpu_offload is not supported (weights and "
                         "optimizer state stay in 288 GB HBM); set it to false")
    from ..models.materialize import has_meta_params, materialize

    if has_meta_params(model):
        materialize(model, ctx.device)
    z = ctx.hw.get("zero_stage")
    gd, rd = grad_dtypes(ctx)
    return DataParallelEngine(model, lr=lr, betas=betas, weight_decay=weight_decay,
                              max_grad_norm=max_grad_norm, zero_stage=None if z is None else min(int(z), 1),
                              bucket_mb=ctx.hw.get("bucket_mb", 256.0),
                              master_weights=ctx.hw.get("master_weights", True), sp_size=sp,
                              grad_dtype=gd, reduce_dtype=rd, **groups)


_DTYPES = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16,
           "bfloat16": torch.bfloat16}


def grad_dtypes(ctx: TrainContext):
    """(grad accumulation dtype, reduce dtype) from hardware.grad_dtype / hardware.reduce_dtype.
    grad_dtype "auto" (default): fp32 main grads once gradient_accumulation_steps >= 16 (bf16
    accumulation of 16-256 micro-batch grads loses the small ones: config/dpo_hh.yaml uses 256),
    else the parameter dtype. reduce_dtype defaults to the grad dtype."""
    g = str(ctx.hw.get("grad_dtype", "auto")).lower()
    if g == "auto":
        gd = torch.float32 if int(ctx.hw.get("grad_accum", 1)) >= 16 else None
    elif g in _DTYPES:
        gd = _DTYPES[g]
    else:
        raise ValueError(f"hardware.grad_dtype must be auto / fp32 / bf16, got {g!r}")
    r = ctx.hw.get("reduce_dtype")
    if r is not None and str(r).lower() not in _DTYPES:
        raise ValueError(f"hardware.reduce_dtype must be fp32 / bf16, got {r!r}")
    return gd, (_DTYPES[str(r).lower()] if r is not None else None)


def effective_batch_msg(ctx: TrainContext, micro: int) -> str:
    eff = micro * ctx.dp_size * ctx.hw["grad_accum"]
    target = (ctx.cfg.get("optimization", {}) or {}).get("total_batch_size", eff)
    return f"Effective global batch size: {eff} (target {target})"


def move_to(batch, device):
    if isinstance(batch, torch.Tensor):
        return batch.to(device, non_blocking=True)
    if isinstance(batch, dict):
        return {k: move_to(v, device) for k, v in batch.items()}
    if isinstance(batch, (list, tuple)):
        return type(batch)(move_to(v, device) for v in batch)
    return batch


def _batch_rows(batch) -> int:
    """Samples in a micro-batch: pairs for preference batches, rows otherwise."""
    if isinstance(batch, torch.Tensor):
        return int(batch.shape[0]) if batch.dim() else 1
    if isinstance(batch, dict):
        for k in ("chosen", "input_ids"):
            if k in batch:
                return _batch_rows(batch[k])
        for v in batch.values():
            return _batch_rows(v)
    if isinstance(batch, (list, tuple)) and batch:
        return _batch_rows(batch[0])
    return 0


StepFn = Callable[[Any], Tuple[torch.Tensor, Dict[str, Any]]]


def _moe_dropped_slots(model) -> Optional[int]:
    """Token slots the capacity-bounded EP dispatch dropped since the last call (None: no EP)."""
    from ..parallel.expert import ExpertParallel

    seen, total = set(), None
    for m in model.modules():
        ep = getattr(m, "ep", None)
        if isinstance(ep, ExpertParallel) and id(ep) not in seen:
            seen.add(id(ep))
            total = (total or 0) + ep.dropped_slots()
    return total


def train_loop(ctx: TrainContext, loader, sampler, engine: DataParallelEngine, step_fn: StepFn,
               total_steps: int, models_to_save: List[Any], tokenizer=None,
               scheduler: Optional[LRSchedule] = None, log_every: int = 10, eval_every: int = 0,
               save_every: int = 0, eval_fn: Optional[Callable[[int], Dict[str, Any]]] = None,
               extra_log_fn: Optional[Callable[[int, Dict[str, Any]], Dict[str, Any]]] = None,
               resume: Optional[str] = None, keep_last: Optional[int] = None) -> int:
    accum = ctx.hw["grad_accum"]
    global_step = 0
    if resume:
        path = resolve_checkpoint(resume)
        if path is not None:
            global_step = load_state(path, models_to_save[:1], engine, scheduler)
            ctx.log(f"Resumed from {path} at step {global_step}")
    lg = ctx.cfg.get("logging", {}) or {}
    dbg = ctx.cfg.get("debug", {}) or {}
    prof = ProfileWindow(lg.get("profile_steps"), lg.get("profile_dir", str(Path(ctx.log_dir) / "profile")),
                         enabled=ctx.is_main or bool(lg.get("profile_all_ranks", False)))
    faults = FaultInjector(dbg.get("fault_at_step"), dbg.get("fault_rank"))
    sync_every = int(dbg.get("check_sync_every", 0) or 0)
    dp_group = ctx.mesh.grad_group if ctx.mesh is not None else None  # params replicated over it
    running = RunningLoss()
    last_metrics: Dict[str, Any] = {}
    done = global_step >= total_steps
    n_batches = len(loader)
    if n_batches == 0:
        raise RuntimeError("empty training dataset")
    # resume at the exact data position: epoch-seeded sampler order, skip consumed batches
    epoch, skip = divmod(global_step, n_batches)
    t_log, rows_log = time.perf_counter(), 0
    while not done:
        if sampler is not None:
            sampler.set_epoch(epoch)
        for bi, batch in enumerate(loader):
            if skip:
                skip -= 1
                continue
            prof.step(global_step + 1)
            faults.maybe_fail(global_step + 1, ctx.dist.rank)
            with trace_range("data"):
                batch = move_to(batch, ctx.device)
            rows_log += _batch_rows(batch)
            micro_idx = global_step % accum
            sync = (micro_idx == accum - 1) or (bi == n_batches - 1)
            ctx_mgr = contextlib.nullcontext() if sync else engine.no_sync()
            with ctx_mgr, trace_range("fwd_bwd"):
                loss, metrics = step_fn(batch)
                (loss / accum).backward()
            if sync:
                with trace_range("optim"):
                    lr = scheduler.lr(global_step) if scheduler is not None else None
                    engine.step(lr)
                if sync_every and (global_step + 1) // accum % sync_every == 0:
                    check_replicas_in_sync(models_to_save[0], dp_group)
            if scheduler is not None:
                scheduler.step()
            running.update(loss.detach())
            last_metrics = metrics
            global_step += 1
            if log_every and global_step % log_every == 0:
                from ..ops.embedding import check_ids

                # out-of-range token ids since the last log (sticky device word), on every rank
                check_ids(collective=True)
                rec = {"train/loss": running.average, "train/grad_norm": engine.last_grad_norm,
                       "train/comm_exposed_ms": engine.comm_timer.last_step_ms()}
                dropped = _moe_dropped_slots(models_to_save[0])
                if dropped is not None:
                    rec["moe/dropped_slots"] = dropped
                    if dropped:
                        ctx.log(f"WARNING: expert-parallel capacity dropped {dropped} token slots "
                                f"since the last log (hardware.ep_capacity_factor; 0 = dropless)")
                if scheduler is not None:
                    rec["train/lr"] = scheduler.lr(global_step)
                if extra_log_fn is not None:
                    rec.update(extra_log_fn(global_step, metrics))
                dt = time.perf_counter() - t_log
                rec["perf/samples_per_s"] = rows_log * ctx.dp_size / max(dt, 1e-9)
                rec["perf/step_s"] = dt / log_every
                if torch.cuda.is_available():
                    rec["perf/max_mem_gb"] = torch.cuda.max_memory_allocated() / 2 ** 30
                rec.update(PHASES.pop())
                ctx.logger.log(rec, global_step)
                running = RunningLoss()
                t_log, rows_log = time.perf_counter(), 0
            if eval_fn is not None and eval_every and global_step % eval_every == 0:
                with trace_range("eval"):
                    ctx.logger.log(eval_fn(global_step), global_step)
            if save_every and global_step % save_every == 0:
                with trace_range("save"):
                    save_state(Path(ctx.output_dir) / f"step_{global_step}", models_to_save, engine,
                               scheduler, global_step, tokenizer, keep_last=keep_last)
            if global_step >= total_steps:
                done = True
                break
        epoch += 1
    prof.close()
    save_state(Path(ctx.output_dir) / "final", models_to_save, engine, scheduler, global_step, tokenizer)
    return global_step
