"""Distillation (reference: src/training/train_distill.py:32-175).

`distill.use_kl and distill.on_policy` with teachers -> token-masked ensemble forward KL
KL(mean_k softmax(teacher_k) || softmax(student)) over every (unshifted) position, fused in one
HIP row kernel (fwd + in-place grad, no [K, B, T, V] fp32 tensors); otherwise causal-LM CE on
the teacher rollouts. Teachers are frozen (Appendix A #15) and must share the student's
vocabulary. Metrics: `train/loss`, `train/reward_mean`. Checkpoint: student, then teachers."""
from __future__ import annotations

import argparse
from typing import Dict, List

import torch

from ..data import TeacherRolloutDataset, build_dataloader
from ..models import load_causal_lm
from ..objectives import distill_loss
from ..utils.config import add_config_args, config_from_args
from .common import meta_init, effective_batch_msg, make_engine, parallelize, setup, train_loop


def parse_args(argv=None) -> argparse.Namespace:
    return add_config_args(argparse.ArgumentParser(description="Distill aligned teacher into student")).parse_args(argv)


def main(argv=None) -> int:
    args = parse_args(argv)
    config = config_from_args(args)
    ctx = setup(config, "distill", default_seed=0)
    model_cfg: Dict = config["model"]
    dcfg: Dict = config.get("distill", {}) or {}
    student = load_causal_lm(model_cfg["student_model_name_or_path"],
                             gradient_checkpointing=model_cfg.get("gradient_checkpointing", True),
                             device=ctx.device, seed=ctx.seed, meta_init=meta_init(ctx))
    use_kl = bool(dcfg.get("use_kl", False) and dcfg.get("on_policy", False))
    teachers: List = []
    if use_kl:
        paths = dcfg.get("teacher_model_names_or_paths") or []
        if not paths:
            single = dcfg.get("teacher_model_name_or_path") or model_cfg.get("teacher_path")
            paths = [single] if single else []
        if not paths:
            raise ValueError("KL distillation requested but no teacher model path provided")
        for i, tp in enumerate(paths):
            tb = load_causal_lm(tp, gradient_checkpointing=False, device=ctx.device, seed=ctx.seed + 1 + i,
                                 meta_init=meta_init(ctx))
            tb.model.eval().requires_grad_(False)
            teachers.append(tb.model)
    parallelize(ctx, student.model)
    for t in teachers:
        parallelize(ctx, t)
    tok = student.tokenizer
    ds = TeacherRolloutDataset(config["data"]["teacher_samples_path"], tok,
                               max_length=model_cfg.get("max_seq_length", 2048))
    opt = config["optimization"]
    micro = opt["micro_batch_size"]
    loader, sampler = build_dataloader(ds, micro, shuffle=True,
                                       num_workers=config["data"].get("num_workers", 4), seed=ctx.seed)
    engine = make_engine(ctx, student.model, lr=opt["learning_rate"],
                         weight_decay=opt.get("weight_decay", 0.0), max_grad_norm=opt.get("max_grad_norm", 1.0))
    lg = config["logging"]
    ctx.log(effective_batch_msg(ctx, micro))
    student.model.train()

    def step_fn(batch):
        reward = batch.pop("reward")
        loss = distill_loss(student.model, teachers, batch, use_kl)
        return loss, {"reward": reward}

    train_loop(ctx, loader, sampler, engine, step_fn, opt["max_train_steps"], [student.model] + teachers, tok,
               log_every=lg.get("log_every_steps", 20), save_every=lg.get("save_every_steps", 400),
               extra_log_fn=lambda s, m: {"train/reward_mean": m["reward"].float().mean()},
               resume=args.resume, keep_last=lg.get("keep_last"))
    ctx.log("Distillation complete")
    ctx.logger.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
