"""Supervised fine-tuning entry point (reference: src/training/train_sft.py:45-174).

    python -m distributed_llm_alignment_amd.training.train_sft --config config/sft_config.yaml
    torchrun --nproc-per-node 8 -m distributed_llm_alignment_amd.training.train_sft --config ...

Same config keys and defaults as the reference: AdamW betas (0.9, 0.95), weight_decay default 0,
cosine schedule with warmup stepped per micro-batch, `train/loss` + `eval/loss` metrics, seed 42.
"""
from __future__ import annotations

import argparse
from typing import Dict

import torch

from ..data import build_dataloader, build_instruction_dataset
from ..models import count_trainable_params, load_causal_lm
from ..objectives import sft_loss
from ..optim.scheduler import LRSchedule
from ..parallel.dist import all_gather_tensor
from ..utils.config import add_config_args, config_from_args
from .common import meta_init, effective_batch_msg, make_engine, move_to, parallelize, setup, train_loop


def parse_args(argv=None) -> argparse.Namespace:
    return add_config_args(argparse.ArgumentParser(description="Distributed SFT training")).parse_args(argv)


@torch.no_grad()
def evaluate_loss(model, loader, device) -> float:
    """Mean eval loss, gathered across ranks (reference train_sft.py:33-42, C5)."""
    model.eval()
    losses = []
    for batch in loader:
        batch = move_to(batch, device)
        loss = sft_loss(model, batch).float()
        n = batch["input_ids"].shape[0]
        losses.append(all_gather_tensor(loss.reshape(1).repeat(n)).mean())
    model.train()
    if not losses:
        return float("nan")
    return float(torch.stack(losses).mean().item())


def main(argv=None) -> int:
    args = parse_args(argv)
    config = config_from_args(args)
    ctx = setup(config, "sft", default_seed=42)
    ctx.log(f"Loaded config from {args.config}")
    model_cfg: Dict = config["model"]
    bundle = load_causal_lm(model_cfg["model_name_or_path"],
                            gradient_checkpointing=model_cfg.get("gradient_checkpointing", True),
                            use_flash_attention=model_cfg.get("use_flash_attention", False),
                            device=ctx.device, seed=ctx.seed, meta_init=meta_init(ctx))
    model, tok = bundle.model, bundle.tokenizer
    parallelize(ctx, model)
    data_cfg = dict(config["data"])
    max_len = model_cfg.get("max_seq_length", 2048)
    opt = config["optimization"]
    micro = opt["micro_batch_size"]
    nw = data_cfg.get("num_workers", 4)
    train_ds = build_instruction_dataset(data_cfg | {"max_seq_length": max_len}, tok, split="train")
    loader, sampler = build_dataloader(train_ds, micro, shuffle=True, num_workers=nw, seed=ctx.seed)
    eval_loader = None
    if data_cfg.get("eval_path") or data_cfg.get("eval_split"):
        eval_ds = build_instruction_dataset(data_cfg | {"max_seq_length": max_len}, tok, split="eval")
        eval_loader, _ = build_dataloader(eval_ds, micro, shuffle=False, num_workers=nw, seed=ctx.seed)

    engine = make_engine(ctx, model, lr=opt["learning_rate"], betas=(0.9, 0.95),
                         weight_decay=opt.get("weight_decay", 0.0),
                         max_grad_norm=opt.get("max_grad_norm", 1.0))
    total = opt["max_train_steps"]
    sched = LRSchedule(opt["learning_rate"], opt.get("lr_scheduler", "cosine"),
                       opt.get("warmup_steps", 0), total)
    lg = config["logging"]
    ctx.log(f"Trainable parameters: {count_trainable_params(model)}")
    ctx.log(effective_batch_msg(ctx, micro))
    model.train()
    train_loop(ctx, loader, sampler, engine, lambda b: (sft_loss(model, b), {}), total, [model], tok,
               scheduler=sched, log_every=lg.get("log_every_steps", 20),
               eval_every=lg.get("eval_every_steps", 200) if eval_loader is not None else 0,
               save_every=lg.get("save_every_steps", 500),
               eval_fn=(lambda s: {"eval/loss": evaluate_loss(model, eval_loader, ctx.device)})
               if eval_loader is not None else None,
               resume=args.resume, keep_last=lg.get("keep_last"))
    ctx.log("Training complete")
    ctx.logger.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
