"""Pairwise reward-model training (reference: src/training/train_reward.py:57-174).

Bradley-Terry loss `-logsigmoid(s_c - s_r).mean()` on a native backbone + Dropout/Linear head,
`eval/loss` and `eval/acc` metrics, AdamW (default betas, weight_decay from config, default 0)."""
from __future__ import annotations

import argparse
from typing import Dict

import torch

from ..data import build_dataloader, build_preference_dataset
from ..models import build_reward_model
from ..objectives import reward_loss
from ..parallel.dist import all_gather_tensor
from ..utils.config import add_config_args, config_from_args
from .common import effective_batch_msg, make_engine, move_to, parallelize, setup, train_loop


def parse_args(argv=None) -> argparse.Namespace:
    return add_config_args(argparse.ArgumentParser(description="Train reward model")).parse_args(argv)


@torch.no_grad()
def evaluate(model, loader, device, pad_id: int = 0) -> Dict[str, float]:
    model.eval()
    correct = total = 0
    losses = []
    for batch in loader:
        batch = move_to(batch, device)
        loss, m = reward_loss(model, batch, pad_id)
        losses.append(all_gather_tensor(loss.float().reshape(1)).mean())
        c = (m["chosen_scores"] > m["rejected_scores"]).float()
        correct += float(all_gather_tensor(c).sum().item())
        total += int(all_gather_tensor(c).numel())
    model.train()
    return {"loss": float(torch.stack(losses).mean().item()) if losses else float("nan"),
            "accuracy": correct / max(total, 1)}


def main(argv=None) -> int:
    args = parse_args(argv)
    config = config_from_args(args)
    ctx = setup(config, "reward", default_seed=0)
    model_cfg: Dict = config["model"]
    rm, tok = build_reward_model(model_cfg["base_model_name_or_path"],
                                 pooling=model_cfg.get("pooling", "last_token"),
                                 dropout=model_cfg.get("dropout", 0.1), device=ctx.device, seed=ctx.seed)
    if model_cfg.get("gradient_checkpointing", False):
        rm.backbone.gradient_checkpointing_enable()
    parallelize(ctx, rm)
    data_cfg = dict(config["data"])
    max_len = model_cfg.get("max_seq_length", 1024)
    opt = config["optimization"]
    micro = opt["micro_batch_size"]
    nw = data_cfg.get("num_workers", 4)
    ds = build_preference_dataset(data_cfg | {"max_seq_length": max_len}, tok, split="train")
    loader, sampler = build_dataloader(ds, micro, shuffle=True, num_workers=nw, seed=ctx.seed)
    eval_loader = None
    if data_cfg.get("eval_path") or data_cfg.get("eval_split"):
        eds = build_preference_dataset(data_cfg | {"max_seq_length": max_len}, tok, split="eval")
        eval_loader, _ = build_dataloader(eds, micro, shuffle=False, num_workers=nw, seed=ctx.seed)
    engine = make_engine(ctx, rm, lr=opt["learning_rate"], weight_decay=opt.get("weight_decay", 0.0),
                         max_grad_norm=opt.get("max_grad_norm", 1.0))
    pad_id = tok.pad_token_id or 0
    lg = config["logging"]
    ctx.log(effective_batch_msg(ctx, micro))
    rm.train()

    def eval_fn(step):
        m = evaluate(rm, eval_loader, ctx.device, pad_id)
        return {"eval/loss": m["loss"], "eval/acc": m["accuracy"]}

    train_loop(ctx, loader, sampler, engine, lambda b: reward_loss(rm, b, pad_id), opt["max_train_steps"],
               [rm], tok, log_every=lg.get("log_every_steps", 10),
               eval_every=lg.get("eval_every_steps", 100) if eval_loader is not None else 0,
               save_every=lg.get("save_every_steps", 200),
               eval_fn=eval_fn if eval_loader is not None else None,
               extra_log_fn=lambda s, m: {"train/accuracy": m["accuracy"]},
               resume=args.resume, keep_last=lg.get("keep_last"))
    ctx.log("Finished reward training")
    ctx.logger.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
