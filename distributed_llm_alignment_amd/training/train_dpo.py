"""Direct Preference Optimization (reference: src/training/train_dpo.py:47-143).

    torchrun --nproc-per-node 8 -m distributed_llm_alignment_amd.training.train_dpo --config config/dpo_config.yaml

Reference semantics kept: length-normalised sequence log-probs over ALL tokens (prompt included,
Appendix A #11), `dpo_loss = -logsigmoid(beta*((pc-pr)-(rc-rr))).mean()`, beta from
`model.beta` (0.1), AdamW default betas with weight_decay 0.01 (hard-coded in the reference), no LR
scheduler (set `optimization.apply_scheduler: true` to use lr_scheduler/warmup_steps),
`train/loss` and `train/preference_rate` metrics, checkpoints contain policy (model.safetensors)
then ref (model_1.safetensors). Options beyond the reference: `model.logprob_reduction: sum`,
`data.mask_prompt: true` (score response tokens only), `model.label_smoothing` (cDPO),
`model.reference_fp8: true` (the frozen reference's layer GEMMs on e4m3 weights and activations
with row scales, hipBLASLt fp8: ops.linear.enable_fp8_inference).

The frozen reference model is co-resident on every GPU (bf16, no grad); chosen and rejected
sequences run as one [2B, T] batch per forward.
"""
from __future__ import annotations

import argparse
from typing import Dict

import torch

from ..data import build_dataloader, build_preference_dataset
from ..models import load_causal_lm
from ..objectives import dpo_step_loss
from ..optim.scheduler import LRSchedule
from ..utils.config import add_config_args, config_from_args
from .common import meta_init, effective_batch_msg, make_engine, parallelize, setup, train_loop


def parse_args(argv=None) -> argparse.Namespace:
    return add_config_args(argparse.ArgumentParser(description="DPO training")).parse_args(argv)


def main(argv=None) -> int:
    args = parse_args(argv)
    config = config_from_args(args)
    ctx = setup(config, "dpo", default_seed=0)
    model_cfg: Dict = config["model"]
    policy = load_causal_lm(model_cfg["policy_model_name_or_path"],
                            gradient_checkpointing=model_cfg.get("gradient_checkpointing", True),
                            device=ctx.device, seed=ctx.seed, meta_init=meta_init(ctx))
    ref = load_causal_lm(model_cfg["reference_model_name_or_path"], gradient_checkpointing=False,
                         device=ctx.device, seed=ctx.seed, meta_init=meta_init(ctx))
    ref.model.eval()
    ref.model.requires_grad_(False)
    if model_cfg.get("reference_fp8", False):  # frozen reference on the fp8 inference GEMMs (opt-in)
        from ..ops import enable_fp8_inference

        enable_fp8_inference(ref.model)
    parallelize(ctx, policy.model)
    parallelize(ctx, ref.model)
    tok = policy.tokenizer
    data_cfg = dict(config["data"])
    data_cfg["preference_path"] = data_cfg.get("preference_path")
    ds = build_preference_dataset(data_cfg | {"max_seq_length": model_cfg.get("max_seq_length", 1024)},
                                  tok, split="train")
    opt = config["optimization"]
    micro = opt["micro_batch_size"]
    loader, sampler = build_dataloader(ds, micro, shuffle=True, num_workers=data_cfg.get("num_workers", 4),
                                       seed=ctx.seed)
    engine = make_engine(ctx, policy.model, lr=opt["learning_rate"],
                         weight_decay=opt.get("weight_decay", 0.01) if opt.get("honor_weight_decay") else 0.01,
                         max_grad_norm=opt.get("max_grad_norm", 1.0))
    sched = None
    if opt.get("apply_scheduler"):
        sched = LRSchedule(opt["learning_rate"], opt.get("lr_scheduler", "cosine"),
                           opt.get("warmup_steps", 0), opt["max_train_steps"])
    beta = model_cfg.get("beta", 0.1)
    ls = model_cfg.get("label_smoothing", 0.0) or 0.0
    reduction = model_cfg.get("logprob_reduction", "mean")
    pad_id = tok.pad_token_id or 0
    lg = config["logging"]
    eval_every = lg.get("eval_every_steps", 100)
    ctx.log(effective_batch_msg(ctx, micro))
    policy.model.train()

    def step_fn(batch):
        return dpo_step_loss(policy.model, ref.model, batch, beta=beta, label_smoothing=ls,
                             reduction=reduction, pad_id=pad_id)

    def extra(step, m):
        out = {"train/reward_accuracy": m["rewards/accuracy"], "train/reward_margin": m["rewards/margin"]}
        if eval_every and step % eval_every == 0:
            out["train/preference_rate"] = (m["policy_chosen_logps"] > m["policy_rejected_logps"]).float().mean()
        return out

    train_loop(ctx, loader, sampler, engine, step_fn, opt["max_train_steps"], [policy.model, ref.model],
               tok, scheduler=sched, log_every=lg.get("log_every_steps", 10), save_every=lg.get("save_every_steps", 200),
               extra_log_fn=extra, resume=args.resume, keep_last=lg.get("keep_last"))
    ctx.log("DPO training complete")
    ctx.logger.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
