"""KL-penalised policy-gradient RLHF ("PPO-style"; reference: src/training/train_rlhf.py:61-166).

Per step: sample `ppo.batch_size` prompts (same seed on every rank), take this rank's contiguous
slice (fixes Appendix A #1), left-pad and generate with the native KV-cache decoder (HIP flash
attention over the cache), score `prompt\\n\\nresponse` with the reward model (eval mode, no grad:
fixes #8), then REINFORCE with a KL-shaped reward and a mean baseline:
    kl = logp_pi - logp_ref ;  r' = r - kl_coef*kl ;  A = r' - mean(r') ;  loss = -mean(A * logp_pi)
(fused HIP kernel). The log-prob mask covers prompt + generated tokens up to and including EOS
(fixes #10). `generation_params.do_sample` defaults to True (#9). `ppo.update_micro_batch: m`
runs the update as gradient-accumulated micro-batches of m rollouts with a baseline each, the
per-process semantics of the reference's multi-process run (`reinforce_update`).

Overlap (BASELINE north star, `ppo.async_rollouts: true`, off by default since it changes the
semantics to one-step-stale rollouts): step k+1's rollouts are generated while step k's gradient
reduce-scatter is still in flight on RCCL's stream. `train/comm_exposed_ms` logs the part of the
gradient collectives the step did not hide (the compute stream's wait at `engine.step`;
parallel/dist.py ExposedCommTimer); tests/test_distributed_cpu.py measures it with 2 gloo ranks.

`ppo.algorithm: ppo` (not in the reference, whose loop is critic-free) switches to token-level
actor-critic PPO, the north-star "PPO RLHF (actor + critic + reward)" configuration: a critic
(`ValueModel`, initialised from `critic.base_model_name_or_path` or the reward backbone) gives
per-token values, the per-token reward is -kl_coef * (logp - logp_ref) plus the reward-model
score on the last generated token, advantages are GAE(gamma, lam) (HIP wave-scan kernel),
whitened; `ppo_epochs` x `num_minibatches` updates of the clipped surrogate + `vf_coef` x the
clipped value loss (fused HIP fwd+bwd kernels), policy and critic each on their own engine.
"""
from __future__ import annotations

import argparse
import contextlib
import random
from pathlib import Path
from typing import Dict, List

import torch

from ..data import read_jsonl
from ..models import (build_reward_model, build_value_model, generate, load_causal_lm,
                      load_reward_checkpoint)
from ..objectives import ppo_backward, ppo_loss, ppo_rollout_stats, rlhf_loss
from ..parallel.dist import barrier, split_for_rank
from ..utils.checkpoint import save_state
from ..utils.config import add_config_args, config_from_args
from ..utils.logging import RunningLoss
from .common import make_engine, parallelize, setup


def parse_args(argv=None) -> argparse.Namespace:
    return add_config_args(argparse.ArgumentParser(description="RLHF PPO loop")).parse_args(argv)


def load_prompts(cfg: Dict[str, str]) -> List[str]:
    source = cfg.get("source", "local")
    if source == "hf":
        try:
            from datasets import load_dataset

            ds = load_dataset(cfg["hf_path"], cfg.get("hf_name"), split=cfg.get("split", "train"))
            key = cfg.get("prompt_key", "prompt")
            return [row[key] for row in ds if row.get(key)]
        except Exception:
            if not (cfg.get("prompt_path") or cfg.get("path")):
                raise
    if source == "synthetic":
        from ..data.synthetic import synthetic_prompt_records

        return [r["prompt"] for r in synthetic_prompt_records(int(cfg.get("num_samples", 256)))]
    path = cfg.get("prompt_path") or cfg.get("path")
    return [r["prompt"] for r in read_jsonl(path) if r.get("prompt")]


def _tokenize_left(tok, texts, max_len, device):
    side = getattr(tok, "padding_side", "right")
    tok.padding_side = "left"
    enc = tok(texts, return_tensors="pt", padding=True, truncation=True, max_length=max_len)
    tok.padding_side = side
    return enc["input_ids"].to(device), enc["attention_mask"].to(device)


def main(argv=None) -> int:
    args = parse_args(argv)
    config = config_from_args(args)
    ctx = setup(config, "rlhf", default_seed=0)
    model_cfg: Dict = config["model"]
    ppo = config["ppo"]
    policy = load_causal_lm(model_cfg["policy_model_name_or_path"],
                            gradient_checkpointing=model_cfg.get("gradient_checkpointing", True),
                            device=ctx.device, seed=ctx.seed)
    ref = load_causal_lm(model_cfg["reference_model_name_or_path"], gradient_checkpointing=False,
                         device=ctx.device, seed=ctx.seed)
    ref.model.eval().requires_grad_(False)
    rcfg = config.get("reward_model", {}) or {}
    rbase = rcfg.get("base_model_name_or_path", model_cfg["policy_model_name_or_path"])
    rpath = rcfg.get("path")
    if rpath and Path(rpath).is_dir() and (Path(rpath) / "config.json").exists() and "base_model_name_or_path" not in rcfg:
        rbase = rpath
    rm, rtok = build_reward_model(rbase, pooling="last_token", dropout=0.1, device=ctx.device, seed=ctx.seed)
    if rpath and Path(rpath).exists():
        ctx.log(f"Loaded reward weights from {load_reward_checkpoint(rm, rpath)}")
    rm.eval().requires_grad_(False)
    if ppo.get("frozen_fp8", False):  # reference + reward model on the fp8 inference GEMMs (opt-in)
        from ..ops import enable_fp8_inference

        enable_fp8_inference(ref.model)
        enable_fp8_inference(rm.backbone)
    for m in (policy.model, ref.model, rm):
        parallelize(ctx, m)

    prompts = load_prompts(config["sampling"])
    gen = dict(ppo.get("generation_params", {"max_new_tokens": 256}))
    gen.setdefault("do_sample", True)
    engine = make_engine(ctx, policy.model, lr=ppo.get("learning_rate", 1e-6), betas=(0.9, 0.95),
                         weight_decay=ppo.get("weight_decay", 0.01),
                         max_grad_norm=ppo.get("max_grad_norm", 1.0))
    steps = ppo.get("steps", 1024)
    batch_size = ppo.get("batch_size", 64)
    kl_coef = ppo.get("kl_coef", 0.1)
    max_len = model_cfg.get("max_seq_length", 1024)
    tok = policy.tokenizer
    rng = random.Random(ctx.seed)
    gen_g = torch.Generator(device=ctx.device)
    gen_g.manual_seed(ctx.seed * 1000 + (ctx.mesh.dp_rank if ctx.mesh is not None else ctx.dist.rank))
    running = RunningLoss()
    log_every = (config.get("logging", {}) or {}).get("log_every_steps", 10)
    algo = str(ppo.get("algorithm", "reinforce")).lower()
    if algo not in ("reinforce", "ppo"):
        raise ValueError(f"ppo.algorithm must be reinforce|ppo, got {algo!r}")

    # reward inputs built on the device when the reward tokenizer equals the policy's (no
    # decode / re-tokenise round trip through the host; training/handoff.py), else the
    # reference's text path (src/training/train_rlhf.py:131-147)
    from .handoff import RewardHandoff

    handoff = RewardHandoff(tok, rtok, policy.model.cfg.vocab_size, ctx.device, max_len,
                            ppo.get("reward_handoff", "auto"),
                            validate_every=int(ppo.get("reward_handoff_validate_every", 16)))
    ctx.log(f"reward hand-off: {'device ids' if handoff.device_path else 'decode + re-tokenise'}")

    def rollout():
        batch_prompts = rng.sample(prompts, k=min(batch_size, len(prompts)))
        mine = split_for_rank(batch_prompts)
        ids, am = _tokenize_left(tok, mine, max_len, ctx.device)
        seqs, mask = generate(policy.model, ids, am, max_new_tokens=gen.get("max_new_tokens", 256),
                              do_sample=gen["do_sample"], temperature=gen.get("temperature", 1.0),
                              top_p=gen.get("top_p", 1.0), top_k=gen.get("top_k", 0),
                              pad_token_id=tok.pad_token_id, eos_token_id=getattr(tok, "eos_token_id", None),
                              generator=gen_g, return_mask=True,
                              weight_dtype=ppo.get("rollout_weight_dtype", "bf16"))
        r_ids, r_mask = handoff(mine, ids, am, seqs, mask)
        with torch.no_grad():
            scores = rm(r_ids, r_mask)
        return seqs, mask, scores, ids.shape[1]

    policy.model.train()
    if algo == "ppo":
        return _ppo_loop(ctx, config, ppo, policy, ref, rm, rollout, engine, steps, kl_coef, log_every)
    micro = int(ppo.get("update_micro_batch", 0) or 0)
    pending = rollout()
    for step in range(steps):
        seqs, mask, scores, _ = pending
        loss, m = reinforce_update(policy.model, ref.model, engine, seqs, mask, scores, kl_coef, micro)
        if ppo.get("async_rollouts", False) and step + 1 < steps:
            # the bucketed reduce-scatter launched by the backward hooks is in flight on RCCL's
            # stream; generating the next rollouts (pre-update weights) overlaps it
            pending = rollout()
            engine.step()
        else:
            engine.step()
            if step + 1 < steps:
                pending = rollout()
        running.update(loss.detach())
        if (step + 1) % log_every == 0:
            ctx.logger.log({"train/loss": running.average, "train/kl": m["kl"],
                            "train/reward_mean": scores.mean(), "train/grad_norm": engine.last_grad_norm,
                            "train/comm_exposed_ms": engine.comm_timer.last_step_ms()},
                           step + 1)
            running = RunningLoss()
    barrier()
    save_state(config["logging"]["output_dir"], [policy.model, ref.model, rm], engine, None, steps, tok)
    ctx.log("RLHF PPO loop complete")
    ctx.logger.close()
    return 0


def micro_bounds(n: int, micro: int):
    """[start, stop) of each update micro-batch. A ragged tail (n % micro != 0) is folded into the
    previous micro-batch instead of standing alone: a 1-rollout micro-batch's mean baseline is its
    own reward, so its advantage (and policy gradient) would be exactly zero while it still
    carried weight."""
    b = [(s, min(n, s + micro)) for s in range(0, n, micro)]
    if len(b) > 1 and b[-1][1] - b[-1][0] < micro:
        b[-2:] = [(b[-2][0], n)]
    return b


def reinforce_update(policy, ref, engine, seqs, mask, scores, kl_coef: float, micro: int = 0):
    """Backward of the KL-penalised policy-gradient loss over this rank's rollouts.

    micro > 0 (`ppo.update_micro_batch`): gradient-accumulated micro-batches of `micro` rollouts,
    each with its own mean baseline and weighted by its share of the rollouts -- the gradient of
    a job with that many rollouts per process (the reference splits `ppo.batch_size` across
    processes and takes `rewards.mean()` per process, src/training/train_rlhf.py:114,151, then
    DDP averages), and no activation recompute is needed for a large one-GPU batch.
    Returns (loss, metrics) like `rlhf_loss`."""
    n = seqs.shape[0]
    if micro <= 0 or micro >= n:
        loss, m = rlhf_loss(policy, ref, seqs, mask, scores, kl_coef)
        loss.backward()
        return loss, m
    bounds = micro_bounds(n, micro)
    tot, kl = 0.0, 0.0
    for i, (s0, s1) in enumerate(bounds):
        sl = slice(s0, s1)
        w = (sl.stop - sl.start) / n
        ctx = engine.no_sync() if i < len(bounds) - 1 else contextlib.nullcontext()
        with ctx:
            loss, m = rlhf_loss(policy, ref, seqs[sl], mask[sl], scores[sl], kl_coef)
            (loss * w).backward()
        tot = tot + loss.detach() * w
        kl = kl + m["kl"] * w
    return tot, {"kl": kl}


def _ppo_loop(ctx, config, ppo, policy, ref, rm, rollout, engine, steps, kl_coef, log_every) -> int:
    """Token-level actor-critic PPO (`ppo.algorithm: ppo`)."""
    model_cfg = config["model"]
    ccfg = config.get("critic", {}) or {}
    rcfg = config.get("reward_model", {}) or {}
    cbase = ccfg.get("base_model_name_or_path") or rcfg.get("base_model_name_or_path") \
        or model_cfg["policy_model_name_or_path"]
    critic, _ = build_value_model(cbase, device=ctx.device, seed=ctx.seed + 1,
                                  gradient_checkpointing=ccfg.get("gradient_checkpointing",
                                                                  model_cfg.get("gradient_checkpointing", True)))
    parallelize(ctx, critic)
    critic.train()
    critic_engine = make_engine(ctx, critic, lr=ccfg.get("learning_rate", ppo.get("learning_rate", 1e-6)),
                                betas=(0.9, 0.95), weight_decay=ppo.get("weight_decay", 0.01),
                                max_grad_norm=ppo.get("max_grad_norm", 1.0))
    gamma, lam = float(ppo.get("gamma", 1.0)), float(ppo.get("lam", 0.95))
    clip, vclip = float(ppo.get("clip_range", 0.2)), float(ppo.get("value_clip_range", 0.2))
    vf_coef = float(ppo.get("vf_coef", 0.1))
    epochs, nmb = int(ppo.get("ppo_epochs", 1)), max(1, int(ppo.get("num_minibatches", 1)))
    overlap = bool(ppo.get("async_rollouts", False))
    running = RunningLoss()
    pending = rollout()
    for step in range(steps):
        seqs, mask, scores, tp = pending
        stats = ppo_rollout_stats(policy.model, ref.model, critic, seqs, mask, tp, scores, kl_coef,
                                  gamma, lam)
        S = seqs.shape[0]
        bounds = [(i * S // nmb, (i + 1) * S // nmb) for i in range(nmb)]
        for ep in range(epochs):
            for mi, (a, b) in enumerate(bounds):
                if b <= a:
                    continue
                mb = {k: v[a:b] for k, v in stats.items() if k in ("old_logp", "values", "advantages", "returns", "act")}
                loss, m = ppo_loss(policy.model, critic, seqs[a:b], mask[a:b], mb, clip, vclip, vf_coef)
                ppo_backward(loss)
                last = ep == epochs - 1 and mi == len(bounds) - 1
                if last and overlap and step + 1 < steps:
                    # overlaps the in-flight ZeRO-0/1 bucket collectives (they are waited on in
                    # step()); an FSDP engine has already drained its reduce-scatters in its
                    # end-of-backward callback, so there the rollout only runs ahead of step()
                    pending = rollout()
                engine.step()
                critic_engine.step()
                running.update(loss.detach())
        if not overlap and step + 1 < steps:
            pending = rollout()
        if (step + 1) % log_every == 0:
            ctx.logger.log({"train/loss": running.average, "train/kl": stats["kl"].mean(),
                            "train/reward_mean": stats["scores"].mean(),
                            "train/policy_loss": m["policy_loss"], "train/value_loss": m["value_loss"],
                            "train/clipfrac": m["clipfrac"], "train/approx_kl": m["approx_kl"],
                            "train/grad_norm": engine.last_grad_norm,
                            "train/comm_exposed_ms": engine.comm_timer.last_step_ms()}, step + 1)
            running = RunningLoss()
    barrier()
    out = save_state(config["logging"]["output_dir"], [policy.model, ref.model, rm, critic], engine, None,
                     steps, policy.tokenizer)
    from ..utils.stream_st import save_streamed

    cst = critic_engine.optimizer_state()
    save_streamed(Path(out) / f"critic_optimizer_shard_{ctx.dist.rank}.safetensors",
                  {k: v for k, v in cst.items() if isinstance(v, torch.Tensor) or v is None},
                  {k: (list(v) if isinstance(v, tuple) else v) for k, v in cst.items()
                   if not (isinstance(v, torch.Tensor) or v is None)})
    ctx.log("RLHF PPO (actor-critic) loop complete")
    ctx.logger.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
