#!/usr/bin/env python
"""One-GPU RLHF step throughput for the BASELINE "Llama-3-8B PPO-style RLHF" config: per step,
generate B rollouts (prompt T_p, up to N new tokens, hipGraph decode + fused sampler), score
them with a Llama-3-8B-backbone reward model, compute policy / reference sequence log-probs and
the KL-penalised policy-gradient loss (fused HIP kernel), backward and fused AdamW. Random init,
synthetic prompts. Prints one JSON line (rollouts/s and the phase split).

--overlap: one-step-stale rollouts (`ppo.async_rollouts`) overlapped on ONE GPU. A snapshot copy of
the policy generates and scores step k+1's rollouts on a side stream, from a helper thread, while
the main thread trains on step k's. Generation is bound by HBM bandwidth (B=8 weight streaming)
and the update by MFMA, so the two share the chip. The snapshot is refreshed from the policy
after each update: rollouts come from the weights one update behind.

--algorithm ppo: BASELINE config 3 as specified, token-level actor-critic PPO (`ppo.algorithm: ppo`,
config/rlhf_ppo_llama3_8b.yaml): policy + frozen reference + reward model + critic (a Llama-3-8B
backbone with a value head), each step generate -> score -> stats (policy / reference log-probs
and critic values, GAE) -> `--ppo-epochs` x `--minibatches` clipped-surrogate + value updates on
two engines. `--zero-shape N` lays both engines out as rank 0 of an N-rank ZeRO-1 job (fp32 master
and moments for 1/N of each model, no collectives), so the memory and per-rank work are those of
one GPU of the N-GPU node (reference: config/rlhf_config.yaml:13 batch 64 over 8 processes = 8
rollouts per rank). Prints the phase split and a per-rank memory plan."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--handoff", choices=("device", "text", "none"), default="device",
                    help="reward inputs: device-built ids (training/handoff.py), the reference's "
                         "decode + re-tokenise text path (byte tokenizer), or the raw sequences")
    ap.add_argument("--overlap", action="store_true",
                    help="generate step k+1's rollouts (policy snapshot, side stream) during step k's update")
    ap.add_argument("--grad-ckpt", default="", help="policy activation recompute: full|mlp|attention "
                    "(the reference's rlhf_config batch of 64 rollouts on one GPU needs mlp)")
    ap.add_argument("--micro", type=int, default=0,
                    help="reinforce: run the policy update as batch/micro gradient-accumulated "
                         "micro-batches, each with its own advantage baseline -- one rank's share of "
                         "a batch/micro-rank DDP job (the reference splits the batch across processes "
                         "and takes rewards.mean() per process), so no activation recompute is needed")
    ap.add_argument("--algorithm", choices=("reinforce", "ppo"), default="reinforce")
    ap.add_argument("--rollout-dtype", choices=("bf16", "fp8"), default="bf16",
                    help="decode weight streams of the rollout generation (ppo.rollout_weight_dtype)")
    ap.add_argument("--frozen-fp8", action="store_true",
                    help="reference + reward model layer GEMMs on fp8 (ppo.frozen_fp8, ops.enable_fp8_inference)")
    ap.add_argument("--force-pg", action="store_true",
                    help="reinforce: a real one-rank RCCL group and the policy engine's N-GPU path on it "
                         "(bucket all-reduces on RCCL's stream during the update's backward), so "
                         "--overlap runs generation beside real collectives")
    ap.add_argument("--zero-shape", type=int, default=1,
                    help="engines laid out as rank 0 of an N-rank ZeRO-1 job (1/N optimizer state)")
    ap.add_argument("--ppo-epochs", type=int, default=2)
    ap.add_argument("--minibatches", type=int, default=2)
    a = ap.parse_args()
    a.overlap = a.overlap or os.environ.get("DLA_BENCH_RLHF_OVERLAP") == "1"  # (A/B arms by env)
    if a.micro and a.batch % a.micro:
        ap.error("--batch must be a multiple of --micro")
    if a.micro and (a.overlap or a.algorithm == "ppo"):
        ap.error("--micro applies to the synchronous reinforce update only")
    if a.algorithm == "ppo":
        return ppo_main(a)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from distributed_llm_alignment_amd.models import build_model, generate, get_config
    from distributed_llm_alignment_amd.models.reward import RewardModel
    from distributed_llm_alignment_amd.objectives import rlhf_loss
    from distributed_llm_alignment_amd.ops import _ext
    from distributed_llm_alignment_amd.training.train_rlhf import reinforce_update
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine
    from distributed_llm_alignment_amd.utils.tuning import enable_gemm_tuning

    dev = torch.device("cuda", 0)
    _ext.require()
    enable_gemm_tuning(0)
    if a.force_pg:
        from distributed_llm_alignment_amd.parallel.dist import init_distributed

        torch.cuda.set_device(dev)
        init_distributed(force_pg=True)
    cfg = get_config(a.model)
    pol = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=1)
    ref = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=1).requires_grad_(False).eval()
    rm = RewardModel(build_model(cfg, device=dev, dtype=torch.bfloat16, seed=2, headless=True)).to(dev, torch.bfloat16)
    if a.frozen_fp8:
        from distributed_llm_alignment_amd.ops import enable_fp8_inference

        enable_fp8_inference(ref)
        enable_fp8_inference(rm.backbone)
    rm.eval().requires_grad_(False)
    if a.grad_ckpt:
        pol.gradient_checkpointing_enable(a.grad_ckpt)
    eng = DataParallelEngine(pol, lr=1e-6, betas=(0.9, 0.95), weight_decay=0.01, max_grad_norm=1.0,
                             # (DLA_BENCH_ENGINE_PLAIN=1: the process group exists, the engine
                             # runs the one-rank path; isolates the group from the engine path)
                             force_comm=a.force_pg and os.environ.get("DLA_BENCH_ENGINE_PLAIN") != "1")
    g = torch.Generator(device=dev).manual_seed(0)
    from distributed_llm_alignment_amd.models.tokenizer import ByteTokenizer
    from distributed_llm_alignment_amd.training.handoff import RewardHandoff

    tok = ByteTokenizer(vocab_size=cfg.vocab_size)
    handoff = RewardHandoff(tok, tok, cfg.vocab_size, dev, a.prompt + a.new + 8,
                            "text" if a.handoff == "text" else "device")
    prompts = ["synthetic prompt"] * a.batch
    phases = {"generate": 0.0, "score": 0.0, "train": 0.0}

    def sync():
        torch.cuda.synchronize()
        return time.perf_counter()

    exposed = []  # the update's gradient-collective wait nothing overlapped, ms per step

    def step(record):
        ids = torch.randint(3, cfg.vocab_size, (a.batch, a.prompt), device=dev, generator=g)
        am = torch.ones_like(ids)
        t0 = sync()
        seqs, mask = generate(pol, ids, am, max_new_tokens=a.new, do_sample=True, temperature=0.7,
                              top_p=0.9, eos_token_id=-1, return_mask=True, seed=3,
                              weight_dtype=a.rollout_dtype)
        t1 = sync()
        with torch.no_grad():
            if a.handoff == "none":
                scores = rm(seqs, mask)
            else:
                r_ids, r_mask = handoff(prompts, ids, am, seqs, mask)
                scores = rm(r_ids, r_mask)
        t2 = sync()
        pol.train()
        reinforce_update(pol, ref, eng, seqs, mask, scores.float(), 0.1, a.micro)
        eng.step()
        t3 = sync()
        if record:
            phases["generate"] += t1 - t0
            phases["score"] += t2 - t1
            phases["train"] += t3 - t2
            exposed.append(eng.comm_timer.last_step_ms())

    if a.overlap:
        import threading

        snap = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=1).requires_grad_(False).eval()
        snap_params = list(snap.parameters())

        @torch.no_grad()
        def refresh():  # snapshot <- policy (main stream, after the update)
            for d, s_ in zip(snap_params, pol.parameters()):
                d.copy_(s_.detach())

        side = torch.cuda.Stream(device=dev)

        def rollout():
            ids = torch.randint(3, cfg.vocab_size, (a.batch, a.prompt), device=dev, generator=g)
            am = torch.ones_like(ids)
            seqs, mask = generate(snap, ids, am, max_new_tokens=a.new, do_sample=True, temperature=0.7,
                                  top_p=0.9, eos_token_id=-1, return_mask=True, seed=3,
                              weight_dtype=a.rollout_dtype)
            with torch.no_grad():
                if a.handoff == "none":
                    scores = rm(seqs, mask)
                else:
                    r_ids, r_mask = handoff(prompts, ids, am, seqs, mask)
                    scores = rm(r_ids, r_mask)
            return seqs, mask, scores

        def train(ro):
            seqs, mask, scores = ro
            pol.train()
            loss, _ = rlhf_loss(pol, ref, seqs, mask, scores.float(), 0.1)
            loss.backward()
            eng.step()

        refresh()
        pending = rollout()  # also captures the snapshot's decode graph (serially)

        def ostep(record):
            nonlocal pending
            out = {}
            main = torch.cuda.current_stream(dev)
            side.wait_stream(main)  # the refreshed snapshot

            def job():
                with torch.cuda.stream(side):
                    t0 = time.perf_counter()
                    out["ro"] = rollout()
                    side.synchronize()
                    out["t"] = time.perf_counter() - t0

            th = threading.Thread(target=job)
            t0 = time.perf_counter()
            th.start()
            train(pending)
            main.synchronize()
            t_train = time.perf_counter() - t0
            th.join()
            main.wait_stream(side)
            for x in out["ro"]:
                x.record_stream(main)
            refresh()
            pending = out["ro"]
            if record:
                phases["generate"] += out["t"]
                phases["train"] += t_train

        for _ in range(a.warmup):
            ostep(False)
        t = sync()
        for _ in range(a.steps):
            ostep(True)
        dt = sync() - t
    else:
        for _ in range(a.warmup):
            step(False)
        t = sync()
        for _ in range(a.steps):
            step(True)
        dt = sync() - t
    print(json.dumps({"bench": "rlhf_step", "model": cfg.name, "rollouts_per_step": a.batch,
                      "rollout_dtype": a.rollout_dtype, "frozen_fp8": a.frozen_fp8,
                      "grad_ckpt": a.grad_ckpt or "none", "handoff": a.handoff,
                      "overlap": bool(a.overlap), "update_micro": a.micro or a.batch,
                      "peak_gib": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1),
                      "prompt": a.prompt, "new_tokens": a.new, "s_per_step": round(dt / a.steps, 3),
                      "rollouts_per_s": round(a.batch * a.steps / dt, 3),
                      **{f"{k}_s": round(v / a.steps, 3) for k, v in phases.items()},
                      "comm_exposed_ms": round(sum(exposed) / len(exposed), 2) if exposed else None}), flush=True)
    return 0


def ppo_main(a) -> int:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from distributed_llm_alignment_amd.models import build_model, generate, get_config
    from distributed_llm_alignment_amd.models.reward import RewardModel, ValueModel
    from distributed_llm_alignment_amd.models.tokenizer import ByteTokenizer
    from distributed_llm_alignment_amd.objectives import ppo_backward, ppo_loss, ppo_rollout_stats
    from distributed_llm_alignment_amd.ops import _ext
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine
    from distributed_llm_alignment_amd.training.handoff import RewardHandoff
    from distributed_llm_alignment_amd.utils.tuning import enable_gemm_tuning

    dev = torch.device("cuda", 0)
    _ext.require()
    enable_gemm_tuning(0)
    cfg = get_config(a.model)
    gib = 2.0 ** 30
    mem = {}

    def note(k):
        torch.cuda.synchronize()
        mem[k] = round(torch.cuda.memory_allocated(dev) / gib, 2)

    note("start")
    pol = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=1)
    note("policy")
    ref = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=1).requires_grad_(False).eval()
    note("reference")
    rm = RewardModel(build_model(cfg, device=dev, dtype=torch.bfloat16, seed=2, headless=True)).to(dev, torch.bfloat16)
    if a.frozen_fp8:
        from distributed_llm_alignment_amd.ops import enable_fp8_inference

        enable_fp8_inference(ref)
        enable_fp8_inference(rm.backbone)
    rm.eval().requires_grad_(False)
    note("reward")
    critic = ValueModel(build_model(cfg, device=dev, dtype=torch.bfloat16, seed=3, headless=True))
    note("critic")
    if a.grad_ckpt:
        pol.gradient_checkpointing_enable(a.grad_ckpt)
        critic.backbone.gradient_checkpointing_enable(a.grad_ckpt)
    kw = dict(betas=(0.9, 0.95), weight_decay=0.01, max_grad_norm=1.0, shape_world=a.zero_shape)
    eng = DataParallelEngine(pol, lr=1e-6, **kw)
    note("policy_engine")
    ceng = DataParallelEngine(critic, lr=5e-6, **kw)
    note("critic_engine")
    g = torch.Generator(device=dev).manual_seed(0)
    tok = ByteTokenizer(vocab_size=cfg.vocab_size)
    handoff = RewardHandoff(tok, tok, cfg.vocab_size, dev, a.prompt + a.new + 8, "device")
    prompts = ["synthetic prompt"] * a.batch
    phases = {"generate": 0.0, "score": 0.0, "stats": 0.0, "update": 0.0}
    peaks = {}

    def sync():
        torch.cuda.synchronize()
        return time.perf_counter()

    def phase_peak(name):
        torch.cuda.synchronize()
        peaks[name] = max(peaks.get(name, 0.0), round(torch.cuda.max_memory_allocated(dev) / gib, 2))
        torch.cuda.reset_peak_memory_stats(dev)

    exposed = []  # the update's gradient-collective wait nothing overlapped, ms per step

    def step(record):
        ids = torch.randint(3, cfg.vocab_size, (a.batch, a.prompt), device=dev, generator=g)
        am = torch.ones_like(ids)
        torch.cuda.reset_peak_memory_stats(dev)
        t0 = sync()
        seqs, mask = generate(pol, ids, am, max_new_tokens=a.new, do_sample=True, temperature=0.7,
                              top_p=0.9, eos_token_id=-1, return_mask=True, seed=3,
                              weight_dtype=a.rollout_dtype)
        t1 = sync()
        phase_peak("generate")
        with torch.no_grad():
            r_ids, r_mask = handoff(prompts, ids, am, seqs, mask)
            scores = rm(r_ids, r_mask)
        t2 = sync()
        phase_peak("score")
        stats = ppo_rollout_stats(pol, ref, critic, seqs, mask, a.prompt, scores, 0.05, 1.0, 0.95)
        t3 = sync()
        phase_peak("stats")
        S = seqs.shape[0]
        nmb = max(1, a.minibatches)
        bounds = [(i * S // nmb, (i + 1) * S // nmb) for i in range(nmb)]
        pol.train()
        critic.train()
        for _ in range(a.ppo_epochs):
            for lo, hi in bounds:
                mb = {k: v[lo:hi] for k, v in stats.items() if k in ("old_logp", "values", "advantages", "returns", "act")}
                loss, m = ppo_loss(pol, critic, seqs[lo:hi], mask[lo:hi], mb, 0.2, 0.2, 0.1)
                ppo_backward(loss)
                eng.step()
                ceng.step()
        t4 = sync()
        phase_peak("update")
        if record:
            phases["generate"] += t1 - t0
            phases["score"] += t2 - t1
            phases["stats"] += t3 - t2
            phases["update"] += t4 - t3
        return loss, m

    for _ in range(a.warmup):
        step(False)
    t = sync()
    for _ in range(a.steps):
        loss, m = step(True)
    dt = sync() - t
    # the update moved both models (finite, nonzero grad norms)
    health = {"loss": round(float(loss), 5), "policy_grad_norm": round(float(eng.last_grad_norm), 5),
              "critic_grad_norm": round(float(ceng.last_grad_norm), 5),
              "clipfrac": round(float(m["clipfrac"]), 4)}
    print(json.dumps({"bench": "ppo_step", "model": cfg.name, "rollouts_per_step": a.batch,
                      "rollout_dtype": a.rollout_dtype, "frozen_fp8": a.frozen_fp8,
                      "zero_shape": a.zero_shape, "ppo_epochs": a.ppo_epochs, "minibatches": a.minibatches,
                      "grad_ckpt": a.grad_ckpt or "none", "prompt": a.prompt, "new_tokens": a.new,
                      "s_per_step": round(dt / a.steps, 3), "rollouts_per_s": round(a.batch * a.steps / dt, 3),
                      **{f"{k}_s": round(v / a.steps, 3) for k, v in phases.items()},
                      "mem_after_gib": mem, "peak_gib_by_phase": peaks,
                      "device_total_gib": round(torch.cuda.get_device_properties(dev).total_memory / gib, 1),
                      **health}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
