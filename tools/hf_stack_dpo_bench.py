#!/usr/bin/env python
"""Comparison point for the headline metric (BASELINE.md "comparison point" column): the
reference's DPO step as it runs on stock PyTorch-ROCm + HF transformers, on the same MI355X.

Re-implements the reference step semantics (src/training/train_dpo.py:31-44, 107-118):
  * HF `LlamaForCausalLM` (SDPA attention) in bf16, random init of the named architecture;
  * policy with HF gradient checkpointing (base_model.py:36-37 / dpo config), frozen reference;
  * four forwards per micro-batch (policy chosen / rejected, reference chosen / rejected), each
    materialising fp32 log_softmax over [B, T, V] then gather + masked mean;
  * -logsigmoid(beta * margin).mean(), backward, clip_grad_norm_(1.0), torch AdamW
    (lr 1e-6, weight_decay 0.01, foreach), step + zero_grad.
Synthetic preference pairs with the shape of bench.py. Prints one JSON line.

    python tools/hf_stack_dpo_bench.py --micro-pairs 4 --accum 4 [--no-ckpt] [--ref-no-grad]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--micro-pairs", type=int, default=4)
    ap.add_argument("--accum", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-ckpt", action="store_true", help="disable gradient checkpointing")
    ap.add_argument("--ref-no-grad", action="store_true",
                    help="run the reference forwards under no_grad (the reference does not)")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from transformers import LlamaConfig, LlamaForCausalLM

    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.models import get_config

    dev = torch.device("cuda", 0)
    cfg = get_config(a.model)
    hf = cfg.to_hf()
    hf.pop("architectures", None)
    hf.pop("model_type", None)
    hf.pop("torch_dtype", None)
    hcfg = LlamaConfig(**hf)
    hcfg._attn_implementation = "sdpa"
    torch.manual_seed(0)
    with torch.device(dev):
        policy = LlamaForCausalLM(hcfg).to(torch.bfloat16)
        ref = LlamaForCausalLM(hcfg).to(torch.bfloat16)
    ref.load_state_dict(policy.state_dict())
    ref.eval().requires_grad_(False)
    if not a.no_ckpt:
        policy.gradient_checkpointing_enable()
    policy.config.use_cache = False
    policy.train()
    opt = torch.optim.AdamW(policy.parameters(), lr=1e-6, weight_decay=0.01)
    gen = torch.Generator().manual_seed(17)
    batches = [synthetic_preference_batch(a.micro_pairs, a.seq_len, cfg.vocab_size, device=dev, generator=gen)
               for _ in range(4)]

    def logps(model, ids, mask):
        logits = model(input_ids=ids, attention_mask=mask).logits[:, :-1]
        labels = ids[:, 1:]
        m = mask[:, 1:]
        lp = torch.log_softmax(logits.float(), dim=-1)
        g = torch.gather(lp, 2, labels.unsqueeze(-1)).squeeze(-1)
        return (g * m).sum(1) / m.sum(1).clamp(min=1)

    state = {"i": 0}

    def step():
        for _ in range(a.accum):
            b = batches[state["i"] % len(batches)]
            state["i"] += 1
            c, r = b["chosen"], b["rejected"]
            pp = logps(policy, c["input_ids"], c["attention_mask"])
            pn = logps(policy, r["input_ids"], r["attention_mask"])
            ctx = torch.no_grad() if a.ref_no_grad else torch.enable_grad()
            with ctx:
                rp = logps(ref, c["input_ids"], c["attention_mask"])
                rn = logps(ref, r["input_ids"], r["attention_mask"])
            loss = -F.logsigmoid(0.1 * ((pp - pn) - (rp - rn))).mean() / a.accum
            loss.backward()
        torch.nn.utils.clip_grad_norm_(policy.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    pairs = a.micro_pairs * a.accum * a.steps
    print(json.dumps({"stack": "pytorch-rocm + HF transformers (SDPA) + torch AdamW",
                      "model": cfg.name, "pairs_per_s": round(pairs / dt, 4),
                      "ms_per_step": round(dt / a.steps * 1e3, 1), "micro_pairs": a.micro_pairs,
                      "accum": a.accum, "seq_len": a.seq_len, "grad_ckpt": not a.no_ckpt,
                      "ref_no_grad": a.ref_no_grad, "loss": float(loss) * a.accum,
                      "max_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
