#!/usr/bin/env python
"""Comparison point for the reference's only perf harness (src/eval/eval_latency.py:22-63): the
same measurement on stock PyTorch-ROCm + HF transformers on the same MI355X — HF
`LlamaForCausalLM` / `MistralForCausalLM` (SDPA) in bf16, random init of the named architecture,
`model(input_ids, attention_mask)` forwards at every (batch, seq) of the grid, `warmup_steps`
untimed then `measure_steps` timed between synchronisations; tokens/s = B*T*steps/dt. Prints one
JSON line per grid point (compare with `eval_latency --config config/eval_latency_mi355x.yaml`).

    python tools/hf_stack_latency.py --model mistral-7b
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--batch-sizes", default="1,4,8")
    ap.add_argument("--seq-lengths", default="256,512,1024")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import transformers

    from distributed_llm_alignment_amd.models import get_config

    dev = torch.device("cuda", 0)
    cfg = get_config(a.model)
    hf = cfg.to_hf()
    arch = hf.pop("architectures", ["LlamaForCausalLM"])[0]
    model_type = hf.pop("model_type", "llama")
    hf.pop("torch_dtype", None)
    hcfg = transformers.AutoConfig.for_model(model_type, **hf)
    hcfg._attn_implementation = "sdpa"
    torch.manual_seed(0)
    with torch.device(dev):
        model = getattr(transformers, arch)(hcfg).to(torch.bfloat16).eval()
    for b in map(int, a.batch_sizes.split(",")):
        for t in map(int, a.seq_lengths.split(",")):
            ids = torch.randint(0, cfg.vocab_size - 1, (b, t), device=dev)
            att = torch.ones_like(ids)
            with torch.no_grad():
                for _ in range(a.warmup):
                    model(input_ids=ids, attention_mask=att)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    model(input_ids=ids, attention_mask=att)
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"stack": "hf-transformers", "model": cfg.name, "batch_size": b, "seq_length": t,
                              "tokens_per_second": round(b * t * a.steps / dt, 1),
                              "latency_ms": round(dt / a.steps * 1000.0, 3)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
