#!/usr/bin/env python
"""Rollout-generation throughput (the RLHF / teacher-generation hot loop):
prefill B prompts of length T, then decode N tokens, eager per-op loop vs the captured-hipGraph
decode step. Prints one JSON line per mode.

    python tools/bench_generate.py --model llama3-8b --batch 8 --prompt 1024 --new 256
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
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=1024)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--modes", default="eager,graph")
    ap.add_argument("--weight-dtype", choices=("bf16", "fp8"), default="bf16",
                    help="decode weight streams (generate(weight_dtype=...))")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from distributed_llm_alignment_amd.models import build_model, generate, get_config
    from distributed_llm_alignment_amd.ops import _ext
    from distributed_llm_alignment_amd.utils.tuning import enable_gemm_tuning

    dev = torch.device("cuda", 0)
    _ext.require()
    enable_gemm_tuning(0)
    cfg = get_config(a.model)
    m = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    g = torch.Generator(device=dev).manual_seed(0)
    ids = torch.randint(3, cfg.vocab_size, (a.batch, a.prompt), device=dev, generator=g)
    am = torch.ones_like(ids)
    for mode in a.modes.split(","):
        kw = dict(max_new_tokens=a.new, do_sample=True, temperature=0.7, top_p=0.9, eos_token_id=-1,
                  use_graph=(mode == "graph"), seed=1, weight_dtype=a.weight_dtype)
        generate(m, ids[:, :64], am[:, :64], **{**kw, "max_new_tokens": 8})  # warm
        generate(m, ids, am, **kw)  # warm at the timed shapes (graph mode: the capture is reused)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = generate(m, ids, am, **kw)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        n = out.shape[1] - a.prompt
        # prefill alone, for the per-token decode latency
        t1 = time.perf_counter()
        generate(m, ids, am, **{**kw, "max_new_tokens": 1})
        torch.cuda.synchronize()
        tp = time.perf_counter() - t1
        print(json.dumps({"mode": mode, "model": cfg.name, "batch": a.batch, "prompt": a.prompt,
                          "weight_dtype": a.weight_dtype,
                          "new_tokens": n, "total_s": round(dt, 3), "prefill_s": round(tp, 3),
                          "decode_ms_per_token": round((dt - tp) / max(n - 1, 1) * 1e3, 3),
                          "decode_tokens_per_s": round(a.batch * (n - 1) / max(dt - tp, 1e-9), 1)}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
