#!/usr/bin/env python
"""Tune hipBLASLt/rocBLAS solution selection (PyTorch TunableOp) for every GEMM shape of a
model's DPO/SFT step on this GPU and write the table used by utils/tuning.py.

    python tools/tune_gemms.py --model llama3-8b --tokens 8192 --chunk 4096 --out <table.csv>

Shapes (M = tokens per micro-batch): forward Y = X W^T, input grad dX = dY W, weight grad
W.main_grad += dY^T X (beta = 1) for qkv / o / gate_up / down / LM head, plus the no-grad LM-head
chunk. Prints one line per shape so long tunings stay observable.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--out", required=True)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--ms", type=int, default=12)
    ap.add_argument("--only", default="", help="comma list of fwd,dx,dw,dxt,dwt,lm")
    ap.add_argument("--rotating-mb", type=int, default=0,
                    help="TunableOp rotating buffer: operands cycle through this many MB so each "
                         "candidate is timed cache-cold, as in the step (0 = cache-warm)")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from distributed_llm_alignment_amd.models import get_config

    cfg = get_config(a.model)
    H, F, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
    q = cfg.q_size + 2 * cfg.kv_size
    up = 2 * F if cfg.activation == "swiglu" else F
    layers = [("qkv", q, H), ("o", H, cfg.q_size), ("up", up, H), ("down", H, F)]
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.record_untuned_enable(False)
    tun.set_max_tuning_iterations(a.iters)
    tun.set_max_tuning_duration(a.ms)
    tun.set_filename(a.out, insert_device_ordinal=False)
    try:
        tun.set_rotating_buffer_size(a.rotating_mb)
    except Exception:
        pass
    dev = torch.device("cuda", 0)
    M = a.tokens
    only = set(a.only.split(",")) if a.only else {"fwd", "dx", "dw", "dxt", "dwt", "lm"}

    def run(tag, fn):
        t0 = time.time()
        fn()
        torch.cuda.synchronize()
        print(f"[tune] {tag} done in {time.time() - t0:.1f}s", flush=True)

    shapes = list(layers)
    if "lm" in only:
        shapes.append(("lm_head", V, H))
    for name, N, K in shapes:
        W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        dY = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        if "fwd" in only:
            run(f"fwd {name} M={M} N={N} K={K}", lambda: torch.nn.functional.linear(X, W))
        if "dx" in only:
            run(f"dx  {name} M={M} N={K} K={N}", lambda: dY @ W)
        if "dw" in only:
            G = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
            run(f"dw  {name} M={N} N={K} K={M}", lambda: G.addmm_(dY.t(), X))
        # layouts the engine actually issues (ops/linear.py): TN input grad through the persistent
        # W^T, TN weight grad on transposed activations accumulated with beta = 1
        if "dxt" in only:
            Wt = W.t().contiguous()
            run(f"dxT {name} M={M} N={K} K={N}", lambda: torch.nn.functional.linear(dY, Wt))
            del Wt
        if "dwt" in only:
            G = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
            dYt, Xt = dY.t().contiguous(), X.t().contiguous()
            run(f"dwT {name} M={N} N={K} K={M}", lambda: G.addmm_(dYt, Xt.t()))
            del G, dYt, Xt
        if name == "lm_head" and a.chunk and a.chunk != M:
            Xc = X[: a.chunk]
            run(f"fwd {name} chunk M={a.chunk}", lambda: torch.nn.functional.linear(Xc, W))
        del W, X, dY
        torch.cuda.empty_cache()
    print("[tune] writing", a.out, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
