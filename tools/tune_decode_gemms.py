#!/usr/bin/env python
"""TunableOp table entries for the decode GEMMs that stay on hipBLASLt: 17-64 rows (larger
rollout batches on one GPU) for qkv / o / gate|up / down / LM head, plus the long-K down
projection and the LM head at 1-16 rows. A 1 GB rotating buffer makes every timed call stream
its weights from HBM, as in a real decode step (16 GB of weights between two uses of one
matrix), instead of finding them in the 256 MB Infinity Cache.

    python tools/tune_decode_gemms.py --out gpurun_out/decode_tune.csv [--rows 32,64]

Result on MI355X (profiles/r2_decode.md): the library's default choice is already within noise of
the best solution at 32 and 64 rows, so the shipped table was left unchanged.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--rows", default="32,64")
    ap.add_argument("--small_rows", default="1,2,4,8,16")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--ms", type=int, default=30)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from distributed_llm_alignment_amd.models import get_config

    cfg = get_config(a.model)
    H, Fd, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
    q = cfg.q_size + 2 * cfg.kv_size
    big = [("qkv", q, H), ("o", H, cfg.q_size), ("gate_up", 2 * Fd, H), ("down", H, Fd), ("lm_head", V, H)]
    small = [("down", H, Fd), ("lm_head", V, H)]  # the 1-16-row shapes the skinny kernels leave
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.record_untuned_enable(False)
    tun.set_max_tuning_iterations(a.iters)
    tun.set_max_tuning_duration(a.ms)
    tun.set_rotating_buffer_size(1024)
    tun.set_filename(a.out, insert_device_ordinal=False)
    dev = torch.device("cuda", 0)
    jobs = [(int(m), s) for m in a.rows.split(",") if m for s in big]
    jobs += [(int(m), s) for m in a.small_rows.split(",") if m for s in small]
    for M, (name, N, K) in jobs:
        W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        t0 = time.time()
        with torch.no_grad():
            F.linear(x, W)
        torch.cuda.synchronize()
        print(f"[tune] {name} M={M} N={N} K={K} {time.time() - t0:.1f}s", flush=True)
        del W, x
    return 0


if __name__ == "__main__":
    sys.exit(main())
