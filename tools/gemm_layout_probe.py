#!/usr/bin/env python
"""Measure the input-gradient GEMM dX = dY @ W in its natural NN layout vs the TN layout
obtained from a persistent transposed weight copy (dX = linear(dY, W^T)), for every linear of a
model, with TunableOp tuning both. Prints one line per shape."""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--tune", type=int, default=1)
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from distributed_llm_alignment_amd.models import get_config

    cfg = get_config(a.model)
    H, Fd = cfg.hidden_size, cfg.intermediate_size
    shapes = [("qkv", cfg.q_size + 2 * cfg.kv_size, H), ("o", H, cfg.q_size), ("up", 2 * Fd, H), ("down", H, Fd)]
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(bool(a.tune))
    tun.record_untuned_enable(False)
    tun.set_max_tuning_iterations(20)
    tun.set_max_tuning_duration(30)
    tun.set_filename("/tmp/probe_tunableop.csv", insert_device_ordinal=False)
    dev = torch.device("cuda", 0)
    M = a.tokens
    for name, N, K in shapes:
        W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        Wt = W.t().contiguous()
        dY = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * M * N * K
        t_nn = bench(lambda: dY @ W)
        t_tn = bench(lambda: F.linear(dY, Wt))
        t_tr = bench(lambda: Wt.copy_(W.t()))
        print(f"[probe] {name:5s} dX M={M} N={K} K={N}: NN {t_nn*1e3:.3f} ms ({flops/t_nn/1e15:.2f} PF/s)  "
              f"TN(W^T copy) {t_tn*1e3:.3f} ms ({flops/t_tn/1e15:.2f} PF/s)  transpose {t_tr*1e3:.3f} ms",
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
