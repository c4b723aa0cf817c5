"""What the token-chunked TP GEMMs cost at Llama-3-70B's per-rank TP = 8 shapes (one MI355X).

The overlapped TP layers (parallel/tensor_parallel.py) split every row-parallel forward GEMM and
every Megatron-SP gather-GEMM / GEMM-reduce-scatter into DLA_TP_CHUNKS token chunks so chunk c's
collective runs under chunk c+1's GEMM. On one GPU there is no collective to hide, so this probe
times only the price of the split: the same GEMMs whole vs in 2 / 4 / 8 row chunks, forward and
input-gradient (the weight gradient stays whole in the implementation). Per-rank shapes
(`models.config.tp_shard_config` of llama3-70b at tp 8): H 8192, qkv 1280 columns, o 1024 input
columns, gate|up 7168 columns, down 3584 input columns; M = 4096 tokens (the 70B config's
2-pair micro-batch at seq 1024).

    python tools/tp_chunk_probe.py [--tokens 4096] [--chunks 1 2 4 8] [--reps 30]

Prints one JSON line per (gemm, chunks) and a per-step estimate for the 70B DPO config (80 layers,
8 micro-batches, policy fwd + bwd and reference fwd).
"""
from __future__ import annotations

import argparse
import json
import statistics

import torch
import torch.nn.functional as F


def _time(fn, reps: int) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def _bounds(M: int, c: int):
    step = max(8, ((M + c - 1) // c + 7) // 8 * 8)
    return [(a, min(M, a + step)) for a in range(0, M, step)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--chunks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--layers", type=int, default=80)
    ap.add_argument("--micro", type=int, default=8)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    M, H = args.tokens, 8192
    g = torch.Generator(device=dev).manual_seed(0)
    # (name, N out, K in); forward y[M, N] = x[M, K] W^T, dgrad dx[M, K] = dy[M, N] W (TN via W^T)
    shapes = [("qkv", 1280, H), ("o", H, 1024), ("gate_up", 7168, H), ("down", H, 3584)]
    per = {}
    for name, N, K in shapes:
        W = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16) * 0.02
        Wt = W.t().contiguous()
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        for c in args.chunks:
            bnd = _bounds(M, c)

            def fwd():
                for a, b in bnd:
                    torch.mm(x[a:b], W.t(), out=y[a:b])

            def dgrad():
                for a, b in bnd:
                    dx[a:b] = F.linear(dy[a:b], Wt)

            tf, tb = _time(fwd, args.reps), _time(dgrad, args.reps)
            fl = 2.0 * M * N * K
            per[(name, c)] = (tf, tb)
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "chunks": c, "fwd_ms": round(tf, 4),
                              "dgrad_ms": round(tb, 4), "fwd_tflops": round(fl / tf / 1e9, 1),
                              "dgrad_tflops": round(fl / tb / 1e9, 1)}), flush=True)
    # per optimizer step: every layer runs 2 forwards (policy + reference) and 1 dgrad per
    # micro-batch for each of the 4 GEMMs
    base = None
    for c in args.chunks:
        tot = sum(2 * per[(n, c)][0] + per[(n, c)][1] for n, _, _ in shapes) * args.layers * args.micro
        base = tot if base is None else base
        print(json.dumps({"chunks": c, "chunked_gemm_ms_per_step": round(tot, 1),
                          "penalty_ms_per_step_vs_first": round(tot - base, 1)}), flush=True)


if __name__ == "__main__":
    main()
