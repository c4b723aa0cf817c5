#!/usr/bin/env python
"""Flash-attention fwd/bwd microbenchmark at the DPO bench shape (B=8 sequences x T=1024,
Llama-3-8B heads: Hq=32, Hkv=8, D=128, causal). Prints TF/s per pass; run under
`rocprofv3 --kernel-trace --stats` or `--pmc ...` for counters."""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=8)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from distributed_llm_alignment_amd import ops

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(a.B, a.T, a.Hq, a.D, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    k = torch.randn(a.B, a.T, a.Hkv, a.D, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    v = torch.randn(a.B, a.T, a.Hkv, a.D, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    do = torch.randn(a.B, a.T, a.Hq, a.D, device=dev, generator=g).to(torch.bfloat16)
    flops_fwd = 4.0 * a.B * a.Hq * a.T * a.T * a.D / 2  # causal
    o = ops.attention_core(q, k, v, causal=True)
    torch.autograd.grad(o, [q, k, v], do)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        o = ops.attention_core(q, k, v, causal=True)
    torch.cuda.synchronize()
    tf = (time.perf_counter() - t0) / a.iters
    t0 = time.perf_counter()
    for _ in range(a.iters):
        torch.autograd.grad(o, [q, k, v], do, retain_graph=True)
    torch.cuda.synchronize()
    tb = (time.perf_counter() - t0) / a.iters
    print(f"[attn] fwd {tf*1e6:.1f} us ({flops_fwd/tf/1e12:.0f} TF/s)  bwd(all kernels) {tb*1e6:.1f} us "
          f"({2.5*flops_fwd/tb/1e12:.0f} TF/s)", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
