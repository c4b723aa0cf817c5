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
    ap.add_argument("--noncausal", action="store_true")
    ap.add_argument("--ab", default="", help="NAME[=v0,v1]: env var to A/B (forward and backward), interleaved")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from distributed_llm_alignment_amd import ops

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(a.B, a.T, a.Hq, a.D, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    k = torch.randn(a.B, a.T, a.Hkv, a.D, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    v = torch.randn(a.B, a.T, a.Hkv, a.D, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    do = torch.randn(a.B, a.T, a.Hq, a.D, device=dev, generator=g).to(torch.bfloat16)
    causal = not a.noncausal
    flops_fwd = 4.0 * a.B * a.Hq * a.T * a.T * a.D / (2 if causal else 1)
    o = ops.attention_core(q, k, v, causal=causal)
    torch.autograd.grad(o, [q, k, v], do)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        o = ops.attention_core(q, k, v, causal=causal)
    torch.cuda.synchronize()
    tf = (time.perf_counter() - t0) / a.iters
    t0 = time.perf_counter()
    for _ in range(a.iters):
        torch.autograd.grad(o, [q, k, v], do, retain_graph=True)
    torch.cuda.synchronize()
    tb = (time.perf_counter() - t0) / a.iters
    if a.ab:
        # interleaved rounds in one process (cdna guide §5.4 rule 24): min per setting
        name, _, vals = a.ab.partition("=")
        vals = tuple(vals.split(",")) if vals else ("0", "1")
        best, outs = {}, {}
        for _ in range(a.rounds):
            for val in vals:
                os.environ[name] = val
                outs[val] = ops.attention_core(q, k, v, causal=causal)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    ops.attention_core(q, k, v, causal=causal)
                torch.cuda.synchronize()
                best[val] = min(best.get(val, 1e9), (time.perf_counter() - t0) / a.iters)
        # backward (all kernels: delta, main, dQ reduce, dK/dV reduce), same interleaving
        bbest, gouts = {}, {}
        for _ in range(a.rounds):
            for val in vals:
                os.environ[name] = val
                gouts[val] = torch.autograd.grad(o, [q, k, v], do, retain_graph=True)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    torch.autograd.grad(o, [q, k, v], do, retain_graph=True)
                torch.cuda.synchronize()
                bbest[val] = min(bbest.get(val, 1e9), (time.perf_counter() - t0) / a.iters)
        os.environ.pop(name)
        diff = (outs[vals[0]].float() - outs[vals[1]].float()).abs().max().item()
        gdiff = max((x.float() - y.float()).abs().max().item() for x, y in zip(gouts[vals[0]], gouts[vals[1]]))
        for val in vals:
            print(f"[attn-ab] {name}={val} fwd {best[val]*1e6:.1f} us ({flops_fwd/best[val]/1e12:.0f} TF/s) "
                  f"bwd {bbest[val]*1e6:.1f} us ({2.5*flops_fwd/bbest[val]/1e12:.0f} TF/s)", flush=True)
        print(f"[attn-ab] max |o0 - o1| = {diff:.3e}  max |grad0 - grad1| = {gdiff:.3e}", flush=True)
    print(f"[attn] B={a.B} T={a.T} Hq={a.Hq} causal={causal} fwd {tf*1e6:.1f} us ({flops_fwd/tf/1e12:.0f} TF/s)  bwd(all kernels) {tb*1e6:.1f} us "
          f"({2.5*flops_fwd/tb/1e12:.0f} TF/s)", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
