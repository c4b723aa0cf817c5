"""Mixtral expert-block microbenchmark on one MI355X: device-driven grouped GEMM
(csrc/grouped_gemm.hip) vs the per-expert hipBLASLt loop, forward and forward+backward.

    python tools/grouped_gemm_bench.py [--tokens 8192] [--hidden 4096] [--ffn 14336] [--experts 8]

Prints one JSON line per measurement (per-op TFLOP/s of the grouped kernel, then the whole
expert block for both paths, bf16 and fp8 forward). Operands are random (N(0,1) activations,
0.02-scaled weights): zero-filled data would run the chip at a higher clock (cdna guide §5.4
rule 25)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, iters=10, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--ffn", type=int, default=14336)
    ap.add_argument("--experts", type=int, default=8)
    ap.add_argument("--topk", type=int, default=2)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--scheds", default="0")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--blocks", type=int, default=1, help="also time the whole expert block (0/1)")
    ap.add_argument("--only", default="", help="substring filter on the per-op cases")
    ap.add_argument("--no-loop", action="store_true")
    a = ap.parse_args(argv)

    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.ops import _ext

    C = _ext.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    T, H, Fd, E, k = a.tokens, a.hidden, a.ffn, a.experts, a.topk
    topi = torch.argsort(torch.rand(T, E, device=dev, generator=g), -1)[:, :k].to(torch.int32)
    pos, counts = ops.moe.expert_positions(topi, E)
    offs = ops.moe.expert_offsets(counts)
    M = T * k
    xs = torch.randn(M, H, device=dev, generator=g).to(torch.bfloat16)
    w_up = (torch.randn(E, 2 * Fd, H, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    w_down = (torch.randn(E, H, Fd, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    dy = torch.randn(M, H, device=dev, generator=g).to(torch.bfloat16)
    gu, act = C.gg_fwd_swiglu(xs, w_up, offs, None, None)
    dgu = torch.randn(M, 2 * Fd, device=dev, generator=g).to(torch.bfloat16)
    gw_up = torch.zeros_like(w_up, dtype=torch.float32)
    gw_down = torch.zeros_like(w_down, dtype=torch.float32)
    gw_up16 = torch.zeros_like(w_up)
    meta = {"tokens": T, "rows": M, "hidden": H, "ffn": Fd, "experts": E, "topk": k,
            "counts": counts.tolist()}
    print(json.dumps({"config": meta}), flush=True)

    def rep(name, ms, flops):
        print(json.dumps({"op": name, "ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1)}),
              flush=True)

    up_f, dn_f = 2.0 * M * H * 2 * Fd, 2.0 * M * Fd * H
    xq, sx = ops.moe.quant_fp8_rows(xs)
    wq, sw = ops.moe.fp8_weight(w_up)
    cases = [
        ("up+swiglu fwd", lambda: C.gg_fwd_swiglu(xs, w_up, offs, None, None), up_f),
        ("down fwd", lambda: C.gg_fwd(act, w_down, offs, None, None), dn_f),
        ("down dgrad+swiglu bwd", lambda: C.gg_dgrad_swiglu(dy, w_down, offs, gu), dn_f),
        ("down wgrad (fp32 acc)", lambda: C.gg_wgrad(dy, act, offs, gw_down, True), dn_f),
        ("up dgrad", lambda: C.gg_dgrad(dgu, w_up, offs), up_f),
        ("up wgrad (fp32 acc)", lambda: C.gg_wgrad(dgu, xs, offs, gw_up, True), up_f),
        ("up wgrad (bf16 acc)", lambda: C.gg_wgrad(dgu, xs, offs, gw_up16, True), up_f),
        ("up+swiglu fwd fp8", lambda: C.gg_fwd_swiglu(xq, wq, offs, sx, sw), up_f),
    ]
    cases = [c for c in cases if a.only in c[0]]
    scheds = [int(x) for x in a.scheds.split(",")]
    # interleaved rounds in one process (cdna guide §5.4 rule 24): min over rounds per schedule
    best = {}
    for _ in range(a.rounds):
        for name, fn, fl in cases:
            for sc in scheds:
                torch.ops.dla.gg_set_sched(sc)
                ms = _time(fn, a.iters)
                best[(name, sc)] = min(ms, best.get((name, sc), 1e9))
    for name, fn, fl in cases:
        for sc in scheds:
            rep(f"grouped {name} sched{sc}", best[(name, sc)], fl)
    torch.ops.dla.gg_set_sched(-1)  # per-layout defaults for the block timings
    cl = counts.tolist()
    # hipBLASLt per-expert reference for the same projections
    def loop_up():
        s = 0
        for e, c in enumerate(cl):
            torch.mm(xs[s:s + c], w_up[e].t(), out=gu[s:s + c])
            s += c
    if not a.no_loop:
        rep("loop up fwd (hipBLASLt)", _time(loop_up, a.iters), up_f)

    fwd_f = up_f + dn_f
    for path in (("grouped", "loop") if a.blocks else ()):
        os.environ["DLA_MOE_GEMM"] = path
        for fp8 in (False, True):
            x = xs.clone().requires_grad_(True)
            wu = w_up.clone().requires_grad_(True)
            wd = w_down.clone().requires_grad_(True)
            cnt = counts if path == "grouped" else cl
            f = lambda: ops.moe.experts_swiglu(x, wu, wd, cnt, fp8=fp8)
            with torch.no_grad():
                rep(f"{path} expert block fwd{' fp8' if fp8 else ''}", _time(f, a.iters), fwd_f)

            def fb():
                y = f()
                torch.autograd.backward(y, dy)
            rep(f"{path} expert block fwd+bwd{' fp8' if fp8 else ''}", _time(fb, a.iters), 3 * fwd_f)
    os.environ.pop("DLA_MOE_GEMM", None)


if __name__ == "__main__":
    main()
