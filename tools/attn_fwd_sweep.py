#!/usr/bin/env python
"""Attention forward kernel time over (B, T) at fixed B*T (the DPO micro-batch's 8192 tokens),
timed as a hipGraph replay of `iters` back-to-back forwards, so host dispatch never shows
(tools/attn_bench.py times eager calls and reads the host's dispatch time at small shapes).

    python tools/attn_fwd_sweep.py [--tokens 8192] [--ab ENV=v0,v1]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--T", default="256,512,1024,2048,4096")
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=8)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ab", default="", help="ENV=v0,v1: interleave the settings per shape")
    ap.add_argument("--v-strided", action="store_true",
                    help="v as the strided view of a fused [B, T, (Hq + 2 Hkv) * D] qkv buffer, as the "
                         "training step passes it (q, k contiguous: the RoPE pass writes them)")
    ap.add_argument("--cfg", action="append", default=[],
                    help="NAME:VAR=VAL[,VAR=VAL...] (repeatable): interleave these env settings per shape")
    a = ap.parse_args()
    from distributed_llm_alignment_amd import ops

    dev = torch.device("cuda", 0)
    cfgs = [("us", {})]
    if a.ab:
        name, _, vs = a.ab.partition("=")
        cfgs = [(f"us[{name}={v}]", {name: v}) for v in (vs.split(",") if vs else ["0", "1"])]
    if a.cfg:
        cfgs = []
        for c in a.cfg:
            label, _, kv = c.partition(":")
            cfgs.append((f"us[{label}]", dict(x.split("=", 1) for x in kv.split(","))))
    for T in map(int, a.T.split(",")):
        B = max(1, a.tokens // T)
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B, T, a.Hq, a.D, device=dev, generator=g).to(torch.bfloat16)
        k = torch.randn(B, T, a.Hkv, a.D, device=dev, generator=g).to(torch.bfloat16)
        v = torch.randn(B, T, a.Hkv, a.D, device=dev, generator=g).to(torch.bfloat16)
        if a.v_strided:
            C = (a.Hq + 2 * a.Hkv) * a.D
            buf = torch.zeros(B, T, C, device=dev, dtype=torch.bfloat16)
            vs = buf[..., (a.Hq + a.Hkv) * a.D:].view(B, T, a.Hkv, a.D)
            vs.copy_(v)
            v = vs
        for causal in (True, False):
            flops = 4.0 * B * a.Hq * T * T * a.D / (2 if causal else 1)
            rec = {"B": B, "T": T, "causal": causal}
            outs = {}
            for key, env in cfgs:
                saved = {k2: os.environ.get(k2) for k2 in env}
                os.environ.update(env)
                with torch.no_grad():
                    outs[key] = ops.attention_core(q, k, v, causal=causal)
                    torch.cuda.synchronize()
                    gr = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gr):
                        for _ in range(a.iters):
                            ops.attention_core(q, k, v, causal=causal)
                best = 1e9
                for _ in range(3):
                    gr.replay()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    gr.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    best = min(best, e0.elapsed_time(e1) * 1e3 / a.iters)
                del gr
                for k2, v2 in saved.items():
                    if v2 is None:
                        os.environ.pop(k2, None)
                    else:
                        os.environ[k2] = v2
                rec[key] = round(best, 1)
                rec[key.replace("us", "tf")] = round(flops / best / 1e6, 0)
            if len(cfgs) > 1:
                o0 = outs[cfgs[0][0]].float()
                rec["max_abs_diff"] = max(float((outs[c[0]].float() - o0).abs().max()) for c in cfgs)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
