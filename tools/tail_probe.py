#!/usr/bin/env python
"""Probe of the persistent decode layer tail (csrc/decode_tail.hip) at Llama-3-8B shapes: time per
call against the four-launch fused layer (o + residual, gate|up + SwiGLU, down + residual, next qkv)
on the same weights, and (DLA_TAIL_STAMPS=1) the per-workgroup phase edges.

    python tools/tail_probe.py [--batch 8] [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--model", default="llama3-8b")
    a = ap.parse_args()
    import distributed_llm_alignment_amd  # noqa: F401
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.models.generation import KVCache

    dev = torch.device("cuda", 0)
    NL = 4  # 4 layers x 436 MB rotate past the 256 MB Infinity Cache, as a real decode step does
    cfg = get_config(a.model, num_layers=NL)
    m = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=1).eval()
    B, H = a.batch, cfg.hidden_size
    cache = KVCache(m, B, 64, None)
    with torch.no_grad():
        m(torch.randint(3, cfg.vocab_size, (B, 16), device=dev), cache=cache)
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.randn(B, H, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    att = (torch.randn(B, m.layers[0].attn.o_proj.shape[1], device=dev, generator=g) * 0.5).to(torch.bfloat16)
    L = m.layers
    eps = cfg.norm_eps

    def tail():  # one "step": every layer's tail once (its counters' epoch), then the next epoch
        out = None
        for i in range(NL):
            out = ops.decode.layer_tail(att, x, L[i], L[(i + 1) % NL], eps, cache, i)
        cache.advance_device()
        return out

    def four():
        out = None
        for i in range(NL):
            l0, l1 = L[i], L[(i + 1) % NL]
            s, ssq = ops.decode.skinny_residual(att, l0.attn.o_proj, x)
            mm = ops.decode.skinny_normed(s, ssq, l0.ln2_w, eps, l0.mlp.up_proj, glu=True)
            s2, ssq2 = ops.decode.skinny_residual(mm, l0.mlp.down_proj, s)
            out = (s2, ops.decode.skinny_normed(s2, ssq2, l1.ln1_w, eps, l1.attn.qkv_proj))
        return out

    def timeit(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.iters / NL  # per layer

    with torch.no_grad():
        xo_t, q_t = tail()
        xo_f, q_f = four()
        torch.cuda.synchronize()
        same = bool(torch.equal(xo_t, xo_f.view_as(xo_t)) and torch.equal(q_t, q_f.view_as(q_t)))
        t_tail, t_four = timeit(tail), timeit(four)
        rec = {"batch": B, "tail_us": round(t_tail, 2), "four_launch_us": round(t_four, 2), "bitwise_equal": same,
               "err": int(cache.sync_err.item())}
        if os.environ.get("DLA_TAIL_STAMPS") == "1":
            tail()
            torch.cuda.synchronize()
            st = torch.ops.dla.decode_tail_stamps(x).cpu()
            nwg = torch.cuda.get_device_properties(0).multi_processor_count
            st = st[:nwg].double() * 10e-3  # 100 MHz ticks -> us
            t0 = st[:, 0].min()
            st = st - t0
            names = ["start", "O_done", "O_released", "GU_done", "GU_released", "DOWN_done", "DOWN_released", "end"]
            rec["edges_us"] = {n: [round(float(st[:, i].min()), 2), round(float(st[:, i].median()), 2),
                                   round(float(st[:, i].max()), 2)] for i, n in enumerate(names)}
            spans = {"O": st[:, 1] - st[:, 0], "wait0": st[:, 2] - st[:, 1], "GU": st[:, 3] - st[:, 2],
                     "wait1": st[:, 4] - st[:, 3], "DOWN": st[:, 5] - st[:, 4], "wait2": st[:, 6] - st[:, 5],
                     "QKV": st[:, 7] - st[:, 6]}
            rec["spans_us_min_med_max"] = {k: [round(float(v.min()), 2), round(float(v.median()), 2),
                                               round(float(v.max()), 2)] for k, v in spans.items()}
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
