"""Decode-attention microbenchmark (Llama-3-8B heads, B=8): fused rope + split-KV attention +
combine per call, timed from a captured hipGraph of 50 calls (no host launch cost), for several
cache lengths, both kernel versions (DLA_DECODE_ATTN_V1 is read once per process: run twice).

    python tools/decode_attn_bench.py [--lens 128,512,1152,4096]"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="128,512,1152,4096")
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=8)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--headmajor", type=int, default=0, help="cache stored [B, Hkv, Tmax, D]")
    a = ap.parse_args()
    from distributed_llm_alignment_amd.ops import RotaryCache, _ext

    C = _ext.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    B, Hq, Hkv, D = a.B, a.Hq, a.Hkv, a.D
    for L in [int(x) for x in a.lens.split(",")]:
        Tmax = L + 1
        rope = RotaryCache(D, 500000.0, Tmax + 8, None)
        cos, sin = rope.tables(dev)
        if a.headmajor:  # same logical [B, Tmax, Hkv, D] tensor, head-major storage
            kc = torch.randn(B, Hkv, Tmax, D, device=dev, generator=g).to(torch.bfloat16).transpose(1, 2)
            vc = torch.randn(B, Hkv, Tmax, D, device=dev, generator=g).to(torch.bfloat16).transpose(1, 2)
        else:
            kc = torch.randn(B, Tmax, Hkv, D, device=dev, generator=g).to(torch.bfloat16)
            vc = torch.randn(B, Tmax, Hkv, D, device=dev, generator=g).to(torch.bfloat16)
        qkv = torch.randn(B, 1, (Hq + 2 * Hkv) * D, device=dev, generator=g).to(torch.bfloat16)
        pos = torch.full((B,), L - 1, device=dev, dtype=torch.int32)
        slot = torch.tensor([L - 1], device=dev, dtype=torch.long)
        kv_len = torch.tensor([L], device=dev, dtype=torch.int32)

        def call():
            return C.decode_attn_rope(qkv, cos, sin, pos, kc, vc, slot, kv_len, None, 0, D ** -0.5,
                                      Hq, Hkv, D, D)

        call()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(50):
                call()
        graph.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            s.record()
            graph.replay()
            e.record()
            torch.cuda.synchronize()
            best = min(best, s.elapsed_time(e) / 50)
        mb = 2 * B * L * Hkv * D * 2 / 1e6
        print(json.dumps({"kv_len": L, "us": round(best * 1e3, 2), "kv_MB": round(mb, 1),
                          "TB_s": round(mb / 1e6 / (best * 1e-3), 2),
                          "v1": os.environ.get("DLA_DECODE_ATTN_V1", "0"),
                          "headmajor": a.headmajor}), flush=True)


if __name__ == "__main__":
    main()
