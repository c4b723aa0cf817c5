#!/usr/bin/env python
"""How far the weight-only fp8 decode (ops.decode.fp8_weights) moves one decode step's logits at a
real model size: Llama-3-8B shapes, random init (no checkpoint is available offline, so this is a
numerics probe, not a quality benchmark), B rows after a prompt prefill. Prints one JSON line:
relative L2 error of the logits, top-1 agreement, mean KL(bf16 || fp8) of the softmax at T = 1.

    python tools/fp8_decode_probe.py [--batch 8 --prompt 512 --layers 32]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--layers", type=int, default=None)
    a = ap.parse_args()
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.models.generation import KVCache

    dev = torch.device("cuda", 0)
    ops._ext.require()
    cfg = get_config(a.model, **({"num_layers": a.layers} if a.layers else {}))
    m = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0).eval()
    g = torch.Generator(device=dev).manual_seed(0)
    ids = torch.randint(3, cfg.vocab_size, (a.batch, a.prompt), device=dev, generator=g)
    nxt = torch.randint(3, cfg.vocab_size, (a.batch, 1), device=dev, generator=g)
    out = {}
    with torch.no_grad():
        for dt in ("bf16", "fp8"):
            with ops.decode.fp8_weights(dt == "fp8"):
                cache = KVCache(m, a.batch, a.prompt + 4, None)
                m(ids, cache=cache)
                out[dt] = m.logits(m(nxt, cache=cache)[:, -1]).float()
        # control: the same bf16 weights, every op in fp32 (plain torch), on the full sequence --
        # what bf16 arithmetic alone moves the logits by at this depth
        ref = _fp32_logits(m, torch.cat([ids, nxt], 1))
    b, f = out["bf16"], out["fp8"]

    def cmp(x, y):
        lx, ly = torch.log_softmax(x, -1), torch.log_softmax(y, -1)
        kl = (ly.exp() * (ly - lx)).sum(-1)  # KL(y || x)
        return {"rel_l2": round(float((x - y).norm() / y.norm()), 5),
                "top1_agree": round(float((x.argmax(-1) == y.argmax(-1)).float().mean()), 4),
                "kl_mean": round(float(kl.mean()), 6)}

    print(json.dumps({"model": cfg.name, "layers": cfg.num_layers, "batch": a.batch, "prompt": a.prompt,
                      "logits_std_fp32": round(float(ref.std()), 4),
                      "bf16_decode_vs_fp32": cmp(b, ref), "fp8_decode_vs_fp32": cmp(f, ref),
                      "fp8_vs_bf16_decode": cmp(f, b),
                      "data": "random-init weights, random prompt ids"}), flush=True)


def _fp32_logits(m, ids):
    """Last-position logits of a native Llama model computed in fp32 with plain torch ops."""
    import math

    from distributed_llm_alignment_amd.ops.attention import _ref_rope, ref_attention
    from distributed_llm_alignment_amd.ops.norm import _ref_norm

    cfg = m.cfg
    B, T = ids.shape
    Hq, Hkv, D = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
    cos, sin = m.rope.tables(ids.device)
    pos = torch.arange(T, device=ids.device).expand(B, T)
    x = m.embed[ids].float()
    for layer in m.layers:
        h = _ref_norm(x, layer.ln1_w.float(), None, cfg.norm_eps, True)
        qkv = h @ layer.attn.qkv_proj.float().t()
        q = qkv[..., : Hq * D].reshape(B, T, Hq, D)
        k = qkv[..., Hq * D:(Hq + Hkv) * D].reshape(B, T, Hkv, D)
        v = qkv[..., (Hq + Hkv) * D:].reshape(B, T, Hkv, D)
        q = _ref_rope(q, cos, sin, pos, m.rope.rot_dim)
        k = _ref_rope(k, cos, sin, pos, m.rope.rot_dim)
        a = ref_attention(q, k, v, 1.0 / math.sqrt(D), True, 0, 0, None, None).float().reshape(B, T, Hq * D)
        x = x + a @ layer.attn.o_proj.float().t()
        h2 = _ref_norm(x, layer.ln2_w.float(), None, cfg.norm_eps, True)
        gu = h2 @ layer.mlp.up_proj.float().t()
        gt, up = gu.chunk(2, -1)
        x = x + (torch.nn.functional.silu(gt) * up) @ layer.mlp.down_proj.float().t()
    x = _ref_norm(x[:, -1], m.norm_w.float(), None, cfg.norm_eps, True)
    return x @ m.head_weight.float().t()


if __name__ == "__main__":
    main()
