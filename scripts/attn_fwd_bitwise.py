"""Forward-attention outputs (O and LSE-dependent backward grads) over a fixed set of shapes,
saved to / compared with a file: run once per kernel variant (e.g. DLA_ATTN_FWD_PERSIST=0, then
=1 with --compare) to check that two builds / paths give bitwise-equal results.

    python scripts/attn_fwd_bitwise.py OUT.pt            # save
    python scripts/attn_fwd_bitwise.py OUT.pt --compare  # compare with the saved file"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from distributed_llm_alignment_amd import ops

    path, compare = sys.argv[1], "--compare" in sys.argv
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    cases = [(8, 1024, 1024, True, False), (2, 1000, 1000, True, True), (3, 517, 517, False, True),
             (2, 300, 812, True, False), (1, 64, 64, True, False)]
    for B, Tq, Tk, causal, pad in cases:
        q = torch.randn(B, Tq, 32, 128, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
        k = torch.randn(B, Tk, 8, 128, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
        v = torch.randn(B, Tk, 8, 128, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
        ks = ke = None
        if pad:
            ks = (torch.arange(B, device=dev) * 37 % 61).to(torch.int32)
            ke = (Tk - torch.arange(B, device=dev) * 13 % 29).to(torch.int32)
        o = ops.attention_core(q, k, v, causal=causal, kv_start=ks, kv_end=ke)
        do = torch.randn(o.shape, device=dev, generator=g).to(torch.bfloat16)
        gq, gk, gv = torch.autograd.grad(o, [q, k, v], do)
        res[f"{B}x{Tq}x{Tk}c{int(causal)}p{int(pad)}"] = [t.detach().cpu() for t in (o, gq, gk, gv)]
    if not compare:
        torch.save(res, path)
        print("saved", len(res))
        return 0
    ref = torch.load(path, weights_only=True)
    bad = 0
    for key, ts in res.items():
        for name, a, b in zip(("o", "dq", "dk", "dv"), ts, ref[key]):
            if not torch.equal(a, b):
                bad += 1
                print("DIFF", key, name, float((a.float() - b.float()).abs().max()))
    print("bitwise equal" if bad == 0 else f"{bad} tensors differ")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
