"""Does reading a decode kernel's operand into the 256 MiB Infinity Cache beforehand make the kernel
faster? Llama-3-8B decode shapes at B = 8 (qkv, o, gate|up, down on the skinny kernels, and the
decode attention over a 1152-slot KV cache).

For each kernel the weights rotate over enough copies (>= 1 GB) that a call never finds its own
operand left over from an earlier call, as in a real decode step. Before each timed call, the first
`frac` of the operand's bytes are read by a reduction; the call alone is timed with events.
`--concurrent` also times the call while a side stream reads the NEXT call's operand.

    python tools/ic_prefetch_probe.py [--iters 40]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _touch(t: torch.Tensor, frac: float, out: torch.Tensor) -> None:
    v = t.reshape(-1)
    n = int(v.numel() * frac) // 4096 * 4096
    if n:
        torch.amax(v[:n].view(-1, 4096), dim=0, out=out)


def probe(name, ops, targets, iters, fracs, concurrent, nbytes):
    dev = targets[0].device
    out = torch.empty(4096, dtype=targets[0].dtype, device=dev)
    out2 = torch.empty(4096, dtype=targets[0].dtype, device=dev)
    side = torch.cuda.Stream(dev)
    n = len(ops)
    for i in range(n):
        ops[i]()
    torch.cuda.synchronize()
    res = {"kernel": name, "MB": round(nbytes / 1e6, 1)}
    for frac in fracs:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for it in range(iters):
            i = it % n
            _touch(targets[i], frac, out)
            ev[it][0].record()
            ops[i]()
            ev[it][1].record()
        torch.cuda.synchronize()
        ts = [a.elapsed_time(b) * 1e3 for a, b in ev[4:]]
        res[f"us_pre{int(frac * 100)}"] = round(statistics.median(ts), 2)
    if concurrent:
        for frac in concurrent:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
            main = torch.cuda.current_stream(dev)
            for it in range(iters):
                i = it % n
                ev[it][0].record()
                side.wait_event(ev[it][0])
                with torch.cuda.stream(side):
                    _touch(targets[(i + 1) % n], frac, out2)
                ops[i]()
                ev[it][1].record()
                main.wait_stream(side)
            torch.cuda.synchronize()
            ts = [a.elapsed_time(b) * 1e3 for a, b in ev[4:]]
            res[f"us_with_side_read{int(frac * 100)}"] = round(statistics.median(ts), 2)
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--rows", type=int, default=8)
    a = ap.parse_args()
    import distributed_llm_alignment_amd  # noqa: F401
    from distributed_llm_alignment_amd.ops import decode

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B, H = a.rows, 4096
    fracs = (0.0, 0.25, 0.5, 1.0)
    eps = 1e-5
    with torch.no_grad():
        x = (torch.randn(B, H, device=dev)).to(torch.bfloat16)
        res = (torch.randn(B, H, device=dev)).to(torch.bfloat16)
        nw = (1 + 0.1 * torch.randn(H, device=dev)).to(torch.bfloat16)
        for name, N, K, kind in (("qkv", 6144, 4096, "normed"), ("o", 4096, 4096, "resid"),
                                 ("gate_up", 28672, 4096, "glu"), ("down", 4096, 14336, "resid")):
            ncopy = max(2, -(-(1 << 30) // (N * K * 2)))
            ws = [(torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16) for _ in range(ncopy)]
            if kind == "resid":
                xin = (torch.randn(B, K, device=dev)).to(torch.bfloat16)
                ops = [lambda w=w: decode.skinny_residual(xin, w, res) for w in ws]
                targets = [decode.tiled_weight(w) for w in ws]
            else:
                s, ssq = decode.skinny_residual(x, torch.randn(H, H, device=dev).to(torch.bfloat16) * 0.01, res)
                ops = [lambda w=w: decode.skinny_normed(s, ssq, nw, eps, w, glu=kind == "glu") for w in ws]
                targets = [decode.folded_weight(w, nw, tiled=True) for w in ws]
            probe(name, ops, targets, a.iters, fracs, (0.25, 1.0), N * K * 2)
            del ws, ops, targets
            torch.cuda.empty_cache()
        # decode attention: q [B, 32, 128], caches [B, 1152, 8, 128], 1024 + 1 keys
        Hq, Hkv, D, T = 32, 8, 128, 1152
        ncopy = max(2, -(-(1 << 30) // (2 * B * T * Hkv * D * 2)))
        kvs = [torch.randn(2, B, T, Hkv, D, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
        q = torch.randn(B, Hq, D, device=dev).to(torch.bfloat16)
        L = torch.tensor([1025], dtype=torch.int32, device=dev)
        ops = [lambda kv=kv: decode.decode_attention(q, kv[0], kv[1], L) for kv in kvs]
        probe("decode_attn", ops, kvs, a.iters, fracs, (0.25, 1.0), kvs[0].numel() * 2)


if __name__ == "__main__":
    main()
