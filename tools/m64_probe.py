"""Decode projections at 17..64 rows (csrc/skinny64.hip m64 kernels + split-K reduce) timed one by
one at Llama-3-8B shapes, weights rotated over >= 1 GB so every call streams from HBM. The split
count is the most that keep the grid within one workgroup per CU; DLA_M64_WG=n (read once per
process) restores the round-3 rule (fewest splits reaching n workgroups), so A/B across processes:

    DLA_M64_WG=512 python tools/m64_probe.py [--rows 64]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--iters", type=int, default=60)
    a = ap.parse_args()
    import distributed_llm_alignment_amd  # noqa: F401
    from distributed_llm_alignment_amd.ops import decode

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    out = {"rows": a.rows, "m64_wg": os.environ.get("DLA_M64_WG", "auto")}
    with torch.no_grad():
        for name, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336)):
            ncopy = max(2, -(-(1 << 30) // (N * K * 2)))
            ws = [(torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16) for _ in range(ncopy)]
            x = torch.randn(a.rows, K, device=dev).to(torch.bfloat16)
            for w in ws:
                decode.skinny64_linear(x, w, tiled=True)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
            for it in range(a.iters):
                ev[it][0].record()
                decode.skinny64_linear(x, ws[it % ncopy], tiled=True)
                ev[it][1].record()
            torch.cuda.synchronize()
            ts = [s.elapsed_time(e) * 1e3 for s, e in ev[5:]]
            out[f"{name}_us"] = round(statistics.median(ts), 2)
            out[f"{name}_TBps"] = round(N * K * 2 / statistics.median(ts) / 1e6, 2)
            del ws
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
