#!/usr/bin/env python
"""Per-block phase times of the persistent attention forward (DLA_ATTN_STAMPS=1 build path:
csrc/attention.hip attn_fwd_persist_kernel `stamp`): for each workgroup and its first 8 blocks,
tiles (compute of the block's K/V tiles), enter (next Q read from LDS + next loads issued),
epilogue (O / LSE stores issued) and wait (barrier before the next block's first tile).

    DLA_ATTN_STAMPS=1 python tools/attn_seam_probe.py [--B 8 --T 1024] [--noncausal]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=8)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--noncausal", action="store_true")
    a = ap.parse_args()
    assert os.environ.get("DLA_ATTN_STAMPS") == "1"
    from distributed_llm_alignment_amd.ops import _ext

    C = _ext.require()
    dev = torch.device("cuda", 0)
    q = torch.randn(a.B, a.T, a.Hq, a.D, device=dev).to(torch.bfloat16)
    k = torch.randn(a.B, a.T, a.Hkv, a.D, device=dev).to(torch.bfloat16)
    v = torch.randn(a.B, a.T, a.Hkv, a.D, device=dev).to(torch.bfloat16)
    for _ in range(3):
        C.attn_fwd(q, k, v, a.D ** -0.5, not a.noncausal, 0, 0, None, None)
    torch.cuda.synchronize()
    st = C.attn_stamps(q).view(-1, 8, 4).double().cpu() * 1e-2  # 100 MHz ticks -> us
    nwg = torch.cuda.get_device_properties(0).multi_processor_count
    st = st[:nwg]
    ok = st[:, :, 0] > 0
    t0 = st[:, 0, 0][ok[:, 0]].min()
    rec = {"B": a.B, "T": a.T, "causal": not a.noncausal}
    spans = {"tiles": st[:, :, 1] - st[:, :, 0], "enter": st[:, :, 2] - st[:, :, 1],
             "epilogue": st[:, :, 3] - st[:, :, 2]}
    nxt = torch.roll(st[:, :, 0], -1, dims=1)
    spans["wait"] = nxt - st[:, :, 3]
    okw = ok & torch.roll(ok, -1, dims=1)
    okw[:, -1] = False
    for name, v in spans.items():
        m = okw if name == "wait" else ok
        x = v[m]
        rec[name + "_us"] = [round(float(x.min()), 2), round(float(x.median()), 2), round(float(x.max()), 2)]
    rec["first_start_us"] = [round(float((st[:, 0, 0] - t0).min()), 2), round(float((st[:, 0, 0] - t0).max()), 2)]
    last = torch.where(ok, st[:, :, 3], torch.zeros_like(st[:, :, 3])).max(dim=1).values
    rec["end_us"] = [round(float((last - t0).min()), 2), round(float((last - t0).max()), 2)]
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
