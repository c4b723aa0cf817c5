#!/usr/bin/env python
"""Rollout -> reward-model hand-off cost in isolation (training/handoff.py): the reference's
decode + re-tokenise text path (src/training/train_rlhf.py:131-147) against the device-built ids,
at equal sequence lengths (byte tokenizer, byte-range token ids so the text path keeps every
token: the full-vocabulary random models of tools/bench_rlhf.py would decode to empty strings
and make the text path look free). Prints one JSON line per (batch, path).

    python tools/bench_handoff.py [--batch 8,64] [--prompt 512] [--new 256]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", default="8,64")
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args(argv)
    from distributed_llm_alignment_amd.models.tokenizer import ByteTokenizer
    from distributed_llm_alignment_amd.training.handoff import RewardHandoff

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    tok = ByteTokenizer(vocab_size=512)
    g = torch.Generator().manual_seed(0)
    for B in (int(x) for x in a.batch.split(",")):
        # printable ASCII bytes: valid UTF-8, so decode -> encode round-trips every token
        ids = torch.randint(32 + tok.offset, 127 + tok.offset, (B, a.prompt), generator=g)
        ids[:, 0] = tok.bos_token_id
        am = torch.ones_like(ids)
        resp = torch.randint(32 + tok.offset, 127 + tok.offset, (B, a.new), generator=g)
        seqs = torch.cat([ids, resp], 1).to(dev)
        ids, am = ids.to(dev), am.to(dev)
        prompts = [tok.decode(r[1:].tolist()) for r in ids.cpu()]
        for path in ("text", "device"):
            h = RewardHandoff(tok, tok, tok.vocab_size, dev, a.prompt + a.new + 8, path)
            out = h(prompts, ids, am, seqs)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                out = h(prompts, ids, am, seqs)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.iters
            print(json.dumps({"bench": "reward_handoff", "path": path, "batch": B,
                              "tokens_per_row": int(out[1][0].sum()), "ms": round(dt * 1e3, 3)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
