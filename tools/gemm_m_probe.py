"""Per-layout GEMM rates of the dense projections at several token counts M, through the shipped
TunableOp table in read mode exactly as bench.py loads it (shapes missing from the table fall to
the library heuristic): forward Y = X W^T, input grad through the cached W^T (TN), weight grad TN.

    python tools/gemm_m_probe.py [--model mixtral-8x7b] [--ms 4096,8192] [--resid] [--cold]

--resid adds the residual-stream forms of the forward: torch.addmm(C, X, W^T) out of place (torch
copies C into the output first, then runs beta = 1) and C.addmm_(X, W^T) in place. --cold streams
a 1 GiB buffer between calls, so operands come from HBM as they do inside a training step.
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return statistics.median(s.elapsed_time(e) for s, e in ev) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mixtral-8x7b")
    ap.add_argument("--ms", default="4096,8192")
    ap.add_argument("--resid", action="store_true")
    ap.add_argument("--cold", action="store_true")
    a = ap.parse_args()
    from distributed_llm_alignment_amd.models import get_config
    from distributed_llm_alignment_amd.utils.tuning import enable_gemm_tuning

    mode = enable_gemm_tuning(0)
    cfg = get_config(a.model)
    H = cfg.hidden_size
    dev = torch.device("cuda", 0)
    shapes = [("qkv", cfg.q_size + 2 * cfg.kv_size, H), ("o", H, cfg.q_size)]
    if a.resid:
        shapes.append(("down", H, cfg.intermediate_size))
    for M in [int(x) for x in a.ms.split(",")]:
        for name, N, K in shapes:
            W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            Wt = W.t().contiguous()
            X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            dY = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
            dYt, Xt = dY.t().contiguous(), X.t().contiguous()
            G = torch.zeros(N, K, device=dev, dtype=torch.float32)
            fl = 2.0 * M * N * K
            r = {"model": a.model, "gemm": name, "M": M, "N": N, "K": K, "tuning": mode}
            C = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
            flush = torch.empty(1 << 29, device=dev, dtype=torch.bfloat16) if a.cold else None
            arms = [("fwd", lambda: F.linear(X, W)), ("dgrad_tn", lambda: F.linear(dY, Wt)),
                    ("wgrad_tn_f32", lambda: torch.addmm(G, dYt, Xt.t(), out_dtype=torch.float32, out=G))]
            if a.resid:
                arms += [("fwd_addmm", lambda: torch.addmm(C, X, W.t())), ("fwd_addmm_", lambda: C.addmm_(X, W.t()))]
            for tag, fn in arms:
                us = timeit((lambda fn=fn: (flush.fill_(1.0), fn())) if a.cold else fn)
                if a.cold:
                    us -= timeit(lambda: flush.fill_(1.0))
                r[f"{tag}_us"] = round(us, 1)
                r[f"{tag}_TFs"] = round(fl / us / 1e6, 0)
            print(json.dumps(r), flush=True)
            del W, Wt, X, dY, dYt, Xt, G, C, flush
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
