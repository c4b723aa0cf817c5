"""Decode GEMM bandwidth: skinny kernel (csrc/skinny.hip) vs the library GEMM (torch F.linear /
hipBLASLt with the TunableOp table) at Llama-3-8B decode shapes, B = 8 rows.

    python tools/skinny_bench.py [--rows 8] [--iters 200]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    import distributed_llm_alignment_amd  # noqa: F401
    from distributed_llm_alignment_amd.ops import decode
    from distributed_llm_alignment_amd.utils.tuning import enable_gemm_tuning

    enable_gemm_tuning(0)
    dev = torch.device("cuda", 0)
    shapes = [("qkv", 6144, 4096, False), ("o", 4096, 4096, False), ("gate_up", 28672, 4096, False),
              ("down(+swiglu)", 4096, 14336, True), ("lm_head", 128256, 4096, False)]
    torch.manual_seed(0)
    for name, N, K, sw in shapes:
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        x = torch.randn(a.rows, 2 * K if sw else K, device=dev).to(torch.bfloat16)
        with torch.no_grad():
            if sw:
                lib = lambda: F.linear(decode._ext.require().swiglu_fwd(x), w)
            else:
                lib = lambda: F.linear(x, w)
            sk = lambda: decode.skinny_linear(x, w, swiglu=sw, min_n=0)
            t_lib, t_sk = timeit(lib, a.iters), timeit(sk, a.iters)
        gb = N * K * 2 / 1e9
        print(json.dumps({"gemm": name, "rows": a.rows, "N": N, "K": K, "library_us": round(t_lib, 1),
                          "skinny_us": round(t_sk, 1), "library_TBps": round(gb / t_lib * 1e3, 2),
                          "skinny_TBps": round(gb / t_sk * 1e3, 2)}), flush=True)
        del w


if __name__ == "__main__":
    main()
