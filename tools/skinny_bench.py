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
        # rotate over enough weight copies (>= 1 GB) that no call finds its weights in the 256 MB
        # Infinity Cache, as in a real decode step (16 GB of weights between two uses)
        ncopy = max(1, -(-(1 << 30) // (N * K * 2)))
        ws = [(torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16) for _ in range(ncopy)]
        x = torch.randn(a.rows, 2 * K if sw else K, device=dev).to(torch.bfloat16)
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % ncopy
            return ws[it[0]]
        with torch.no_grad():
            if sw:
                lib = lambda: F.linear(decode._ext.require().swiglu_fwd(x), nxt())
            else:
                lib = lambda: F.linear(x, nxt())
            sk = lambda: decode.skinny_linear(x, nxt(), swiglu=sw, min_n=0)
            t_lib, t_sk = timeit(lib, a.iters), timeit(sk, a.iters)
            extra = {}
            if name == "gate_up":
                for mode in ("lds", "ks"):
                    extra[f"glu_{mode}_us"] = round(timeit(lambda: decode.skinny_glu(x, nxt(), mode=mode), a.iters), 1)
        gb = N * K * 2 / 1e9
        print(json.dumps({"gemm": name, "rows": a.rows, "N": N, "K": K, "library_us": round(t_lib, 1),
                          "skinny_us": round(t_sk, 1), "library_TBps": round(gb / t_lib * 1e3, 2),
                          "skinny_TBps": round(gb / t_sk * 1e3, 2), **extra}), flush=True)
        del ws


if __name__ == "__main__":
    main()
