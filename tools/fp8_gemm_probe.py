#!/usr/bin/env python
"""Is hipBLASLt's fp8 GEMM (torch._scaled_mm, e4m3fn, per-row / per-tensor scales) available and
how fast is it against bf16 at the Llama-3-8B DPO GEMM shapes (M = 8192 tokens)? One JSON line per
shape; errors are reported, not raised."""
import json
import time

import torch


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    dev = torch.device("cuda", 0)
    for N, K in ((6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)):
        M = 8192
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        flops = 2.0 * M * N * K
        rec = {"M": M, "N": N, "K": K}
        rec["bf16_tflops"] = round(flops / bench(lambda: x @ w.t()) / 1e12, 1)
        for mode in ("tensor", "row"):
            try:
                if mode == "tensor":
                    sx = (x.abs().amax().float() / 448).reshape(())
                    sw = (w.abs().amax().float() / 448).reshape(())
                    xq = (x.float() / sx).to(torch.float8_e4m3fn)
                    wq = (w.float() / sw).to(torch.float8_e4m3fn)
                    fn = lambda: torch._scaled_mm(xq, wq.t(), scale_a=sx, scale_b=sw, out_dtype=torch.bfloat16)
                else:
                    sx = (x.abs().amax(1, keepdim=True).float() / 448)
                    sw = (w.abs().amax(1, keepdim=True).float() / 448)
                    xq = (x.float() / sx).to(torch.float8_e4m3fn)
                    wq = (w.float() / sw).to(torch.float8_e4m3fn)
                    fn = lambda: torch._scaled_mm(xq, wq.t(), scale_a=sx, scale_b=sw.t(), out_dtype=torch.bfloat16)
                y = fn()
                ref = (x.float() @ w.float().t())
                rec[f"fp8_{mode}_tflops"] = round(flops / bench(fn) / 1e12, 1)
                rec[f"fp8_{mode}_rel_err"] = round(float((y.float() - ref).norm() / ref.norm()), 4)
            except Exception as e:  # noqa: BLE001
                rec[f"fp8_{mode}_error"] = f"{type(e).__name__}: {str(e)[:160]}"
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
