"""Bandwidth of the HIP bf16 transpose (and the SwiGLU transposed-output kernels) at Llama-3-8B
DPO micro-batch shapes (8192 tokens)."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import distributed_llm_alignment_amd  # noqa: F401
from distributed_llm_alignment_amd.ops import _ext


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


C = _ext.require()
for R, K in [(8192, 4096), (8192, 6144), (8192, 14336), (4096, 14336)]:
    x = torch.randn(R, K, device="cuda", dtype=torch.bfloat16)
    o = torch.empty(K, R, device="cuda", dtype=torch.bfloat16)
    us = timeit(lambda: C.transpose_bf16(x, o))
    print(f"transpose [{R},{K}]: {us:.1f} us  {2 * x.numel() * 2 / us / 1e6:.2f} TB/s", flush=True)
gu = torch.randn(8192, 28672, device="cuda", dtype=torch.bfloat16)
d = torch.randn(8192, 14336, device="cuda", dtype=torch.bfloat16)
us = timeit(lambda: C.swiglu_fwd_t(gu), 20)
print(f"swiglu_fwd_t: {us:.1f} us  {(gu.numel() + 2 * d.numel()) * 2 / us / 1e6:.2f} TB/s", flush=True)
us = timeit(lambda: C.swiglu_bwd_t(gu, d), 20)
print(f"swiglu_bwd_t: {us:.1f} us  {(3 * gu.numel() + d.numel()) * 2 / us / 1e6:.2f} TB/s", flush=True)
us = timeit(lambda: C.swiglu_fwd(gu), 20)
print(f"swiglu_fwd:   {us:.1f} us  {(gu.numel() + d.numel()) * 2 / us / 1e6:.2f} TB/s", flush=True)
us = timeit(lambda: C.swiglu_bwd(gu, d), 20)
print(f"swiglu_bwd:   {us:.1f} us  {(2 * gu.numel() + d.numel()) * 2 / us / 1e6:.2f} TB/s", flush=True)
