"""Is the GEMM rate bounded by the kernel or by power/clock? Times one large bf16 GEMM
(8192 x 8192 x 8192, hipBLASLt) on operands with different bit activity: zeros, constant ones,
N(0,1) random, and sparse-random. A data-dependent rate means the clock is power-limited."""
import sys
import time

import torch


def rate(a, b, iters=30):
    for _ in range(5):
        a @ b
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        a @ b
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / iters
    return 2 * a.shape[0] * a.shape[1] * b.shape[1] / dt / 1e15


n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dev = "cuda"
cases = {
    "zeros": lambda: torch.zeros(n, n, device=dev, dtype=torch.bfloat16),
    "ones": lambda: torch.ones(n, n, device=dev, dtype=torch.bfloat16),
    "randn": lambda: torch.randn(n, n, device=dev, dtype=torch.bfloat16),
    "randn*1e-2": lambda: (torch.randn(n, n, device=dev) * 1e-2).bfloat16(),
    "10% nonzero": lambda: (torch.randn(n, n, device=dev) * (torch.rand(n, n, device=dev) < 0.1)).bfloat16(),
}
for name, mk in cases.items():
    a, b = mk(), mk()
    print(f"{name:12s} {rate(a, b):.3f} PF/s", flush=True)
a, b = cases["zeros"](), cases["zeros"]()
print(f"zeros again  {rate(a, b):.3f} PF/s", flush=True)
