import os, sys, time, torch, torch.nn.functional as F
sys.path.insert(0, "/root/repo")
from distributed_llm_alignment_amd.utils.tuning import enable_gemm_tuning
from distributed_llm_alignment_amd.ops.linear import _LinearMainGradFn
print("mode", enable_gemm_tuning(0), flush=True)
dev = torch.device("cuda", 0)
M = 8192
def bench(fn, iters=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / iters
for name, N, K in [("qkv", 6144, 4096), ("o", 4096, 4096), ("up", 28672, 4096), ("down", 4096, 14336)]:
    W = (torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02).requires_grad_(True)
    W.main_grad = torch.zeros_like(W)
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16).requires_grad_(True)
    dY = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    t_direct = bench(lambda: dY @ W.detach())
    def ag():
        y = _LinearMainGradFn.apply(X, W, None)
        torch.autograd.backward(y, dY)
    t_fwd = bench(lambda: F.linear(X, W.detach()))
    t_ag = bench(ag)
    t_dw = bench(lambda: W.main_grad.addmm_(dY.t(), X.detach()))
    print(f"[p2] {name}: direct NN {t_direct*1e3:.3f} ms | fwd {t_fwd*1e3:.3f} | dW {t_dw*1e3:.3f} | autograd fwd+dX+dW {t_ag*1e3:.3f} (implied dX {1e3*(t_ag-t_fwd-t_dw):.3f})", flush=True)
