import sys, time, torch
sys.path.insert(0, "/root/repo")
from distributed_llm_alignment_amd.utils.tuning import enable_gemm_tuning
print("mode", enable_gemm_tuning(0), flush=True)
dev = torch.device("cuda", 0)
M = 8192
def bench(fn, iters=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / iters
buf = torch.zeros(400_000_000, device=dev, dtype=torch.bfloat16)
for name, N, K in [("qkv", 6144, 4096), ("o", 4096, 4096), ("up", 28672, 4096), ("down", 4096, 14336)]:
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    dY = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    res = []
    for off in (0, 64, 128, 256, 1024):
        G = buf[off:off + N * K].view(N, K)
        res.append((off, bench(lambda: G.addmm_(dY.t(), X)) * 1e3))
    Gf = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
    t_own = bench(lambda: Gf.addmm_(dY.t(), X)) * 1e3
    t_mm = bench(lambda: torch.mm(dY.t(), X)) * 1e3
    print(f"[dw] {name}: own {t_own:.3f} ms, mm(no beta) {t_mm:.3f} | views " + " ".join(f"off{o}:{t:.3f}" for o, t in res), flush=True)
