import sys, time, torch
sys.path.insert(0, "/root/repo")
from distributed_llm_alignment_amd.ops import _ext
tun = torch.cuda.tunable
tun.enable(True); tun.tuning_enable(True); tun.record_untuned_enable(False)
tun.set_max_tuning_iterations(20); tun.set_max_tuning_duration(30)
tun.set_filename("/tmp/probe_dw.csv", insert_device_ordinal=False)
dev = torch.device("cuda", 0)
M = 8192
T = _ext.require().transpose_bf16
def bench(fn, iters=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / iters * 1e3
for name, N, K in [("qkv", 6144, 4096), ("o", 4096, 4096), ("up", 28672, 4096), ("down", 4096, 14336)]:
    X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    dY = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    G = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
    Xt = torch.empty(K, M, device=dev, dtype=torch.bfloat16)
    dYt = torch.empty(N, M, device=dev, dtype=torch.bfloat16)
    t_nt = bench(lambda: G.addmm_(dY.t(), X))
    t_tx = bench(lambda: T(X, Xt))
    t_ty = bench(lambda: T(dY, dYt))
    T(X, Xt); T(dY, dYt)
    t_tn = bench(lambda: G.addmm_(dYt, Xt.t()))
    fl = 2.0 * M * N * K
    print(f"[dwtn] {name}: NT {t_nt:.3f} ms ({fl/t_nt/1e12:.0f} TF/s) | TN {t_tn:.3f} ms ({fl/t_tn/1e12:.0f} TF/s) + T(X) {t_tx:.3f} + T(dY) {t_ty:.3f}", flush=True)
