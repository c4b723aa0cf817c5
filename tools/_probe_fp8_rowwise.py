import torch, time
dev = torch.device("cuda", 0)
M, K, N = 4096, 4096, 14336
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
def q_rows(t):
    amax = t.abs().amax(dim=1, keepdim=True).float().clamp(min=1e-12)
    s = 448.0 / amax
    return (t.float() * s).clamp(-448, 448).to(torch.float8_e4m3fn), (1.0 / s)
xq, sx = q_rows(x)
wq, sw = q_rows(w)
try:
    y = torch._scaled_mm(xq, wq.t(), scale_a=sx, scale_b=sw.t(), out_dtype=torch.bfloat16)
    ref = x.float() @ w.float().t()
    print("rowwise ok rel", ((y.float() - ref).norm() / ref.norm()).item(), flush=True)
    for _ in range(3): torch._scaled_mm(xq, wq.t(), scale_a=sx, scale_b=sw.t(), out_dtype=torch.bfloat16)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(20): torch._scaled_mm(xq, wq.t(), scale_a=sx, scale_b=sw.t(), out_dtype=torch.bfloat16)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 20
    print(f"fp8 rowwise {dt*1e3:.3f} ms {2*M*N*K/dt/1e15:.2f} PF/s", flush=True)
except Exception as e:
    print("rowwise failed:", repr(e)[:300], flush=True)
st = torch.tensor(1.0, device=dev)
for _ in range(3): torch._scaled_mm(xq, wq.t(), scale_a=st, scale_b=st, out_dtype=torch.bfloat16)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(20): torch._scaled_mm(xq, wq.t(), scale_a=st, scale_b=st, out_dtype=torch.bfloat16)
torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 20
print(f"fp8 tensorwise {dt*1e3:.3f} ms {2*M*N*K/dt/1e15:.2f} PF/s", flush=True)
for _ in range(3): x @ w.t()
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(20): x @ w.t()
torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 20
print(f"bf16 {dt*1e3:.3f} ms {2*M*N*K/dt/1e15:.2f} PF/s", flush=True)
