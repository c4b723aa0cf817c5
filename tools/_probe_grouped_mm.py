"""Probe: torch._grouped_mm on ROCm at the Mixtral expert shapes -- does it run device-driven
(graph-capturable, no host sync) and how fast vs the per-expert hipBLASLt loop."""
import time

import torch

dev = torch.device("cuda", 0)
E, H, F, rows = 8, 4096, 14336, 16384
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(rows, H, device=dev, generator=g).to(torch.bfloat16)
w = (torch.randn(E, 2 * F, H, device=dev, generator=g) * H ** -0.5).to(torch.bfloat16)
cnt = torch.full((E,), rows // E, dtype=torch.int32)
cnt[0] += 37
cnt[1] -= 37
offs = torch.cumsum(cnt, 0).to(torch.int32).to(dev)
wt = w.transpose(1, 2)  # [E, H, 2F]


def gm():
    return torch._grouped_mm(x, wt, offs=offs)


def loop():
    outs, a = [], 0
    for e, c in enumerate(cnt.tolist()):
        outs.append(x[a:a + c] @ w[e].t())
        a += c
    return torch.cat(outs)


try:
    y = gm()
    ref = loop()
    print("grouped_mm ok, rel err", float((y.float() - ref.float()).norm() / ref.float().norm()))
except Exception as e:  # noqa: BLE001
    print("grouped_mm failed:", repr(e)[:300])
    raise SystemExit(0)
for name, fn in (("grouped_mm", gm), ("loop", loop)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    print(f"{name}: {dt * 1e3:.3f} ms  {2 * rows * H * 2 * F / dt / 1e12:.0f} TFLOP/s", flush=True)
s = torch.cuda.Stream()
try:
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            yy = gm()
    gr.replay()
    torch.cuda.synchronize()
    print("graph capture ok (no host sync)")
except Exception as e:  # noqa: BLE001
    print("graph capture failed:", repr(e)[:300])
