import sys, time, torch
sys.path.insert(0, "/root/repo")
from distributed_llm_alignment_amd.ops import decode, _ext
_ext.require()
dev = torch.device("cuda", 0)
for dist in ("randn", "peaked"):
    g = torch.Generator(device=dev).manual_seed(0)
    lg = torch.randn(8, 128256, device=dev, generator=g)
    if dist == "peaked":
        lg = lg * 4.0
    lg = lg.to(torch.bfloat16)
    rng = torch.tensor([1, 0], dtype=torch.long, device=dev)
    for name, (t, k, p, gr) in {"greedy": (1.0, 0, 1.0, True), "temp": (0.7, 0, 1.0, False),
                                "top_p": (0.7, 0, 0.9, False), "top_k": (0.7, 50, 1.0, False),
                                "k+p": (0.7, 50, 0.9, False)}.items():
        for _ in range(3): decode.sample_tokens(lg, t, k, p, gr, rng)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(20): decode.sample_tokens(lg, t, k, p, gr, rng)
        torch.cuda.synchronize()
        print(f"[samp] {dist:6s} {name:7s} {(time.perf_counter()-t0)/20*1e6:8.1f} us", flush=True)
