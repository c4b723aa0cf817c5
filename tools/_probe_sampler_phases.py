"""Time the fused sampler per configuration (which phase costs what), 8 x 128256 bf16 logits."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_alignment_amd.ops import _ext, decode
_ext.require()
dev = torch.device("cuda", 0)
for scale in (0.05, 3.0):
    lg = (torch.randn(8, 128256, device=dev) * scale).to(torch.bfloat16)
    rng = torch.tensor([1, 0], dtype=torch.long, device=dev)
    for name, (t, k, p, g) in {"greedy": (0.7, 0, 1.0, True), "plain": (0.7, 0, 1.0, False),
                               "topk50": (0.7, 50, 1.0, False), "topp0.9": (0.7, 0, 0.9, False),
                               "topk50+topp0.9": (0.7, 50, 0.9, False)}.items():
        for _ in range(5):
            decode.sample_tokens(lg, t, k, p, g, rng)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            decode.sample_tokens(lg, t, k, p, g, rng)
        e.record()
        torch.cuda.synchronize()
        print(f"logit std {scale}: {name:16s} {s.elapsed_time(e) / 50 * 1e3:8.1f} us", flush=True)
