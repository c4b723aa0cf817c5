"""Debug probe: per-parameter gradient differences between no recompute and a selective policy
over 3 DPO steps on the GPU (tiny-llama-d128, DataParallelEngine)."""
import sys

import torch

from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
from distributed_llm_alignment_amd.models import build_model, get_config
from distributed_llm_alignment_amd.objectives import dpo_step_loss
from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine

policy = sys.argv[1] if len(sys.argv) > 1 else "mlp"
dev = torch.device("cuda", 0)


def run(pol_name):
    cfg = get_config("tiny-llama-d128")
    pol = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    ref = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0).requires_grad_(False)
    if pol_name:
        pol.gradient_checkpointing_enable(pol_name)
    eng = DataParallelEngine(pol, lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
    b = synthetic_preference_batch(2, 128, cfg.vocab_size, device=dev, generator=torch.Generator().manual_seed(5))
    grads, norms = [], []
    for _ in range(3):
        loss, _ = dpo_step_loss(pol, ref, b)
        loss.backward()
        grads.append({n: p.main_grad.float().clone() if getattr(p, "main_grad", None) is not None
                      else p.grad.float().clone() for n, p in pol.named_parameters()})
        norms.append(float(eng.step()))
    return grads, norms


ga, na = run(None)
gb, nb = run(policy)
print("norms", na, nb)
for s in range(3):
    bad = [(n, (ga[s][n] - gb[s][n]).abs().max().item(), ga[s][n].abs().max().item()) for n in ga[s]
           if not torch.allclose(ga[s][n], gb[s][n], rtol=2e-2, atol=1e-4)]
    print("step", s, "mismatching params:", len(bad))
    for x in bad[:12]:
        print("   ", x)
