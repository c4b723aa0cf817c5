import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_alignment_amd.models import build_model, get_config
from distributed_llm_alignment_amd.models import generation as G
from distributed_llm_alignment_amd.ops import _ext
from distributed_llm_alignment_amd.utils.tuning import enable_gemm_tuning
dev = torch.device("cuda", 0); _ext.require(); enable_gemm_tuning(0)
cfg = get_config("llama3-8b"); m = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
ids = torch.randint(3, cfg.vocab_size, (8, 1024), device=dev)
orig_cap, orig_rep = G._DecodeGraph.capture, G._DecodeGraph.replay
T = {}
def cap(self):
    torch.cuda.synchronize(); t = time.perf_counter(); orig_cap(self); torch.cuda.synchronize(); T["capture"] = time.perf_counter() - t
G._DecodeGraph.capture = cap
for it in range(3):
    torch.cuda.synchronize(); t = time.perf_counter()
    G.generate(m, ids, torch.ones_like(ids), max_new_tokens=64, do_sample=True, temperature=0.7, top_p=0.9, eos_token_id=-1, use_graph=True, seed=1)
    torch.cuda.synchronize(); print(os.environ.get("DLA_SKINNY"), "total", round(time.perf_counter() - t, 3), "capture", round(T["capture"], 3), flush=True)
