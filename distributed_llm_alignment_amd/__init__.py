"""distributed_llm_alignment_amd — MI355X-native (gfx950 / CDNA4) distributed LLM alignment.

SFT, pairwise reward modelling, DPO, KL-penalised policy-gradient RLHF, teacher rollout
generation and CE / ensemble-KL distillation, with the reference's CLI, YAML schema, JSONL data
schemas and accelerate-style checkpoint layout (nikhil-lalgudi/distributed-llm-alignment), on
native models whose hot path runs hand-written HIP kernels (`csrc/`, `torch.ops.dla`) and whose
scaling runs RCCL collectives over xGMI (`parallel/`).
"""
__version__ = "0.1.0"

from .ops import _ext as _ext  # noqa: F401  (loads csrc/_C.so when present)

_ext.load()
