"""distributed_llm_alignment_amd — MI355X-native (gfx950 / CDNA4) distributed LLM alignment.

SFT, pairwise reward modelling, DPO, KL-penalised policy-gradient RLHF, teacher rollout
generation and CE / ensemble-KL distillation, with the reference's CLI, YAML schema, JSONL data
schemas and accelerate-style checkpoint layout (nikhil-lalgudi/distributed-llm-alignment), on
native models whose hot path runs hand-written HIP kernels (`csrc/`, `torch.ops.dla`) and whose
scaling runs RCCL collectives over xGMI (`parallel/`).
"""
__version__ = "0.1.0"

import os as _os

from .ops import _ext as _ext  # noqa: F401  (loads csrc/_C.so when present)

# DLA_SKIP_EXT_LOAD=1: do not load _C.so at import (the build entry sets it, so a stale library
# from an older source tree -- whose op schemas no longer match -- is rebuilt, never loaded first)
if _os.environ.get("DLA_SKIP_EXT_LOAD") != "1":
    _ext.load()
