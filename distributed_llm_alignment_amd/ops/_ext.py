"""Loader for the in-tree gfx950 extension (`_C.so`, ops under `torch.ops.dla`).

Policy (no silent fallbacks on the GPU):
  * GPU tensors ALWAYS go through the HIP kernels. If `_C.so` is missing or fails to load and a
    GPU op is requested, `require()` raises with the build command to run.
  * CPU tensors use the pure-PyTorch reference implementations in each op module (used by the
    CPU / gloo test tier and as numerics oracles), never the other way round.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

_LOCK = threading.Lock()
_STATE = {"loaded": False, "error": None}
# DLA_EXT_PATH: load an alternative build of the extension (A/B kernel experiments on one box)
SO_PATH = Path(os.environ.get("DLA_EXT_PATH") or Path(__file__).resolve().parent.parent / "_C.so")


def load(build_if_missing: bool | None = None) -> bool:
    """Load `_C.so` once. Optionally build it first (env DLA_AUTOBUILD=1 or argument)."""
    with _LOCK:
        if _STATE["loaded"]:
            return True
        if build_if_missing is None:
            build_if_missing = os.environ.get("DLA_AUTOBUILD", "0") == "1"
        try:
            if not SO_PATH.exists() and build_if_missing:
                from .. import _build

                _build.build()
            if not SO_PATH.exists():
                raise FileNotFoundError(str(SO_PATH))
            torch.ops.load_library(str(SO_PATH))
            _STATE["loaded"] = True
            _STATE["error"] = None
        except Exception as exc:  # surfaced by require()
            _STATE["error"] = exc
        return _STATE["loaded"]


def available() -> bool:
    return _STATE["loaded"] or load()


def require():
    """Return the op namespace or raise loudly (GPU path must never fall back silently)."""
    if not available():
        raise RuntimeError(
            "distributed_llm_alignment_amd HIP extension is not loaded "
            f"({_STATE['error']!r}). Build it with: "
            "DLA_SKIP_EXT_LOAD=1 python -m distributed_llm_alignment_amd._build"
        )
    return torch.ops.dla


def use_native(*tensors: torch.Tensor) -> bool:
    """True when the op must run on the HIP kernels (any operand on the GPU)."""
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            return True
    return False
