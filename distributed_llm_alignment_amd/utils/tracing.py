"""Tracing and profiling (the reference has none beyond `time.perf_counter` in
src/eval/eval_latency.py:45-53).

* `trace_range(name)`: a roctx range (ROCm's marker API, `libroctx64.so`, loaded with ctypes —
  no CUDA NVTX shim) around a host phase, visible in `rocprofv3 --marker-trace` timelines next to
  the kernels it launched; a no-op when roctx is absent (CPU containers). Also accumulates host
  wall time per phase for the metrics log.
* `ProfileWindow`: `torch.profiler` over a step window (config `logging.profile_steps: [a, b]`,
  `logging.profile_dir`), exporting a Chrome trace and a per-kernel table; the rocprofv3 recipe
  for counters is in README (run the trainer under `rocprofv3 --kernel-trace --stats`).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict
from pathlib import Path
from typing import Dict, Optional, Sequence

_ROCTX = None
_ROCTX_TRIED = False


def _roctx():
    global _ROCTX, _ROCTX_TRIED
    if _ROCTX_TRIED:
        return _ROCTX
    _ROCTX_TRIED = True
    if os.environ.get("DLA_ROCTX", "1") == "0":
        return None
    for name in ("libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _ROCTX = lib
            break
        except OSError:
            continue
    return _ROCTX


class PhaseTimes:
    """Host wall time per traced phase since the last `pop()`."""

    def __init__(self):
        self.t: Dict[str, float] = defaultdict(float)

    def add(self, name: str, dt: float):
        self.t[name] += dt

    def pop(self) -> Dict[str, float]:
        out = {f"time/{k}_s": v for k, v in self.t.items()}
        self.t = defaultdict(float)
        return out


PHASES = PhaseTimes()


@contextlib.contextmanager
def trace_range(name: str):
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    try:
        yield
    finally:
        PHASES.add(name, time.perf_counter() - t0)
        if lib is not None:
            lib.roctxRangePop()


def mark(msg: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(msg.encode())


class ProfileWindow:
    """torch.profiler active for steps [start, end) (1-based global steps)."""

    def __init__(self, steps: Optional[Sequence[int]], out_dir: str, enabled: bool = True):
        self.start, self.end = (int(steps[0]), int(steps[1])) if steps else (0, 0)
        self.dir = Path(out_dir)
        self.enabled = enabled and self.end > self.start
        self.prof = None

    def step(self, global_step: int) -> None:
        if not self.enabled:
            return
        if global_step == self.start and self.prof is None:
            import torch
            from torch.profiler import ProfilerActivity, profile

            acts = [ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(ProfilerActivity.CUDA)
            self.prof = profile(activities=acts, record_shapes=False)
            self.prof.__enter__()
        elif global_step == self.end and self.prof is not None:
            self.close()

    def close(self) -> None:
        if self.prof is None:
            return
        import torch

        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.prof.__exit__(None, None, None)
        self.dir.mkdir(parents=True, exist_ok=True)
        self.prof.export_chrome_trace(str(self.dir / "trace.json"))
        key = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
        (self.dir / "kernels.txt").write_text(self.prof.key_averages().table(sort_by=key, row_limit=80))
        self.prof = None
        self.enabled = False
