"""Metrics / logging: the reference logs through `accelerator.log` but never calls
`init_trackers`, so nothing is recorded (Appendix A #3). Here a JSONL sink in `logging.log_dir`
is always on (rank 0), wandb is optional, and metric names follow the reference
(`train/loss`, `eval/loss`, `eval/acc`, `train/preference_rate`, `train/kl`,
`train/reward_mean`). Device tensors are converted only when a line is written."""
from __future__ import annotations

import json
import os
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, Optional

import torch


@dataclass
class RunningLoss:
    """Streaming mean between log points (reference utils.py:39-52). Accepts device tensors
    and defers the host sync to `.average`."""

    total: Any = 0.0
    count: int = 0

    def update(self, value, n: int = 1) -> None:
        if isinstance(value, torch.Tensor):
            value = value.detach().float()
        self.total = self.total + value * n
        self.count += n

    @property
    def average(self) -> float:
        t = self.total
        if isinstance(t, torch.Tensor):
            t = float(t.item())
        return t / max(self.count, 1)


def _to_py(v):
    if isinstance(v, torch.Tensor):
        return v.detach().float().item() if v.numel() == 1 else v.detach().float().cpu().tolist()
    return v


class MetricsLogger:
    def __init__(self, log_dir: Optional[str], is_main: bool = True, use_wandb: bool = False,
                 project: str = "distributed-llm-alignment-amd", config: Optional[dict] = None,
                 run_name: Optional[str] = None):
        self.is_main = is_main
        self.fh = None
        self.wandb = None
        if is_main and log_dir:
            Path(log_dir).mkdir(parents=True, exist_ok=True)
            self.path = Path(log_dir) / "metrics.jsonl"
            self.fh = self.path.open("a", encoding="utf-8")
        if is_main and use_wandb:
            try:
                import wandb  # noqa: WPS433

                self.wandb = wandb.init(project=project, config=config or {}, name=run_name,
                                        mode=os.environ.get("WANDB_MODE", "offline"))
            except Exception:  # wandb absent/offline: JSONL remains the source of truth
                self.wandb = None

    def log(self, metrics: Dict[str, Any], step: int) -> None:
        if not self.is_main:
            return
        rec = {k: _to_py(v) for k, v in metrics.items()}
        rec["step"] = step
        rec["time"] = time.time()
        if self.fh:
            self.fh.write(json.dumps(rec) + "\n")
            self.fh.flush()
        if self.wandb is not None:
            self.wandb.log({k: v for k, v in rec.items() if k not in ("step", "time")}, step=step)

    def close(self):
        if self.fh:
            self.fh.close()
            self.fh = None
        if self.wandb is not None:
            self.wandb.finish()


def log_rank_zero(message: str, is_main: Optional[bool] = None) -> None:
    if is_main is None:
        from ..parallel.dist import is_main as _im

        is_main = _im()
    if is_main:
        print(message, flush=True)


class StepTimer:
    """Wall-clock throughput / MFU tracker."""

    def __init__(self, flops_per_sample: float = 0.0, peak_tflops: float = 2500.0):
        self.flops = flops_per_sample
        self.peak = peak_tflops
        self.t0 = None
        self.samples = 0

    def start(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.t0 = time.perf_counter()
        self.samples = 0

    def add(self, n: int):
        self.samples += n

    def stats(self, world: int = 1) -> Dict[str, float]:
        if self.t0 is None:
            return {}
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dt = time.perf_counter() - self.t0
        sps = self.samples * world / max(dt, 1e-9)
        out = {"perf/samples_per_s": sps}
        if self.flops:
            tf = sps * self.flops / world / 1e12
            out["perf/tflops_per_gpu"] = tf
            out["perf/mfu"] = tf / self.peak
        return out
