"""Host-side LR schedules with the HF `get_scheduler` formulas the reference uses
for SFT (src/training/train_sft.py:105-110): cosine / linear with linear warmup, constant."""
from __future__ import annotations

import math


class LRSchedule:
    def __init__(self, base_lr: float, name: str = "constant", warmup_steps: int = 0,
                 total_steps: int = 0, num_cycles: float = 0.5):
        self.base_lr = base_lr
        self.name = (name or "constant").lower()
        self.warmup = int(warmup_steps or 0)
        self.total = int(total_steps or 0)
        self.num_cycles = num_cycles
        self.last_step = 0

    def factor(self, step: int) -> float:
        if self.name in ("constant", "none"):
            return 1.0
        if step < self.warmup:
            return step / max(1, self.warmup)
        if self.name == "constant_with_warmup":
            return 1.0
        progress = (step - self.warmup) / max(1, self.total - self.warmup)
        if self.name == "linear":
            return max(0.0, 1.0 - progress)
        if self.name == "cosine":
            return max(0.0, 0.5 * (1.0 + math.cos(math.pi * self.num_cycles * 2.0 * progress)))
        raise ValueError(f"unknown lr_scheduler {self.name!r}")

    def lr(self, step: int = None) -> float:
        return self.base_lr * self.factor(self.last_step if step is None else step)

    def step(self):
        self.last_step += 1

    def state_dict(self):
        return {"base_lr": self.base_lr, "name": self.name, "warmup": self.warmup,
                "total": self.total, "last_step": self.last_step}

    def load_state_dict(self, d):
        self.last_step = int(d.get("last_step", 0))
