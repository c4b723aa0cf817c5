"""Fused flat AdamW (HIP) + grad-norm clipping, and host-side LR schedules."""
from .adamw import adamw_update, clip_coefficient, grad_sumsq
from .scheduler import LRSchedule

__all__ = ["adamw_update", "clip_coefficient", "grad_sumsq", "LRSchedule"]
