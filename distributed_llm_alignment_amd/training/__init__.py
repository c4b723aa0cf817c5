"""Trainer entry points (reference layer L6/L7): SFT, reward, DPO, RLHF, distillation, teacher
rollout generation. Each module exposes `main(argv=None)` with the reference CLI contract."""
from .common import TrainContext, make_engine, seed_everything, setup, train_loop

__all__ = ["TrainContext", "make_engine", "seed_everything", "setup", "train_loop"]
