"""`src.training.utils` helpers. `get_accelerator` returns the native runtime handle (RCCL
process group + device) exposing the accelerate attributes the reference scripts read."""
from __future__ import annotations

from pathlib import Path

import torch

from distributed_llm_alignment_amd.data.loader import get_distributed_sampler as _sampler
from distributed_llm_alignment_amd.parallel import dist as _dist
from distributed_llm_alignment_amd.training.common import seed_everything  # noqa: F401
from distributed_llm_alignment_amd.utils.config import flatten_dict, load_config, save_json  # noqa: F401
from distributed_llm_alignment_amd.utils.logging import RunningLoss  # noqa: F401


class Runtime:
    """accelerate-like view of the process group: is_main_process, num_processes,
    process_index, device, gather(), wait_for_everyone(), backward(), clip_grad_norm_()."""

    def __init__(self, config):
        self.state = _dist.init_distributed()
        self.gradient_accumulation_steps = int((config.get("hardware", {}) or {}).get("gradient_accumulation_steps", 1))

    @property
    def is_main_process(self):
        return self.state.is_main

    @property
    def num_processes(self):
        return self.state.world_size

    @property
    def process_index(self):
        return self.state.rank

    @property
    def device(self):
        return self.state.device

    def gather(self, t):
        return _dist.all_gather_tensor(t)

    def wait_for_everyone(self):
        _dist.barrier()

    def backward(self, loss):
        (loss / self.gradient_accumulation_steps).backward()

    def clip_grad_norm_(self, params, max_norm):
        return torch.nn.utils.clip_grad_norm_(list(params), max_norm)

    def broadcast(self, obj):
        return _dist.broadcast_object(obj)


def get_accelerator(config):
    return Runtime(config)


def prepare_output_dirs(*paths):
    for p in paths:
        Path(p).mkdir(parents=True, exist_ok=True)


def broadcast_config(accelerator, config):
    return _dist.broadcast_object(config)


def save_accelerator_state(accelerator, output_dir, tag, models=(), engine=None):
    from distributed_llm_alignment_amd.utils.checkpoint import save_state

    return save_state(Path(output_dir) / tag, list(models), engine)


def log_rank_zero(accelerator, message):
    if accelerator is None or accelerator.is_main_process:
        print(message, flush=True)


def get_distributed_sampler(dataset, accelerator=None, shuffle=True):
    return _sampler(dataset, shuffle=shuffle)


def maybe_clip_gradients(accelerator, model, max_norm):
    if max_norm and max_norm > 0:
        torch.nn.utils.clip_grad_norm_([p for p in model.parameters() if p.grad is not None], max_norm)


def yield_batch(iterable, accelerator):
    for batch in iterable:
        yield {k: (v.to(accelerator.device) if hasattr(v, "to") else v) for k, v in batch.items()}
