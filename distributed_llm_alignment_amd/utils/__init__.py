"""Config, logging/metrics, checkpointing utilities."""
from .checkpoint import load_model_weights, load_state, resolve_checkpoint, save_state
from .config import (add_config_args, apply_override, config_from_args, deep_merge, flatten_dict,
                     hardware_parallel, load_config, save_json)
from .logging import MetricsLogger, RunningLoss, StepTimer, log_rank_zero

__all__ = ["load_model_weights", "load_state", "resolve_checkpoint", "save_state", "add_config_args",
           "apply_override", "config_from_args", "deep_merge", "flatten_dict", "hardware_parallel",
           "load_config", "save_json", "MetricsLogger", "RunningLoss", "StepTimer", "log_rank_zero"]
