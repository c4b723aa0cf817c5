"""Distributed runtime over RCCL (xGMI) / gloo: process groups, data parallel + ZeRO engine."""
from .data_parallel import DataParallelEngine
from .dist import (DistState, all_gather_tensor, all_reduce_, barrier, broadcast_object, destroy,
                   gather_objects, init_distributed, is_main, split_for_rank, state)

__all__ = ["DataParallelEngine", "DistState", "all_gather_tensor", "all_reduce_", "barrier",
           "broadcast_object", "destroy", "gather_objects", "init_distributed", "is_main",
           "split_for_rank", "state"]
