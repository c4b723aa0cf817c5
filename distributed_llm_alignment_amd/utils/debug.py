"""Correctness tooling for distributed runs (SURVEY §5.2 race detection / sanitizers and §5.3
failure detection / fault injection; the reference has none).

* `replica_checksums` / `check_replicas_in_sync`: after an optimizer step every data-parallel
  replica must hold bit-identical weights (ZeRO shards all-gathered, TP shards compared within
  their own DP group); a per-rank fp64 checksum of the parameters is all-gathered over the DP
  group and compared — catches a missed/duplicated gradient bucket, a stream race between the
  reduce-scatter and AdamW, or a rank that silently diverged.
* `determinism_check`: run the same closure twice from identical seeds and compare the losses
  bitwise (atomics-free kernels: the flash-attention dQ uses fp32 atomics, so the check is
  opt-in per op set).
* `FaultInjector`: `DLA_FAULT_STEP=<s>` (optionally `DLA_FAULT_RANK=<r>`) makes the training loop
  die at global step s — exercised by the resume tests (kill, restart from `latest`, compare the
  loss trajectory with an uninterrupted run).
* `debug_env()`: the HIP settings for a serialised debug run (`AMD_SERIALIZE_KERNEL=3`,
  `HIP_LAUNCH_BLOCKING=1`) and RCCL async error handling, to export BEFORE the process starts
  (scripts/_launch_common.sh does this when DLA_DEBUG=1).
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist


def param_checksum(module: torch.nn.Module) -> torch.Tensor:
    s = torch.zeros((), dtype=torch.float64, device=next(module.parameters()).device)
    for i, p in enumerate(module.parameters()):
        if p.numel() == 0 or p.untyped_storage().size() == 0:  # resharded ZeRO-3 unit
            continue
        s += p.detach().double().sum() * (1.0 + 1e-3 * (i % 97))
    return s


def replica_checksums(module: torch.nn.Module, group=None) -> List[float]:
    c = param_checksum(module).reshape(1)
    if not (dist.is_available() and dist.is_initialized()):
        return [float(c)]
    ws = dist.get_world_size(group)
    out = [torch.zeros_like(c) for _ in range(ws)]
    dist.all_gather(out, c, group=group)
    return [float(x) for x in out]


def check_replicas_in_sync(module: torch.nn.Module, group=None, rtol: float = 0.0) -> None:
    """Raise if data-parallel replicas hold different weights (collective over `group`)."""
    eng = getattr(module, "_dla_fsdp", None)
    if eng is not None:
        return  # ZeRO-3: ranks hold disjoint shards by design
    dp = getattr(module, "_dla_dp_engine", None)
    if dp is not None:
        dp.wait_params()  # overlapped ZeRO-1 all-gathers
    sums = replica_checksums(module, group)
    ref = sums[0]
    bad = [i for i, s in enumerate(sums) if abs(s - ref) > rtol * max(abs(ref), 1.0)]
    if bad:
        raise RuntimeError(f"data-parallel replicas diverged: checksums {sums} (ranks {bad} differ)")


def determinism_check(fn: Callable[[], torch.Tensor], seed: int = 0, runs: int = 2) -> Dict[str, object]:
    vals = []
    for _ in range(runs):
        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed_all(seed)
        v = fn()
        vals.append(v.detach().double().cpu().clone())
    same = all(torch.equal(vals[0], v) for v in vals[1:])
    return {"deterministic": same, "values": [v.tolist() for v in vals]}


class FaultInjected(RuntimeError):
    pass


class FaultInjector:
    def __init__(self, step: Optional[int] = None, rank: Optional[int] = None):
        env_s = os.environ.get("DLA_FAULT_STEP")
        env_r = os.environ.get("DLA_FAULT_RANK")
        self.step = step if step is not None else (int(env_s) if env_s else None)
        self.rank = rank if rank is not None else (int(env_r) if env_r else None)

    def maybe_fail(self, global_step: int, rank: int) -> None:
        if self.step is not None and global_step == self.step and (self.rank is None or self.rank == rank):
            raise FaultInjected(f"injected fault at step {global_step} on rank {rank}")


def debug_env() -> Dict[str, str]:
    return {"AMD_SERIALIZE_KERNEL": "3", "HIP_LAUNCH_BLOCKING": "1",
            "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1", "NCCL_DEBUG": "WARN"}
