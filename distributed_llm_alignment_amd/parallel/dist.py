"""Process-group runtime: one process per GPU, RCCL (torch backend "nccl") over xGMI on MI355X,
gloo on CPU (test tier).

Replaces accelerate's `Accelerator()` process-group creation (src/training/utils.py:55-75,
config/accelerate_config.yaml: MULTI_GPU, 8 processes, static rendezvous). Reads the standard
torchrun env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT); a single process with no
env runs world_size=1 without creating a group.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistState:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None
    # a ONE-rank process group that the engines drive like a real one (force_pg): every bucket
    # hook, reduce-scatter, all-gather and all-to-all is issued on the communicator
    forced: bool = False

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def initialized(self) -> bool:
        return (self.world_size > 1 or self.forced) and dist.is_available() and dist.is_initialized()


_STATE = DistState()


def init_distributed(backend: Optional[str] = None, timeout_s: int = 1800,
                     device: Optional[str] = None, force_pg: Optional[bool] = None) -> DistState:
    """Initialise (idempotent). backend defaults to nccl(=RCCL) on GPU, gloo on CPU.

    `force_pg` (default: env DLA_FORCE_PG=1) with a single process: create a real 1-rank
    process group anyway and mark the state `forced`, so the communication engines run their
    collective code paths (hooks, async works, RCCL's stream and events) on one GPU -- the same
    code the N-GPU job runs, exercised where there is only one device (bench.py --force-pg,
    tests/test_force_comm.py)."""
    global _STATE
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if force_pg is None:
        force_pg = os.environ.get("DLA_FORCE_PG", "0") == "1"
    forced = bool(force_pg) and world == 1
    use_gpu = torch.cuda.is_available() and device != "cpu"
    if use_gpu:
        n = torch.cuda.device_count()
        dev = torch.device("cuda", local % max(n, 1))
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    be = backend or ("nccl" if use_gpu else "gloo")
    # a hung / failed collective raises (with the op and group in the message) instead of
    # blocking the job forever; DLA_COLLECTIVE_TIMEOUT_S overrides the timeout
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    timeout_s = int(os.environ.get("DLA_COLLECTIVE_TIMEOUT_S", timeout_s))
    if (world > 1 or forced) and not dist.is_initialized():
        kwargs = dict(backend=be, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if forced:
            # the one-rank group rendezvous in-process: no TCP port to race for, nothing written
            # into MASTER_PORT for later inits or child processes to inherit
            kwargs["store"] = dist.HashStore()
        else:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29500")
        if be == "nccl":
            kwargs["device_id"] = dev
            opts = comm_pg_options(world)
            if opts is not None:
                kwargs["pg_options"] = opts
        dist.init_process_group(**kwargs)
    forced = forced and dist.is_initialized()
    _STATE = DistState(rank=rank, world_size=world, local_rank=local, device=dev,
                       backend=be if (world > 1 or forced) else None, forced=forced)
    return _STATE


# RCCL's internal streams at HIGH priority. HIP maps streams round-robin onto a few hardware queues
# per process (GPU_MAX_HW_QUEUES, 4 by default) and one hardware queue runs its kernels in order:
# a rocprofv3 trace of the ZeRO-1 bench on a forced one-rank group showed RCCL's stream on the SAME
# hardware queue as torch's compute stream, its bucket kernels 0 % concurrent with the backward
# (profiles/r5_force_pg_streams.md). A high-priority stream gets its own (priority) queue, so the
# gradient collectives really run beside the backward GEMMs. DLA_RCCL_HIGH_PRIORITY=0 keeps torch's
# default (normal-priority pool stream).
# The priority queue is not free: with the one-rank group's collectives in place (no RCCL kernels
# at all), the RLHF update ran 0.405 s with it vs 0.353 s without (= the no-group run, 0.354 s),
# and the 70B TP-8 rank step 2132 vs 2034 ms: its pending stream waits alone slow the
# bandwidth-bound kernels of the compute queue 2-3x (profiles/r6_rlhf_forced.md). So a ONE-rank
# group, which has nothing to overlap, keeps the normal-priority stream; groups of >= 2 ranks
# take the high-priority one for the overlap.
RCCL_HIGH_PRIORITY = os.environ.get("DLA_RCCL_HIGH_PRIORITY", "1") != "0"


def comm_pg_options(group_size: int = 2):
    """ProcessGroupNCCL options for every RCCL group this framework creates (world + sub-groups)."""
    if not RCCL_HIGH_PRIORITY or group_size < 2 or not hasattr(dist, "ProcessGroupNCCL"):
        return None
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    return opts


def new_group(ranks, **kw):
    """dist.new_group with the framework's RCCL options (high-priority comm streams)."""
    if _STATE.backend == "nccl" and "pg_options" not in kw:
        opts = comm_pg_options(len(ranks))
        if opts is not None:
            kw["pg_options"] = opts
    return dist.new_group(ranks, **kw)


def state() -> DistState:
    return _STATE


def is_main() -> bool:
    return _STATE.rank == 0


def barrier():
    if _STATE.initialized:
        if _STATE.backend == "nccl":
            dist.barrier(device_ids=[_STATE.device.index])
        else:
            dist.barrier()


def all_reduce_(t: torch.Tensor, op: str = "sum", group=None) -> torch.Tensor:
    if _STATE.initialized:
        dist.all_reduce(t, op=dist.ReduceOp.SUM if op in ("sum", "mean") else dist.ReduceOp.MAX,
                        group=group)
        if op == "mean":
            t.div_(dist.get_world_size(group))
    return t


def all_gather_tensor(t: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenate equal-shape tensors from all ranks along dim 0 (C5 eval gather)."""
    if not _STATE.initialized:
        return t
    ws = dist.get_world_size(group)
    out = torch.empty((ws * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


def broadcast_object(obj: Any, src: int = 0) -> Any:
    if not _STATE.initialized:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


def gather_objects(obj: Any) -> List[Any]:
    if not _STATE.initialized:
        return [obj]
    out: List[Any] = [None] * _STATE.world_size
    dist.all_gather_object(out, obj)
    return out


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def split_for_rank(items: list, rank: Optional[int] = None, world: Optional[int] = None) -> list:
    """Contiguous slice of `items` for this rank (fixes the reference's misuse of
    `split_between_processes` at train_rlhf.py:114)."""
    if rank is None or world is None:
        from .mesh import current_mesh

        m = current_mesh()  # data-parallel replicas: TP ranks of one replica share a slice
        r0, w0 = (m.dp_rank, m.dp) if m is not None else (_STATE.rank, _STATE.world_size)
        rank = r0 if rank is None else rank
        world = w0 if world is None else world
    n = len(items)
    per, extra = divmod(n, world)
    start = rank * per + min(rank, extra)
    return items[start:start + per + (1 if rank < extra else 0)]


class ExposedCommTimer:
    """Time the training step spends waiting for its gradient collectives at the step boundary
    (`finish_grad_sync`): the part of the reduce-scatter / all-reduce that nothing overlapped.

    On a GPU, events go on the compute stream around the waits. `Work.wait()` makes that stream
    wait for RCCL's stream, so the device time between the two events is exactly the stall. It is
    about 0 when the collectives finished behind earlier work (backward compute, the next RLHF
    rollout), and the whole tail of the reduce otherwise. On the CPU (gloo) `wait()` blocks the
    host, and host time is measured. `last_ms()` reads the most recent interval; it synchronises
    on the end event, so call it at logging time, not inside the step."""

    def __init__(self, device: torch.device):
        self.cuda = device.type == "cuda"
        self._a = self._b = None
        self._t0 = self._host_ms = 0.0
        self._hist: list = []  # every interval since reset(): (start, end) events or host ms
        self._step_from, self._last_step = 0, []  # close_step() / last_step_ms()

    def begin(self):
        if self.cuda:
            self._a = torch.cuda.Event(enable_timing=True)
            self._a.record()
        else:
            import time

            self._t0 = time.perf_counter()

    def end(self):
        if self.cuda:
            self._b = torch.cuda.Event(enable_timing=True)
            self._b.record()
            self._hist.append((self._a, self._b))
        else:
            import time

            self._host_ms = (time.perf_counter() - self._t0) * 1e3
            self._hist.append(self._host_ms)
        if len(self._hist) > 4096:
            del self._hist[:2048]
            self._step_from = max(0, getattr(self, "_step_from", 0) - 2048)

    def reset(self):
        self._hist = []
        self._step_from, self._last_step = 0, []

    def close_step(self):
        """Mark an optimizer-step boundary: the intervals recorded since the previous boundary
        (one per drained backward pass under FSDP, plus the step's own wait) become the step's
        exposed comm, read by `last_step_ms()`."""
        start = getattr(self, "_step_from", 0)
        self._last_step = self._hist[start:]
        self._step_from = len(self._hist)

    def last_step_ms(self) -> float:
        """Exposed comm of the last closed step: the SUM of its intervals (synchronises)."""
        iv = getattr(self, "_last_step", [])
        if self.cuda:
            if not iv:
                return 0.0
            iv[-1][1].synchronize()
            return float(sum(a.elapsed_time(b) for a, b in iv))
        return float(sum(iv))

    def total_ms(self) -> float:
        """Sum over every interval since reset() (synchronises on the last one)."""
        if self.cuda:
            if self._hist:
                self._hist[-1][1].synchronize()
            return float(sum(a.elapsed_time(b) for a, b in self._hist))
        return float(sum(self._hist))

    def last_ms(self) -> float:
        if self.cuda:
            if self._b is None:
                return 0.0
            self._b.synchronize()
            return float(self._a.elapsed_time(self._b))
        return self._host_ms

