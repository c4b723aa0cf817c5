"""Data-parallel training engine: flat buffers, bucketed RCCL gradient reduction overlapped with
backward, ZeRO-1 optimizer sharding and the fused flat AdamW.

Replaces DDP / DeepSpeed ZeRO / FSDP as reached through accelerate in the reference
(SURVEY §2.3 P1-P4, §2.5 C2-C4, C8-C9):
  * every trainable parameter lives in ONE flat bf16 buffer, laid out in reverse registration
    order (~ backward order) and cut into buckets (default 256 MiB: a few large collectives
    keep the 7 xGMI links busy instead of many small latency-bound ones);
  * `.grad` of each parameter is a view into a flat grad buffer, so autograd accumulates
    micro-batches in place (`no_sync()` suppresses communication on accumulation steps, C4);
  * on the sync micro-step a post-accumulate-grad hook launches the bucket's collective as soon
    as its last gradient lands (strictly in bucket order on every rank), on RCCL's stream,
    overlapping the remaining backward;
  * ZeRO-1 (default for world > 1): buckets are reduce-scattered; rank r owns chunk r of every
    bucket and keeps fp32 master / Adam moments only for its 1/world of the model; after the
    fused AdamW the bf16 shards are all-gathered back (C8/C9 semantics without per-layer
    gathers, which an 8B model on 288 GB HBM does not need);
  * ZeRO-0: classic all-reduce + replicated optimizer;
  * identical seeded init on every rank replaces DDP's rank-0 broadcast (C2); `broadcast_params`
    is available for loaded checkpoints.
Gradients are SUM-reduced; the 1/world mean is folded into the AdamW kernel's grad scale and the
clip-norm computation (no extra pass over the gradients).

fp32 gradient accumulation (`grad_dtype=torch.float32`, chosen automatically by the trainers for
gradient_accumulation_steps >= 16, e.g. config/dpo_hh.yaml's 256): the flat grad buffer is fp32
(`main_grad`), weight gradients are accumulated into it by the GEMMs themselves (hipBLASLt
bf16 x bf16 -> fp32 C, beta = 1), the few autograd-produced grads (norm weights, embeddings)
are folded in by the post-accumulate hook, and the fused AdamW reads fp32 grads. The bucket
collectives reduce in fp32 (`reduce_dtype=torch.float32`) or, to halve xGMI bytes, in bf16
(`reduce_dtype=torch.bfloat16`: the bucket is rounded once, after accumulation).
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..optim.adamw import adamw_update, clip_coefficient, grad_sumsq
from .dist import DistState, ExposedCommTimer, state as dist_state
from . import collectives as coll

ALIGN = 64  # elements; keeps every param view 128-byte aligned for 16-byte vector kernels


@dataclass
class Bucket:
    start: int
    end: int
    params: List[nn.Parameter] = field(default_factory=list)
    shard_off: int = 0  # offset of this rank's chunk inside the local shard buffers
    expert: bool = False  # holds expert-parallel weights (reduced over the expert-DP group)
    group: object = None
    world: int = 1
    rank: int = 0

    @property
    def size(self) -> int:
        return self.end - self.start


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class DataParallelEngine:
    def __init__(self, module: nn.Module, lr: float = 1e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, max_grad_norm: float = 1.0, zero_stage: Optional[int] = None,
                 bucket_mb: float = 256.0, master_weights: bool = True,
                 dist_st: Optional[DistState] = None, group=None, tp_group=None, expert_group=None,
                 overlap_param_gather: bool = os.environ.get("DLA_OVERLAP_AG", "1") != "0",
                 sp_size: int = 1,
                 grad_dtype: Optional[torch.dtype] = None, reduce_dtype: Optional[torch.dtype] = None,
                 shape_world: int = 1, force_comm: Optional[bool] = None):
        """`shape_world` > 1 (debug / benchmarking, one process only): lay the engine out as rank 0
        of a ZeRO-1 group of that size without any process group -- fp32 master weights and Adam
        moments exist (and are updated) only for this rank's 1/shape_world chunk of every bucket,
        the reduce-scatter becomes a local copy of that chunk and the all-gather a copy back.
        The memory and per-rank optimizer work are those of one rank of the N-GPU job; the
        communication is not run (tools/bench_rlhf.py --zero-shape, like bench.py --tp-shape).

        `force_comm` (default: the process group was created with `force_pg`, or env
        DLA_FORCE_COMM=1) with a ONE-rank group: run the multi-rank code path anyway -- ZeRO-1
        layout, grad-ready bucket hooks, async reduce-scatters on RCCL's stream during backward,
        the shard AdamW and the overlapped all-gathers -- so every line the N-GPU job runs
        executes on one GPU (bench.py --force-pg, tests/test_force_comm.py)."""
        self.module = module
        # sequence parallel (parallel.sequence): `group` is DP x SP and the sp ranks of a replica
        # hold partial (token-slice) gradients of one replicated loss -> sum over SP, mean over DP
        self.sp_size = int(sp_size)
        self.dist = dist_st or dist_state()
        # tensor parallel: grads of TP-sharded params differ per TP rank; params marked
        # `_dla_tp_replicated` are identical across TP ranks (counted once in the clip norm)
        self.tp_group = tp_group
        # (a parallel.collectives.ShapeGroup stands in for N ranks inside one process)
        self.tp_size = coll.world_size(tp_group) if (tp_group is not None and (
            self.dist.initialized or coll.is_shape(tp_group))) else 1
        if group is not None and coll.is_shape(group):
            self.world, self.rank = coll.world_size(group), coll.rank(group)
        elif self.dist.initialized:
            if group is not None:
                self.world, self.rank = coll.world_size(group), coll.rank(group)
            elif self.tp_size > 1 and not coll.is_shape(tp_group):
                # TP without a DP group: only legal when TP spans the whole world (dp = 1)
                if self.tp_size != self.dist.world_size:
                    raise ValueError("pass the data-parallel group (mesh.dp_group) when tp < world")
                self.world, self.rank = 1, 0
            else:
                self.world, self.rank = self.dist.world_size, self.dist.rank
        else:
            self.world, self.rank = 1, 0
        self.shape_group = coll.is_shape(group)
        self.shape_only = int(shape_world) > 1
        if self.shape_only:
            if self.world != 1:
                raise ValueError("shape_world is a single-process mode (no data-parallel group)")
            self.world, self.rank = int(shape_world), 0
        self.group = group
        if force_comm is None:
            force_comm = self.dist.forced or os.environ.get("DLA_FORCE_COMM", "0") == "1"
        # a one-rank group driven like an N-rank one (needs an initialised process group)
        self.force_comm = bool(force_comm) and not self.shape_only and dist.is_available() \
            and dist.is_initialized()
        multi = self.world > 1 or self.force_comm
        self.zero = (1 if multi else 0) if zero_stage is None else (zero_stage if multi else 0)
        self.lr, self.betas, self.eps, self.wd = lr, tuple(betas), eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        self._sync = True
        self._handles = []
        self._launched = 0
        self._seen = set()
        self._pass_armed = False  # an end-of-backward callback is queued for this sync pass
        self._pass_launched = False  # every bucket of the accumulated grads is in flight

        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError("no trainable parameters")
        dtypes = {p.dtype for p in params}
        if len(dtypes) != 1:
            raise ValueError(f"mixed parameter dtypes {dtypes}")
        self.dtype = params[0].dtype
        self.device = params[0].device
        self.comm_timer = ExposedCommTimer(self.device)  # exposed gradient-comm wait per step
        self.grad_dtype = grad_dtype or self.dtype
        self.grad_fp32 = self.grad_dtype == torch.float32 and self.dtype != torch.float32
        self.reduce_dtype = reduce_dtype or self.grad_dtype
        params = list(reversed(params))  # ~ the order gradients are produced in
        bucket_elems = max(ALIGN, int(bucket_mb * (1 << 20)) // params[0].element_size())
        # expert-parallel weights (parallel.expert) are reduced over the group of ranks holding
        # the SAME experts; dense weights over the data-parallel group
        self.expert_group = expert_group
        if expert_group is not None and (self.dist.initialized or self.force_comm
                                         or coll.is_shape(expert_group)):
            ew, er = coll.world_size(expert_group), coll.rank(expert_group)
        else:
            ew, er = 1, 0
        kinds = {False: (group, self.world, self.rank), True: (expert_group, ew, er)}
        # ---- layout
        self.buckets: List[Bucket] = []
        offsets: Dict[int, int] = {}

        def new_bucket(pos, expert):
            g, w, r = kinds[expert]
            return Bucket(pos, pos, expert=expert, group=g, world=w, rank=r)

        cur = new_bucket(0, bool(getattr(params[0], "_dla_expert", False)))
        pos = 0
        for p in params:
            n = _round_up(p.numel(), ALIGN)
            is_exp = bool(getattr(p, "_dla_expert", False))
            if cur.params and ((pos - cur.start) + n > bucket_elems or is_exp != cur.expert):
                cur.end = cur.start + _round_up(pos - cur.start, ALIGN * cur.world)
                self.buckets.append(cur)
                pos = cur.end
                cur = new_bucket(pos, is_exp)
            offsets[id(p)] = pos
            cur.params.append(p)
            pos += n
        cur.end = cur.start + _round_up(pos - cur.start, ALIGN * cur.world)
        self.buckets.append(cur)
        self.numel = cur.end
        self.has_experts = any(b.expert for b in self.buckets)
        # communication needed at all? (ZeRO with a 1-rank expert group still copies shards)
        self._comm = multi and not self.shape_only
        self.comm_ops = 0  # collectives issued by this engine (tests check the comm path ran)
        # ---- flat storage (params re-pointed into it)
        self.param_buf = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        self.grad_buf = torch.zeros(self.numel, dtype=self.grad_dtype, device=self.device)
        self.params = params
        # weights change in place inside the flat buffer (fused AdamW, all-gathers): the
        # per-parameter _version does not move, so caches key on this shared epoch too
        self._wt_epoch = [0]
        with torch.no_grad():
            for p in params:
                o = offsets[id(p)]
                view = self.param_buf[o:o + p.numel()].view_as(p)
                view.copy_(p.data)
                p.data = view
                gview = self.grad_buf[o:o + p.numel()].view_as(p)
                if self.grad_fp32:
                    # autograd grads must match the param dtype: they arrive in p.grad (bf16) and
                    # the post-accumulate hook folds them into the fp32 main_grad
                    p.grad = None
                else:
                    p.grad = gview
                # ops.linear / linear_logprob accumulate weight grads here inside the GEMM
                p.main_grad = gview
                p._dla_grad_hook = self._on_grad
                # persistent W^T for the TN-layout input-gradient GEMM (ops.linear.input_grad)
                p._dla_wt_ok = p.dim() == 2 and not getattr(p, "_dla_shared", False)
                p._dla_epoch = self._wt_epoch
        self._offsets = offsets
        # ---- shard layout
        shard = 0
        for b in self.buckets:
            b.shard_off = shard
            shard += b.size // b.world
        self.shard_numel = shard
        # every bucket over a ONE-rank group (the forced one-rank RCCL path, or EP buckets whose
        # experts live on this rank only): a rank's chunk IS its bucket, in the same order, so the
        # shards alias the flat buffers -- the reduce-scatter and all-gather are issued in place
        # (sendbuff == recvbuff: nothing to move) instead of copying 2 x 16 GB per Llama-3-8B
        # step into and out of separate shard buffers (profiles/r6_rlhf_forced.md), and the
        # 16 GB + 16 GB of shard memory are not allocated
        self.shard_alias = self.zero and not self.shape_only and all(b.world == 1 for b in self.buckets)
        if self.zero and self.shard_alias:
            self.grad_shard = self.grad_buf
            self.param_shard = self.param_buf
        elif self.zero:
            self.grad_shard = torch.zeros(shard, dtype=self.grad_dtype, device=self.device)
            self.param_shard = torch.empty(shard, dtype=self.dtype, device=self.device)
            torch.cat([self._chunk(self.param_buf, b) for b in self.buckets], out=self.param_shard)
        else:
            self.grad_shard = self.grad_buf
            self.param_shard = self.param_buf
        # shard-coordinate ranges of TP-replicated params (for the clip norm)
        self._repl_ranges = []
        if self.tp_size > 1:
            for b in self.buckets:
                c = b.size // b.world
                lo, hi = (b.start + b.rank * c, b.start + (b.rank + 1) * c) if self.zero else (b.start, b.end)
                base = (b.shard_off - lo) if self.zero else 0
                for p in b.params:
                    if getattr(p, "_dla_tp_replicated", False):
                        o = offsets[id(p)]
                        a, e = max(lo, o), min(hi, o + p.numel())
                        if a < e:
                            self._repl_ranges.append((a + base, e + base))
        n_state = self.param_shard.numel()
        self.master = self.param_shard.to(torch.float32, copy=True) if master_weights else None  # one allocation (.float().clone() made two)
        self.exp_avg = torch.zeros(n_state, dtype=torch.float32, device=self.device)
        self.exp_avg_sq = torch.zeros(n_state, dtype=torch.float32, device=self.device)
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.last_grad_norm = torch.zeros((), dtype=torch.float32, device=self.device)
        # ---- hooks
        self._bucket_of = {}
        self._ready = [0] * len(self.buckets)
        for bi, b in enumerate(self.buckets):
            for p in b.params:
                self._bucket_of[id(p)] = bi
                p.register_post_accumulate_grad_hook(self._on_grad)
        # ZeRO-1 parameter all-gather overlapped with the next forward: step() issues the
        # per-bucket all-gathers asynchronously in forward order (the last buckets hold the
        # first-used parameters); a forward pre-hook on every module that owns parameters waits
        # only for the buckets of its own weights, so layer i computes while later layers'
        # weights are still in flight on RCCL's stream.
        self._ag_pending: Dict[int, object] = {}
        module._dla_dp_engine = self
        self.overlap_param_gather = overlap_param_gather and self.zero and self._comm
        # (A per-bucket AdamW on a side stream overlapped with the next forward measured 0.3-0.5 %
        # slower on 1x MI355X -- the bandwidth-bound update only takes HBM and power from the
        # forward GEMMs -- and was removed; README "Tried".)
        if self.overlap_param_gather:
            for mod in module.modules():
                own = [self._bucket_of[id(p)] for p in mod.parameters(recurse=False) if id(p) in self._bucket_of]
                if own:
                    mod.register_forward_pre_hook(self._make_wait_hook(sorted(set(own))))

    # ------------------------------------------------------------------------ helpers
    def _make_wait_hook(self, buckets):
        def hook(_mod, _inp):
            if self._ag_pending:
                for bi in buckets:
                    h = self._ag_pending.pop(bi, None)
                    if h is not None:
                        h.wait()
        return hook

    def wait_params(self):
        """Block (on the current stream) until every in-flight parameter all-gather landed.
        Needed before reading weights outside a module forward (checkpoints, exports)."""
        for h in self._ag_pending.values():
            h.wait()
        self._ag_pending.clear()

    def _chunk(self, buf: torch.Tensor, b: Bucket) -> torch.Tensor:
        c = b.size // b.world
        return buf[b.start + b.rank * c: b.start + (b.rank + 1) * c]

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    def _on_grad(self, p: nn.Parameter):
        if self.grad_fp32 and p.grad is not None:
            # an autograd-produced (bf16) grad: fold into the fp32 main_grad, every micro-step
            p.main_grad.add_(p.grad)
            p.grad = None
        if not self._sync or not self._comm:
            return
        # a main_grad (GEMM-accumulated) weight reports twice: from the GEMM epilogue and from
        # its AccumulateGrad node (which still runs with an undefined grad) -> count once
        if id(p) in self._seen:
            return
        if not self._pass_armed:
            self._begin_sync_pass()
        self._seen.add(id(p))
        bi = self._bucket_of[id(p)]
        self._ready[bi] += 1
        # launch strictly in bucket order so every rank issues identical collective sequences
        while self._launched < len(self.buckets) and \
                self._ready[self._launched] == len(self.buckets[self._launched].params):
            self._launch(self._launched)
            self._launched += 1

    def _begin_sync_pass(self):
        """First gradient of a synchronising backward pass: queue `_end_sync_pass` for the end of
        this pass. A second sync pass before step() (backward called twice without no_sync)
        re-launches every bucket: ZeRO-1's reduce-scatter reads the locally accumulated buffer
        and overwrites the shard (in order on RCCL's stream), so the sum over both passes lands;
        ZeRO-0's in-place all-reduce would sum the first pass's already-summed values again, so
        that case is refused."""
        if self._pass_launched and not self.zero:
            raise RuntimeError("a second synchronising backward before step() under ZeRO-0: wrap the "
                               "accumulation micro-batches in engine.no_sync()")
        self._pass_armed = True
        torch.autograd.Variable._execution_engine.queue_callback(self._end_sync_pass)

    def _end_sync_pass(self):
        # buckets whose params got no gradient this pass (unused params), in bucket order
        while self._launched < len(self.buckets):
            self._launch(self._launched)
            self._launched += 1
        self._launched = 0
        self._ready = [0] * len(self.buckets)
        self._seen = set()
        self._pass_armed = False
        self._pass_launched = True

    def _launch(self, bi: int):
        b = self.buckets[bi]
        g = self.grad_buf[b.start:b.end]
        if b.world == 1 and not self.force_comm:  # expert bucket whose experts live here only
            if self.zero and not self.shard_alias:
                self.grad_shard[b.shard_off:b.shard_off + b.size].copy_(g)
            return
        self.comm_ops += 1
        if self.reduce_dtype != self.grad_dtype:
            # reduce in the (narrower) communication dtype: round the accumulated bucket once
            gc = g.to(self.reduce_dtype)
            if self.zero:
                oc = torch.empty(b.size // b.world, dtype=self.reduce_dtype, device=g.device)
                h = coll.reduce_scatter_tensor(oc, gc, op=dist.ReduceOp.SUM, group=b.group, async_op=True)
                dst = self.grad_shard[b.shard_off:b.shard_off + b.size // b.world]
                self._handles.append((h, lambda oc=oc, dst=dst: dst.copy_(oc)))
            else:
                h = coll.all_reduce(gc, op=dist.ReduceOp.SUM, group=b.group, async_op=True)
                self._handles.append((h, lambda gc=gc, g=g: g.copy_(gc)))
            return
        if self.zero:
            out = self.grad_shard[b.shard_off:b.shard_off + b.size // b.world]
            h = coll.reduce_scatter_tensor(out, g, op=dist.ReduceOp.SUM, group=b.group, async_op=True)
        else:
            h = coll.all_reduce(g, op=dist.ReduceOp.SUM, group=b.group, async_op=True)
        self._handles.append((h, None))

    def finish_grad_sync(self):
        """Launch buckets whose params got no gradient (unused params), then wait for all."""
        if self.shape_only:  # the reduce-scatter's output: this rank's chunks (overwritten)
            for b in self.buckets:
                c = b.size // b.world
                self.grad_shard[b.shard_off:b.shard_off + c].copy_(self._chunk(self.grad_buf, b))
        if self._comm:
            if not self._pass_launched:  # no synchronising backward since the last step
                while self._launched < len(self.buckets):
                    self._launch(self._launched)
                    self._launched += 1
            self.comm_timer.begin()
            for h, post in self._handles:
                h.wait()
                if post is not None:
                    post()
            self.comm_timer.end()
        self._reset_pass_state()

    def _reset_pass_state(self):
        # also clears _pass_armed: a backward that raised after its first gradient hook (OOM)
        # never ran its queued _end_sync_pass, and a stuck flag would stop later sync passes
        # from arming theirs
        self._handles = []
        self._launched = 0
        self._ready = [0] * len(self.buckets)
        self._seen = set()
        self._pass_launched = False
        self._pass_armed = False

    # ------------------------------------------------------------------------ step
    @property
    def grad_scale(self) -> float:
        if self.shape_only or self.shape_group:  # local gradients, nothing summed over ranks
            return float(self.sp_size)
        return self.sp_size / self.world

    def clip_and_norm(self):
        gs = self.grad_scale
        grad_sumsq(self.grad_shard, self._sumsq, accumulate=False)
        if self._repl_ranges:
            rep = sum(self.grad_shard[a:e].float().pow(2).sum() for a, e in self._repl_ranges)
            self._sumsq -= (1.0 - 1.0 / self.tp_size) * rep
        if self.has_experts and self._comm:
            # weight every element by 1/(#ranks holding it) and sum over the DP group: dense
            # grads are replicated dp times (ZeRO-0) or unique (ZeRO-1); expert grads are
            # replicated over the expert-DP group (ZeRO-0) or unique, and differ across EP ranks
            if not hasattr(self, "_esumsq"):
                self._esumsq = torch.zeros(1, dtype=torch.float32, device=self.device)
            self._esumsq.zero_()
            for b in self.buckets:
                if b.expert:
                    n = b.size // b.world if self.zero else b.size
                    o = b.shard_off if self.zero else b.start
                    grad_sumsq(self.grad_shard[o:o + n], self._esumsq, accumulate=True)
            dense = self._sumsq - self._esumsq
            if self.zero:
                self._sumsq = dense + self._esumsq
            else:
                ew = self.buckets[[b.expert for b in self.buckets].index(True)].world
                self._sumsq = dense / self.world + self._esumsq / ew
            coll.all_reduce(self._sumsq, op=dist.ReduceOp.SUM, group=self.group)
        elif self.zero and self._comm:
            coll.all_reduce(self._sumsq, op=dist.ReduceOp.SUM, group=self.group)
        if self.tp_size > 1:
            coll.all_reduce(self._sumsq, op=dist.ReduceOp.SUM, group=self.tp_group)
        sumsq = self._sumsq * (gs * gs)
        norm, coef = clip_coefficient(sumsq, self.max_grad_norm if self.max_grad_norm else 0.0)
        self.last_grad_norm = norm
        return coef

    def step(self, lr: Optional[float] = None) -> torch.Tensor:
        """Finish comm, clip, fused AdamW on the local shard, all-gather weights, zero grads.
        Returns the (device) global grad norm."""
        self.finish_grad_sync()
        self.comm_timer.close_step()
        lr = self.lr if lr is None else lr
        coef = self.clip_and_norm()
        self.step_count += 1
        adamw_update(self.param_shard, self.master, self.grad_shard, self.exp_avg, self.exp_avg_sq,
                     lr, self.betas[0], self.betas[1], self.eps, self.wd, self.step_count,
                     clip=coef if self.max_grad_norm else None, grad_scale=self.grad_scale)
        if self.zero:
            self.wait_params()
            for bi in reversed(range(len(self.buckets))):  # forward order
                b = self.buckets[bi]
                c = b.size // b.world
                if b.world == 1 and not self.force_comm:
                    if not self.shard_alias:
                        self.param_buf[b.start:b.end].copy_(self.param_shard[b.shard_off:b.shard_off + c])
                elif self.shape_only:  # the all-gather's local part
                    self._chunk(self.param_buf, b).copy_(self.param_shard[b.shard_off:b.shard_off + c])
                else:
                    self.comm_ops += 1
                    h = coll.all_gather_into_tensor(self.param_buf[b.start:b.end],
                                                    self.param_shard[b.shard_off:b.shard_off + c],
                                                    group=b.group, async_op=self.overlap_param_gather)
                    if self.overlap_param_gather:
                        self._ag_pending[bi] = h
        self._wt_epoch[0] += 1  # invalidates weight-derived caches (ops.linear W^T)
        self.zero_grad()
        return self.last_grad_norm

    def zero_grad(self):
        for h, _ in self._handles:  # collectives still reading/writing the buffers (an aborted pass)
            h.wait()
        self._reset_pass_state()
        self.grad_buf.zero_()
        if self.grad_fp32:
            for p in self.params:
                p.grad = None
        if self.zero and not (self._comm or self.shape_only):
            # with a collective (or its shape-only local copy) every bucket's reduce-scatter
            # OVERWRITES its shard each step (finish_grad_sync launches the buckets no gradient
            # reached), so zeroing it too only costs a pass over the shard: 16 GB of HBM writes
            # per step on the forced one-rank Llama-3-8B layout (profiles/r6_rlhf_forced.md)
            self.grad_shard.zero_()

    @torch.no_grad()
    def broadcast_params(self, src: int = 0):
        self.wait_params()
        self._wt_epoch[0] += 1
        if self.world > 1:
            for b in self.buckets:
                if b.world > 1:
                    gsrc = coll.get_global_rank(b.group, src) if b.group is not None else src
                    coll.broadcast(self.param_buf[b.start:b.end], src=gsrc, group=b.group)
            if self.zero and not self.shard_alias:
                torch.cat([self._chunk(self.param_buf, b) for b in self.buckets], out=self.param_shard)
            if self.master is not None:
                self.master.copy_(self.param_shard)  # (copy_ converts in place: no fp32 temporary)

    @torch.no_grad()
    def sync_master_from_params(self):
        self.wait_params()
        self._wt_epoch[0] += 1
        if self.zero and not self.shard_alias:
            torch.cat([self._chunk(self.param_buf, b) for b in self.buckets], out=self.param_shard)
        if self.master is not None:
            self.master.copy_(self.param_shard)  # (copy_ converts in place: no fp32 temporary)

    # ------------------------------------------------------------------------ state
    def optimizer_state(self) -> Dict[str, object]:
        """Local (possibly sharded) optimizer state."""
        if self.shape_only:
            raise RuntimeError("a shape_world engine holds one rank's optimizer shard of a job that "
                               "does not exist: it has no checkpointable state")
        self.wait_params()
        return {"step": self.step_count, "lr": self.lr, "betas": self.betas, "eps": self.eps,
                "weight_decay": self.wd, "world": self.world, "zero": self.zero,
                "rank": self.rank, "numel": self.numel,
                "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "master": self.master}

    @torch.no_grad()
    def load_optimizer_state(self, sd: Dict[str, object]):
        self.wait_params()
        if int(sd.get("numel", self.numel)) != self.numel or int(sd.get("world", self.world)) != self.world:
            raise ValueError("optimizer state layout does not match (numel/world)")
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        if self.master is not None and sd.get("master") is not None:
            self.master.copy_(sd["master"])

    def layout(self) -> Dict[str, object]:
        """Where every parameter's optimizer state lives in the per-rank shards (written next to
        the shards as dla_optimizer_layout.json; tools/consolidate_checkpoint.py rebuilds a
        torch-format optimizer.bin offline from it)."""
        self.wait_params()
        all_params = [p for p in self.module.parameters() if p.requires_grad]
        index = {id(p): i for i, p in enumerate(all_params)}
        names = {id(p): n for n, p in self.module.named_parameters()}
        return {"kind": "flat", "zero": self.zero, "world": self.world, "numel": self.numel,
                "tp_size": self.tp_size,
                "buckets": [{"start": b.start, "end": b.end, "world": b.world, "shard_off": b.shard_off,
                             "expert": b.expert} for b in self.buckets],
                "params": [{"index": index[id(p)], "name": names.get(id(p), ""), "shape": list(p.shape),
                            "offset": self._offsets[id(p)]} for p in self.params]}

    def torch_optimizer_state_dict(self) -> Dict[str, object]:
        """Consolidated torch.optim.AdamW-format state dict (param index -> step/exp_avg/
        exp_avg_sq), as accelerate writes to optimizer.bin. Gathers shards under ZeRO."""
        self.wait_params()
        ea, es = self.exp_avg, self.exp_avg_sq
        if self.zero:
            ea, es = self._gather_full(ea), self._gather_full(es)
        state = {}
        all_params = [p for p in self.module.parameters() if p.requires_grad]
        for i, p in enumerate(all_params):
            o = self._offsets[id(p)]
            state[i] = {"step": torch.tensor(float(self.step_count)),
                        "exp_avg": ea[o:o + p.numel()].view(p.shape).cpu(),
                        "exp_avg_sq": es[o:o + p.numel()].view(p.shape).cpu()}
        group = {"lr": self.lr, "betas": self.betas, "eps": self.eps, "weight_decay": self.wd,
                 "amsgrad": False, "foreach": None, "maximize": False, "capturable": False,
                 "differentiable": False, "fused": None, "params": list(range(len(all_params)))}
        return {"state": state, "param_groups": [group]}

    def _gather_full(self, shard: torch.Tensor) -> torch.Tensor:
        full = torch.empty(self.numel, dtype=shard.dtype, device=shard.device)
        for b in self.buckets:
            c = b.size // b.world
            if b.world == 1:
                full[b.start:b.end].copy_(shard[b.shard_off:b.shard_off + c])
            else:
                coll.all_gather_into_tensor(full[b.start:b.end], shard[b.shard_off:b.shard_off + c].contiguous(),
                                            group=b.group)
        return full
