"""Fully-sharded data parallel (ZeRO-3 / FSDP FULL_SHARD) over an RCCL group.

Replaces DeepSpeed ZeRO-3 (`config/deepspeed_zero3.json:5-15`) and FSDP FULL_SHARD
(`config/fsdp_config.yaml:6-10`) reached through accelerate (`src/training/utils.py:55-75`),
SURVEY §2.3 P2/P3, §2.5 C8-C10. Needed when a model's parameters + fp32 optimizer state do not
fit one GPU replicated (Llama-3-70B: 140 GB bf16 weights + 840 GB fp32 master/m/v).

Design (MI355X-first):
  * one *unit* per decoder layer plus a *root* unit (embeddings, final norm, LM head). Each unit
    is ONE flat bf16 tensor whose storage exists only while the unit is gathered; parameters are
    permanent views of it (storage resized to 0 when resharded, so autograd-saved views stay
    valid and are simply re-filled by the next all-gather);
  * rank r permanently owns chunk r of every unit (`param_shard`), the fp32 master copy and Adam
    moments of that chunk — the fused HIP AdamW runs on the local shard only, and unlike ZeRO-1
    no post-step all-gather is needed: updated weights are gathered lazily by the next forward;
  * forward: a pre-hook all-gathers the unit (already in flight if prefetched) and prefetches the
    next one on RCCL's stream; a post-hook frees it (reshard-after-forward) and arms a grad hook
    on the unit's outputs;
  * backward: that grad hook re-gathers the unit (and prefetches the previous one) BEFORE the
    unit's backward/recompute runs; weight grads land in a transient full-size unit grad buffer
    (GEMM epilogue `main_grad` accumulation); when the unit's last grad arrives its buffer is
    reduce-scattered (async, at most 2 in flight) into the local grad shard and freed;
  * the root unit (≈ 2 GB for Llama-3, 4 GB for 70B) stays resident: the LM-head log-prob is
    computed outside `forward`;
  * gradient accumulation reduce-scatters every micro-batch (the full grads are never kept) —
    `no_sync()` is accepted and ignored, as in FSDP with `NO_SHARD` disabled;
  * frozen models (the DPO/RLHF reference, distillation teachers) use `ShardedInference`: the same
    units and hooks with no gradients or optimizer.
Checkpoints use `summon_full_params()` (see utils/checkpoint.py), producing the same full HF
layout as unsharded training.
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..optim.adamw import adamw_update, clip_coefficient, grad_sumsq
from .dist import DistState, ExposedCommTimer, state as dist_state
from . import collectives as coll

ALIGN = 64


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _free(t: torch.Tensor) -> None:
    st = t.untyped_storage()
    if st.size() != 0:
        st.resize_(0)


def _alloc(t: torch.Tensor) -> None:
    st = t.untyped_storage()
    nbytes = t.numel() * t.element_size()
    if st.size() != nbytes:
        st.resize_(nbytes)


def default_units(module: nn.Module, min_num_params: int = 0) -> List[List[nn.Module]]:
    """Consecutive decoder layers grouped into FSDP units. `min_num_params` is the size-based wrap
    policy of the reference's FSDP plugin (config/fsdp_config.yaml:9-10, accelerate
    SIZE_BASED_WRAP): layers are merged until a unit holds at least that many parameters (every
    Llama/Mistral layer is far above the reference's 1e6, so that gives one unit per layer)."""
    base = getattr(module, "backbone", module)
    layers = getattr(base, "layers", None)
    if layers is None:
        raise ValueError("cannot infer FSDP units: module has no `.layers`")
    units, cur, n = [], [], 0
    for layer in layers:
        cur.append(layer)
        n += sum(p.numel() for p in layer.parameters())
        if n >= min_num_params:
            units.append(cur)
            cur, n = [], 0
    if cur:
        units.append(cur)
    return units


class _Unit:
    def __init__(self, idx: int, modules: Optional[List[nn.Module]], params: List[nn.Parameter],
                 world: int):
        self.idx = idx
        self.modules = modules or []
        self.module = self.modules[-1] if self.modules else None
        self.params = params
        self.offsets: Dict[int, int] = {}
        pos = 0
        for p in params:
            self.offsets[id(p)] = pos
            pos += _round_up(p.numel(), ALIGN)
        self.numel = _round_up(max(pos, 1), ALIGN * world)
        self.chunk = self.numel // world
        self.shard_off = 0
        self.full: Optional[torch.Tensor] = None
        self.gfull: Optional[torch.Tensor] = None
        self.resident = True
        self.handle = None
        self.in_backward = False
        self.ready = 0
        self.reduced = False

    @property
    def is_root(self) -> bool:
        return self.module is None


class _ShardedBase:
    """Unit layout, gather/free and the forward/backward hooks (shared by training and frozen)."""

    trainable = False

    def _init_sharding(self, module: nn.Module, group, params: List[nn.Parameter], prefetch: bool,
                       dist_st: Optional[DistState], single: bool = False, min_num_params: int = 0,
                       force_comm: Optional[bool] = None):
        self.module = module
        self.dist = dist_st or dist_state()
        self.group = group
        if coll.is_shape(group) and not single:  # one rank of an N-rank group, in this process
            self.world, self.rank = coll.world_size(group), coll.rank(group)
        elif self.dist.initialized and not single:
            self.world = coll.world_size(group) if group is not None else coll.world_size()
            self.rank = coll.rank(group) if group is not None else coll.rank()
        else:
            self.world, self.rank = 1, 0
        if force_comm is None:
            force_comm = self.dist.forced or os.environ.get("DLA_FORCE_COMM", "0") == "1"
        # `_comm`: gathers / reduce-scatters go through the communicator. A one-rank group with
        # force_comm runs them too (the N-GPU code path on one GPU, tests/test_force_comm.py)
        self._comm = self.world > 1 or (bool(force_comm) and not single and dist.is_available()
                                         and dist.is_initialized())
        self.comm_ops = 0  # collectives issued (tests check that the comm path ran)
        self.prefetch = prefetch
        self.dtype = params[0].dtype
        # meta parameters (models/materialize.py): values are produced unit by unit below, on
        # this rank's device, and never exist for the whole model at once
        meta = any(p.is_meta for p in params)
        self.device = self.dist.device if meta else params[0].device
        pset = {id(p) for p in params}
        unit_mods = default_units(module, min_num_params)
        owner: Dict[int, int] = {}
        units: List[_Unit] = []
        for i, mods in enumerate(unit_mods):
            ps = [p for m in mods for p in m.parameters() if id(p) in pset and id(p) not in owner]
            for p in ps:
                owner[id(p)] = i
            units.append(_Unit(i, mods, ps, self.world))
        root = [p for p in params if id(p) not in owner]
        for p in root:
            owner[id(p)] = len(units)
        units.append(_Unit(len(units), None, root, self.world))
        self.units = units
        self.unit_of = owner
        shard = 0
        for u in units:
            u.shard_off = shard
            shard += u.chunk
        self.shard_numel = shard
        self.numel = sum(u.numel for u in units)
        self.param_shard = torch.empty(shard, dtype=self.dtype, device=self.device)
        if meta:
            from ..models.materialize import _account, _owners, local_value, replace_param

            owners_map = _owners(module)
            esz = torch.empty(0, dtype=self.dtype).element_size()
            _account(shard * esz)  # this rank's shards, kept
        with torch.no_grad():
            for u in units:
                u.full = torch.zeros(u.numel, dtype=self.dtype, device=self.device)
                if meta:
                    _account(u.numel * esz)
                for i, p in enumerate(u.params):
                    o = u.offsets[id(p)]
                    view = u.full[o:o + p.numel()].view(p.shape)
                    if p.is_meta:
                        val = local_value(module, p, self.device)
                        view.copy_(val)
                        _account(-val.numel() * val.element_size())  # lives on in the unit buffer
                        del val
                        newp = replace_param(module, p, view, owners_map)
                        u.offsets[id(newp)] = u.offsets.pop(id(p))
                        owner[id(newp)] = owner.pop(id(p))
                        u.params[i] = newp
                    else:
                        view.copy_(p.data)
                        p.data = view
                self.param_shard[u.shard_off:u.shard_off + u.chunk].copy_(self._my_chunk(u.full, u))
                if not u.is_root:  # one full unit at a time: bounded construction peak
                    _free(u.full)
                    u.resident = False
                    if meta:
                        _account(-u.numel * esz)
        # weight epoch: bumped whenever the shards change (step / load / writeback). Gathers keep
        # the params' version counters untouched, so caches derived from weights (the decode
        # kernels' folded / tiled copies, ops.decode._wkey) key on this instead
        self._wt_epoch = [0]
        for u in units:
            for p in u.params:
                p._dla_epoch = self._wt_epoch
        self._pending = []  # in-flight reduce-scatters: (handle, tmp, unit)
        self.comm_timer = ExposedCommTimer(self.device)  # exposed gradient-comm wait per step
        self._seen = set()
        for u in units:  # gather before the unit's first layer, free after its last
            for m in u.modules:  # callers that bypass Module.__call__ (fused decode) check this
                m._dla_sharded = self
            if u.modules:
                u.modules[0].register_forward_pre_hook(self._make_pre_forward(u))
                u.modules[-1].register_forward_hook(self._make_post_forward(u))

    # ------------------------------------------------------------------ gather / free
    def _my_chunk(self, buf: torch.Tensor, u: _Unit) -> torch.Tensor:
        return buf[self.rank * u.chunk:(self.rank + 1) * u.chunk]

    def _gather(self, u: _Unit, async_op: bool = False):
        if u.resident:
            if u.handle is not None and not async_op:
                u.handle.wait()
                u.handle = None
            return
        _alloc(u.full)
        src = self.param_shard[u.shard_off:u.shard_off + u.chunk]
        with torch.autograd._unsafe_preserve_version_counter(u.full):
            if self._comm:
                self.comm_ops += 1
                h = coll.all_gather_into_tensor(u.full, src, group=self.group, async_op=True)
            else:
                u.full.copy_(src)
                h = None
        u.resident = True
        u.handle = h
        if not async_op and h is not None:
            h.wait()
            u.handle = None

    _pinned = False  # gathered_for_inference(): every unit stays resident

    def _reshard(self, u: _Unit):
        if u.is_root or self._pinned:
            return
        if u.handle is not None:
            u.handle.wait()
            u.handle = None
        _free(u.full)
        u.resident = False

    @contextlib.contextmanager
    def gathered_for_inference(self):
        """Every unit gathered once and kept resident (the forward hooks neither re-gather nor
        free) for the duration: rollout generation of a ZeRO-3 policy then runs like an unsharded
        model -- the fused decode kernels and the captured decode graph -- instead of one
        all-gather per layer per generated token ("hybrid engine"). Costs the full weights of the
        model on every rank while inside."""
        if self._pinned:
            yield
            return
        for u in self.units:
            self._gather(u)
        self._pinned = True
        try:
            yield
        finally:
            self._pinned = False
            for u in self.units:
                self._reshard(u)

    # ------------------------------------------------------------------ hooks
    def _make_pre_forward(self, u: _Unit):
        def hook(_mod, _inp):
            self._gather(u)
            if self.prefetch and not u.in_backward and u.idx + 1 < len(self.units) - 1:
                self._gather(self.units[u.idx + 1], async_op=True)
        return hook

    def _make_post_forward(self, u: _Unit):
        def hook(_mod, _inp, out):
            if u.in_backward:  # activation-checkpoint recompute inside backward: keep resident
                return out
            if self.trainable and torch.is_grad_enabled():
                outs = out if isinstance(out, (tuple, list)) else (out,)
                for t in outs:
                    if isinstance(t, torch.Tensor) and t.requires_grad:
                        t.register_hook(self._make_pre_backward(u))
            self._reshard(u)
            return out
        return hook

    def _make_pre_backward(self, u: _Unit):
        def hook(grad):
            self._pre_backward(u)
            return grad
        return hook

    def _pre_backward(self, u: _Unit):
        pass


class ShardedInference(_ShardedBase):
    """ZeRO-3 sharding of a frozen model (reference / teachers): 1/world of the weights resident,
    each layer gathered just in time for its forward."""

    def __init__(self, module: nn.Module, group=None, prefetch: bool = True,
                 dist_st: Optional[DistState] = None, min_num_params: int = 0,
                 force_comm: Optional[bool] = None):
        params = list(module.parameters())
        self._init_sharding(module, group, params, prefetch, dist_st, min_num_params=min_num_params,
                            force_comm=force_comm)
        module._dla_fsdp = self

    @contextlib.contextmanager
    def summon_full_params(self, writeback: bool = False):
        for u in self.units:
            self._gather(u)
        try:
            yield
        finally:
            if writeback:
                with torch.no_grad():
                    for u in self.units:
                        self.param_shard[u.shard_off:u.shard_off + u.chunk].copy_(self._my_chunk(u.full, u))
                self._wt_epoch[0] += 1
            for u in self.units:
                self._reshard(u)


class FullyShardedEngine(_ShardedBase):
    """Training engine with the DataParallelEngine interface (step / zero_grad / no_sync /
    optimizer_state / torch_optimizer_state_dict / ...), zero stage 3."""

    trainable = True

    def __init__(self, module: nn.Module, lr: float = 1e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, max_grad_norm: float = 1.0, master_weights: bool = True,
                 dist_st: Optional[DistState] = None, group=None, tp_group=None, prefetch: bool = True,
                 min_num_params: int = 0, cpu_offload: bool = False,
                 grad_dtype: Optional[torch.dtype] = None, force_comm: Optional[bool] = None, **_unused):
        if cpu_offload:
            raise ValueError("FSDP parameter CPU offload is not supported: sharded weights, fp32 "
                             "master and moments stay in HBM (288 GB per MI355X); set "
                             "hardware.fsdp.offload_params: false")
        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError("no trainable parameters")
        if len({p.dtype for p in params}) != 1:
            raise ValueError("mixed parameter dtypes")
        if any(getattr(p, "_dla_expert", False) for p in params):
            raise NotImplementedError("expert-parallel weights: use the ZeRO-1 engine (zero_stage <= 2)")
        if any(not p.requires_grad for p in module.parameters()):
            raise ValueError("FullyShardedEngine shards every parameter; freeze by wrapping the "
                             "frozen part in ShardedInference instead")
        st = dist_st or dist_state()
        self.tp_group = tp_group
        self.tp_size = coll.world_size(tp_group) if (tp_group is not None and (
            st.initialized or coll.is_shape(tp_group))) else 1
        if group is None and self.tp_size > 1 and self.tp_size != st.world_size:
            raise ValueError("pass the data-parallel group (mesh.dp_group) when tp < world")
        # TP spanning the whole world: dp = 1, nothing to shard over (kept for uniformity)
        self._init_sharding(module, group, params, prefetch, st, single=group is None and self.tp_size > 1,
                            min_num_params=min_num_params, force_comm=force_comm)
        self.zero = 3
        self.lr, self.betas, self.eps, self.wd = lr, tuple(betas), eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        self.params = [p for p in module.parameters() if p.requires_grad]  # (meta ones replaced)
        self._cb_armed = False
        n = self.shard_numel
        # micro-batch grads are reduce-scattered per unit in the param dtype and accumulated here:
        # fp32 (grad_dtype) keeps 16-256 micro-batch accumulations exact to fp32 rounding
        self.grad_shard = torch.zeros(n, dtype=grad_dtype or self.dtype, device=self.device)
        self.master = self.param_shard.to(torch.float32, copy=True) if master_weights else None  # one allocation (.float().clone() made two)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=self.device)
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.last_grad_norm = torch.zeros((), dtype=torch.float32, device=self.device)
        with torch.no_grad():
            for u in self.units:
                u.gfull = torch.zeros(u.numel, dtype=self.dtype, device=self.device)
                for p in u.params:
                    o = u.offsets[id(p)]
                    p.grad = u.gfull[o:o + p.numel()].view_as(p)
                    p.main_grad = p.grad
                    p._dla_grad_hook = self._on_grad
                    p.register_post_accumulate_grad_hook(self._on_grad)
                if not u.is_root:
                    _free(u.gfull)
        # shard-coordinate ranges of TP-replicated params (counted once in the clip norm)
        self._repl_ranges = []
        if self.tp_size > 1:
            for u in self.units:
                lo, hi = self.rank * u.chunk, (self.rank + 1) * u.chunk
                for p in u.params:
                    if getattr(p, "_dla_tp_replicated", False):
                        o = u.offsets[id(p)]
                        a, e = max(lo, o), min(hi, o + p.numel())
                        if a < e:
                            self._repl_ranges.append((u.shard_off + a - lo, u.shard_off + e - lo))
        module._dla_fsdp = self

    # ------------------------------------------------------------------ backward
    def _arm_post_backward(self):
        """Queue `_post_backward` to run when the current backward pass ends (once per pass)."""
        if not self._cb_armed:
            self._cb_armed = True
            torch.autograd.Variable._execution_engine.queue_callback(self._post_backward)

    def _post_backward(self):
        """End of one backward pass (one micro-batch): reduce-scatter the units whose grads are
        complete but not yet launched (the root), drain every pending reduce-scatter into the
        grad shard and reset the per-pass state, so the next micro-batch's backward re-arms every
        unit. Without this, a second micro-batch before step() found every parameter already
        `seen` and every unit `reduced`: its gradients were never reduced (and a unit buffer still
        pending from the first pass was zeroed under it)."""
        self._cb_armed = False
        self.finish_grad_sync()

    def _pre_backward(self, u: _Unit):
        if u.in_backward:
            return
        self._arm_post_backward()
        u.in_backward = True
        self._gather(u)
        if not u.is_root:
            _alloc(u.gfull)
            u.gfull.zero_()
        if self.prefetch and u.idx > 0:
            self._gather(self.units[u.idx - 1], async_op=True)

    def _on_grad(self, p: nn.Parameter):
        if id(p) in self._seen:  # GEMM-epilogue + AccumulateGrad report the same grad
            return
        self._arm_post_backward()
        self._seen.add(id(p))
        u = self.units[self.unit_of[id(p)]]
        u.ready += 1
        if u.ready == len(u.params):
            self._reduce(u)

    def _reduce(self, u: _Unit):
        if u.reduced:
            return
        u.reduced = True
        if not u.is_root and u.gfull.untyped_storage().size() == 0:  # unit saw no backward
            _alloc(u.gfull)
            u.gfull.zero_()
        if self._comm:
            self.comm_ops += 1
            tmp = torch.empty(u.chunk, dtype=self.dtype, device=self.device)
            h = coll.reduce_scatter_tensor(tmp, u.gfull, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        else:
            tmp, h = u.gfull, None
        self._pending.append((h, tmp, u))
        if not u.is_root:
            self._reshard(u)
            u.in_backward = False
        while len(self._pending) > 2:
            self._drain_one()

    def _drain_one(self):
        h, tmp, u = self._pending.pop(0)
        if h is not None:
            h.wait()
        self.grad_shard[u.shard_off:u.shard_off + u.chunk].add_(tmp if h is not None else self._my_chunk(tmp, u))
        if u.is_root:
            u.gfull.zero_()
        else:
            _free(u.gfull)

    def finish_grad_sync(self, timed: bool = True):
        # identical order on every rank: layer units as they completed, then the rest by index
        if self._seen or any(u.in_backward for u in self.units):
            for u in sorted(self.units, key=lambda x: -x.idx):
                if not u.reduced and (u.ready > 0 or u.in_backward or u.is_root):
                    self._reduce(u)
        # one interval per drain that has something to wait for: the end-of-backward callback
        # (_post_backward) drains every pass, so step()'s own call usually finds nothing and
        # must not record an empty interval (the step's exposed comm is the sum: close_step)
        timed = timed and bool(self._pending)
        if timed:
            self.comm_timer.begin()
        while self._pending:
            self._drain_one()
        if timed:
            self.comm_timer.end()
        self._seen = set()
        for u in self.units:
            u.ready = 0
            u.reduced = False
            u.in_backward = False
            if not u.is_root:
                self._reshard(u)

    @contextlib.contextmanager
    def no_sync(self):
        yield  # every micro-batch is reduce-scattered (full grads are never kept)

    # ------------------------------------------------------------------ step
    @property
    def grad_scale(self) -> float:
        # a shape group's reduce-scatter copies this rank's own slot (nothing is summed)
        return 1.0 if coll.is_shape(self.group) else 1.0 / self.world

    def clip_and_norm(self):
        gs = self.grad_scale
        grad_sumsq(self.grad_shard, self._sumsq, accumulate=False)
        if self._repl_ranges:
            rep = sum(self.grad_shard[a:e].float().pow(2).sum() for a, e in self._repl_ranges)
            self._sumsq -= (1.0 - 1.0 / self.tp_size) * rep
        if self._comm:
            coll.all_reduce(self._sumsq, op=dist.ReduceOp.SUM, group=self.group)
        if self.tp_size > 1:
            coll.all_reduce(self._sumsq, op=dist.ReduceOp.SUM, group=self.tp_group)
        norm, coef = clip_coefficient(self._sumsq * (gs * gs), self.max_grad_norm or 0.0)
        self.last_grad_norm = norm
        return coef

    def step(self, lr: Optional[float] = None) -> torch.Tensor:
        self.finish_grad_sync()
        self.comm_timer.close_step()
        lr = self.lr if lr is None else lr
        coef = self.clip_and_norm()
        self.step_count += 1
        self._wt_epoch[0] += 1
        adamw_update(self.param_shard, self.master, self.grad_shard, self.exp_avg, self.exp_avg_sq,
                     lr, self.betas[0], self.betas[1], self.eps, self.wd, self.step_count,
                     clip=coef if self.max_grad_norm else None, grad_scale=self.grad_scale)
        root = self.units[-1]
        root.resident = False  # stale: re-gather the (resident) root from the updated shards
        self._gather(root)
        self.zero_grad()
        return self.last_grad_norm

    def zero_grad(self):
        self.grad_shard.zero_()
        self.units[-1].gfull.zero_()

    # ------------------------------------------------------------------ full params / state
    @contextlib.contextmanager
    def summon_full_params(self, writeback: bool = False):
        for u in self.units:
            self._gather(u)
        try:
            yield
        finally:
            if writeback:
                self._shards_from_full()
            for u in self.units:
                self._reshard(u)

    @torch.no_grad()
    def _shards_from_full(self):
        for u in self.units:
            self.param_shard[u.shard_off:u.shard_off + u.chunk].copy_(self._my_chunk(u.full, u))
        self._wt_epoch[0] += 1
        if self.master is not None:
            self.master.copy_(self.param_shard)  # (copy_ converts in place: no fp32 temporary)

    @torch.no_grad()
    def broadcast_params(self, src: int = 0):
        if self.world > 1:
            with self.summon_full_params(writeback=True):
                gsrc = coll.get_global_rank(self.group, src) if self.group is not None else src
                for u in self.units:
                    coll.broadcast(u.full, src=gsrc, group=self.group)

    @torch.no_grad()
    def sync_master_from_params(self):
        if self.master is not None:
            self.master.copy_(self.param_shard)  # (copy_ converts in place: no fp32 temporary)

    def optimizer_state(self) -> Dict[str, object]:
        return {"step": self.step_count, "lr": self.lr, "betas": self.betas, "eps": self.eps,
                "weight_decay": self.wd, "world": self.world, "zero": 3, "rank": self.rank,
                "numel": self.numel, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "master": self.master}

    @torch.no_grad()
    def load_optimizer_state(self, sd: Dict[str, object]):
        if int(sd.get("numel", self.numel)) != self.numel or int(sd.get("world", self.world)) != self.world:
            raise ValueError("optimizer state layout does not match (numel/world)")
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        if self.master is not None and sd.get("master") is not None:
            self.master.copy_(sd["master"])
            self.param_shard.copy_(self.master.to(self.dtype))
            self._wt_epoch[0] += 1

    def _gather_unit(self, shard: torch.Tensor, u: _Unit) -> torch.Tensor:
        out = torch.empty(u.numel, dtype=shard.dtype, device=shard.device)
        src = shard[u.shard_off:u.shard_off + u.chunk].contiguous()
        if self._comm:
            coll.all_gather_into_tensor(out, src, group=self.group)
        else:
            out.copy_(src)
        return out

    def layout(self) -> Dict[str, object]:
        """Per-unit shard layout of the optimizer state (see DataParallelEngine.layout)."""
        all_params = [p for p in self.module.parameters() if p.requires_grad]
        index = {id(p): i for i, p in enumerate(all_params)}
        names = {id(p): n for n, p in self.module.named_parameters()}
        return {"kind": "fsdp", "zero": 3, "world": self.world, "numel": self.numel,
                "tp_size": self.tp_size,
                "units": [{"numel": u.numel, "chunk": u.chunk, "shard_off": u.shard_off,
                           "params": [{"index": index[id(p)], "name": names.get(id(p), ""),
                                       "shape": list(p.shape), "offset": u.offsets[id(p)]} for p in u.params]}
                          for u in self.units]}

    def torch_optimizer_state_dict(self) -> Dict[str, object]:
        """torch.optim.AdamW-format state (param index in module order), gathered per unit."""
        state = {}
        all_params = [p for p in self.module.parameters() if p.requires_grad]
        index = {id(p): i for i, p in enumerate(all_params)}
        for u in self.units:
            ea, es = self._gather_unit(self.exp_avg, u), self._gather_unit(self.exp_avg_sq, u)
            for p in u.params:
                o = u.offsets[id(p)]
                state[index[id(p)]] = {"step": torch.tensor(float(self.step_count)),
                                       "exp_avg": ea[o:o + p.numel()].view(p.shape).cpu(),
                                       "exp_avg_sq": es[o:o + p.numel()].view(p.shape).cpu()}
        group = {"lr": self.lr, "betas": self.betas, "eps": self.eps, "weight_decay": self.wd,
                 "amsgrad": False, "foreach": None, "maximize": False, "capturable": False,
                 "differentiable": False, "fused": None, "params": list(range(len(all_params)))}
        return {"state": dict(sorted(state.items())), "param_groups": [group]}


@contextlib.contextmanager
def fsdp_full_params(model, writeback: bool = False):
    """Full parameters of a model sharded by FullyShardedEngine / ShardedInference (no-op
    otherwise). Collective over the sharding group."""
    eng = getattr(model, "_dla_fsdp", None)
    if eng is None:
        yield model
        return
    with eng.summon_full_params(writeback=writeback):
        yield model
