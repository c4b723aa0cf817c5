"""Memory-bounded weight I/O for sharded models (reference: accelerate
`save_state`, src/training/utils.py:99-102, which writes per-rank FSDP/DeepSpeed shards).

A 70B policy + frozen reference under FSDP x TP must never be gathered whole (that is ~280 GB of
bf16 on every GPU). Everything here walks a model ONE UNIT AT A TIME — an FSDP unit (one decoder
layer) or, for unsharded / TP / EP models, one decoder layer — and then the root (embeddings,
final norm, LM head):

  * `full_params(...)`   — make one unit's parameters full (FSDP all-gather of the unit, TP
    all-gather of sharded matrices, EP all-gather of expert stacks), optionally write modified
    values back into the shards, free again. Collective: every rank walks the same units.
  * `save_consolidated`  — HF-named tensors, streamed: `model.safetensors` (reference layout) up
    to DLA_CKPT_SINGLE_FILE_GB (default 40), else HF index shards
    `model-0000k-of-0000n.safetensors` + `model.safetensors.index.json` flushed every
    DLA_CKPT_SHARD_GB (default 5). Rank 0 holds at most one flush buffer on the host.
  * `load_consolidated`  — the inverse, reading tensors lazily (safetensors `safe_open`).
  * `save_rank_shards` / `load_rank_shards` — per-rank files of the rank's LOCAL tensors (no
    collective, no gather): `{stem}.fsdp{r}-tp{t}-ep{e}.safetensors` + `{stem}.shards.json`
    (layout). Exact fast resume on the same layout; `tools/consolidate_checkpoint.py --weights`
    rebuilds the HF-named files offline from them on the host, one unit at a time.
"""
from __future__ import annotations

import json
import os
from contextlib import contextmanager
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

SINGLE_FILE_MAX_BYTES = int(float(os.environ.get("DLA_CKPT_SINGLE_FILE_GB", "40")) * 2 ** 30)
SHARD_BYTES = int(float(os.environ.get("DLA_CKPT_SHARD_GB", "5")) * 2 ** 30)
FSDP_KEY = "__fsdp_param_shard__"

# diagnostics for tests: most non-root FSDP units simultaneously full during a walk
STATS = {"max_full_units": 0}


def _base(model):
    return getattr(model, "backbone", model)


def unit_groups(model) -> List[Tuple[object, object, list]]:
    """[(fsdp_engine | None, unit | None, params)] in the same order on every rank."""
    eng = getattr(model, "_dla_fsdp", None)
    groups, seen = [], set()
    if eng is not None:
        for u in eng.units:
            groups.append((eng, u, list(u.params)))
            seen.update(id(p) for p in u.params)
    else:
        for layer in getattr(_base(model), "layers", []):
            ps = list(layer.parameters())
            groups.append((None, None, ps))
            seen.update(id(p) for p in ps)
    rest = [p for p in model.parameters() if id(p) not in seen]
    if rest:
        groups.append((None, None, rest))
    return groups


def _fsdp_writeback(eng, u) -> None:
    sl = slice(u.shard_off, u.shard_off + u.chunk)
    eng.param_shard[sl].copy_(eng._my_chunk(u.full, u))
    master = getattr(eng, "master", None)
    if master is not None:
        master[sl].copy_(eng.param_shard[sl].float())


@contextmanager
def full_params(model, eng, unit, params, writeback: bool = False):
    """Within the context every parameter in `params` holds its FULL tensor. Collective over the
    FSDP / TP / EP groups involved (all ranks must enter with the same unit)."""
    from ..parallel.tensor_parallel import gather_tensor, shard_tensor

    base = _base(model)
    fsdp = eng is not None and unit is not None
    if fsdp:
        eng._gather(unit)
        STATS["max_full_units"] = max(STATS["max_full_units"],
                                      sum(1 for u in eng.units if u.resident and not u.is_root))
    saved = []
    try:
        with torch.no_grad():
            for p in params:
                spec = getattr(p, "_dla_tp_spec", None)
                ep = getattr(p, "_dla_ep", None)
                if spec is not None and getattr(base, "tp_size", 1) > 1:
                    saved.append((p, p.data, "tp", spec))
                    p.data = gather_tensor(p.data, spec, base.tp)
                elif ep is not None and ep[2] > 1:
                    full = p.data.new_empty((p.shape[0] * ep[2],) + tuple(p.shape[1:]))
                    dist.all_gather_into_tensor(full, p.data.contiguous(), group=ep[0])
                    saved.append((p, p.data, "ep", ep))
                    p.data = full
        yield
    finally:
        with torch.no_grad():
            for p, local, kind, info in reversed(saved):
                if writeback:
                    if kind == "tp":
                        local.copy_(shard_tensor(p.data, info, base.tp_rank, base.tp_size))
                    else:
                        n = local.shape[0]
                        local.copy_(p.data[info[1] * n:(info[1] + 1) * n])
                p.data = local
            if fsdp:
                if writeback:
                    _fsdp_writeback(eng, unit)
                eng._reshard(unit)


def full_nbytes(model) -> int:
    """Bytes of the unsharded model (TP / EP slices scaled back up; FSDP views keep full shapes)."""
    base = _base(model)
    tot = 0
    for p in model.parameters():
        n = p.numel()
        if getattr(p, "_dla_tp_spec", None) is not None and getattr(base, "tp_size", 1) > 1:
            n *= base.tp_size
        ep = getattr(p, "_dla_ep", None)
        if ep is not None:
            n *= ep[2]
        tot += n * p.element_size()
    return tot


def _hf_subset(model, only):
    if hasattr(model, "hf_state_dict"):
        return model.hf_state_dict(only=only)
    return {n: p for n, p in model.named_parameters() if n in only}


def iter_hf_groups(model, keep: bool = True):
    """Yield {hf_key: cpu tensor} per unit (None on ranks with keep=False). Collective."""
    names = {id(p): n for n, p in model.named_parameters()}
    for eng, u, ps in unit_groups(model):
        with full_params(model, eng, u, ps):
            out = None
            if keep:
                sd = _hf_subset(model, {names[id(p)] for p in ps})
                out = {k: v.detach().to("cpu", copy=True).contiguous() for k, v in sd.items()}
        yield out


class ConsolidatedWriter:
    """Host-side writer of HF-named tensors: one `{stem}.safetensors` when the whole model fits
    `single_max` bytes, else HF index shards flushed every `shard_bytes` (bounded host memory)."""

    def __init__(self, out_dir, stem: str, total_bytes: int, single_max: int = None,
                 shard_bytes: int = None):
        self.dir = Path(out_dir)
        self.stem = stem
        self.single = total_bytes <= (SINGLE_FILE_MAX_BYTES if single_max is None else single_max)
        self.shard_bytes = SHARD_BYTES if shard_bytes is None else shard_bytes
        self.buf: Dict[str, torch.Tensor] = {}
        self.buf_bytes = 0
        self.files: List[Tuple[str, List[str]]] = []
        self.total = 0

    def add(self, tensors: Dict[str, torch.Tensor]) -> None:
        for k, v in tensors.items():
            self.buf[k] = v
            nb = v.numel() * v.element_size()
            self.buf_bytes += nb
            self.total += nb
        if not self.single and self.buf_bytes >= self.shard_bytes:
            self._flush()

    def _flush(self) -> None:
        from safetensors.torch import save_file

        if not self.buf:
            return
        tmp = f"{self.stem}.part{len(self.files):05d}.tmp"
        save_file(self.buf, str(self.dir / tmp), metadata={"format": "pt"})
        self.files.append((tmp, list(self.buf)))
        self.buf, self.buf_bytes = {}, 0

    def close(self) -> List[str]:
        from safetensors.torch import save_file

        if self.single:
            name = f"{self.stem}.safetensors"
            save_file(self.buf, str(self.dir / name), metadata={"format": "pt"})
            self.buf = {}
            return [name]
        self._flush()
        n = len(self.files)
        weight_map, names = {}, []
        for i, (tmp, keys) in enumerate(self.files):
            name = f"{self.stem}-{i + 1:05d}-of-{n:05d}.safetensors"
            os.replace(self.dir / tmp, self.dir / name)
            names.append(name)
            for k in keys:
                weight_map[k] = name
        index = {"metadata": {"total_size": self.total}, "weight_map": dict(sorted(weight_map.items()))}
        (self.dir / f"{self.stem}.safetensors.index.json").write_text(json.dumps(index, indent=2))
        return names


def save_consolidated(model, out_dir, stem: str, is_main: bool) -> Optional[List[str]]:
    """Stream HF-named weights of `model` into `out_dir` (collective; rank 0 writes)."""
    w = ConsolidatedWriter(out_dir, stem, full_nbytes(model)) if is_main else None
    for tensors in iter_hf_groups(model, keep=is_main):
        if w is not None:
            w.add(tensors)
    return w.close() if w is not None else None


def open_consolidated(d, stem: str):
    """LazyTensors over `{stem}.safetensors` or `{stem}.safetensors.index.json` (None if absent)."""
    from safetensors import safe_open

    from ..models.hf_io import LazyTensors

    d = Path(d)
    single = d / f"{stem}.safetensors"
    index = d / f"{stem}.safetensors.index.json"
    if single.exists():
        h = safe_open(str(single), framework="pt")
        keys = list(h.keys())
        return LazyTensors(keys, lambda k: h.get_tensor(k))
    if index.exists():
        wm = json.loads(index.read_text())["weight_map"]
        handles = {}

        def get(k):
            f = wm[k]
            if f not in handles:
                handles[f] = safe_open(str(d / f), framework="pt")
            return handles[f].get_tensor(k)
        return LazyTensors(wm.keys(), get)
    return None


_IGNORABLE = ("rotary_emb.inv_freq", ".attn.bias", ".attn.masked_bias")


def load_consolidated(model, sd, strict: bool = True):
    """Load HF-named tensors (a mapping, typically lazy) into a possibly sharded model, one unit
    at a time (collective)."""
    names = {id(p): n for n, p in model.named_parameters()}
    used: set = set()
    missing: List[str] = []
    for eng, u, ps in unit_groups(model):
        only = {names[id(p)] for p in ps}
        with full_params(model, eng, u, ps, writeback=True):
            if hasattr(model, "load_hf_state_dict"):
                m, _ = model.load_hf_state_dict(sd, strict=False, only=only, used_out=used)
                missing += m
            else:
                for n, p in model.named_parameters():
                    if n in only:
                        key = n if n in sd else f"module.{n}"
                        if key in sd:
                            p.data.copy_(sd[key].to(p.dtype))
                            used.add(key)
                        else:
                            missing.append(n)
    if getattr(_base(model).cfg, "tie_word_embeddings", False):
        missing = [m for m in missing if not m.startswith("lm_head")]
    unexpected = [k for k in sd if k not in used and not k.startswith("lm_head")
                  and not any(s in k for s in _IGNORABLE)]
    if strict and (missing or unexpected):
        raise KeyError(f"missing={missing[:8]} unexpected={unexpected[:8]}")
    return missing, unexpected


# ------------------------------------------------------------------------------ per-rank shards
def _coords(model) -> Dict[str, int]:
    from ..parallel.mesh import current_mesh

    base = _base(model)
    eng = getattr(model, "_dla_fsdp", None)
    mesh = current_mesh()
    ep_rank = 0
    for p in model.parameters():
        ep = getattr(p, "_dla_ep", None)
        if ep is not None:
            ep_rank = ep[1]
            break
    c = {"fsdp": eng.rank if eng is not None else 0, "tp": getattr(base, "tp_rank", 0)
         if getattr(base, "tp_size", 1) > 1 else 0, "ep": ep_rank}
    # a rank writes when no other rank holds identical local tensors before it
    if eng is not None:
        writer = True if mesh is None else mesh.sp_rank == 0
    elif mesh is None:
        writer = (dist.get_rank() if dist.is_initialized() else 0) == 0
    elif any(getattr(p, "_dla_ep", None) is not None for p in model.parameters()):
        writer = dist.get_rank(mesh.edp_group) == 0 if mesh.edp_group is not None else True
    else:
        writer = mesh.dp_rank == 0 and mesh.sp_rank == 0
    c["writer"] = writer
    return c


def _shard_file(stem: str, c) -> str:
    return f"{stem}.fsdp{c['fsdp']}-tp{c['tp']}-ep{c['ep']}.safetensors"


def save_rank_shards(model, out_dir, stem: str) -> Optional[str]:
    """Write this rank's LOCAL tensors (no collective). Returns the file written (or None)."""
    from safetensors.torch import save_file

    c = _coords(model)
    base = _base(model)
    eng = getattr(model, "_dla_fsdp", None)
    out = Path(out_dir)
    if c["writer"]:
        t: Dict[str, torch.Tensor] = {}
        in_fsdp = set()
        if eng is not None:
            t[FSDP_KEY] = eng.param_shard.detach().to("cpu", copy=True)
            in_fsdp = {id(p) for u in eng.units for p in u.params}
        for n, p in model.named_parameters():
            if id(p) not in in_fsdp:
                t[n] = p.detach().to("cpu", copy=True).contiguous()
        save_file(t, str(out / _shard_file(stem, c)), metadata={"format": "pt"})
    is_main = (dist.get_rank() if dist.is_initialized() else 0) == 0
    if is_main:
        params = {}
        for n, p in model.named_parameters():
            spec = getattr(p, "_dla_tp_spec", None)
            ep = getattr(p, "_dla_ep", None)
            params[n] = {"shape": list(p.shape), "dtype": str(p.dtype).replace("torch.", ""),
                         "tp_spec": [spec[0], list(spec[1])] if spec is not None and getattr(base, "tp_size", 1) > 1 else None,
                         "ep": ep[2] if ep is not None else 1}
        lay = {"stem": stem, "tp_size": getattr(base, "tp_size", 1),
               "ep_size": max([v["ep"] for v in params.values()] + [1]),
               "fsdp_world": eng.world if eng is not None else 1,
               "kind": type(model).__name__, "params": params,
               "cfg": base.cfg.to_dict() if hasattr(base, "cfg") else None,
               "fsdp_units": [{"numel": u.numel, "chunk": u.chunk, "shard_off": u.shard_off,
                               "params": [{"name": n, "offset": u.offsets[id(p)]}
                                          for n, p in model.named_parameters() if id(p) in u.offsets]}
                              for u in eng.units] if eng is not None else None}
        (out / f"{stem}.shards.json").write_text(json.dumps(lay, indent=1))
    return _shard_file(stem, c) if c["writer"] else None


def load_rank_shards(model, d, stem: str) -> bool:
    """Exact resume from this rank's shard file; False when the layout does not match."""
    from safetensors import safe_open

    d = Path(d)
    lay_f = d / f"{stem}.shards.json"
    if not lay_f.exists():
        return False
    lay = json.loads(lay_f.read_text())
    base = _base(model)
    eng = getattr(model, "_dla_fsdp", None)
    c = _coords(model)
    f = d / _shard_file(stem, c)
    ok = (f.exists() and int(lay["tp_size"]) == getattr(base, "tp_size", 1)
          and int(lay["fsdp_world"]) == (eng.world if eng is not None else 1))
    in_fsdp = {id(p) for u in eng.units for p in u.params} if eng is not None else set()
    if ok and eng is not None:
        # the flat shard is only meaningful under the SAME unit grouping: a different
        # fsdp_min_num_params can keep the total length and still move every element
        names = {id(p): n for n, p in model.named_parameters()}
        saved = lay.get("fsdp_units") or []
        now = [{"numel": u.numel, "chunk": u.chunk, "shard_off": u.shard_off,
                "params": sorted((names[id(p)], u.offsets[id(p)]) for p in u.params)} for u in eng.units]
        ok = len(saved) == len(now) and all(
            int(a["numel"]) == b["numel"] and int(a["chunk"]) == b["chunk"]
            and int(a["shard_off"]) == b["shard_off"]
            and sorted((q["name"], int(q["offset"])) for q in a["params"]) == b["params"]
            for a, b in zip(saved, now))
    if ok:
        with safe_open(str(f), framework="pt") as h:
            keys = set(h.keys())
            ok = (eng is not None) == (FSDP_KEY in keys)
            if ok and eng is not None:
                ok = h.get_slice(FSDP_KEY).get_shape() == [eng.param_shard.numel()]
            ok = ok and all(n in keys and list(h.get_slice(n).get_shape()) == list(p.shape)
                            for n, p in model.named_parameters() if id(p) not in in_fsdp)
    if dist.is_initialized():  # every rank takes the same branch (the FSDP root re-gather is collective)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                            device=eng.device if eng is not None else next(model.parameters()).device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = bool(flag.item())
    if not ok:
        return False
    with safe_open(str(f), framework="pt") as h, torch.no_grad():
        if eng is not None:
            eng.param_shard.copy_(h.get_tensor(FSDP_KEY).to(eng.param_shard.device))
            if getattr(eng, "master", None) is not None:
                eng.master.copy_(eng.param_shard.float())
            for u in eng.units:  # resident units (the root) re-gather from the new shards
                if u.resident:
                    u.resident = False
                    eng._gather(u)
        for n, p in model.named_parameters():
            if id(p) not in in_fsdp:
                p.data.copy_(h.get_tensor(n).to(p.device))
    return True
