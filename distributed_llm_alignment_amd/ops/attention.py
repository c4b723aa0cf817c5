"""Rotary embedding + flash attention.

Entry points
  * `qkv_attention(qkv, ...)`: the training/prefill path. Takes the fused QKV projection output
    `[B, T, (Hq + 2*Hkv) * D]` and returns `[B, T, Hq * D]` (ready for o_proj). On the GPU this
    is ONE autograd node: HIP RoPE -> HIP flash-attention forward; the backward runs the HIP
    flash-attention backward and the HIP RoPE backward and returns a single fused dQKV buffer
    (dV is written in place by the attention kernel, dQ/dK un-rotated straight into it).
  * `attention_core(q, k, v, ...)`: [B, T, H, D] tensors (KV-cache decode, odd head dims).
  * `RotaryCache`: host-precomputed fp32 cos/sin tables (HF `rotate_half` convention, optional
    partial rotary and Llama-3.1 frequency scaling).

Masking semantics (all paths, matching HF SDPA with a causal + padding mask): key j is visible
to query i of batch b iff kv_start[b] <= j < kv_end[b], and for causal attention
j <= i + causal_off (causal_off = Tk - Tq), and with a sliding window j > i + causal_off - window.
Fully-masked query rows produce zeros.
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from . import _ext


class RotaryCache:
    """cos/sin tables [max_pos, rot_dim/2] in fp32, one copy per device."""

    def __init__(self, rot_dim: int, theta: float = 10000.0, max_pos: int = 4096,
                 scaling: Optional[dict] = None):
        self.rot_dim = rot_dim
        self.theta = theta
        self.max_pos = max_pos
        inv = 1.0 / (theta ** (torch.arange(0, rot_dim, 2, dtype=torch.float64) / rot_dim))
        if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
            factor = scaling.get("factor", 8.0)
            lo = scaling.get("low_freq_factor", 1.0)
            hi = scaling.get("high_freq_factor", 4.0)
            old = scaling.get("original_max_position_embeddings", 8192)
            lo_wl, hi_wl = old / lo, old / hi
            wl = 2 * math.pi / inv
            scaled = torch.where(wl > lo_wl, inv / factor, inv)
            smooth = (old / wl - lo) / (hi - lo)
            mid = (1 - smooth) * scaled / factor + smooth * scaled
            is_mid = (wl >= hi_wl) & (wl <= lo_wl)
            inv = torch.where(is_mid, mid, scaled)
        elif scaling and scaling.get("rope_type", scaling.get("type")) == "linear":
            inv = inv / scaling.get("factor", 1.0)
        t = torch.arange(max_pos, dtype=torch.float64)
        freqs = torch.outer(t, inv)
        self._cos = freqs.cos().float()
        self._sin = freqs.sin().float()
        self._dev: Dict[torch.device, tuple] = {}

    def tables(self, device: torch.device):
        device = torch.device(device)
        if device.type == "cpu":
            return self._cos, self._sin
        if device not in self._dev:
            self._dev[device] = (self._cos.to(device), self._sin.to(device))
        return self._dev[device]


# ---------------------------------------------------------------------------------------------
# pure-PyTorch reference (CPU path + numerics oracle)
# ---------------------------------------------------------------------------------------------
def _ref_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor,
              rot: int) -> torch.Tensor:
    """x [B, T, H, D]; pos [B, T] long. rotate-half over the first `rot` dims."""
    xf = x.float()
    c = cos[pos].unsqueeze(2)  # [B, T, 1, rot/2]
    s = sin[pos].unsqueeze(2)
    half = rot // 2
    x1, x2, rest = xf[..., :half], xf[..., half:rot], xf[..., rot:]
    o1 = x1 * c - x2 * s
    o2 = x2 * c + x1 * s
    return torch.cat([o1, o2, rest], dim=-1).to(x.dtype)


def _visibility(B, Tq, Tk, causal, causal_off, window, kv_start, kv_end, device, segs=None):
    qi = torch.arange(Tq, device=device).view(1, Tq, 1)
    kj = torch.arange(Tk, device=device).view(1, 1, Tk)
    ok = torch.ones(B, Tq, Tk, dtype=torch.bool, device=device)
    if segs is not None:  # packed sequences: query i sees keys >= seg_start[i] (block diagonal)
        ok = ok & (kj >= segs[0].view(B, Tq, 1).to(device))
    if kv_start is not None:
        ok = ok & (kj >= kv_start.view(B, 1, 1).to(device))
    if kv_end is not None:
        ok = ok & (kj < kv_end.view(B, 1, 1).to(device))
    if causal:
        ok = ok & (kj <= qi + causal_off)
        if window and window > 0:
            ok = ok & (kj > qi + causal_off - window)
    return ok


def ref_attention(q, k, v, scale, causal=True, causal_off=0, window=0, kv_start=None,
                  kv_end=None, segs=None) -> torch.Tensor:
    """q [B, Tq, Hq, D], k/v [B, Tk, Hkv, D] -> [B, Tq, Hq, D] (fp32 math)."""
    B, Tq, Hq, D = q.shape
    Tk, Hkv = k.shape[1], k.shape[2]
    rep = Hq // Hkv
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    ok = _visibility(B, Tq, Tk, causal, causal_off, window, kv_start, kv_end, q.device, segs)
    s = s.masked_fill(~ok.unsqueeze(1), float("-inf"))
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    o = torch.matmul(p, vf).transpose(1, 2)
    return o.to(q.dtype)


# ---------------------------------------------------------------------------------------------
# GPU autograd nodes
# ---------------------------------------------------------------------------------------------
def _i32(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if t is None else t.to(dtype=torch.int32).contiguous()


# Full-rotary RoPE backward folded into the attention backward's dQ reduce / dK-dV passes (no
# separate rope_bwd launch, no rotated-space dq/dk temporaries); DLA_FUSED_ROPE_BWD=0 restores
# the separate kernel for A/B runs.
FUSED_ROPE_BWD = os.environ.get("DLA_FUSED_ROPE_BWD", "1") != "0"
# Full-rotary RoPE forward folded into the attention kernels ("RoPE on load": no rope_fwd launch,
# no rotated K copy; the forward writes the rotated Q only when a backward needs it). Off by
# default: same-box A/B on the Llama-3-8B DPO step 1611-1613 (on) vs 1608-1609 ms (off) — every
# forward workgroup re-rotates each K tile it stages (16 query blocks per sequence at T = 1024),
# which costs more than the one 40 us rope pass it replaces. DLA_FUSED_ROPE_FWD=1 enables it.
FUSED_ROPE_FWD = os.environ.get("DLA_FUSED_ROPE_FWD", "0") == "1"
# Q-only RoPE on load (the default at full rotary, D 64 / 128): the forward kernel rotates the
# Q rows it loads once per workgroup (and writes the rotated Q for the backward when there is
# one), and the rope kernel rotates only K -- a fifth of the bytes of the q + k pass (Llama-3
# GQA 32 / 8) -- so no workgroup re-rotates K tiles. DLA_ROPE_Q_ON_LOAD=0 restores the q + k pass.
ROPE_Q_ON_LOAD = os.environ.get("DLA_ROPE_Q_ON_LOAD", "1") != "0"


class _FusedQKVAttnFn(torch.autograd.Function):
    """qkv [B, T, C] -> o [B, T, Hq*D]; RoPE (optional) fused in; returns one dqkv."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, pos, Hq, Hkv, D, rot, scale, causal, window, kv_start, kv_end,
                segs=None):
        ops = _ext.require()
        B, T, C = qkv.shape
        q2 = qkv.reshape(B * T, C)
        off = qkv.storage_offset()
        v4 = qkv.as_strided((B, T, Hkv, D), (T * C, C, D, 1), off + (Hq + Hkv) * D)
        on_load = rot == D and D in (64, 128) and FUSED_ROPE_FWD
        q_load = rot == D and D in (64, 128) and ROPE_Q_ON_LOAD and not on_load
        if q_load:
            # K rotated by the rope kernel over the K columns only; Q rotated on load
            _, k_r = ops.rope_fwd(q2[:, Hq * D:], cos, sin, pos, 0, Hkv, D, rot, T, 0)
            q4 = qkv.as_strided((B, T, Hq, D), (T * C, C, D, 1), off)
            k4 = k_r.view(B, T, Hkv, D)
            q_rot = torch.empty((B, T, Hq, D), dtype=qkv.dtype, device=qkv.device) \
                if ctx.needs_input_grad[0] else None
            o, lse2 = ops.attn_fwd(q4, k4, v4, float(scale), bool(causal), 0, int(window), kv_start,
                                   kv_end, segs, cos, sin, pos, q_rot, False)
            ctx.save_for_backward(qkv, q_rot, k4, o, lse2, cos, sin, pos, kv_start, kv_end, segs)
        elif on_load:
            # RoPE on load: the kernel rotates Q in registers and K as it stages it; the rotated
            # Q leaves as a side output only when a backward will read it
            q4 = qkv.as_strided((B, T, Hq, D), (T * C, C, D, 1), off)
            k4 = qkv.as_strided((B, T, Hkv, D), (T * C, C, D, 1), off + Hq * D)
            q_rot = torch.empty((B, T, Hq, D), dtype=qkv.dtype, device=qkv.device) \
                if ctx.needs_input_grad[0] else None
            o, lse2 = ops.attn_fwd(q4, k4, v4, float(scale), bool(causal), 0, int(window), kv_start,
                                   kv_end, segs, cos, sin, pos, q_rot)
            ctx.save_for_backward(qkv, q_rot, None, o, lse2, cos, sin, pos, kv_start, kv_end, segs)
        else:
            if rot > 0:
                q_r, k_r = ops.rope_fwd(q2, cos, sin, pos, Hq, Hkv, D, rot, T, 0)
                q4 = q_r.view(B, T, Hq, D)
                k4 = k_r.view(B, T, Hkv, D)
            else:
                q4 = qkv.as_strided((B, T, Hq, D), (T * C, C, D, 1), off)
                k4 = qkv.as_strided((B, T, Hkv, D), (T * C, C, D, 1), off + Hq * D)
            o, lse2 = ops.attn_fwd(q4, k4, v4, float(scale), bool(causal), 0, int(window), kv_start,
                                   kv_end, segs)
            ctx.save_for_backward(qkv, q4 if rot > 0 else None, k4 if rot > 0 else None, o, lse2,
                                  cos, sin, pos, kv_start, kv_end, segs)
        ctx.on_load = on_load
        ctx.cfg = (B, T, C, Hq, Hkv, D, rot, scale, causal, window)
        return o.view(B, T, Hq * D)

    @staticmethod
    def backward(ctx, do):
        ops = _ext.require()
        qkv, q4, k4, o, lse2, cos, sin, pos, kv_start, kv_end, segs = ctx.saved_tensors
        B, T, C, Hq, Hkv, D, rot, scale, causal, window = ctx.cfg
        off = qkv.storage_offset()
        if ctx.on_load:  # q4 = the forward's rotated Q; K is rotated again as it is staged
            k4 = qkv.as_strided((B, T, Hkv, D), (T * C, C, D, 1), off + Hq * D)
        elif rot == 0:
            q4 = qkv.as_strided((B, T, Hq, D), (T * C, C, D, 1), off)
            k4 = qkv.as_strided((B, T, Hkv, D), (T * C, C, D, 1), off + Hq * D)
        v4 = qkv.as_strided((B, T, Hkv, D), (T * C, C, D, 1), off + (Hq + Hkv) * D)
        do4 = do.contiguous().view(B, T, Hq, D)
        dqkv = torch.empty((B, T, C), dtype=qkv.dtype, device=qkv.device)
        dv = dqkv.as_strided((B, T, Hkv, D), (T * C, C, D, 1), (Hq + Hkv) * D)
        # full rotary at D 64 / 128, or phi-2's partial rotary (32 of D = 80 dims: the dK
        # epilogue un-rotates column tile 0, the reduce passes the rotary chunk pairs)
        fused_rope = (rot == D and D in (64, 128) or (D == 80 and rot == 32)) and \
            (FUSED_ROPE_BWD or ctx.on_load)
        if rot > 0 and not fused_rope:  # rotated-space dq / dk, un-rotated by the RoPE backward
            dq = torch.empty((B, T, Hq, D), dtype=qkv.dtype, device=qkv.device)
            dk = torch.empty((B, T, Hkv, D), dtype=qkv.dtype, device=qkv.device)
        else:  # written straight into the fused dqkv buffer (un-rotated in the attention passes)
            dq = dqkv.as_strided((B, T, Hq, D), (T * C, C, D, 1), 0)
            dk = dqkv.as_strided((B, T, Hkv, D), (T * C, C, D, 1), Hq * D)
        if fused_rope:
            ops.attn_bwd(do4, q4, k4, v4, o, lse2, dq, dk, dv, float(scale), bool(causal), 0,
                         int(window), kv_start, kv_end, segs, cos, sin, pos, bool(ctx.on_load))
        else:
            ops.attn_bwd(do4, q4, k4, v4, o, lse2, dq, dk, dv, float(scale), bool(causal), 0,
                         int(window), kv_start, kv_end, segs)
        if rot > 0 and not fused_rope:
            ops.rope_bwd(dq.view(B * T, Hq * D), dk.view(B * T, Hkv * D), dqkv.view(B * T, C),
                         cos, sin, pos, Hq, Hkv, D, rot, T, 0)
        return dqkv, None, None, None, None, None, None, None, None, None, None, None, None, None


class _AttnCoreFn(torch.autograd.Function):
    """[B, T, H, D] q/k/v -> o. Used for KV-cache decode and padded head dims."""

    @staticmethod
    def forward(ctx, q, k, v, scale, causal, causal_off, window, kv_start, kv_end, segs=None):
        ops = _ext.require()
        o, lse2 = ops.attn_fwd(q, k, v, float(scale), bool(causal), int(causal_off), int(window),
                               kv_start, kv_end, segs)
        ctx.save_for_backward(q, k, v, o, lse2, kv_start, kv_end, segs)
        ctx.cfg = (scale, causal, causal_off, window)
        return o

    @staticmethod
    def backward(ctx, do):
        ops = _ext.require()
        q, k, v, o, lse2, kv_start, kv_end, segs = ctx.saved_tensors
        scale, causal, causal_off, window = ctx.cfg
        dq = torch.empty_like(q, memory_format=torch.contiguous_format)
        dk = torch.empty_like(k, memory_format=torch.contiguous_format)
        dv = torch.empty_like(v, memory_format=torch.contiguous_format)
        ops.attn_bwd(do.contiguous(), q, k, v, o, lse2, dq, dk, dv, float(scale), bool(causal),
                     int(causal_off), int(window), kv_start, kv_end, segs)
        return dq, dk, dv, None, None, None, None, None, None, None


# head dims with a native kernel tile: 64 / 128, and 80 (phi-2: Q.K^T over exactly 5 MFMA k-steps,
# 96-wide LDS images whose 16 zero pad columns cost only the P.V / dK / dV tiles; csrc/attention.hip
# attn_dp). Others are zero-padded to the next native size. DLA_ATTN_D80=0 pads D = 80 to 128.
NATIVE_HEAD_DIMS = (64, 80, 128) if os.environ.get("DLA_ATTN_D80", "1") != "0" else (64, 128)


def _pad_d(x: torch.Tensor, Dp: int) -> torch.Tensor:
    return F.pad(x, (0, Dp - x.shape[-1]))


def attention_core(q, k, v, scale=None, causal=True, causal_off=None, window=0, kv_start=None,
                   kv_end=None, segs=None) -> torch.Tensor:
    """q [B, Tq, Hq, D], k/v [B, Tk, Hkv, D] (unit stride on D) -> [B, Tq, Hq, D]."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if causal_off is None:
        causal_off = k.shape[1] - q.shape[1]
    if not _ext.use_native(q):
        return ref_attention(q, k, v, scale, causal, causal_off, window, kv_start, kv_end, segs)
    ks, ke, sg = _i32(kv_start), _i32(kv_end), _i32(segs)
    if D in NATIVE_HEAD_DIMS:
        return _AttnCoreFn.apply(q, k, v, scale, causal, causal_off, window, ks, ke, sg)
    Dp = 64 if D < 64 else 128
    o = _AttnCoreFn.apply(_pad_d(q, Dp), _pad_d(k, Dp), _pad_d(v, Dp), scale, causal, causal_off,
                          window, ks, ke, sg)
    return o[..., :D]


def apply_rope(x: torch.Tensor, rope: RotaryCache, positions: torch.Tensor) -> torch.Tensor:
    """x [B, T, H, D] -> rotated (reference math; used on small decode tensors and CPU)."""
    cos, sin = rope.tables(x.device)
    return _ref_rope(x, cos, sin, positions.long(), rope.rot_dim)


def qkv_attention(qkv: torch.Tensor, Hq: int, Hkv: int, D: int, rope: Optional[RotaryCache],
                  causal: bool = True, window: int = 0, kv_start=None, kv_end=None,
                  positions: Optional[torch.Tensor] = None, scale: Optional[float] = None,
                  segs: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused QKV -> (RoPE) -> attention. qkv [B, T, (Hq+2Hkv)*D] -> [B, T, Hq*D].
    `segs` [2, B, T] int32 (seg_start; seg_end): packed sequences, block-diagonal causal mask."""
    B, T, C = qkv.shape
    assert C == (Hq + 2 * Hkv) * D, "qkv width mismatch"
    if rope is not None and T > rope.max_pos:
        raise ValueError(f"sequence length {T} exceeds the rotary table ({rope.max_pos})")
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    rot = rope.rot_dim if rope is not None else 0
    if not _ext.use_native(qkv):
        q = qkv[..., : Hq * D].reshape(B, T, Hq, D)
        k = qkv[..., Hq * D:(Hq + Hkv) * D].reshape(B, T, Hkv, D)
        v = qkv[..., (Hq + Hkv) * D:].reshape(B, T, Hkv, D)
        if rope is not None:
            pos = positions if positions is not None else torch.arange(T, device=qkv.device).expand(B, T)
            q = apply_rope(q, rope, pos)
            k = apply_rope(k, rope, pos)
        o = ref_attention(q, k, v, scale, causal, 0, window, kv_start, kv_end, segs)
        return o.reshape(B, T, Hq * D)
    ks, ke, sg = _i32(kv_start), _i32(kv_end), _i32(segs)
    pos32 = _i32(positions.reshape(-1)) if positions is not None else None
    if D in NATIVE_HEAD_DIMS:
        if rope is not None:
            cos, sin = rope.tables(qkv.device)
        else:
            cos = sin = torch.empty(0, device=qkv.device)
        return _FusedQKVAttnFn.apply(qkv.contiguous(), cos, sin, pos32, Hq, Hkv, D, rot, scale,
                                     causal, window, ks, ke, sg)
    # other head dims (e.g. 96, 256): HIP RoPE forward/backward on the fused
    # qkv buffer (the kernels take any D % 8 == 0), then the native attention core on head dims
    # zero-padded to the next supported size
    if rope is not None and D % 8 == 0 and rot % 16 == 0:
        cos, sin = rope.tables(qkv.device)
        q, k, v = _RopeQKFn.apply(qkv.contiguous(), cos, sin, pos32, Hq, Hkv, D, rot)
    else:
        q = qkv[..., : Hq * D].reshape(B, T, Hq, D)
        k = qkv[..., Hq * D:(Hq + Hkv) * D].reshape(B, T, Hkv, D)
        v = qkv[..., (Hq + Hkv) * D:].reshape(B, T, Hkv, D)
        if rope is not None:
            pos = positions if positions is not None else torch.arange(T, device=qkv.device).expand(B, T)
            q = apply_rope(q, rope, pos)
            k = apply_rope(k, rope, pos)
    o = attention_core(q, k, v, scale, causal, 0, window, kv_start, kv_end, segs)
    return o.reshape(B, T, Hq * D)


class _RopeQKFn(torch.autograd.Function):
    """qkv [B, T, (Hq+2Hkv)D] -> rotated q [B,T,Hq,D], k [B,T,Hkv,D] and v [B,T,Hkv,D] on the
    HIP rope kernels (forward rope_fwd; backward rope_bwd un-rotates dq/dk straight into dqkv)."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, pos32, Hq, Hkv, D, rot):
        B, T, C = qkv.shape
        q, k = _ext.require().rope_fwd(qkv.reshape(B * T, C), cos, sin, pos32, Hq, Hkv, D, rot, T, 0)
        v = qkv[..., (Hq + Hkv) * D:].reshape(B, T, Hkv, D)
        ctx.save_for_backward(cos, sin, pos32)
        ctx.cfg = (B, T, C, Hq, Hkv, D, rot)
        return q.view(B, T, Hq, D), k.view(B, T, Hkv, D), v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin, pos32 = ctx.saved_tensors
        B, T, C, Hq, Hkv, D, rot = ctx.cfg
        dqkv = torch.empty((B, T, C), dtype=dq.dtype, device=dq.device)
        _ext.require().rope_bwd(dq.contiguous().view(B * T, Hq * D), dk.contiguous().view(B * T, Hkv * D),
                                dqkv.view(B * T, C), cos, sin, pos32, Hq, Hkv, D, rot, T, 0)
        dqkv[..., (Hq + Hkv) * D:] = dv.reshape(B, T, Hkv * D)
        return dqkv, None, None, None, None, None, None, None


def rope_qk(qkv: torch.Tensor, rope: Optional[RotaryCache], Hq: int, Hkv: int, D: int,
            positions: Optional[torch.Tensor] = None, pos_offset: int = 0):
    """Inference helper (no autograd): qkv [B, T, C] -> rotated q [B,T,Hq,D], k [B,T,Hkv,D] and
    the v view [B,T,Hkv,D]. positions [B, T] (or t + pos_offset when None)."""
    B, T, C = qkv.shape
    v = qkv[..., (Hq + Hkv) * D:].reshape(B, T, Hkv, D)
    if rope is not None and T + pos_offset > rope.max_pos:
        raise ValueError("positions exceed the rotary table")
    if rope is None:
        return (qkv[..., : Hq * D].reshape(B, T, Hq, D),
                qkv[..., Hq * D:(Hq + Hkv) * D].reshape(B, T, Hkv, D), v)
    if _ext.use_native(qkv) and D % 8 == 0 and rope.rot_dim % 16 == 0:
        cos, sin = rope.tables(qkv.device)
        pos32 = _i32(positions.reshape(-1)) if positions is not None else None
        q, k = _ext.require().rope_fwd(qkv.reshape(B * T, C).contiguous(), cos, sin, pos32, Hq, Hkv,
                                       D, rope.rot_dim, T, int(pos_offset))
        return q.view(B, T, Hq, D), k.view(B, T, Hkv, D), v
    if positions is None:
        positions = (torch.arange(T, device=qkv.device) + pos_offset).expand(B, T)
    q = apply_rope(qkv[..., : Hq * D].reshape(B, T, Hq, D), rope, positions)
    k = apply_rope(qkv[..., Hq * D:(Hq + Hkv) * D].reshape(B, T, Hkv, D), rope, positions)
    return q, k, v
