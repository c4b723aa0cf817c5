"""Decode-path ops: split-KV GQA decode attention and the fused top-k/top-p sampler.

GPU tensors run `torch.ops.dla.decode_attn` / `torch.ops.dla.sample_tokens` (csrc/decode.hip,
csrc/sampling.hip); both take their lengths / RNG counter from device memory so a decode step can
be captured once in a hipGraph and replayed per token. CPU tensors use PyTorch references.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import _ext


def decode_supported(q_heads: int, kv_heads: int, head_dim: int) -> bool:
    return head_dim in (64, 128) and q_heads % kv_heads == 0 and (q_heads // kv_heads) in (1, 2, 4, 8)


def decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                     kv_len: torch.Tensor, kv_start: Optional[torch.Tensor] = None, window: int = 0,
                     scale: Optional[float] = None) -> torch.Tensor:
    """q [B, Hq, D] (the newest token), caches [B, Tmax, Hkv, D]; keys [kv_start, kv_len) are
    attended (kv_len: int32 [1] on device). Returns [B, Hq, D]."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if _ext.use_native(q):
        return _ext.require().decode_attn(q, k_cache, v_cache, kv_len.to(torch.int32),
                                          kv_start.to(torch.int32) if kv_start is not None else None,
                                          int(window), float(scale))
    return ref_decode_attention(q, k_cache, v_cache, int(kv_len.reshape(-1)[0]), kv_start, window, scale)


def ref_decode_attention(q, k_cache, v_cache, L: int, kv_start=None, window: int = 0, scale=None):
    B, Hq, D = q.shape
    Hkv = k_cache.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    k = k_cache[:, :L].float().repeat_interleave(Hq // Hkv, dim=2)  # [B, L, Hq, D]
    v = v_cache[:, :L].float().repeat_interleave(Hq // Hkv, dim=2)
    s = torch.einsum("bhd,blhd->bhl", q.float(), k) * scale
    idx = torch.arange(L, device=q.device)
    lo = kv_start.view(B, 1).long() if kv_start is not None else torch.zeros(B, 1, dtype=torch.long, device=q.device)
    if window and window > 0:
        lo = torch.clamp(lo, min=L - window)
    mask = idx.view(1, L) < lo
    s = s.masked_fill(mask.view(B, 1, L), float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("bhl,blhd->bhd", p, v).to(q.dtype)


def sample_tokens(logits: torch.Tensor, temperature: float, top_k: int, top_p: float, greedy: bool,
                  rng: torch.Tensor, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """logits [B, V] -> token ids [B] (int64). rng: int64 [2] device tensor (seed, counter) for
    the fused kernel; CPU falls back to `models.generation.sample_next` semantics."""
    if _ext.use_native(logits):
        return _ext.require().sample_tokens(logits, float(temperature), int(top_k), float(top_p),
                                            bool(greedy), rng)
    from ..models.generation import sample_next

    return sample_next(logits.float(), not greedy, temperature, top_p, top_k, generator)


# ------------------------------------------------------------------------- skinny GEMM (M <= 16)
SKINNY = os.environ.get("DLA_SKINNY", "1") != "0"
# Every decode GEMM takes the skinny kernels: wide outputs (>= 128 column blocks) the LDS-staged
# kernel without split-K, narrow ones the in-workgroup split-K kernel. The cross-workgroup
# split-K form (agent-scope release per workgroup) stays only for shapes neither fits, since inside
# a real decode step it was 1.66x slower (profiles/r1_decode_skinny.md). DLA_SKINNY_MIN_N raises
# the width threshold for A/B runs.
SKINNY_MIN_N = int(os.environ.get("DLA_SKINNY_MIN_N", "0"))
SKINNY_WIDE_N = 128 * 128  # >= this many output columns: the kernel runs without any split-K
# measured in a decode step (profiles/r1_decode_skinny.md): hipBLASLt stays ahead for the LM head
# (N = 128256) and for the long-K narrow down projection (K = 14336), so those keep the library
SKINNY_MAX_N = int(os.environ.get("DLA_SKINNY_MAX_N", "65536"))
SKINNY_MAX_NARROW_K = int(os.environ.get("DLA_SKINNY_MAX_NARROW_K", "8192"))
_COUNTERS = {}


def _skinny_counters(dev: torch.device) -> Optional[torch.Tensor]:
    """Per-device split-K arrival counters (zeroed once; the kernel re-arms them). Never created
    inside a hipGraph capture (it would become a graph-pool allocation + memset node)."""
    key = dev.index
    c = _COUNTERS.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return None
        c = torch.zeros(8192, dtype=torch.int32, device=dev)
        _COUNTERS[key] = c
    return c


# 17..64 decode rows can run on the split-K kernels with 2 or 4 row tiles per weight fragment
# (narrow outputs N < 16384 with K % 1024 == 0, and the gate|up GLU kernel; DLA_SKINNY_MAX_ROWS=64).
# Off by default: measured on 1x MI355X (Llama-3-8B, prompt 512, graph decode) 11.57 vs 6.11
# ms/token at 64 rows and 7.12 vs 5.09 at 32 -- every workgroup re-reads all of x for its 16
# output columns (~1.7 GB of L2 -> CU traffic per layer at 64 rows), which costs more than the
# weight stream it shares; hipBLASLt's 16-64 x 64 tiles keep 17+ rows.
SKINNY_MAX_ROWS = int(os.environ.get("DLA_SKINNY_MAX_ROWS", "16"))
SKINNY_KS_MAX_K = int(os.environ.get("DLA_SKINNY_KS_MAX_K", str(1 << 20)))  # A/B: long-K down on hipBLASLt


SKINNY_GLU_MAX_ROWS = int(os.environ.get("DLA_SKINNY_GLU_MAX_ROWS", "64"))


def _ks_rows_ok(rows: int, N: int, K: int, glu: bool) -> bool:
    if glu:
        return rows <= min(SKINNY_MAX_ROWS, SKINNY_GLU_MAX_ROWS) and K % 512 == 0 and N % 32 == 0
    return (rows <= SKINNY_MAX_ROWS and N < SKINNY_WIDE_N and K % 1024 == 0 and N % 16 == 0
            and K <= SKINNY_KS_MAX_K)


def skinny_ok(x: torch.Tensor, weight: torch.Tensor, swiglu: bool = False,
              min_n: Optional[int] = None, glu: bool = False) -> bool:
    """Inference-only decode GEMM: <= 16 rows (<= 64 on the split-K kernels), bf16,
    K % 256 == 0, N % 16 == 0, no autograd. `glu`: the gate|up GEMM with the SwiGLU epilogue."""
    if not (SKINNY and _ext.use_native(x)) or torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad):
        return False
    rows = x.numel() // x.shape[-1] if x.dim() else 0
    N, K = weight.shape if weight.dim() == 2 else (0, 0)
    if rows > 16:
        if swiglu or not _ks_rows_ok(rows, N, K, glu):
            return False
    elif min_n is None and (N > SKINNY_MAX_N or (N < SKINNY_WIDE_N and K > SKINNY_MAX_NARROW_K)):
        return False
    return (1 <= rows <= 64 and N >= (SKINNY_MIN_N if min_n is None else min_n) and x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and weight.dim() == 2 and weight.stride(1) == 1 and weight.stride(0) % 8 == 0
            and x.shape[-1] == (2 * K if swiglu else K) and K % 256 == 0 and N % 16 == 0
            and (N + 127) // 128 <= 8192 and x.device == weight.device)


def skinny_linear(x: torch.Tensor, weight: torch.Tensor, swiglu: bool = False,
                  min_n: Optional[int] = None) -> Optional[torch.Tensor]:
    """y = x @ weight^T (or swiglu(x) @ weight^T) with the decode skinny-GEMM kernel
    (csrc/skinny.hip). Returns None when the shape/state is not eligible (caller falls back)."""
    if not skinny_ok(x, weight, swiglu, min_n):
        return None
    cnt = _skinny_counters(x.device)
    if cnt is None:
        return None
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(-1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    y = _ext.require().skinny_gemm(x2, weight, cnt, bool(swiglu))
    return y.view(*x.shape[:-1], weight.shape[0])


# gate|up kernel: "ks" = in-workgroup split-K (F / 16 workgroups, 4 waves per gate / up K
# quarter), "lds" = x staged in LDS, one wave per 16 rows over all of K (F / 64 workgroups)
SKINNY_GLU = os.environ.get("DLA_SKINNY_GLU", "lds")


def skinny_glu(x: torch.Tensor, weight: torch.Tensor, mode: Optional[str] = None) -> Optional[torch.Tensor]:
    """Decode gate|up projection with SwiGLU in the epilogue: weight = [gate; up] (2F rows) ->
    silu(x gate^T) * (x up^T) [.., F] in one kernel (csrc/skinny.hip). None if the
    shape/state is not eligible (the caller runs GEMM + swiglu)."""
    if not skinny_ok(x, weight, glu=True):
        return None
    rows = x.numel() // x.shape[-1]
    if ((mode or SKINNY_GLU) == "ks" or rows > 16) and x.shape[-1] % 512 == 0 and weight.shape[0] % 32 == 0:
        x2 = x.reshape(-1, x.shape[-1])
        if x2.stride(-1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
            x2 = x2.contiguous()
        return _ext.require().skinny_glu_ks(x2, weight).view(*x.shape[:-1], weight.shape[0] // 2)
    if weight.shape[0] % 128 or x.shape[-1] * min(x.numel() // x.shape[-1], 16) > 80 * 1024:
        return None
    cnt = _skinny_counters(x.device)
    if cnt is None:
        return None
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(-1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    m = _ext.require().skinny_gemm(x2, weight, cnt, False, True)
    return m.view(*x.shape[:-1], weight.shape[0] // 2)


def ref_skinny_linear(x: torch.Tensor, weight: torch.Tensor, swiglu: bool = False) -> torch.Tensor:
    if swiglu:
        g, u = x.float().chunk(2, dim=-1)
        x = (torch.nn.functional.silu(g) * u).to(x.dtype)
    return (x.float() @ weight.float().t()).to(x.dtype)


# ------------------------------------------------------- fused decode layer (residual + norm)
# Each decode layer's two residual-add + RMSNorm launches (4.8 us each at Llama-3-8B B=8,
# profiles/r2_decode.md: pure launch ramp / latency on 64 KB) are split across the neighbouring
# projections instead (csrc/skinny.hip KsFuse): the o and down projections write the new
# residual stream s = x + y plus per-(row, 16 columns) partial sums of s^2, and the next
# projection (gate|up, or the next layer's qkv) computes RMSNorm(s) W^T = rstd * (s (W o w)^T):
# a plain GEMM on s against a cached copy of W with the norm weight w folded into its columns,
# whose epilogue scales each row by rstd (from the producer's partials). DLA_DECODE_FUSED_NORM=0
# keeps the separate norm launches.
DECODE_FUSED_NORM = os.environ.get("DLA_DECODE_FUSED_NORM", "1") != "0"


# 17..64 decode rows (the reference's 64-rollout RLHF batch): the fused layer runs on the
# csrc/skinny64.hip kernels -- x streamed through an LDS ring shared by 8 waves x 16 columns,
# split-K slabs reduced by a second launch that applies the residual / norm epilogue.
# DLA_DECODE_M64=0 keeps those rows on hipBLASLt + separate norm / SwiGLU launches.
DECODE_M64 = os.environ.get("DLA_DECODE_M64", "1") != "0"  # A/B: profiles/r3_decode_b64.md


def _m64_layer_ok(H: int, qkv_w, o_w, up_w, down_w) -> bool:
    F2 = up_w.shape[0]
    return (H % 256 == 0 and H <= 8192 and qkv_w.shape[0] % 128 == 0 and o_w.shape[0] == H
            and H % 128 == 0 and o_w.shape[1] % 256 == 0 and F2 % 128 == 0
            and down_w.shape == (H, F2 // 2) and (F2 // 2) % 256 == 0)


def fused_layer_ok(x: torch.Tensor, H: int, qkv_w: torch.Tensor, o_w: torch.Tensor,
                   up_w: torch.Tensor, down_w: torch.Tensor) -> bool:
    """Shapes / state the fused decode layer supports (M <= 16 bf16 rows on csrc/skinny.hip,
    17..64 on csrc/skinny64.hip; no autograd)."""
    if not (DECODE_FUSED_NORM and SKINNY and _ext.use_native(x)) or torch.is_grad_enabled():
        return False
    rows = x.numel() // x.shape[-1]
    if not (1 <= rows <= 64 and x.dtype == torch.bfloat16 and x.shape[-1] == H):
        return False
    if rows > 16:
        return (DECODE_M64 and _m64_layer_ok(H, qkv_w, o_w, up_w, down_w)
                and all(w.dtype == torch.bfloat16 and w.stride(-1) == 1 and w.stride(0) % 8 == 0
                        for w in (qkv_w, o_w, up_w, down_w)))
    F2 = up_w.shape[0]
    ok = (H % 1024 == 0 and H < 16384 and H // 16 <= 512 and qkv_w.shape == (qkv_w.shape[0], H)
          and qkv_w.shape[0] < 16384 and qkv_w.shape[0] % 16 == 0 and o_w.shape[0] == H
          and o_w.shape[1] % 1024 == 0 and down_w.shape == (H, F2 // 2) and (F2 // 2) % 1024 == 0
          and F2 % 128 == 0 and rows * (H + 8) * 2 <= 148 * 1024)
    return ok and all(w.dtype == torch.bfloat16 and w.stride(-1) == 1 and w.stride(0) % 8 == 0
                      for w in (qkv_w, o_w, up_w, down_w))


def _rows(t: torch.Tensor) -> torch.Tensor:
    t2 = t.reshape(-1, t.shape[-1])
    if t2.stride(-1) != 1 or t2.stride(0) % 8 or t2.data_ptr() % 16:
        t2 = t2.contiguous()
    return t2


def _wkey(t: torch.Tensor):
    ep = getattr(t, "_dla_epoch", None)
    return (t.data_ptr(), t._version, ep[0] if ep is not None else 0)


# The fused decode layer's kernels read their weights in a tiled layout (csrc/skinny64.hip TW:
# [N/16, K/32, 4, 16, 8], each weight load 1 KB contiguous instead of 16 rows x 64 B at a K-row
# stride). DLA_DECODE_TILED: 1 = the folded qkv / gate|up copies (which exist anyway) are kept
# tiled; 2 (default) = also tiled copies of o / down (one extra copy of those two weights, ~4.8 GB
# for Llama-3-8B, made the first time the fused decode layer runs); 0 = row-major.
DECODE_TILED = int(os.environ.get("DLA_DECODE_TILED", "2"))


# B <= 16 gate|up, opt-in (DLA_DECODE_GLU_IL=1): one wave per 16-row tile holding 8 gate + the
# matching 8 up rows (interleaved tiled copy), SwiGLU by a lane swap, 7 waves per workgroup =
# exactly 256 workgroups at Llama-3-8B (csrc/skinny.hip skinny_glu_il_kernel). Bitwise equal to the
# default 8-wave kernel (224 workgroups) and no faster: 3.72 vs 3.72 ms/token, 47.0 vs 46.6 us per
# layer (same box), 3.69-3.70 with a 3- or 4-deep ring (DLA_GLU_IL_DEPTH) -- the gate|up stream is
# HBM-bound at ~5 TB/s, not short of CUs.
DECODE_GLU_IL = os.environ.get("DLA_DECODE_GLU_IL", "0") != "0"


def _glu_interleave(w: torch.Tensor) -> torch.Tensor:
    """[gate; up] rows (2F) -> row order gate 8t..8t+7, up 8t..8t+7 per 16-row tile."""
    F = w.shape[0] // 2
    return torch.stack((w[:F].reshape(F // 8, 8, -1), w[F:].reshape(F // 8, 8, -1)), 1).reshape(2 * F, -1)


def _tile_into(t: torch.Tensor, w: torch.Tensor, norm_w: Optional[torch.Tensor] = None,
               glu_il: bool = False) -> None:
    """t <- w (with norm_w: bf16(w * norm_w); glu_il: gate / up rows interleaved 8 + 8 per tile) in
    the tiled layout: one HIP pass on the GPU."""
    N, K = w.shape
    if _ext.use_native(w) and w.stride(-1) == 1 and w.stride(0) % 8 == 0:
        _ext.require().tile_weight(w, norm_w.contiguous() if norm_w is not None else None, t, bool(glu_il))
        return
    src = w * norm_w.view(1, -1) if norm_w is not None else w
    if glu_il:
        src = _glu_interleave(src)
    t.copy_(src.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4))


def _cached(w: torch.Tensor, attr: str, key, make) -> torch.Tensor:
    """Weight-derived cache on `w` (attr), refreshed IN PLACE when `key` moved: a captured decode
    graph keeps reading the same storage. Never made inside a capture (call
    `refresh_folded_weights` before capturing / replaying)."""
    c = getattr(w, attr, None)
    if c is None or c[0] != key:
        if w.is_cuda and torch.cuda.is_current_stream_capturing():
            if c is None:
                raise RuntimeError("derived decode weight first requested inside a graph capture")
            return c[1]
        with torch.no_grad():
            t = make(c[1] if c is not None else None)
        c = (key, t)
        setattr(w, attr, c)
    return c[1]


def folded_weight(w: torch.Tensor, norm_w: torch.Tensor, tiled: bool = False,
                  glu_il: bool = False) -> torch.Tensor:
    """Cached W o norm_w (the RMSNorm weight folded into W's input columns; `tiled`: in the
    skinny64 tiled layout, `glu_il`: tiled with gate / up rows interleaved), refreshed in place
    when either tensor changed (version counter / engine weight epoch)."""
    N, K = w.shape

    def make(t):
        if not tiled:
            t = t if t is not None else torch.empty_like(w, memory_format=torch.contiguous_format)
            torch.mul(w.detach(), norm_w.detach().view(1, -1), out=t)
            return t
        t = t if t is not None else torch.empty((N // 16, K // 32, 4, 16, 8), dtype=w.dtype, device=w.device)
        _tile_into(t, w.detach(), norm_w.detach(), glu_il)
        return t

    attr = "_dla_fold_g" if glu_il else ("_dla_fold_t" if tiled else "_dla_fold")
    return _cached(w, attr, (_wkey(w), _wkey(norm_w)), make)


def tiled_weight(w: torch.Tensor) -> torch.Tensor:
    """Cached copy of W in the skinny64 tiled layout (refreshed like `folded_weight`)."""
    N, K = w.shape

    def make(t):
        t = t if t is not None else torch.empty((N // 16, K // 32, 4, 16, 8), dtype=w.dtype, device=w.device)
        _tile_into(t, w.detach())
        return t

    return _cached(w, "_dla_tile", _wkey(w), make)


# ---------------------------------------------------------------------------------------------
# Weight-only fp8 decode (opt-in): the fused decode layer's four weight streams (qkv, o, gate|up,
# down: 74 % of the bytes per token at Llama-3-8B B=8) read an e4m3 copy with one fp32 scale per
# weight row (amax / 448), half the bf16 bytes; activations, the KV cache, the LM head and every
# accumulation stay bf16 / fp32 (csrc/skinny_ks.h F8, csrc/skinny.hip skinny_glu_il_kernel F8). For
# RLHF rollouts (`generate(..., weight_dtype="fp8")`, `ppo.rollout_weight_dtype`): the update's
# old-policy log-probs are recomputed in bf16 on the sampled tokens (training/train_rlhf.py), so
# the fp8 copy only changes which tokens are sampled. DLA_DECODE_FP8=1 turns it on process-wide.
_FP8 = [os.environ.get("DLA_DECODE_FP8", "0") == "1"]


class fp8_weights:
    """Context manager: decode projections on fp8 weight copies inside the block."""

    def __init__(self, enabled: bool = True):
        self.enabled = bool(enabled)

    def __enter__(self):
        self.prev = _FP8[0]
        _FP8[0] = self.enabled
        return self

    def __exit__(self, *exc):
        _FP8[0] = self.prev
        return False


def fp8_enabled() -> bool:
    return _FP8[0]


F8_MAX = 448.0  # largest finite e4m3 (OCP e4m3fn) value


def quantize_rows_f8(src: torch.Tensor):
    """src [N, K] -> (e4m3 values as uint8 [N, K], fp32 scales [N]): per-row amax scaling."""
    a = src.float()
    sc = (a.abs().amax(dim=1) / F8_MAX).clamp_min(1e-12)
    q = (a / sc[:, None]).clamp_(-F8_MAX, F8_MAX).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), sc.contiguous()


def tile_f8(q: torch.Tensor) -> torch.Tensor:
    """uint8 [N, K] -> the F8 tiled layout [N/16, K/64, 64, 16]: lane r + 16 qd of k-tile kt holds
    row r's k = 64 kt + 8 qd + [0, 8) then 64 kt + 32 + 8 qd + [0, 8) (csrc/skinny_ks.h F8)."""
    N, K = q.shape
    return (q.view(N // 16, 16, K // 64, 2, 4, 8).permute(0, 2, 4, 1, 3, 5)
            .reshape(N // 16, K // 64, 64, 16).contiguous())


def fp8_tiled_weight(w: torch.Tensor, norm_w: Optional[torch.Tensor] = None, glu_il: bool = False):
    """Cached (e4m3 tiled copy, per-row scales) of W (o norm_w folded in; glu_il: gate / up rows
    interleaved 8 + 8 per 16-row tile), refreshed when W or norm_w moved (as folded_weight)."""
    N, K = w.shape

    def make(prev):
        if _ext.use_native(w) and w.stride(-1) == 1 and w.stride(0) % 8 == 0:
            # one HIP pass (csrc/skinny64.hip quant_tile_f8_kernel), in place when refreshing: a
            # captured decode graph keeps reading the same storage
            t, sc = prev if prev is not None else (
                torch.empty((N // 16, K // 64, 64, 16), dtype=torch.uint8, device=w.device),
                torch.empty(N, dtype=torch.float32, device=w.device))
            _ext.require().quant_tile_f8(w.detach(), norm_w.detach().contiguous() if norm_w is not None else None,
                                         t, sc, bool(glu_il))
            return (t, sc)
        src = w.detach() if norm_w is None else w.detach() * norm_w.detach().view(1, -1)
        if glu_il:
            src = _glu_interleave(src)
        q, sc = quantize_rows_f8(src)
        t = tile_f8(q)
        if prev is not None:
            prev[0].copy_(t)
            prev[1].copy_(sc)
            return prev
        return (t, sc)

    attr = "_dla_f8_g" if glu_il else ("_dla_f8_n" if norm_w is not None else "_dla_f8")
    key = (_wkey(w), _wkey(norm_w) if norm_w is not None else None)
    return _cached(w, attr, key, make)


def _f8_ok(rows: int, w: torch.Tensor) -> bool:
    """fp8 mode and a shape the fp8 kernels take: <= 16 rows csrc/skinny_ks.h F8 / skinny_glu_il F8,
    17..64 rows csrc/skinny64.hip F8."""
    if not _FP8[0]:
        return False
    if rows <= 16:
        return w.shape[0] % 32 == 0 and w.shape[1] % 1024 == 0
    return DECODE_M64 and rows <= 64 and w.shape[0] % 128 == 0 and w.shape[1] % 256 == 0


def head_f8(x: torch.Tensor, w: torch.Tensor) -> Optional[torch.Tensor]:
    """LM-head logits x @ w^T on the fp8 copy of w (decode rows, fp8 mode), else None."""
    if not (_FP8[0] and x.is_cuda and _ext.use_native(x)) or torch.is_grad_enabled() and x.requires_grad:
        return None
    rows = x.numel() // x.shape[-1]
    if not (1 <= rows <= 64 and _f8_ok(rows, w) and x.dtype == torch.bfloat16):
        return None
    w8, sc = fp8_tiled_weight(w)
    if rows > 16:
        y, _ = _ext.require().skinny64_f8(_rows(x), w8, sc, None, None, 0.0, False)
    else:
        y, _ = _ext.require().skinny_fused_f8(_rows(x), w8, sc, None, None, 0.0)
    return y.view(*x.shape[:-1], w.shape[0])


DERIVED_ATTRS = ("_dla_fold", "_dla_fold_t", "_dla_fold_g", "_dla_tile", "_dla_f8", "_dla_f8_n", "_dla_f8_g",
                 "_dla_fp8")  # (the last: ops.moe.fp8_weight, the fp8 prefill GEMMs' weight copy)


def drop_derived_weights(model) -> int:
    """Free every derived decode weight copy (folded / tiled qkv, gate|up, o, down) held on the
    parameters of `model`; returns the bytes released. A ZeRO-3 policy gathered for one rollout
    (`gathered_for_inference`) calls this on exit: the copies are a second full-model-sized set of
    layer weights, and keeping them would defeat the sharding for the rest of training."""
    freed = 0
    for p in model.parameters():
        for k in DERIVED_ATTRS:
            c = p.__dict__.pop(k, None)
            if c is None:
                continue
            for t in (c[1] if isinstance(c[1], tuple) else (c[1],)):  # fp8 copies: (bytes, scales)
                if isinstance(t, torch.Tensor):
                    freed += t.numel() * t.element_size()
    return freed


def refresh_folded_weights(model) -> None:
    """Bring every derived decode weight of `model` up to date (before a graph replay). A model
    whose layers are ZeRO-3 sharded right now is skipped: its weights are not resident (the
    per-layer decode path does not use these copies), and they refresh once it is gathered."""
    ls = getattr(model, "layers_sharded", None)
    if ls is not None and ls():
        return
    hw = getattr(model, "head_weight", None)
    if isinstance(hw, torch.Tensor) and getattr(hw, "_dla_f8", None) is not None:
        fp8_tiled_weight(hw)
    for layer in getattr(model, "layers", []):
        for w, nw in ((getattr(layer.attn, "qkv_proj", None), getattr(layer, "ln1_w", None)),
                      (getattr(layer.mlp, "up_proj", None), getattr(layer, "ln2_w", None))):
            if w is None or nw is None:
                continue
            if getattr(w, "_dla_fold", None) is not None:
                folded_weight(w, nw)
            if getattr(w, "_dla_fold_t", None) is not None:
                folded_weight(w, nw, tiled=True)
            if getattr(w, "_dla_fold_g", None) is not None:
                folded_weight(w, nw, tiled=True, glu_il=True)
            if getattr(w, "_dla_f8_n", None) is not None:
                fp8_tiled_weight(w, nw)
            if getattr(w, "_dla_f8_g", None) is not None:
                fp8_tiled_weight(w, nw, glu_il=True)
        for w in (getattr(layer.attn, "o_proj", None), getattr(layer.mlp, "down_proj", None)):
            if w is not None and getattr(w, "_dla_tile", None) is not None:
                tiled_weight(w)
            if w is not None and getattr(w, "_dla_f8", None) is not None:
                fp8_tiled_weight(w)


def skinny_residual(x: torch.Tensor, w: torch.Tensor, res: torch.Tensor):
    """s = res + x @ w^T (bf16 rounding as linear + add), plus the row-norm partials of s."""
    x2 = _rows(x)
    if _f8_ok(x2.shape[0], w):
        w8, sc = fp8_tiled_weight(w)
        if x2.shape[0] > 16:
            s, ssq = _ext.require().skinny64_f8(x2, w8, sc, _rows(res), None, 0.0, False)
        else:
            s, ssq = _ext.require().skinny_fused_f8(x2, w8, sc, _rows(res), None, 0.0)
        return s.view(*res.shape[:-1], w.shape[0]), ssq
    wk = tiled_weight(w) if DECODE_TILED >= 2 else w
    if x2.shape[0] > 16:
        s, ssq = _ext.require().skinny64(x2, wk, _rows(res), None, 0.0, False)
    else:
        s, ssq = _ext.require().skinny_fused(x2, wk, _rows(res), None, 0.0, False)
    return s.view(*res.shape[:-1], w.shape[0]), ssq


def skinny_normed(s: torch.Tensor, ssq: torch.Tensor, norm_w: torch.Tensor, eps: float,
                  w: torch.Tensor, glu: bool = False) -> torch.Tensor:
    """RMSNorm(s) * norm_w @ w^T from the producer's partials (glu: gate|up + SwiGLU epilogue)."""
    s2 = _rows(s)
    if _f8_ok(s2.shape[0], w) and s2.shape[0] > 16:
        # 17..64 rows: gate|up in the plain [gate; up] row order (the m64 GLU epilogue pairs them)
        w8, sc = fp8_tiled_weight(w, norm_w)
        y, _ = _ext.require().skinny64_f8(s2, w8, sc, None, ssq, float(eps), bool(glu))
        return y.view(*s.shape[:-1], y.shape[-1])
    if _f8_ok(s2.shape[0], w):
        if glu:
            w8, sc = fp8_tiled_weight(w, norm_w, glu_il=True)
            m = _ext.require().skinny_glu_il_f8(s2, w8, sc, ssq, float(eps))
            return m.view(*s.shape[:-1], m.shape[-1])
        w8, sc = fp8_tiled_weight(w, norm_w)
        y, _ = _ext.require().skinny_fused_f8(s2, w8, sc, None, ssq, float(eps))
        return y.view(*s.shape[:-1], y.shape[-1])
    if (glu and DECODE_GLU_IL and DECODE_TILED >= 1 and s2.shape[0] <= 16 and w.shape[0] % 32 == 0
            and w.shape[1] % 512 == 0):
        m = _ext.require().skinny_glu_il(s2, folded_weight(w, norm_w, tiled=True, glu_il=True), ssq, float(eps))
        return m.view(*s.shape[:-1], m.shape[-1])
    wf = folded_weight(w, norm_w, tiled=DECODE_TILED >= 1)
    if s2.shape[0] > 16:
        y, _ = _ext.require().skinny64(s2, wf, None, ssq, float(eps), bool(glu))
    else:
        y, _ = _ext.require().skinny_fused(s2, wf, None, ssq, float(eps), bool(glu))
    return y.view(*s.shape[:-1], y.shape[-1])


def skinny64_linear(x: torch.Tensor, w: torch.Tensor, tiled: bool = False) -> torch.Tensor:
    """y = x @ w^T at 17..64 rows on csrc/skinny64.hip (tests / A/B; `tiled`: through the
    tiled-layout copy of w)."""
    x2 = _rows(x)
    y, _ = _ext.require().skinny64(x2, tiled_weight(w) if tiled else w, None, None, 0.0, False)
    return y.view(*x.shape[:-1], w.shape[0])
