"""Native decoder-only transformer for every model family the reference touches.

One implementation, configured by `ModelConfig`, covers Llama-3 / Mistral (RMSNorm, GQA, RoPE,
SwiGLU, optional sliding window), Mixtral (top-k routed SwiGLU experts), GPT-2 (LayerNorm,
learned positions, GELU, tied head) and phi-2 (parallel attn+MLP block, partial rotary, biases).
It replaces the HF modeling code the reference runs through `AutoModelForCausalLM`
(src/models/base_model.py:17-42) with the gfx950 op set of `..ops`:

  layer:  (h, s) = add_norm(x, s)          HIP fused residual-add + norm
          qkv    = h @ Wqkv^T              ONE fused QKV GEMM (hipBLASLt)
          a      = qkv_attention(qkv)      HIP RoPE + HIP flash attention (fwd/bwd)
          x      = a @ Wo^T
          (h, s) = add_norm(x, s)
          x      = down(swiglu(h @ Wgu^T)) ONE fused gate|up GEMM + HIP SwiGLU
Parameters are stored fused (`qkv_proj`, `gate_up_proj`); `hf_state_dict()` /
`load_hf_state_dict()` convert to/from the HF key layout the reference checkpoints use.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

from .. import ops
from .config import ModelConfig


def _param(*shape, device=None, dtype=None) -> nn.Parameter:
    return nn.Parameter(torch.empty(*shape, device=device, dtype=dtype))


def attention_layout(attention_mask: Optional[torch.Tensor]):
    """From a [B, T] 0/1 mask with one contiguous valid span per row (left or right padding)
    return (kv_start, kv_end, positions) on device, no host sync."""
    if attention_mask is None:
        return None, None, None
    m = attention_mask.to(torch.int32)
    first = (m.cumsum(1) == 0).sum(1).to(torch.int32)
    end = first + m.sum(1).to(torch.int32)
    T = m.shape[1]
    pos = (torch.arange(T, device=m.device, dtype=torch.int32).unsqueeze(0) - first.unsqueeze(1)).clamp(min=0)
    return first, end, pos


def packed_layout(segment_ids: torch.Tensor):
    """Packed rows: `segment_ids` [B, T] labels each token with its sequence (runs of equal ids,
    e.g. 1, 1, 1, 2, 2, 0, 0 with 0 = trailing padding). Returns (positions [B, T] restarting at
    0 in every run, segs [2, B, T] int32 = (first index of the token's run, one past its last)),
    on device, no host sync. Attention is then block-diagonal causal: the packed sequences do
    not see each other (makes `data.packing` real)."""
    B, T = segment_ids.shape
    dev = segment_ids.device
    t = torch.arange(T, device=dev, dtype=torch.int64).expand(B, T)
    new = torch.ones_like(segment_ids, dtype=torch.bool)
    new[:, 1:] = segment_ids[:, 1:] != segment_ids[:, :-1]
    start = torch.where(new, t, torch.zeros_like(t)).cummax(1).values
    last = torch.ones_like(new)
    last[:, :-1] = new[:, 1:]
    end_at = torch.where(last, t + 1, torch.full_like(t, T))
    end = end_at.flip(1).cummin(1).values.flip(1)
    pos = (t - start).to(torch.int32)
    return pos, torch.stack([start, end]).to(torch.int32).contiguous()


class Attention(nn.Module):
    def __init__(self, cfg: ModelConfig, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        H = cfg.hidden_size
        self.qkv_proj = _param(cfg.q_size + 2 * cfg.kv_size, H, device=device, dtype=dtype)
        self.qkv_bias = _param(cfg.q_size + 2 * cfg.kv_size, device=device, dtype=dtype) if cfg.attn_bias else None
        self.o_proj = _param(H, cfg.q_size, device=device, dtype=dtype)
        o_bias = cfg.attn_bias and cfg.arch in ("gpt2", "phi")
        self.o_bias = _param(H, device=device, dtype=dtype) if o_bias else None
        self.tp = None  # tensor-parallel group (parallel.tensor_parallel.apply_tensor_parallel)
        self.tp_seq = None  # Megatron sequence parallel over the TP group (token-sharded stream)
        self.sp = None  # Ulysses sequence parallel (parallel.sequence.apply_sequence_parallel)
        self.h_local, self.kv_local = cfg.num_heads, cfg.num_kv_heads

    def forward(self, h, rope, kv_start, kv_end, positions, cache=None, layer_idx=0, segs=None,
                resid=None):
        """`resid` (no TP, no o bias): return resid + o_proj(attention), the add inside the o GEMM."""
        cfg = self.cfg
        seq = self.tp_seq if (h.dim() == 2 and cache is None) else None
        from ..parallel import tensor_parallel as tpm

        sp_overlap = seq is not None and tpm.TP_OVERLAP and self.qkv_bias is None
        if sp_overlap:  # gather chunk-pipelined under the qkv GEMM
            B, T = positions.shape
            qkv = tpm.sp_gather_linear(h, self.qkv_proj, seq).view(B, T, -1)
        elif seq is not None:
            B, T = positions.shape
            h = tpm.sp_gather(h, seq).view(B, T, -1)
        if sp_overlap:
            pass
        elif seq is None and self.tp is not None and torch.is_grad_enabled():
            from ..parallel.tensor_parallel import col_parallel_linear

            qkv = col_parallel_linear(h, self.qkv_proj, self.qkv_bias, self.tp)
        else:  # (no autograd: the TP input copy is the identity; decode keeps the skinny GEMMs)
            qkv = _lin(h, self.qkv_proj, self.qkv_bias)
        window = cfg.sliding_window if cfg.sliding_window else 0
        if cache is None and self.sp is not None:
            # Ulysses: all-to-all to (all tokens, 1/P of the heads), attention, all-to-all back
            a = self.sp.attention(
                qkv, self.h_local, self.kv_local, cfg.head_dim,
                lambda full, hq, hkv: ops.qkv_attention(full, hq, hkv, cfg.head_dim, rope, causal=True,
                                                        window=window, kv_start=kv_start, kv_end=kv_end,
                                                        positions=positions, segs=segs))
        elif cache is None:
            a = ops.qkv_attention(qkv, self.h_local, self.kv_local, cfg.head_dim, rope,
                                  causal=True, window=window, kv_start=kv_start, kv_end=kv_end,
                                  positions=positions, segs=segs)
        else:
            a = cache.attend(layer_idx, qkv, rope, window)
        if self.tp is None:
            if resid is not None:
                assert self.o_bias is None
                return ops.linear_add(a, self.o_proj, resid)
            return _lin(a, self.o_proj, self.o_bias)
        assert resid is None
        from ..parallel.tensor_parallel import sp_reduce_scatter, tp_grad_sum, tp_reduce

        if seq is not None:
            if tpm.TP_OVERLAP:  # reduce-scatter chunk-pipelined behind the o GEMM
                out = tpm.sp_linear_reduce_scatter(a.reshape(-1, a.shape[-1]), self.o_proj, seq)
            else:
                out = sp_reduce_scatter(ops.linear(a, self.o_proj, None).reshape(-1, cfg.hidden_size), seq)
            return out + tp_grad_sum(self.o_bias, seq) if self.o_bias is not None else out
        from ..parallel.tensor_parallel import row_parallel_linear

        out = row_parallel_linear(a, self.o_proj, self.tp)
        return out + self.o_bias if self.o_bias is not None else out


class MLP(nn.Module):
    def __init__(self, cfg: ModelConfig, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        H, Fd = cfg.hidden_size, cfg.intermediate_size
        if cfg.activation == "swiglu":
            self.up_proj = _param(2 * Fd, H, device=device, dtype=dtype)  # [gate; up]
        else:
            self.up_proj = _param(Fd, H, device=device, dtype=dtype)
        self.up_bias = _param(self.up_proj.shape[0], device=device, dtype=dtype) if cfg.mlp_bias else None
        self.down_proj = _param(H, Fd, device=device, dtype=dtype)
        self.down_bias = _param(H, device=device, dtype=dtype) if cfg.mlp_bias else None
        self.tp = None
        self.tp_seq = None

    def forward(self, h, resid=None):
        """`resid` (no TP): return resid + MLP(h); on the fused SwiGLU node the add runs inside
        the down GEMM (its C input), elsewhere as a plain add."""
        if resid is not None:
            if (self.cfg.activation == "swiglu" and self.up_bias is None and self.down_bias is None
                    and self.tp is None and self.tp_seq is None
                    and ops.swiglu_mlp_ok(h, self.up_proj, self.down_proj)):
                return ops.swiglu_mlp(h, self.up_proj, self.down_proj, resid=resid)
            if self.tp is None and self.tp_seq is None and self.down_bias is None:
                # (no autograd, e.g. the frozen DPO reference: the same add inside the down GEMM)
                u = ops.linear(h, self.up_proj, self.up_bias)
                m = ops.swiglu(u) if self.cfg.activation == "swiglu" else ops.gelu_new(u)
                return ops.linear_add(m, self.down_proj, resid)
            return self.forward(h) + resid
        seq = self.tp_seq if h.dim() == 2 else None
        if seq is not None:
            from ..parallel import tensor_parallel as tpm

            if tpm.TP_OVERLAP and self.up_bias is None and self.down_bias is None:
                # Megatron-SP MLP in chunk-major token order (per-token block): the all-gather
                # pipelined under gate|up, the reduce-scatter behind the down GEMM chunks
                C = tpm.tp_chunks("mlp")  # (one count for both: chunk-major rows)
                u = tpm.sp_gather_linear(h, self.up_proj, seq, chunks=C, token_order=False)
                m = ops.swiglu(u) if self.cfg.activation == "swiglu" else ops.gelu_new(u)
                return tpm.sp_linear_reduce_scatter(m, self.down_proj, seq, chunks=C, token_order=False)
            h = tpm.sp_gather(h, seq)
        elif self.tp is not None:
            from ..parallel import tensor_parallel as tpm

            if (tpm.TP_OVERLAP and self.cfg.activation == "swiglu" and self.up_bias is None
                    and self.down_bias is None and ops.swiglu_mlp_ok(h, self.up_proj, self.down_proj)):
                # the whole Megatron MLP as one node, collectives overlapped (ops.activations)
                return ops.swiglu_mlp(h, self.up_proj, self.down_proj, tp_group=self.tp,
                                      chunks=tpm.tp_chunks("mlp"))
            if tpm.TP_OVERLAP:
                u = tpm.col_parallel_linear(h, self.up_proj, self.up_bias, self.tp)
                m = ops.swiglu(u) if self.cfg.activation == "swiglu" else ops.gelu_new(u)
                out = tpm.row_parallel_linear(m, self.down_proj, self.tp, chunks=tpm.tp_chunks("mlp"))
                return out + self.down_bias if self.down_bias is not None else out
            h = tpm.tp_copy(h, self.tp)
        if (self.cfg.activation == "swiglu" and self.up_bias is None and self.down_bias is None
                and self.tp is None and ops.decode.skinny_ok(h, self.up_proj, glu=True)):
            # decode (<= 16 rows, no autograd): skinny GEMMs, SwiGLU fused into the down GEMM
            m = ops.decode.skinny_glu(h, self.up_proj)  # gate|up GEMM with SwiGLU epilogue
            if m is not None:
                return _lin(m, self.down_proj, None)
            u = ops.decode.skinny_linear(h, self.up_proj)
            if u is not None:
                # SwiGLU fused into the down GEMM only where that GEMM needs no split-K combine
                y = (ops.decode.skinny_linear(u, self.down_proj, swiglu=True)
                     if self.down_proj.shape[0] >= ops.decode.SKINNY_WIDE_N else None)
                return y if y is not None else _lin(ops.swiglu(u), self.down_proj, None)
        if (self.cfg.activation == "swiglu" and self.up_bias is None and self.down_bias is None
                and ops.swiglu_mlp_ok(h, self.up_proj, self.down_proj)):
            out = ops.swiglu_mlp(h, self.up_proj, self.down_proj)
            if self.tp is None:
                return out
            from ..parallel.tensor_parallel import sp_reduce_scatter, tp_reduce

            return sp_reduce_scatter(out, seq) if seq is not None else tp_reduce(out, self.tp)
        u = ops.linear(h, self.up_proj, self.up_bias)
        m = ops.swiglu(u) if self.cfg.activation == "swiglu" else ops.gelu_new(u)
        if self.tp is None:
            return ops.linear(m, self.down_proj, self.down_bias)
        from ..parallel.tensor_parallel import sp_reduce_scatter, tp_grad_sum, tp_reduce

        if seq is not None:
            out = sp_reduce_scatter(ops.linear(m, self.down_proj, None), seq)
            return out + tp_grad_sum(self.down_bias, seq) if self.down_bias is not None else out
        out = tp_reduce(ops.linear(m, self.down_proj, None), self.tp)
        return out + self.down_bias if self.down_bias is not None else out


class MoE(nn.Module):
    """Top-k routed SwiGLU experts (Mixtral). Softmax router in fp32, top-k renormalised,
    dropless token dispatch (sort by expert, one device-driven grouped GEMM per projection,
    weighted gather-combine); no host sync in the local (non-EP) path.
    Under expert parallelism `ep_group` routes tokens with all-to-all (see parallel.expert)."""

    def __init__(self, cfg: ModelConfig, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        H, Fd, E = cfg.hidden_size, cfg.intermediate_size, cfg.num_experts
        self.router = _param(E, H, device=device, dtype=dtype)
        self.expert_up = _param(E, 2 * Fd, H, device=device, dtype=dtype)
        self.expert_down = _param(E, H, Fd, device=device, dtype=dtype)
        self.ep = None  # set by parallel.expert.shard_experts
        self.last_aux_loss = None

    fp8 = False  # e4m3 expert GEMMs in the forward (north star; bf16 backward)
    collect_aux = False  # HF `output_router_logits`: off by default, as in MixtralConfig

    def route(self, h2: torch.Tensor):
        logits = ops.linear(h2, self.router)
        topv, topi = ops.moe.route_topk(logits, self.cfg.num_experts_per_tok)
        if self.collect_aux and self.training and self.cfg.router_aux_loss_coef > 0 and torch.is_grad_enabled():
            E = self.cfg.num_experts
            probs = torch.softmax(logits.float(), dim=-1)
            frac = F.one_hot(topi.long(), E).float().sum(1).mean(0)
            self.last_aux_loss = E * (frac * probs.mean(0)).sum() * self.cfg.router_aux_loss_coef
        return topv, topi

    def forward(self, h):
        shp = h.shape
        h2 = h.reshape(-1, shp[-1])
        topv, topi = self.route(h2)
        if self.ep is not None:
            out = self.ep.dispatch_combine(self, h2, topv, topi)
            return out.view(shp)
        pos, counts = ops.moe.expert_positions(topi, self.cfg.num_experts)
        xs = ops.moe.dispatch(h2, pos)
        ys = ops.moe.experts_swiglu(xs, self.expert_up, self.expert_down, counts, fp8=self.fp8)
        return ops.moe.combine(ys, pos, topv, permutation=True).view(shp)


# Residual adds inside the o / down GEMMs (ops.linear.linear_add); DLA_FUSED_RESIDUAL=0 restores
# the separate fused add + norm kernels for A/B runs.
FUSED_RESIDUAL = os.environ.get("DLA_FUSED_RESIDUAL", "1") != "0"


class DecoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        H = cfg.hidden_size
        bias = cfg.norm_type == "layer"
        self.ln1_w = _param(H, device=device, dtype=dtype)
        self.ln1_b = _param(H, device=device, dtype=dtype) if bias else None
        if not cfg.parallel_block:
            self.ln2_w = _param(H, device=device, dtype=dtype)
            self.ln2_b = _param(H, device=device, dtype=dtype) if bias else None
        self.attn = Attention(cfg, device, dtype)
        self.mlp = MoE(cfg, device, dtype) if cfg.is_moe else MLP(cfg, device, dtype)
        self.tp_seq = None  # Megatron-SP: x / resid are this rank's [N/tp, H] token rows
        self.recompute = None  # selective activation recompute: None | "attention" | "mlp"

    def decode_fused_ok(self, x) -> bool:
        """This layer's decode step can run on the fused residual/norm kernels."""
        cfg, at, mlp = self.cfg, self.attn, self.mlp
        return (cfg.norm_type == "rms" and not cfg.parallel_block and isinstance(mlp, MLP)
                and cfg.activation == "swiglu" and mlp.up_bias is None and mlp.down_bias is None
                and at.qkv_bias is None and at.o_bias is None and at.tp is None and mlp.tp is None
                and at.sp is None and self.ln1_b is None and self.ln2_b is None
                and ops.decode.fused_layer_ok(x, cfg.hidden_size, at.qkv_proj, at.o_proj,
                                              mlp.up_proj, mlp.down_proj))

    def decode_fused(self, s, ssq, rope, cache, layer_idx):
        """One decode step of the layer with no norm launch (ops.decode fused layer): `s` is the
        residual stream after the previous layer and `ssq` its row-norm partials (None for the
        first layer). Returns the next (s, ssq)."""
        cfg, at, mlp = self.cfg, self.attn, self.mlp
        if ssq is None:
            h, _ = ops.add_norm(s, None, self.ln1_w, None, cfg.norm_eps, True)
            qkv = _lin(h, at.qkv_proj, None)
            a = cache.attend(layer_idx, qkv, rope, cfg.sliding_window if cfg.sliding_window else 0)
        else:
            window = cfg.sliding_window if cfg.sliding_window else 0
            qkv = ops.decode.skinny_normed(s, ssq, self.ln1_w, cfg.norm_eps, at.qkv_proj)
            a = cache.attend(layer_idx, qkv, rope, window)
        s2, ssq2 = ops.decode.skinny_residual(a, at.o_proj, s)
        m = ops.decode.skinny_normed(s2, ssq2, self.ln2_w, cfg.norm_eps, mlp.up_proj, glu=True)
        return ops.decode.skinny_residual(m, mlp.down_proj, s2)

    def fused_residual_ok(self, x, cache, seq) -> bool:
        at, mlp = self.attn, self.mlp
        return (FUSED_RESIDUAL and cache is None and seq is None and not self.cfg.parallel_block
                and isinstance(mlp, MLP) and at.tp is None and mlp.tp is None and at.o_bias is None
                and mlp.down_bias is None)

    def forward(self, x, resid, rope, kv_start, kv_end, positions, cache=None, layer_idx=0, segs=None):
        cfg = self.cfg
        rms = cfg.norm_type == "rms"
        seq = self.tp_seq if x.dim() == 2 else None
        if seq is not None:
            from ..parallel.tensor_parallel import tp_grad_sum as w_
        else:
            w_ = _ident
        rc = self.recompute if (cache is None and self.training and torch.is_grad_enabled()) else None
        if self.fused_residual_ok(x, cache, seq):
            # the residual stream rides as the C input of the o and down GEMMs (beta = 1), so each
            # norm reads and writes one [N, H] tensor instead of two each; the layer hands on the
            # summed stream with resid = None
            h, s = ops.add_norm(x, resid, self.ln1_w, self.ln1_b, cfg.norm_eps, rms, keep_stream=True)
            if rc == "attention":
                s = checkpoint(self.attn, h, rope, kv_start, kv_end, positions, None, layer_idx, segs, s,
                               use_reentrant=False)
            else:
                s = self.attn(h, rope, kv_start, kv_end, positions, None, layer_idx, segs, resid=s)
            h, s = ops.add_norm(s, None, self.ln2_w, self.ln2_b, cfg.norm_eps, rms, keep_stream=True)
            if rc == "mlp":
                return checkpoint(self.mlp, h, s, use_reentrant=False), None
            return self.mlp(h, s), None
        h, resid = ops.add_norm(x, resid, w_(self.ln1_w, seq), w_(self.ln1_b, seq), cfg.norm_eps, rms)
        if rc == "attention":  # keep h; drop q/k/v, O and the LSE; recompute them in backward
            a = checkpoint(self.attn, h, rope, kv_start, kv_end, positions, None, layer_idx, segs,
                           use_reentrant=False)
        else:
            a = self.attn(h, rope, kv_start, kv_end, positions, cache, layer_idx, segs)
        mlp = (lambda t: checkpoint(self.mlp, t, use_reentrant=False)) if rc == "mlp" else self.mlp
        if cfg.parallel_block:
            return a + mlp(h), resid
        h, resid = ops.add_norm(a, resid, w_(self.ln2_w, seq), w_(self.ln2_b, seq), cfg.norm_eps, rms)
        return mlp(h), resid


def _ident(w, _seq=None):
    return w


class CausalLM(nn.Module):
    """Decoder-only LM. forward() returns the final normed hidden states [B, T, H]; the LM head
    is applied by the fused log-prob / CE ops (or `logits()` for generation)."""

    def __init__(self, cfg: ModelConfig, device=None, dtype=None, headless: bool = False):
        super().__init__()
        self.cfg = cfg
        self.headless = headless
        H, V = cfg.hidden_size, cfg.vocab_size
        self.embed = _param(V, H, device=device, dtype=dtype)
        self.wpe = _param(cfg.max_position_embeddings, H, device=device, dtype=dtype) if cfg.learned_pos_emb else None
        self.layers = nn.ModuleList([DecoderLayer(cfg, device, dtype) for _ in range(cfg.num_layers)])
        self.norm_w = _param(H, device=device, dtype=dtype)
        self.norm_b = _param(H, device=device, dtype=dtype) if cfg.norm_type == "layer" else None
        self.lm_head = None if (cfg.tie_word_embeddings or headless) else _param(V, H, device=device, dtype=dtype)
        self.lm_head_bias = _param(V, device=device, dtype=dtype) if (cfg.lm_head_bias and not headless) else None
        self.rope = (ops.RotaryCache(cfg.rot_dim, cfg.rope_theta, cfg.max_position_embeddings,
                                     cfg.rope_scaling) if cfg.rot_dim > 0 else None)
        self.gradient_checkpointing = False
        self.tp = None             # set by parallel.tensor_parallel.apply_tensor_parallel
        self.tp_size = 1
        self.tp_rank = 0
        self.vocab_parallel = None  # (vocab offset, local vocab) when embed/head are vocab-sharded
        self.tp_seq = None          # Megatron sequence parallel over the TP group
        self.sp = None              # parallel.sequence.SequenceParallel: this rank holds 1/P of T
        self.layer_devices = None   # per-layer devices under parallel.layer_split (device_map)
        if self.lm_head is None and not headless:
            # tied input/output embedding: its gradient arrives from two ops, so it must go through
            # autograd's AccumulateGrad (one hook call) rather than the GEMM main-grad path
            self.embed._dla_shared = True

    @property
    def moe_device_dispatch(self) -> bool:
        """True when every MoE layer routes without a host sync (grouped GEMM path, no EP, no
        cached fp8 expert copies that a captured graph could replay stale): the condition for a
        hipGraph-captured MoE decode step."""
        cfg = self.cfg
        if not cfg.is_moe:
            return True
        return (ops.moe.grouped_gemm_enabled() and getattr(self, "ep_size", 1) == 1
                and all(getattr(layer.mlp, "ep", None) is None for layer in self.layers)
                and cfg.intermediate_size % 128 == 0 and cfg.hidden_size % 16 == 0
                and not any(getattr(layer.mlp, "fp8", False) for layer in self.layers))

    # --------------------------------------------------------------------------------- init
    @torch.no_grad()
    def init_weights(self, seed: int = 0):
        """Deterministic random init, identical on every rank (no broadcast needed). Each
        parameter draws from its own generator seeded by (seed, parameter index), so any subset
        can be produced alone and in any order: the memory-bounded construction path
        (models/materialize.py) materialises one parameter / FSDP unit at a time and gets
        bitwise the same weights as this whole-model init."""
        for idx, (name, p) in enumerate(self.named_parameters()):
            p.copy_(init_param_tensor(self.cfg, name, idx, tuple(p.shape), seed, p.device, p.dtype))
        return self

    # Activation recompute policies. "full" (= True, the reference's HF
    # gradient checkpointing): every decoder layer keeps only its input and is re-run in
    # backward. Selective: "mlp" re-runs only the MLP block (gate|up GEMM, SwiGLU, down GEMM), so
    # its [T, 2F] / [T, F] intermediates — the largest activations of a Llama layer — are never
    # kept; "attention" re-runs only the attention block (qkv GEMM, RoPE, flash attention, o
    # GEMM). With 288 GB of HBM the 8B DPO bench needs none; they serve long context and 70B.
    RECOMPUTE_POLICIES = ("full", "mlp", "attention")

    def gradient_checkpointing_enable(self, policy="full", gradient_checkpointing_kwargs=None):
        if policy is True or policy is None:
            policy = "full"
        policy = str(policy).lower()
        if policy not in self.RECOMPUTE_POLICIES:
            raise ValueError(f"gradient checkpointing policy must be one of {self.RECOMPUTE_POLICIES}, "
                             f"got {policy!r}")
        self.gradient_checkpointing = policy == "full"
        for layer in self.layers:
            layer.recompute = None if policy == "full" else policy
        self.recompute_policy = policy

    def gradient_checkpointing_disable(self):
        self.gradient_checkpointing = False
        for layer in self.layers:
            layer.recompute = None
        self.recompute_policy = None

    # ------------------------------------------------------------------------------ forward
    @property
    def head_weight(self) -> torch.Tensor:
        return self.embed if self.lm_head is None else self.lm_head

    def embed_tokens(self, input_ids, positions=None):
        if self.vocab_parallel is not None:
            from ..parallel.tensor_parallel import vocab_parallel_embedding

            x = vocab_parallel_embedding(input_ids, self.embed, self.vocab_parallel[0], self.tp)
        else:
            x = ops.embedding(input_ids, self.embed)
        if self.wpe is not None:
            T = input_ids.shape[1]
            pos = positions.long() if positions is not None else torch.arange(T, device=input_ids.device)
            x = x + F.embedding(pos, self.wpe)
        return x

    def _embed_tp_seq(self, input_ids, positions):
        """Megatron-SP entry: this rank's [N/tp, H] token rows of the embedding (vocab-parallel
        partial sums reduce-scattered straight into the token shards)."""
        from ..parallel.tensor_parallel import sp_reduce_scatter, tp_grad_sum

        seq = self.tp_seq
        H = self.cfg.hidden_size
        if self.vocab_parallel is not None:
            off, V_l = self.vocab_parallel
            local = input_ids - off
            own = (local >= 0) & (local < V_l)
            xp = F.embedding(local.clamp(0, V_l - 1), self.embed) * own.unsqueeze(-1).to(self.embed.dtype)
            x = sp_reduce_scatter(xp.reshape(-1, H), seq)
        else:
            x = seq.local(F.embedding(input_ids, tp_grad_sum(self.embed, seq)).reshape(-1, H))
        if self.wpe is not None:
            x = x + seq.local(F.embedding(positions.long(), tp_grad_sum(self.wpe, seq)).reshape(-1, H))
        return x

    def forward(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                cache=None, segment_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
        """`segment_ids` (optional, [B, T]): several sequences packed per row (see packed_layout)."""
        if cache is not None:
            return self._forward_cached(input_ids, attention_mask, cache)
        sp = self.sp
        if sp is not None:  # full (padded) masks / positions drive attention; tokens are sliced
            from ..parallel.sequence import sp_shard_inputs

            input_ids, attention_mask, segment_ids = sp_shard_inputs(sp, input_ids, attention_mask,
                                                                     segment_ids)
        kv_start, kv_end, positions = attention_layout(attention_mask)
        segs = None
        if segment_ids is not None:
            positions, segs = packed_layout(segment_ids)
        tp_seq = self.tp_seq if (sp is None and self.tp_seq is not None
                                 and input_ids.numel() % self.tp_seq.tp == 0) else None
        if sp is not None or tp_seq is not None:
            if positions is None:  # explicit [B, T] positions also carry the shape to the layers
                B, T = input_ids.shape
                positions = torch.arange(T, device=input_ids.device, dtype=torch.int32).expand(B, T)
        if sp is not None:
            x = self.embed_tokens(sp.local(input_ids), sp.local(positions))
        elif tp_seq is not None:
            x = self._embed_tp_seq(input_ids, positions)
        else:
            x = self.embed_tokens(input_ids, positions)
        resid = None
        for i, layer in enumerate(self.layers):
            if self.layer_devices is not None:
                x, resid, kv_start, kv_end, positions, segs = _hop(self.layer_devices[i], x, resid,
                                                                   kv_start, kv_end, positions, segs)
            if self.gradient_checkpointing and self.training and torch.is_grad_enabled():
                x, resid = checkpoint(layer, x, resid, self.rope, kv_start, kv_end, positions, None, 0,
                                      segs, use_reentrant=False)
            else:
                x, resid = layer(x, resid, self.rope, kv_start, kv_end, positions, segs=segs)
        if self.layer_devices is not None:
            x, resid = _hop(self.norm_w.device, x, resid)
        if tp_seq is not None:
            from ..parallel.tensor_parallel import sp_gather_replicated_grad, tp_grad_sum

            h, _ = ops.add_norm(x, resid, tp_grad_sum(self.norm_w, tp_seq), tp_grad_sum(self.norm_b, tp_seq),
                                self.cfg.norm_eps, self.cfg.norm_type == "rms")
            return sp_gather_replicated_grad(h, tp_seq).view(*input_ids.shape, -1)
        h, _ = ops.add_norm(x, resid, self.norm_w, self.norm_b, self.cfg.norm_eps,
                            self.cfg.norm_type == "rms")
        return h

    def sharding_engines(self) -> list:
        """The ZeRO-3 engines whose shards some of this model's layers live in."""
        out = []
        for e in [getattr(self, "_dla_fsdp", None)] + [getattr(l, "_dla_sharded", None) for l in self.layers]:
            if e is not None and all(e is not o for o in out):
                out.append(e)
        return out

    def layers_sharded(self) -> bool:
        """Some decoder layer's weights are ZeRO-3 shards gathered only inside its forward (not
        pinned resident by `gathered_for_inference`)."""
        return any(not getattr(e, "_pinned", False) for e in self.sharding_engines())

    def _forward_cached(self, input_ids, attention_mask, cache):
        positions = cache.positions_for(input_ids.shape[1])
        x = self.embed_tokens(input_ids, positions)
        # decode_fused calls the layers' kernels directly, skipping Module.__call__: a ZeRO-3
        # policy's layers are gathered by forward hooks, so sharded layers take the hooked path
        if (input_ids.shape[1] == 1 and self.layer_devices is None and self.layers
                and not self.layers_sharded() and self.layers[0].decode_fused_ok(x)):
            # decode step: residual add + RMSNorm folded into the neighbouring projections
            s, ssq = x, None
            for i, layer in enumerate(self.layers):
                s, ssq = layer.decode_fused(s, ssq, self.rope, cache, i)
            h, _ = ops.add_norm(s, None, self.norm_w, self.norm_b, self.cfg.norm_eps, True)
            cache.step_done(1)
            return h
        resid = None
        for i, layer in enumerate(self.layers):
            if self.layer_devices is not None:
                x, resid = _hop(self.layer_devices[i], x, resid)
            x, resid = layer(x, resid, self.rope, None, None, None, cache, i)
        if self.layer_devices is not None:
            x, resid = _hop(self.norm_w.device, x, resid)
        h, _ = ops.add_norm(x, resid, self.norm_w, self.norm_b, self.cfg.norm_eps,
                            self.cfg.norm_type == "rms")
        cache.step_done(input_ids.shape[1])
        return h

    def logits(self, hidden: torch.Tensor) -> torch.Tensor:
        lg = None
        if self.lm_head_bias is None and self.vocab_parallel is None:
            lg = ops.decode.head_f8(hidden, self.head_weight)  # fp8 decode mode only
        if lg is None and self.lm_head_bias is None:
            lg = ops.decode.skinny_linear(hidden, self.head_weight)  # decode rows only
        if lg is None:
            lg = F.linear(hidden, self.head_weight, self.lm_head_bias)
        if self.vocab_parallel is not None:
            from ..parallel.tensor_parallel import tp_all_gather_last

            lg = tp_all_gather_last(lg, self.tp)
        return lg

    def _token_logprob(self, h2: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        """Per-token log p(target) from final hidden rows [N, H] (fused HIP LM-head path)."""
        if self.vocab_parallel is not None:
            from ..parallel.tensor_parallel import vocab_parallel_logprob

            return vocab_parallel_logprob(h2, self.head_weight, targets, self.vocab_parallel[0], self.tp)
        return ops.linear_logprob(h2, self.head_weight, targets)

    def aux_loss(self):
        if not self.cfg.is_moe:
            return None
        terms = [l.mlp.last_aux_loss for l in self.layers if l.mlp.last_aux_loss is not None]
        return sum(terms) if terms else None

    # ----------------------------------------------------------------- objective helpers
    def _sp_targets(self, tgt: torch.Tensor, mask: Optional[torch.Tensor] = None):
        """Full [S, T] targets / mask -> this rank's token slice (identity without SP)."""
        sp = self.sp
        if sp is None:
            return tgt, mask
        return sp.local(sp.pad(tgt, -100)), (None if mask is None else sp.local(sp.pad(mask, 0)))

    def _masked_token_logprob(self, h: torch.Tensor, tgt: torch.Tensor) -> torch.Tensor:
        """[S, T', H] hidden + [S, T'] targets (-100 = ignore) -> [S, T'] fp32 log-probs (0 where
        ignored); the LM-head bias models (phi-2) go through full logits."""
        S, T, H = h.shape
        if self.lm_head_bias is not None:
            lg = self.logits(h).float()
            lp = torch.log_softmax(lg, -1).gather(-1, tgt.clamp(min=0).unsqueeze(-1)).squeeze(-1)
            return torch.where(tgt >= 0, lp, torch.zeros_like(lp))
        return self._token_logprob(h.reshape(S * T, H), tgt.reshape(-1)).view(S, T)

    def sequence_logprob(self, input_ids, attention_mask=None, reduction: str = "mean"):
        """Reference `compute_logprobs` (train_dpo.py:31-39): masked mean log p per sequence."""
        h = self(input_ids, attention_mask)  # __call__: module hooks (param all-gather waits) run
        tgt, mask = self._sp_targets(*ops.shifted_targets(input_ids, attention_mask))
        lp = self._masked_token_logprob(h, tgt)
        return sp_seq_reduce(self.sp, lp, mask, reduction == "mean")

    def token_logprobs(self, input_ids, attention_mask=None):
        """[S, T] log p(x_{t+1} | x_<=t) at every scored position (0 elsewhere): the per-action
        grid of token-level RL objectives (PPO)."""
        h = self(input_ids, attention_mask)
        tgt, _ = self._sp_targets(ops.shifted_targets(input_ids, attention_mask)[0])
        lp = self._masked_token_logprob(h, tgt)
        if self.sp is not None:
            lp = self.sp.gather(lp, dim=1)[:, :input_ids.shape[1]]
        return lp

    def causal_lm_loss(self, input_ids, labels, attention_mask=None, segment_ids=None):
        """HF ForCausalLMLoss (train_sft.py:145-146): mean token NLL over labels != -100.
        With `segment_ids` the rows hold packed sequences (labels -100 at each sequence start)."""
        h = self(input_ids, attention_mask, segment_ids=segment_ids)  # __call__: module hooks run
        tgt = torch.full_like(labels, -100)
        tgt[:, :-1] = labels[:, 1:]
        tgt, _ = self._sp_targets(tgt)
        lp = self._masked_token_logprob(h, tgt)
        total, count = lp.sum(), (tgt >= 0).sum().float()
        if self.sp is not None:
            total = self.sp.reduce(total)
            count = self.sp.reduce(count)
        return -(total / count.clamp(min=1))

    # ----------------------------------------------------------------- HF key mapping
    def hf_state_dict(self, only=None) -> Dict[str, torch.Tensor]:
        from .hf_io import to_hf_state_dict

        return to_hf_state_dict(self, only=only)

    def load_hf_state_dict(self, sd, strict: bool = True, only=None, used_out=None):
        from .hf_io import load_hf_state_dict

        return load_hf_state_dict(self, sd, strict=strict, only=only, used_out=used_out)


def _lin(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor]) -> torch.Tensor:
    """ops.linear, with the decode skinny-GEMM kernel for <= 16 rows without autograd."""
    if b is None:
        y = ops.decode.skinny_linear(x, w)
        if y is not None:
            return y
    return ops.linear(x, w, b)


def _hop(dev, *ts):
    """Move activations to the next layer range's device (layer-split model parallel)."""
    return tuple(t if (t is None or t.device == dev) else t.to(dev, non_blocking=True) for t in ts)


def _chunked_randn(p: torch.Tensor, gen: torch.Generator, std: float) -> torch.Tensor:
    flat = p.view(-1)
    step = 1 << 24
    for s in range(0, flat.numel(), step):
        e = min(flat.numel(), s + step)
        flat[s:e] = torch.randn(e - s, generator=gen, device=p.device, dtype=torch.float32).mul_(std).to(p.dtype)
    return p


def _param_seed(seed: int, idx: int) -> int:
    return (int(seed) * 1_000_003 + int(idx) * 7_919 + 17) % (2 ** 62)


def init_param_tensor(cfg: ModelConfig, name: str, idx: int, shape, seed: int, device, dtype) -> torch.Tensor:
    """The init value of parameter `name` (index `idx` in named_parameters order) as a fresh
    tensor: norm weights 1, other vectors 0, matrices N(0, init_std) with the GPT-2 style
    1/sqrt(2L) scaling on the residual-output projections."""
    device = torch.device(device)
    if len(shape) == 1:
        val = 1.0 if name.endswith(("ln1_w", "ln2_w", "norm_w")) else 0.0
        return torch.full(shape, val, device=device, dtype=dtype)
    std = cfg.init_std
    if name.endswith(("o_proj", "down_proj", "expert_down")):
        std = std / math.sqrt(2 * cfg.num_layers)
    gen = torch.Generator(device=device)
    gen.manual_seed(_param_seed(seed, idx))
    t = torch.empty(shape, device=device, dtype=dtype)
    if t.numel() < (1 << 26):
        t.copy_(torch.randn(shape, generator=gen, device=device, dtype=torch.float32).mul_(std))
        return t
    return _chunked_randn(t, gen, std)


def sp_seq_reduce(sp, lp: torch.Tensor, mask: torch.Tensor, mean: bool) -> torch.Tensor:
    """Masked per-sequence sum / mean of token log-probs; under sequence parallelism the partial
    sums and token counts of the local slices are all-reduced over the SP group."""
    if sp is None:
        return ops.seq_reduce(lp, mask, mean=mean)
    s = sp.reduce(ops.seq_reduce(lp, mask, mean=False))
    if not mean:
        return s
    n = sp.reduce(mask.float().sum(1))
    return s / n.clamp(min=1)


def default_dtype(device) -> torch.dtype:
    """bf16 on the GPU, fp32 on CPU (the reference: bf16 if CUDA else fp32, base_model.py:27-29)."""
    return torch.bfloat16 if (device is not None and torch.device(device).type == "cuda") else torch.float32


def build_model(cfg: ModelConfig, device=None, dtype=None, seed: int = 0, init: bool = True,
                headless: bool = False, meta: bool = False) -> CausalLM:
    """`meta=True`: parameters on the meta device, values produced later and only for this rank's
    shard (models/materialize.py; memory-bounded construction for 70B-class models)."""
    dtype = dtype or default_dtype(device)
    if meta:
        from .materialize import build_meta

        return build_meta(cfg, dtype, seed=seed, headless=headless)
    model = CausalLM(cfg, device=device, dtype=dtype, headless=headless)
    if init:
        model.init_weights(seed)
    return model
