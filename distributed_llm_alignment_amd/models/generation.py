"""Autoregressive generation with a preallocated KV cache.

Replaces HF `model.generate` used by the reference's RLHF rollouts (src/training/train_rlhf.py:123-124),
teacher data generation (generate_teacher_data.py:72-79) and alignment eval
(eval_alignment.py:68-79). Prompts are LEFT-padded (fixing Appendix A #10); positions start at
each row's first real token; finished rows emit `pad_token_id`. The cache is contiguous
[L, B, T_max, Hkv, D] per K/V sized once for prompt + max_new_tokens (HBM is plentiful), the
prefill runs the flash-attention kernel over the whole prompt and each decode step attends
to the cache through the same kernel with causal offset.
"""
from __future__ import annotations

import math
import os
import weakref
from dataclasses import dataclass
from typing import Optional

import torch

from .. import ops
from .transformer import CausalLM, attention_layout


class KVCache:
    """Contiguous per-layer K/V cache [L, B, T_max, Hkv, D] sized once for prompt + new tokens.

    The write slot, attended length and next positions also live on the device (`slot`,
    `kv_len`, `pos`), so a single-token decode step touches no host value: it can be captured
    in a hipGraph and replayed (`advance_device`)."""

    def __init__(self, model: CausalLM, batch: int, max_len: int, kv_start: Optional[torch.Tensor]):
        cfg = model.cfg
        dev, dt = model.embed.device, model.embed.dtype
        L, Hkv, D = cfg.num_layers, model.layers[0].attn.kv_local, cfg.head_dim
        self.h_local, self.kv_local = model.layers[0].attn.h_local, Hkv
        self.cfg = cfg
        self.split = model.layer_devices is not None
        if self.split:  # layer-split model: each layer's K/V on that layer's device
            self.k = [torch.empty((batch, max_len, Hkv, D), device=d, dtype=dt) for d in model.layer_devices]
            self.v = [torch.empty((batch, max_len, Hkv, D), device=d, dtype=dt) for d in model.layer_devices]
        elif KV_HEAD_MAJOR:
            # storage [L, B, Hkv, T_max, D] (a head's keys contiguous: one 128-key decode chunk is
            # 32 KB in one run), seen through a [L, B, T_max, Hkv, D] view: every consumer is
            # stride-generic
            self.k = torch.empty((L, batch, Hkv, max_len, D), device=dev, dtype=dt).transpose(2, 3)
            self.v = torch.empty((L, batch, Hkv, max_len, D), device=dev, dtype=dt).transpose(2, 3)
        else:
            self.k = torch.empty((L, batch, max_len, Hkv, D), device=dev, dtype=dt)
            self.v = torch.empty((L, batch, max_len, Hkv, D), device=dev, dtype=dt)
        self.max_len = max_len
        self.len = 0
        self.batch = batch
        self.kv_start = kv_start.to(torch.int32).clone() if kv_start is not None else None
        self._pos = None
        self.slot = torch.zeros(1, dtype=torch.long, device=dev)
        self.kv_len = torch.ones(1, dtype=torch.int32, device=dev)
        self.pos = torch.zeros((batch, 1), dtype=torch.int32, device=dev)
        self.fast_decode = (not self.split and dev.type == "cuda" and dt == torch.bfloat16
                            and ops.decode.decode_supported(self.h_local, Hkv, D))

    def nbytes(self) -> int:
        ks = self.k if isinstance(self.k, list) else [self.k]
        return 2 * sum(t.numel() * t.element_size() for t in ks)

    def reset(self, kv_start: Optional[torch.Tensor]):
        """Empty the cache for a new batch of the same shape, keeping every buffer (and so every
        address a captured decode graph reads) in place."""
        self.len = 0
        self._pos = None
        self.capturing = False
        if kv_start is not None:
            self.kv_start.copy_(kv_start.to(torch.int32))

    def positions_for(self, T: int) -> torch.Tensor:
        if T == 1 and self.len > 0:
            self._pos = self.pos
            return self.pos
        dev = self.slot.device
        t = torch.arange(self.len, self.len + T, device=dev, dtype=torch.int32).unsqueeze(0)
        start = self.kv_start.unsqueeze(1) if self.kv_start is not None else 0
        self._pos = (t - start).clamp(min=0).expand(self.batch, T).contiguous()
        return self._pos

    def attend(self, layer: int, qkv: torch.Tensor, rope, window: int) -> torch.Tensor:
        cfg = self.cfg
        B, T, _ = qkv.shape
        if self.len + T > self.max_len:
            raise RuntimeError("KV cache overflow")
        if T == 1 and self.len > 0 and self.fast_decode:
            # device-indexed cache write + split-KV decode kernel (graph-capturable)
            D = cfg.head_dim
            if rope is not None and rope.rot_dim % 16 == 0 and FUSED_DECODE_ROPE:
                # rope + cache write of the newest token fused into the attention launch
                cos, sin = rope.tables(qkv.device)
                o = ops._ext.require().decode_attn_rope(
                    qkv, cos, sin, self.pos.view(-1), self.k[layer], self.v[layer], self.slot,
                    self.kv_len, self.kv_start, window, 1.0 / math.sqrt(D), self.h_local, self.kv_local, D,
                    rope.rot_dim)
                return o.reshape(B, 1, self.h_local * D)
            if rope is not None and rope.rot_dim % 16 == 0:
                cos, sin = rope.tables(qkv.device)
                q = ops._ext.require().rope_cache_write(qkv, cos, sin, self.pos.view(-1), self.k[layer],
                                                        self.v[layer], self.slot, self.h_local,
                                                        self.kv_local, D, rope.rot_dim)
            else:
                q, k, v = ops.attention.rope_qk(qkv, rope, self.h_local, self.kv_local, D,
                                                positions=self._pos)
                self.k[layer].index_copy_(1, self.slot, k)
                self.v[layer].index_copy_(1, self.slot, v)
            o = ops.decode.decode_attention(q.reshape(B, self.h_local, D), self.k[layer],
                                            self.v[layer], self.kv_len, self.kv_start, window)
            return o.reshape(B, 1, self.h_local * D)
        pos, kv_start = self._pos, self.kv_start
        if self.split:
            pos = pos.to(qkv.device) if pos is not None else None
            kv_start = kv_start.to(qkv.device) if kv_start is not None else None
        q, k, v = ops.attention.rope_qk(qkv, rope, self.h_local, self.kv_local, cfg.head_dim,
                                        positions=pos)
        self.k[layer][:, self.len:self.len + T] = k
        self.v[layer][:, self.len:self.len + T] = v
        end = self.len + T
        o = ops.attention_core(q.contiguous(), self.k[layer][:, :end], self.v[layer][:, :end],
                               causal=True, causal_off=self.len, window=window,
                               kv_start=kv_start, kv_end=None)
        return o.reshape(B, T, self.h_local * cfg.head_dim)

    def advance(self, T: int):
        """Host-driven advance (prefill / eager decode) keeping the device state in step."""
        self.len += T
        self.slot.fill_(self.len)
        self.kv_len.fill_(self.len + 1)
        start = self.kv_start.view(-1, 1) if self.kv_start is not None else 0
        self.pos.copy_((self.len - start) if self.kv_start is not None
                       else torch.full_like(self.pos, self.len))

    capturing = False  # set while a decode step is being captured / replayed as a graph

    def step_done(self, T: int):
        if self.capturing:
            self.advance_device()
        else:
            self.advance(T)

    def advance_device(self):
        """Device-only advance for a captured decode step (host `len` is tracked by the caller)."""
        self.slot.add_(1)
        self.kv_len.add_(1)
        self.pos.add_(1)


@dataclass
class GenerationConfig:
    max_new_tokens: int = 256
    do_sample: bool = True
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    eos_token_id: Optional[int] = None
    pad_token_id: Optional[int] = None


def sample_next(logits: torch.Tensor, do_sample: bool, temperature: float, top_p: float,
                top_k: int = 0, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """logits [B, V] fp32 -> token ids [B]. Temperature, top-k, nucleus (top-p) filtering."""
    if not do_sample or temperature <= 0:
        return logits.argmax(-1)
    logits = logits / temperature
    if top_k and top_k > 0:
        kth = torch.topk(logits, top_k, dim=-1).values[:, -1:]
        logits = logits.masked_fill(logits < kth, float("-inf"))
    if top_p < 1.0:
        sl, si = torch.sort(logits, descending=True, dim=-1)
        probs = torch.softmax(sl, dim=-1)
        cum = probs.cumsum(-1)
        remove = (cum - probs) > top_p
        sl = sl.masked_fill(remove, float("-inf"))
        logits = torch.full_like(logits, float("-inf")).scatter(-1, si, sl)
    probs = torch.softmax(logits, dim=-1)
    return torch.multinomial(probs, 1, generator=generator).squeeze(-1)


def _graph_capable(model: CausalLM) -> bool:
    """Model-level conditions for a captured decode step: single-device, unsharded, and no host
    sync inside the forward (MoE routing still reads per-expert counts on the host unless the
    device-driven grouped expert GEMM is active)."""
    moe_host_sync = model.cfg.is_moe and not getattr(model, "moe_device_dispatch", False)
    return (model.tp_size == 1 and not model.layers_sharded()
            and model.layer_devices is None and not moe_host_sync)


def _graph_ok(model: CausalLM, cache: KVCache) -> bool:
    return (cache.fast_decode and _graph_capable(model) and not cache.split
            and ops._ext.use_native(cache.k))


class _DecodeGraph:
    """One captured decode step: embed -> layers (device-indexed cache writes, decode kernel)
    -> norm -> LM head -> fused sampler -> finished/pad bookkeeping, all on device."""

    def __init__(self, model, cache, B, max_new, eos, pad, greedy, temperature, top_k, top_p, seed):
        dev = cache.k.device
        self.model, self.cache = model, cache
        self.tok = torch.zeros((B, 1), dtype=torch.long, device=dev)
        self.finished = torch.zeros(B, dtype=torch.bool, device=dev)
        self.out = torch.full((B, max_new), pad, dtype=torch.long, device=dev)
        self.gen_mask = torch.zeros((B, max_new), dtype=torch.long, device=dev)
        self.col = torch.zeros(1, dtype=torch.long, device=dev)
        self.rng = torch.tensor([seed, 0], dtype=torch.long, device=dev)
        self.eos, self.pad = eos, pad
        self.args = (temperature, top_k, top_p, greedy)
        self.graph = None

    def _body(self):
        h = self.model(self.tok, cache=self.cache)
        logits = self.model.logits(h[:, -1])
        self.sample(logits)

    def sample(self, logits):
        t, k, p, g = self.args
        nxt = ops.decode.sample_tokens(logits, t, k, p, g, self.rng)
        nxt = torch.where(self.finished, torch.full_like(nxt, self.pad), nxt)
        self.gen_mask.index_copy_(1, self.col, (~self.finished).long().unsqueeze(1))
        self.out.index_copy_(1, self.col, nxt.unsqueeze(1))
        self.finished |= nxt == self.eos
        self.tok.copy_(nxt.unsqueeze(1))
        self.col.add_(1)
        self.rng[1:].add_(1)

    def reset(self, seed: int):
        self.tok.zero_()
        self.finished.zero_()
        self.out.fill_(self.pad)
        self.gen_mask.zero_()
        self.col.zero_()
        self.rng[0].fill_(seed)
        self.rng[1].fill_(0)

    def capture(self):
        self.cache.capturing = True
        ops.decode._skinny_counters(self.tok.device)  # split-K counters: never allocated in a capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            # thread_local: RCCL's watchdog thread (and in-flight gradient collectives of an
            # overlapped RLHF step) keep making HIP calls while this stream captures
            with torch.cuda.graph(self.graph, stream=s, capture_error_mode="thread_local"):
                self._body()
        torch.cuda.current_stream().wait_stream(s)
        self.model = None  # the graph holds the weight addresses; do not keep the module alive

    def replay(self):
        self.graph.replay()
        self.cache.len += 1


# One captured decode step is kept per model and replayed by later generate() calls of the same
# shape and sampling settings (RLHF generates every step at fixed shapes): no re-capture and no
# new KV cache per call. The key includes every parameter/buffer address, so a module whose
# weights moved (`.to()`, re-materialised shards) captures afresh. DLA_GRAPH_REUSE=0 disables.
# The cached KV cache + graph pool stay resident between calls (through the RLHF backward and
# optimizer step); caches larger than DLA_GRAPH_REUSE_MAX_GB (default 24 GB, << 288 GB HBM) are
# not kept, entries die with their model (weakref callback), and `release_graph_cache(model)`
# frees one model's entry on demand.
GRAPH_REUSE = os.environ.get("DLA_GRAPH_REUSE", "1") != "0"
# rope + KV-cache write of the newest token fused into the decode attention launch
FUSED_DECODE_ROPE = os.environ.get("DLA_FUSED_DECODE_ROPE", "1") != "0"
# ZeRO-3 (FSDP) policies are gathered once per generate() call (DLA_DECODE_GATHER=0: per-layer
# gathers inside every decode step, eager only)
DECODE_GATHER = os.environ.get("DLA_DECODE_GATHER", "1") != "0"
GRAPH_REUSE_MAX_BYTES = int(float(os.environ.get("DLA_GRAPH_REUSE_MAX_GB", "24")) * 2 ** 30)
PROMPT_BUCKET = 64
# KV cache storage head-major ([L, B, Hkv, T_max, D] behind the usual view; DLA_KV_HEAD_MAJOR=0 for
# the token-major layout): B = 64 graph decode 4.984 / 4.991 vs 4.994 / 5.012 ms/token, B = 8 noise
# (same box, round 4 end; the whole GPU tier passes on it, tools/gpu_passes.py ab-kv-head-major)
KV_HEAD_MAJOR = os.environ.get("DLA_KV_HEAD_MAJOR", "1") != "0"
_GRAPH_SLOT: dict = {}  # id(model) -> (weakref(model), key, cache, decode graph)


def clear_graph_cache() -> None:
    _GRAPH_SLOT.clear()


def release_graph_cache(model: CausalLM) -> None:
    """Drop the cached decode graph + KV cache of `model` (e.g. before a memory-heavy step)."""
    _GRAPH_SLOT.pop(id(model), None)


def graph_cache_bytes() -> int:
    return sum(e[2].nbytes() for e in _GRAPH_SLOT.values())


def _remember(model: CausalLM, key, cache, dg) -> None:
    if cache.nbytes() > GRAPH_REUSE_MAX_BYTES:
        return
    mid = id(model)
    _GRAPH_SLOT[mid] = (weakref.ref(model, lambda _r, mid=mid: _GRAPH_SLOT.pop(mid, None)), key, cache, dg)


def _weights_key(model: CausalLM) -> tuple:
    return tuple(t.data_ptr() for t in model.parameters()) + tuple(t.data_ptr() for t in model.buffers())


# fp8 rollouts also prefill on the fp8 inference GEMMs (DLA_PREFILL_FP8=0: bf16 prefill, A/B)
PREFILL_FP8 = os.environ.get("DLA_PREFILL_FP8", "1") != "0"


@torch.no_grad()
def generate(model: CausalLM, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
             max_new_tokens: int = 256, do_sample: bool = True, temperature: float = 1.0,
             top_p: float = 1.0, top_k: int = 0, eos_token_id: Optional[int] = None,
             pad_token_id: Optional[int] = None, generator: Optional[torch.Generator] = None,
             return_mask: bool = False, use_graph: Optional[bool] = None, seed: Optional[int] = None,
             weight_dtype: str = "bf16"):
    """Left-padded prompts [B, Tp] -> sequences [B, Tp + n] (n <= max_new_tokens).

    With `return_mask`, also returns the attention mask of the full sequence (prompt mask, then
    1 for every generated token up to and including EOS, 0 afterwards) — the correct mask for
    the RLHF log-prob pass (fixes Appendix A #10's `generated != pad` which drops real EOS).

    On MI355X the prompt is prefilled with the flash-attention kernel, then every new token is
    ONE replay of a captured hipGraph (decode kernel + fused sampler, no host sync except an
    all-finished check every 16 tokens). `use_graph=False` forces the eager per-op loop.

    `weight_dtype="fp8"`: the decode steps' qkv / o / gate|up / down projections and the LM head
    stream an e4m3 copy of the weights with per-row scales (ops.decode.fp8_weights; half the
    bytes of the dominant weight streams), and the prompt prefill runs those projections on the
    fp8 inference GEMMs (ops.fp8_inference_scope: e4m3 weights and activations, row
    scales, hipBLASLt fp8). Attention, norms and the KV cache stay bf16."""
    if weight_dtype not in ("bf16", "fp8"):
        raise ValueError(f"weight_dtype must be 'bf16' or 'fp8', got {weight_dtype!r}")
    f8 = weight_dtype == "fp8" or ops.decode.fp8_enabled()
    with ops.decode.fp8_weights(f8), ops.fp8_inference_scope(model, f8 and PREFILL_FP8):
        return _generate(model, input_ids, attention_mask, max_new_tokens, do_sample, temperature, top_p,
                         top_k, eos_token_id, pad_token_id, generator, return_mask, use_graph, seed)


def _generate(model: CausalLM, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor],
              max_new_tokens: int, do_sample: bool, temperature: float, top_p: float, top_k: int,
              eos_token_id: Optional[int], pad_token_id: Optional[int],
              generator: Optional[torch.Generator], return_mask: bool, use_graph: Optional[bool],
              seed: Optional[int]):
    if DECODE_GATHER and model.layers_sharded():
        # ZeRO-3 policy: gather it once for the whole rollout (fused decode kernels + captured
        # graph) instead of an all-gather per layer per token
        import contextlib

        try:
            with contextlib.ExitStack() as stack:
                for eng in model.sharding_engines():
                    stack.enter_context(eng.gathered_for_inference())
                return _generate(model, input_ids, attention_mask, max_new_tokens, do_sample, temperature,
                                 top_p, top_k, eos_token_id, pad_token_id, generator, return_mask, use_graph,
                                 seed)
        finally:
            # the gathered units are freed on exit: the captured graph (it reads their addresses),
            # its KV cache and the derived decode weight copies (a second full set of layer
            # weights) go with them, so between rollouts each rank holds only its shards
            release_graph_cache(model)
            ops.decode.drop_derived_weights(model)
    was_training = model.training
    model.eval()
    eos = eos_token_id if eos_token_id is not None else model.cfg.eos_token_id
    pad = pad_token_id if pad_token_id is not None else eos
    extra = 0
    # (gated on the model, not on use_graph: eager and graph decoding of a graph-capable model
    # see the same padded prefill, so their outputs stay bitwise comparable)
    if (GRAPH_REUSE and input_ids.is_cuda and max_new_tokens > 2
            and ops._ext.use_native(input_ids) and _graph_capable(model)):
        # left-pad the prompt to a multiple of PROMPT_BUCKET so batches whose longest prompt
        # differs share one decode graph / KV cache (masked prefix: same tokens, stripped below)
        extra = -input_ids.shape[1] % PROMPT_BUCKET
        if extra:
            fill = pad if pad is not None and 0 <= pad < model.cfg.vocab_size else 0
            input_ids = torch.nn.functional.pad(input_ids, (extra, 0), value=fill)
            am0 = attention_mask if attention_mask is not None else torch.ones_like(input_ids[:, extra:])
            attention_mask = torch.nn.functional.pad(am0, (extra, 0), value=0)
    B, Tp = input_ids.shape
    kv_start = None
    if attention_mask is not None:
        kv_start, _, _ = attention_layout(attention_mask)
    greedy = not do_sample or temperature <= 0
    reuse_key, dg = None, None
    if GRAPH_REUSE and use_graph is not False and max_new_tokens > 2 and input_ids.is_cuda \
            and _graph_capable(model):
        reuse_key = (B, Tp, max_new_tokens, kv_start is None, greedy, float(temperature), int(top_k),
                     float(top_p), eos, pad, input_ids.device, _weights_key(model), ops.decode.fp8_enabled())
        hit = _GRAPH_SLOT.get(id(model))
        if hit is not None and hit[0]() is model and hit[1] == reuse_key:
            cache, dg = hit[2], hit[3]
            cache.reset(kv_start)
        else:
            _GRAPH_SLOT.pop(id(model), None)  # free the old cache before sizing a new one
    if dg is None:
        cache = KVCache(model, B, Tp + max_new_tokens, kv_start)
    # folded RMSNorm weights of the fused decode layer are refreshed in place (never inside the
    # captured step): a cached graph replays the same buffers with the current weights
    ops.decode.refresh_folded_weights(model)
    h = model(input_ids, cache=cache)
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,), generator=generator).item()) if generator is not None \
            and generator.device.type == "cpu" else int(torch.randint(0, 2 ** 62, (1,)).item())
    graph_ok = _graph_ok(model, cache) if use_graph is None else (use_graph and _graph_ok(model, cache))
    if graph_ok and max_new_tokens > 2:
        if dg is None:
            dg = _DecodeGraph(model, cache, B, max_new_tokens, eos, pad, greedy, temperature, top_k,
                              top_p, seed)
        else:
            dg.reset(seed)
        dg.sample(model.logits(h[:, -1]))  # token 1 from the prefill, eager
        h = model(dg.tok, cache=cache)  # token 2 eagerly: warms every decode-shape kernel/GEMM
        dg.sample(model.logits(h[:, -1]))
        n = 2
        if n < max_new_tokens and dg.graph is None:
            dg.model = model
            dg.capture()  # records (does not run) one decode step
            if reuse_key is not None:
                _remember(model, reuse_key, cache, dg)
        while n < max_new_tokens:
            dg.replay()
            n += 1
            if n % 16 == 0 and bool(dg.finished.all()):
                break
        cache.capturing = False
        seqs = torch.cat([input_ids, dg.out[:, :n]], dim=1)
        gm = dg.gen_mask[:, :n]
    else:
        out, gen_mask = [input_ids], []
        finished = torch.zeros(B, dtype=torch.bool, device=input_ids.device)
        rng = torch.tensor([seed, 0], dtype=torch.long, device=input_ids.device)
        last = h[:, -1]
        for step in range(max_new_tokens):
            logits = model.logits(last)
            if ops._ext.use_native(logits):
                nxt = ops.decode.sample_tokens(logits, temperature, top_k, top_p, greedy, rng)
                rng[1:].add_(1)
            else:
                nxt = sample_next(logits.float(), do_sample, temperature, top_p, top_k, generator)
            if model.tp_size > 1:  # every TP rank must continue with the same token
                import torch.distributed as dist

                dist.broadcast(nxt, src=dist.get_global_rank(model.tp, 0), group=model.tp)
            nxt = torch.where(finished, torch.full_like(nxt, pad), nxt)
            gen_mask.append((~finished).long())
            out.append(nxt.unsqueeze(1))
            finished = finished | (nxt == eos)
            if step + 1 < max_new_tokens:
                if step % 16 == 15 and bool(finished.all()):
                    break
                last = model(nxt.unsqueeze(1), cache=cache)[:, -1]
        seqs = torch.cat(out, dim=1)
        gm = torch.stack(gen_mask, 1)
    if was_training:
        model.train()
    pm = attention_mask if attention_mask is not None else torch.ones_like(input_ids)
    if extra:
        seqs, pm = seqs[:, extra:].contiguous(), pm[:, extra:]
    if not return_mask:
        return seqs
    return seqs, torch.cat([pm.long(), gm], dim=1)
