"""MI355X numerics of the decode path: split-KV decode attention and the fused sampler against
PyTorch references, and graph-captured generation == eager generation (greedy)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _native():
    from distributed_llm_alignment_amd.ops import _ext

    _ext.require()


@pytest.mark.parametrize("blocks", [None, "16", "60", "one-chunk"])
@pytest.mark.parametrize("D,Hq,Hkv,window", [(128, 32, 8, 0), (64, 8, 8, 0), (128, 16, 2, 300), (64, 16, 8, 0)])
def test_decode_attention_matches_reference(D, Hq, Hkv, window, blocks, monkeypatch):
    """blocks: DLA_DECODE_BLOCKS target -- None keeps the default (the loop kernel, 2 chunks per
    block at this size), 16 / 60 force 1 / 2 splits per sequence, "one-chunk" the one-chunk kernel
    + combine launch (DLA_DECODE_LOOP=0)."""
    from distributed_llm_alignment_amd.ops import decode

    if blocks == "one-chunk":
        monkeypatch.setenv("DLA_DECODE_LOOP", "0")
    elif blocks is not None:
        monkeypatch.setenv("DLA_DECODE_BLOCKS", blocks)

    g = torch.Generator(device=DEV).manual_seed(0)
    B, Tmax, L = 5, 1100, 777
    kc = torch.randn(B, Tmax, Hkv, D, device=DEV, generator=g).to(torch.bfloat16)
    vc = torch.randn(B, Tmax, Hkv, D, device=DEV, generator=g).to(torch.bfloat16)
    q = torch.randn(B, Hq, D, device=DEV, generator=g).to(torch.bfloat16)
    ks = torch.tensor([0, 3, 100, 700, 0], dtype=torch.int32, device=DEV)
    kv_len = torch.tensor([L], dtype=torch.int32, device=DEV)
    o = decode.decode_attention(q, kc, vc, kv_len, ks, window)
    r = decode.ref_decode_attention(q, kc, vc, L, ks, window)
    assert torch.allclose(o.float(), r.float(), atol=2e-2, rtol=2e-2), (o.float() - r.float()).abs().max()


def test_decode_attention_strided_cache_view():
    """The model passes a [B, Tmax, Hkv, D] view of an [L, B, Tmax, Hkv, D] cache."""
    from distributed_llm_alignment_amd.ops import decode

    g = torch.Generator(device=DEV).manual_seed(1)
    big = torch.randn(3, 2, 300, 8, 128, device=DEV, generator=g).to(torch.bfloat16)
    vbig = torch.randn(3, 2, 300, 8, 128, device=DEV, generator=g).to(torch.bfloat16)
    q = torch.randn(2, 32, 128, device=DEV, generator=g).to(torch.bfloat16)
    kv_len = torch.tensor([257], dtype=torch.int32, device=DEV)
    o = decode.decode_attention(q, big[1], vbig[1], kv_len)
    r = decode.ref_decode_attention(q, big[1], vbig[1], 257)
    assert torch.allclose(o.float(), r.float(), atol=2e-2, rtol=2e-2)


def test_sampler_greedy_and_topk1_are_argmax():
    from distributed_llm_alignment_amd.ops import decode

    g = torch.Generator(device=DEV).manual_seed(2)
    logits = torch.randn(7, 128256, device=DEV, generator=g).to(torch.bfloat16)
    rng = torch.tensor([123, 0], dtype=torch.long, device=DEV)
    ref = logits.float().argmax(-1)
    assert torch.equal(decode.sample_tokens(logits, 1.0, 0, 1.0, True, rng), ref)
    assert torch.equal(decode.sample_tokens(logits, 0.7, 1, 1.0, False, rng), ref)


@pytest.mark.parametrize("top_k,top_p", [(0, 1.0), (0, 0.8), (3, 1.0), (4, 0.7)])
def test_sampler_distribution(top_k, top_p):
    from distributed_llm_alignment_amd.ops import decode

    base = torch.tensor([2.0, 1.5, 1.0, 0.5, 0.0, -0.5, -1.0, -3.0], device=DEV)
    T = 0.9
    rows = 20000
    logits = base.expand(rows, -1).contiguous()
    rng = torch.tensor([7, 11], dtype=torch.long, device=DEV)
    tok = decode.sample_tokens(logits, T, top_k, top_p, False, rng)
    freq = torch.bincount(tok, minlength=8).float() / rows
    z = base / T
    if top_k:
        z = torch.where(z >= torch.topk(z, top_k).values[-1], z, torch.tensor(float("-inf"), device=DEV))
    p = torch.softmax(z, 0)
    if top_p < 1.0:
        sp, si = torch.sort(p, descending=True)
        keep = (sp.cumsum(0) - sp) < top_p
        p2 = torch.zeros_like(p)
        p2[si[keep]] = sp[keep]
        p = p2 / p2.sum()
    assert torch.allclose(freq, p, atol=0.015), (freq, p)


@pytest.mark.parametrize("top_k,top_p", [(0, 1.0), (0, 0.8), (3, 1.0), (4, 0.7), (6, 0.5)])
def test_split_sampler_distribution_large_vocab(top_k, top_p):
    """Row-split sampler (V >= 32768 with top-k / top-p): 8 planted logits spread over
    different chunks of a 128256 vocabulary, the rest far below the -64 z window."""
    from distributed_llm_alignment_amd.ops import decode

    V, rows, T = 128256, 12000, 0.9
    base = torch.tensor([2.0, 1.5, 1.0, 0.5, 0.0, -0.5, -1.0, -3.0], device=DEV)
    pos = torch.tensor([5, 17000, 33333, 50008, 70001, 90000, 110007, 128255], device=DEV)
    logits = torch.full((rows, V), -100.0, device=DEV, dtype=torch.bfloat16)
    logits[:, pos] = base.to(torch.bfloat16)
    rng = torch.tensor([7, 11], dtype=torch.long, device=DEV)
    tok = decode.sample_tokens(logits, T, top_k, top_p, False, rng)
    assert bool(torch.isin(tok, pos).all())
    freq = (tok.unsqueeze(1) == pos.unsqueeze(0)).float().mean(0)
    z = base / T
    if top_k:
        z = torch.where(z >= torch.topk(z, top_k).values[-1], z, torch.tensor(float("-inf"), device=DEV))
    p = torch.softmax(z, 0)
    if top_p < 1.0:
        sp, si = torch.sort(p, descending=True)
        keep = (sp.cumsum(0) - sp) < top_p
        p2 = torch.zeros_like(p)
        p2[si[keep]] = sp[keep]
        p = p2 / p2.sum()
    assert torch.allclose(freq, p, atol=0.02), (freq, p)


@pytest.mark.parametrize("top_k,top_p", [(50, 1.0), (0, 0.9), (50, 0.9)])
def test_split_sampler_support_random_logits(top_k, top_p):
    """Every draw of the row-split sampler lies inside the top-k set / the nucleus of a
    plain fp32 reference, on dense random logits (the shape a decode step sees)."""
    from distributed_llm_alignment_amd.ops import decode

    g = torch.Generator(device=DEV).manual_seed(5)
    B, V, T = 8, 128256, 0.7
    logits = (torch.randn(B, V, device=DEV, generator=g) * 3.0).to(torch.bfloat16)
    z = logits.float() / T
    sz, _ = torch.sort(z, dim=-1, descending=True)
    floor = torch.full((B,), -float("inf"), device=DEV)
    if top_k:  # ties of the k-th value are kept, as in the kernel
        floor = sz[:, top_k - 1]
    if top_p < 1.0:
        pz = torch.softmax(torch.where(sz >= floor[:, None] - 1e-4, sz,
                                       torch.tensor(float("-inf"), device=DEV)), -1)
        nucleus = (pz.cumsum(-1) - pz) < top_p + 1e-3
        edge = torch.where(nucleus, sz, torch.tensor(float("inf"), device=DEV)).min(-1).values
        floor = torch.maximum(floor, edge)
    allowed = z >= floor[:, None] - 1e-4
    seen = set()
    for step in range(64):
        rng = torch.tensor([3, step], dtype=torch.long, device=DEV)
        tok = decode.sample_tokens(logits, T, top_k, top_p, False, rng)
        assert bool(allowed.gather(1, tok[:, None]).all()), step
        seen.update(tok.tolist())
    assert len(seen) > 16  # it samples, not argmax


@pytest.mark.parametrize("blocks", [None, "2"])
def test_graph_generation_matches_eager_greedy(blocks, monkeypatch):
    from distributed_llm_alignment_amd.models import build_model, generate, get_config

    if blocks is not None:  # the multi-chunk decode attention kernel inside the captured graph
        monkeypatch.setenv("DLA_DECODE_BLOCKS", blocks)

    cfg = get_config("tiny-llama-d128")
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=0)
    g = torch.Generator(device=DEV).manual_seed(3)
    ids = torch.randint(3, cfg.vocab_size, (3, 20), device=DEV, generator=g)
    am = torch.ones_like(ids)
    am[1, :5] = 0  # left padding
    ids[1, :5] = 0
    a = generate(m, ids, am, max_new_tokens=24, do_sample=False, eos_token_id=-1, use_graph=False)
    b = generate(m, ids, am, max_new_tokens=24, do_sample=False, eos_token_id=-1, use_graph=True)
    assert torch.equal(a, b), (a, b)
    # and both equal a no-cache full-forward greedy continuation for row 0
    x = ids[:1]
    for _ in range(8):
        h = m(x)
        nxt = m.logits(h[:, -1]).float().argmax(-1, keepdim=True)
        x = torch.cat([x, nxt], 1)
    assert torch.equal(x[0, 20:28], a[0, 20:28])


@pytest.mark.parametrize("top_k,top_p", [(0, 1.0), (50, 0.9)])
def test_graph_generation_matches_eager_sampled_large_vocab(top_k, top_p):
    """Sampled decoding with a 65536-token vocabulary takes the row-split sampler (several
    launches + a workspace per step); a captured hipGraph replay draws the same tokens as eager
    decoding for the same seed (device-side Philox counter, order-independent histograms)."""
    import dataclasses

    from distributed_llm_alignment_amd.models import build_model, generate, get_config

    cfg = dataclasses.replace(get_config("tiny-llama-d128"), vocab_size=65536)
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=0)
    g = torch.Generator(device=DEV).manual_seed(4)
    ids = torch.randint(3, cfg.vocab_size, (4, 16), device=DEV, generator=g)
    am = torch.ones_like(ids)
    kw = dict(max_new_tokens=24, do_sample=True, temperature=0.8, top_k=top_k, top_p=top_p,
              eos_token_id=-1, seed=11)
    a = generate(m, ids, am, use_graph=False, **kw)
    b = generate(m, ids, am, use_graph=True, **kw)
    assert torch.equal(a, b), (a, b)
    assert len(set(a[:, 16:].flatten().tolist())) > 24  # sampled, not a fixed point


@pytest.mark.parametrize("fp8", [False, True])
def test_moe_generation_graph_matches_eager(fp8):
    """Mixtral-style policy: routing + device-driven grouped expert GEMMs (no host sync) inside
    the captured decode step give the same greedy tokens as eager decoding and the graph is
    actually used. With fp8 experts (quantised weight copies cached outside the graph) capture
    is refused and use_graph=True falls back to eager decoding, still with the same tokens."""
    from distributed_llm_alignment_amd.models import build_model, generate, get_config
    from distributed_llm_alignment_amd.models import generation as gen

    gen.clear_graph_cache()
    cfg = get_config("tiny-mixtral", hidden_size=256, head_dim=64, intermediate_size=512, num_experts=8)
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=3)
    for layer in m.layers:
        layer.mlp.fp8 = fp8
    assert gen._graph_capable(m) == (not fp8)
    g = torch.Generator(device=DEV).manual_seed(6)
    ids = torch.randint(3, cfg.vocab_size, (3, 17), device=DEV, generator=g)
    am = torch.ones_like(ids)
    am[2, :4] = 0
    ids[2, :4] = 0
    a = generate(m, ids, am, max_new_tokens=16, do_sample=False, eos_token_id=-1, use_graph=False)
    b = generate(m, ids, am, max_new_tokens=16, do_sample=False, eos_token_id=-1, use_graph=True)
    assert torch.equal(a, b), (a, b)
    captured = id(m) in gen._GRAPH_SLOT and gen._GRAPH_SLOT[id(m)][3].graph is not None
    assert captured == (not fp8)
    gen.clear_graph_cache()


def test_decode_graph_reused_across_generate_calls():
    """The second generate() of the same shape replays the first call's captured decode step
    (no new KV cache, no re-capture) and still matches eager decoding on new prompts and new
    left padding; moving the weights forces a fresh capture."""
    from distributed_llm_alignment_amd.models import build_model, generate, get_config
    from distributed_llm_alignment_amd.models import generation as gen

    gen.clear_graph_cache()
    cfg = get_config("tiny-llama-d128")
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=0)
    g = torch.Generator(device=DEV).manual_seed(5)
    kw = dict(max_new_tokens=20, do_sample=True, temperature=0.9, top_p=0.9, eos_token_id=-1)
    graphs = []
    for call, padrow in enumerate((1, 2, 0)):
        ids = torch.randint(3, cfg.vocab_size, (3, 18), device=DEV, generator=g)
        am = torch.ones_like(ids)
        am[padrow, : 3 + call] = 0
        ids[padrow, : 3 + call] = 0
        a = generate(m, ids, am, use_graph=False, seed=call, **kw)
        b, mb = generate(m, ids, am, use_graph=True, seed=call, return_mask=True, **kw)
        assert torch.equal(a, b), (call, a, b)
        assert torch.equal(mb[:, :18], am.long()) and bool(mb[:, 18:].eq(1).all())
        graphs.append(gen._GRAPH_SLOT[id(m)][3].graph)
    assert graphs[0] is graphs[1] is graphs[2]
    # new weight addresses -> fresh capture, still correct
    for p in m.parameters():
        p.data = p.data.clone()
    ids = torch.randint(3, cfg.vocab_size, (3, 18), device=DEV, generator=g)
    am = torch.ones_like(ids)
    a = generate(m, ids, am, use_graph=False, seed=9, **kw)
    b = generate(m, ids, am, use_graph=True, seed=9, **kw)
    assert torch.equal(a, b)
    assert gen._GRAPH_SLOT[id(m)][3].graph is not graphs[0]
    gen.clear_graph_cache()


def test_layer_split_gpu_host_matches_single_gpu():
    """Layer-split model parallel (device_map, parallel/layer_split.py) with a real device hop:
    first half of the layers on the GPU (HIP kernels), second half on the host (reference ops),
    embedding + head on the GPU. Log-probs match the one-GPU model to bf16 tolerance and
    gradients reach every layer on both devices."""
    from distributed_llm_alignment_amd.models import build_model, generate, get_config
    from distributed_llm_alignment_amd.parallel.layer_split import dispatch_layers

    cfg = get_config("tiny-llama-d128")
    a = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=0)
    b = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=0)
    devs = dispatch_layers(b, [DEV, "cpu"])
    assert {d.type for d in devs} == {"cuda", "cpu"} and b.embed.device.type == "cuda"
    g = torch.Generator(device=DEV).manual_seed(5)
    ids = torch.randint(3, cfg.vocab_size, (2, 40), device=DEV, generator=g)
    am = torch.ones_like(ids)
    am[1, :7] = 0
    la, lb = a.sequence_logprob(ids, am), b.sequence_logprob(ids, am)
    assert lb.device.type == "cuda" and (la.float() - lb.float()).abs().max().item() < 0.05
    lb.sum().backward()
    assert all(p.grad is not None and torch.isfinite(p.grad.float()).all() for p in b.parameters())
    out = generate(b, ids, am, max_new_tokens=6, do_sample=False, eos_token_id=-1)
    assert out.shape == (2, 46) and out.device.type == "cuda"


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("N,K,swiglu", [(4096, 4096, False), (6144, 4096, False), (1040, 512, False),
                                         (4096, 14336, False), (16, 2048, False),
                                         (4096, 14336, True), (28672, 4096, False), (2048, 768, True)])
def test_skinny_gemm_matches_fp32(M, N, K, swiglu):
    """Decode skinny GEMM (csrc/skinny.hip) vs an fp32 PyTorch reference, split-K and not, with
    the fused SwiGLU input; bitwise repeatable (fixed-order split-K reduction)."""
    from distributed_llm_alignment_amd.ops import decode

    g = torch.Generator(device=DEV).manual_seed(M * 7 + N)
    x = torch.randn(M, 2 * K if swiglu else K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).to(torch.bfloat16)
    with torch.no_grad():
        y = decode.skinny_linear(x, w, swiglu=swiglu, min_n=0)
        assert y is not None and y.shape == (M, N)
        r = decode.ref_skinny_linear(x, w, swiglu)
        err = (y.float() - r.float()).abs().max().item()
        assert err <= 2e-2 * max(1.0, r.float().abs().max().item()), err
        y2 = decode.skinny_linear(x, w, swiglu=swiglu, min_n=0)  # counters re-armed, same bits
        assert torch.equal(y, y2)


def test_skinny_gemm_strided_rows_and_eligibility():
    from distributed_llm_alignment_amd.ops import decode

    g = torch.Generator(device=DEV).manual_seed(3)
    big = torch.randn(4, 1, 3 * 1024, device=DEV, generator=g).to(torch.bfloat16)
    x = big[..., 1024:2048]                                     # [4, 1, 1024] row stride 3072
    w = torch.randn(512, 1024, device=DEV, generator=g).to(torch.bfloat16)
    with torch.no_grad():
        y = decode.skinny_linear(x, w, min_n=0)
        assert y.shape == (4, 1, 512)
        assert torch.allclose(y.float(), decode.ref_skinny_linear(x, w).float(), atol=0.25, rtol=2e-2)
        assert decode.skinny_linear(torch.zeros(65, 1024, device=DEV, dtype=torch.bfloat16), w, min_n=0) is None
        assert decode.skinny_linear(torch.zeros(2, 1000, device=DEV, dtype=torch.bfloat16),
                                    torch.zeros(512, 1000, device=DEV, dtype=torch.bfloat16), min_n=0) is None
        assert decode.skinny_linear(x, w, min_n=1 << 20) is None  # width threshold respected
    xg = x.detach().clone().requires_grad_(True)
    assert decode.skinny_linear(xg, w, min_n=0) is None  # autograd: library GEMM path


@pytest.mark.parametrize("mode", ["lds", "ks"])
@pytest.mark.parametrize("M", [1, 8, 16])
@pytest.mark.parametrize("F,K", [(14336, 4096), (192, 512)])
def test_skinny_glu_epilogue_matches_unfused(M, F, K, mode):
    """gate|up skinny GEMM with the SwiGLU epilogue == swiglu(bf16 GEMM output), fp32 reference;
    both gate|up kernels (LDS-staged and in-workgroup split-K)."""
    from distributed_llm_alignment_amd.ops import decode

    g = torch.Generator(device=DEV).manual_seed(M + F)
    x = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(2 * F, K, device=DEV, generator=g) * K ** -0.5).to(torch.bfloat16)
    with torch.no_grad():
        m = decode.skinny_glu(x, w, mode=mode)
        assert m is not None and m.shape == (M, F)
        u = (x.float() @ w.float().t()).to(torch.bfloat16)
        gg, uu = u.float().chunk(2, dim=-1)
        r = (torch.nn.functional.silu(gg) * uu)
        err = (m.float() - r).abs().max().item()
        assert err <= 3e-2 * max(1.0, r.abs().max().item()), err


@pytest.mark.parametrize("D,Hq,Hkv,rot", [(128, 32, 8, 128), (64, 8, 8, 32), (128, 8, 1, 64)])
@pytest.mark.parametrize("blocks", [None, "4", "one-chunk"])
def test_fused_rope_decode_attention_matches_unfused(D, Hq, Hkv, rot, blocks, monkeypatch):
    """decode_attn_rope (rope + cache write of the newest token inside the attention launch) ==
    rope_cache_write + decode_attn, bitwise: output and the written cache row (blocks = 4: both
    on the multi-chunk loop kernel, the newest key's V patched into the DMA'd LDS image)."""
    from distributed_llm_alignment_amd.ops import RotaryCache, _ext

    if blocks == "one-chunk":
        monkeypatch.setenv("DLA_DECODE_LOOP", "0")
    elif blocks is not None:
        monkeypatch.setenv("DLA_DECODE_BLOCKS", blocks)

    C = _ext.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    B, Tmax, L = 3, 300, 257  # newest token at slot 256: first key of a fresh 128-key split
    rope = RotaryCache(rot, 10000.0, 4096, None)
    cos, sin = rope.tables(dev)
    kc = torch.randn(B, Tmax, Hkv, D, device=dev, generator=g).to(torch.bfloat16)
    vc = torch.randn(B, Tmax, Hkv, D, device=dev, generator=g).to(torch.bfloat16)
    qkv = torch.randn(B, 1, (Hq + 2 * Hkv) * D, device=dev, generator=g).to(torch.bfloat16)
    kv_start = torch.tensor([0, 5, 40], device=dev, dtype=torch.int32)
    pos = (L - 1 - kv_start).to(torch.int32)
    slot = torch.tensor([L - 1], device=dev, dtype=torch.long)
    kv_len = torch.tensor([L], device=dev, dtype=torch.int32)
    k1, v1 = kc.clone(), vc.clone()
    q = C.rope_cache_write(qkv, cos, sin, pos, k1, v1, slot, Hq, Hkv, D, rot)
    ref = C.decode_attn(q, k1, v1, kv_len, kv_start, 0, D ** -0.5)
    k2, v2 = kc.clone(), vc.clone()
    out = C.decode_attn_rope(qkv, cos, sin, pos, k2, v2, slot, kv_len, kv_start, 0, D ** -0.5, Hq, Hkv, D, rot)
    torch.cuda.synchronize()
    assert torch.equal(k1, k2) and torch.equal(v1, v2)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("M", [17, 24, 32, 40, 64])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336), (1040, 1024)])
def test_skinny_split_k_many_rows_matches_fp32(M, N, K, monkeypatch):
    """17..64 decode rows on the in-workgroup split-K kernel (2 or 4 row tiles of 16 per weight
    fragment, rows past M masked; opt-in, DLA_SKINNY_MAX_ROWS) vs an fp32 reference; bitwise
    repeatable."""
    from distributed_llm_alignment_amd.ops import decode

    monkeypatch.setattr(decode, "SKINNY_MAX_ROWS", 64)
    g = torch.Generator(device=DEV).manual_seed(M * 31 + N)
    x = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).to(torch.bfloat16)
    with torch.no_grad():
        y = decode.skinny_linear(x, w)
        assert y is not None and y.shape == (M, N)
        r = decode.ref_skinny_linear(x, w)
        err = (y.float() - r.float()).abs().max().item()
        assert err <= 2e-2 * max(1.0, r.float().abs().max().item()), err
        assert torch.equal(y, decode.skinny_linear(x, w))
        # wide outputs and fused-swiglu inputs are not taken above 16 rows
        assert decode.skinny_linear(torch.zeros(M, 4096, device=DEV, dtype=torch.bfloat16),
                                    torch.zeros(16384, 4096, device=DEV, dtype=torch.bfloat16)) is None


@pytest.mark.parametrize("M", [20, 33, 64])
def test_skinny_glu_many_rows_matches_unfused(M, monkeypatch):
    """gate|up + SwiGLU epilogue at 17..64 rows (split-K GLU kernel, 4 row tiles) vs fp32."""
    from distributed_llm_alignment_amd.ops import decode

    monkeypatch.setattr(decode, "SKINNY_MAX_ROWS", 64)
    F, K = 1024, 4096
    g = torch.Generator(device=DEV).manual_seed(M)
    x = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(2 * F, K, device=DEV, generator=g) * K ** -0.5).to(torch.bfloat16)
    with torch.no_grad():
        m = decode.skinny_glu(x, w)
        assert m is not None and m.shape == (M, F)
        u = (x.float() @ w.float().t()).to(torch.bfloat16)
        gg, uu = u.float().chunk(2, dim=-1)
        r = torch.nn.functional.silu(gg) * uu
        err = (m.float() - r).abs().max().item()
        assert err <= 3e-2 * max(1.0, r.abs().max().item()), err


@pytest.mark.parametrize("max_rows", [16, 64])
def test_generation_batch_48_graph_matches_eager(max_rows, monkeypatch):
    """A 48-row decode batch (library GEMMs, or the opt-in many-row split-K skinny kernels): the
    captured hipGraph decode draws the same tokens as eager decoding."""
    from distributed_llm_alignment_amd.models import build_model, generate, get_config
    from distributed_llm_alignment_amd.models import generation as gen
    from distributed_llm_alignment_amd.ops import decode

    monkeypatch.setattr(decode, "SKINNY_MAX_ROWS", max_rows)
    gen.clear_graph_cache()
    # H = 1024: qkv / o / down / gate|up all on the split-K kernels
    cfg = get_config("tiny-llama-d128", hidden_size=1024, num_heads=8, num_kv_heads=2)
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=0)
    g = torch.Generator(device=DEV).manual_seed(12)
    ids = torch.randint(3, cfg.vocab_size, (48, 21), device=DEV, generator=g)
    am = torch.ones_like(ids)
    am[5, :6] = 0
    ids[5, :6] = 0
    kw = dict(max_new_tokens=16, do_sample=True, temperature=0.9, top_p=0.9, eos_token_id=-1, seed=4)
    a = generate(m, ids, am, use_graph=False, **kw)
    b = generate(m, ids, am, use_graph=True, **kw)
    assert torch.equal(a, b)
    gen.clear_graph_cache()


def _fused_cfg():
    from distributed_llm_alignment_amd.models import get_config

    # the smallest Llama shape the fused decode layer takes (H and F multiples of 1024)
    return get_config("tiny-llama-d128", hidden_size=1024, num_heads=8, num_kv_heads=2, head_dim=128,
                      intermediate_size=2048, num_layers=3, vocab_size=4096)


@pytest.mark.parametrize("B", [1, 5, 16, 24, 64])
def test_fused_decode_layer_matches_unfused(B, monkeypatch):
    """Decode step with the residual add + RMSNorm folded into the projections (producer row
    partials, consumer-side normalisation; ops.decode fused layer) against the separate-norm
    path and an fp32 full forward, and graph == eager on the fused kernels."""
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, generate
    from distributed_llm_alignment_amd.models.generation import KVCache, clear_graph_cache

    cfg = _fused_cfg()
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=2).eval()
    g = torch.Generator(device=DEV).manual_seed(7)
    ids = torch.randint(3, cfg.vocab_size, (B, 40), device=DEV, generator=g)
    nxt = torch.randint(3, cfg.vocab_size, (B, 1), device=DEV, generator=g)
    outs = {}
    with torch.no_grad():
        for fused in (False, True):
            monkeypatch.setattr(ops.decode, "DECODE_FUSED_NORM", fused)
            cache = KVCache(m, B, 48, None)
            m(ids, cache=cache)
            assert m.layers[0].decode_fused_ok(m.embed_tokens(nxt)) == fused
            outs[fused] = m(nxt, cache=cache).float()
        ref = m(torch.cat([ids, nxt], 1))[:, -1:].float()
    err = lambda a, b: float((a - b).norm() / b.norm())
    assert err(outs[True], outs[False]) < 1e-2
    assert err(outs[True], ref) < 2e-2
    monkeypatch.setattr(ops.decode, "DECODE_FUSED_NORM", True)
    clear_graph_cache()
    a = generate(m, ids, max_new_tokens=12, do_sample=False, eos_token_id=-1, use_graph=False)
    b = generate(m, ids, max_new_tokens=12, do_sample=False, eos_token_id=-1, use_graph=True)
    clear_graph_cache()
    assert torch.equal(a, b)


def test_fsdp_sharded_policy_generation_matches_unsharded(monkeypatch):
    """A ZeRO-3 policy: generate() gathers it once for the rollout (gathered_for_inference: the
    fused decode kernels and the captured graph on resident weights) and its greedy rollouts equal
    the unsharded model's bitwise; with DLA_DECODE_GATHER off the decode steps take the per-layer
    hooked path (never the fused kernels, which would read freed unit storage) and equal the
    unsharded model on that same path. The units are resharded afterwards."""
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, generate, generation
    from distributed_llm_alignment_amd.models.generation import PROMPT_BUCKET, clear_graph_cache
    from distributed_llm_alignment_amd.parallel.fsdp import FullyShardedEngine

    cfg = _fused_cfg()
    a_m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=2).eval()
    b_m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=2)
    eng = FullyShardedEngine(b_m, lr=1e-3)
    b_m.eval()
    assert b_m.layers_sharded() and not a_m.layers_sharded()
    ids = torch.randint(3, cfg.vocab_size, (4, PROMPT_BUCKET), device=DEV,
                        generator=torch.Generator(device=DEV).manual_seed(3))
    clear_graph_cache()
    a = generate(a_m, ids, max_new_tokens=10, do_sample=False, eos_token_id=-1, use_graph=False)
    torch.cuda.synchronize()
    mem0 = torch.cuda.memory_allocated(DEV)
    b = generate(b_m, ids, max_new_tokens=10, do_sample=False, eos_token_id=-1)
    torch.cuda.synchronize()
    # the rollout's gathered units, captured graph, KV cache and derived decode weight copies are
    # all released: the sharded policy costs its shards again, not a second full model
    mem1 = torch.cuda.memory_allocated(DEV)
    layer_bytes = sum(p.numel() * p.element_size() for p in a_m.layers.parameters())
    assert mem1 - mem0 < 0.1 * layer_bytes, (mem0, mem1, layer_bytes)
    assert not any(k in p.__dict__ for p in b_m.parameters() for k in ops.decode.DERIVED_ATTRS)
    clear_graph_cache()
    assert torch.equal(a, b)
    assert b_m.layers_sharded() and not any(u.resident for u in eng.units if not u.is_root)
    monkeypatch.setattr(generation, "DECODE_GATHER", False)
    b2 = generate(b_m, ids, max_new_tokens=10, do_sample=False, eos_token_id=-1)
    monkeypatch.setattr(ops.decode, "DECODE_FUSED_NORM", False)  # same per-layer kernels
    a2 = generate(a_m, ids, max_new_tokens=10, do_sample=False, eos_token_id=-1, use_graph=False)
    clear_graph_cache()
    assert torch.equal(a2, b2)


def test_fused_decode_projection_kernels_match_fp32():
    """The two fused kernel forms in isolation: residual producer (s, row partials of s^2) and the
    norm-on-input consumer (ksplit and the gate|up GLU), against fp32 math on the same bf16 data."""
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.ops.norm import _ref_norm

    M, H, F = 7, 4096, 14336
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(M, F, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(H, F, device=DEV, generator=g) * F ** -0.5).to(torch.bfloat16)
    res = torch.randn(M, H, device=DEV, generator=g).to(torch.bfloat16)
    s, ssq = ops.decode.skinny_residual(x, w, res)
    s_ref = ((x.float() @ w.float().t()).to(torch.bfloat16).float() + res.float())
    assert float((s.float() - s_ref).abs().max()) < 0.05
    sums = ssq[:M].sum(1)
    assert torch.allclose(sums, (s.float() ** 2).sum(1), rtol=1e-4)
    nw = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).to(torch.bfloat16)
    h_ref = _ref_norm(s.float(), nw.float(), None, 1e-5, True)
    wq = (torch.randn(6144, H, device=DEV, generator=g) * H ** -0.5).to(torch.bfloat16)
    y = ops.decode.skinny_normed(s, ssq, nw, 1e-5, wq)
    y_ref = h_ref @ wq.float().t()
    assert float((y.float() - y_ref).norm() / y_ref.norm()) < 1e-2
    wgu = (torch.randn(2 * F, H, device=DEV, generator=g) * H ** -0.5).to(torch.bfloat16)
    mm = ops.decode.skinny_normed(s, ssq, nw, 1e-5, wgu, glu=True)
    gu = h_ref @ wgu.float().t()
    m_ref = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
    assert float((mm.float() - m_ref).norm() / m_ref.norm()) < 1e-2
    # tiled weight layout (the default, DLA_DECODE_TILED) == row-major weights, bitwise
    C = ops._ext.require()
    s_rm, ssq_rm = C.skinny_fused(x, w, res, None, 0.0, False)
    assert torch.equal(s_rm, s) and torch.equal(ssq_rm[:M], ssq[:M])  # rows >= M are not written
    s_t, _ = C.skinny_fused(x, ops.decode.tiled_weight(w), res, None, 0.0, False)
    assert torch.equal(s_t, s)
    y_rm, _ = C.skinny_fused(s, ops.decode.folded_weight(wq, nw), None, ssq, 1e-5, False)
    assert torch.equal(y_rm, y)
    mm_rm, _ = C.skinny_fused(s, ops.decode.folded_weight(wgu, nw), None, ssq, 1e-5, True)
    assert torch.equal(mm_rm, mm)
    # the interleaved-tile gate|up kernel (7 waves per workgroup) == the 8-wave LDS-exchange kernel
    mm_t, _ = C.skinny_fused(s, ops.decode.folded_weight(wgu, nw, tiled=True), None, ssq, 1e-5, True)
    mm_il = C.skinny_glu_il(s, ops.decode.folded_weight(wgu, nw, tiled=True, glu_il=True), ssq, 1e-5)
    assert torch.equal(mm_il, mm_t)
    for Mx in (1, 15, 16):  # every row count the rstd waves cover
        sx = torch.randn(Mx, H, device=DEV, generator=g).to(torch.bfloat16)
        sq = torch.zeros(16, H // 16, device=DEV)
        sq[:Mx] = (sx.float() ** 2).view(Mx, H // 16, 16).sum(-1)
        a, _ = C.skinny_fused(sx, ops.decode.folded_weight(wgu, nw, tiled=True), None, sq, 1e-5, True)
        b = C.skinny_glu_il(sx, ops.decode.folded_weight(wgu, nw, tiled=True, glu_il=True), sq, 1e-5)
        assert torch.equal(a, b), Mx


def test_tile_weight_kernel_matches_permute():
    """csrc/skinny64.hip tile_weight_kernel == the torch permute definition of the tiled layout,
    bitwise, plain and with the RMSNorm weight folded in (torch.mul rounding)."""
    from distributed_llm_alignment_amd import ops

    g = torch.Generator(device=DEV).manual_seed(3)
    N, K = 6144, 4096
    w = torch.randn(N, K, device=DEV, generator=g).to(torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(K, device=DEV, generator=g)).to(torch.bfloat16)
    for norm in (None, nw):
        for il in (False, True):
            out = torch.empty((N // 16, K // 32, 4, 16, 8), dtype=torch.bfloat16, device=DEV)
            ops._ext.require().tile_weight(w, norm, out, il)
            src = w if norm is None else w * norm.view(1, -1)
            if il:
                src = ops.decode._glu_interleave(src)
            ref = src.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4)
            assert torch.equal(out, ref)


@pytest.mark.parametrize("M", [17, 32, 33, 64])
def test_skinny64_kernels_match_fp32(M):
    """csrc/skinny64.hip (17..64 decode rows): plain split-K GEMMs at the Llama-3-8B projection
    shapes and a no-split wide shape, the residual producer (s, row partials of s^2 per 1024
    columns), and the norm-on-input consumers (qkv via the reduce, gate|up via the GLU
    epilogue), each against fp32 math on the same bf16 data."""
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.ops.norm import _ref_norm

    g = torch.Generator(device=DEV).manual_seed(M)
    rel = lambda a, b: float((a.float() - b).norm() / b.norm())
    for N, K in ((6144, 4096), (4096, 14336), (32768, 512), (1152, 1024)):
        x = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).to(torch.bfloat16)
        y = ops.decode.skinny64_linear(x, w)
        assert y.shape == (M, N)
        assert rel(y, x.float() @ w.float().t()) < 5e-3, (N, K)
        # the tiled weight layout is only a different load order: bitwise the same result
        assert torch.equal(ops.decode.skinny64_linear(x, w, tiled=True), y), (N, K)
    H, F = 4096, 14336
    x = torch.randn(M, F, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(H, F, device=DEV, generator=g) * F ** -0.5).to(torch.bfloat16)
    res = torch.randn(M, H, device=DEV, generator=g).to(torch.bfloat16)
    s, ssq = ops.decode.skinny_residual(x, w, res)
    assert ssq.shape == (M, H // 1024)
    s_ref = (x.float() @ w.float().t()).to(torch.bfloat16).float() + res.float()
    assert float((s.float() - s_ref).abs().max()) < 0.05
    assert torch.allclose(ssq.sum(1), (s.float() ** 2).sum(1), rtol=1e-4)
    s_t, ssq_t = ops._ext.require().skinny64(x, ops.decode.tiled_weight(w), res, None, 0.0, False)
    assert torch.equal(s_t, s) and torch.equal(ssq_t, ssq)
    nw = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).to(torch.bfloat16)
    h_ref = _ref_norm(s.float(), nw.float(), None, 1e-5, True)
    wq = (torch.randn(6144, H, device=DEV, generator=g) * H ** -0.5).to(torch.bfloat16)
    y = ops.decode.skinny_normed(s, ssq, nw, 1e-5, wq)
    assert rel(y, h_ref @ wq.float().t()) < 1e-2
    wgu = (torch.randn(2 * F, H, device=DEV, generator=g) * H ** -0.5).to(torch.bfloat16)
    mm = ops.decode.skinny_normed(s, ssq, nw, 1e-5, wgu, glu=True)
    gu = h_ref @ wgu.float().t()
    assert rel(mm, torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]) < 1e-2
    # row-major folded weight (DLA_M64_TILED=0) == the tiled default, bitwise
    mm_rm, _ = ops._ext.require().skinny64(s, ops.decode.folded_weight(wgu, nw), None, ssq, 1e-5, True)
    assert torch.equal(mm_rm, mm)


# ------------------------------------------------------------------ weight-only fp8 decode
def _dequant(w, norm_w=None):
    from distributed_llm_alignment_amd import ops

    src = w if norm_w is None else w * norm_w.view(1, -1)
    q, sc = ops.decode.quantize_rows_f8(src)
    return q.view(torch.float8_e4m3fn).float() * sc[:, None]


@pytest.mark.parametrize("M", [1, 7, 16, 24, 64])
def test_fp8_decode_projection_kernels_match_dequant_fp32(M):
    """The e4m3 weight streams (csrc/skinny_ks.h F8, skinny_glu_il_kernel F8 at <= 16 rows,
    csrc/skinny64.hip F8 at 17..64 rows, both m64 tile heights): residual producer,
    norm-on-input qkv and the gate|up GLU against fp32 math on the DEQUANTISED weights (so only
    accumulation order and bf16 output rounding differ), and within fp8 quantisation error of the
    bf16 kernels."""
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.ops.norm import _ref_norm

    H, F = 4096, 14336
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(M, F, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(H, F, device=DEV, generator=g) * F ** -0.5).to(torch.bfloat16)
    res = torch.randn(M, H, device=DEV, generator=g).to(torch.bfloat16)
    rel = lambda a, b: float((a.float() - b.float()).norm() / b.float().norm())
    s16, _ = ops.decode.skinny_residual(x, w, res)
    with ops.decode.fp8_weights(True):
        s, ssq = ops.decode.skinny_residual(x, w, res)
    s_ref = ((x.float() @ _dequant(w).t()).to(torch.bfloat16).float() + res.float())
    assert float((s.float() - s_ref).abs().max()) < 0.05
    assert torch.allclose(ssq[:M].sum(1), (s.float() ** 2).sum(1), rtol=1e-4)
    assert rel(s - res, s16 - res) < 0.06  # the projection part, fp8 vs bf16 weights
    nw = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).to(torch.bfloat16)
    h_ref = _ref_norm(s.float(), nw.float(), None, 1e-5, True)
    wq = (torch.randn(6144, H, device=DEV, generator=g) * H ** -0.5).to(torch.bfloat16)
    wgu = (torch.randn(2 * F, H, device=DEV, generator=g) * H ** -0.5).to(torch.bfloat16)
    y16 = ops.decode.skinny_normed(s, ssq, nw, 1e-5, wq)
    m16 = ops.decode.skinny_normed(s, ssq, nw, 1e-5, wgu, glu=True)
    with ops.decode.fp8_weights(True):
        y = ops.decode.skinny_normed(s, ssq, nw, 1e-5, wq)
        mm = ops.decode.skinny_normed(s, ssq, nw, 1e-5, wgu, glu=True)
    rstd = torch.rsqrt((s.float() ** 2).mean(1, keepdim=True) + 1e-5)
    y_ref = (s.float() * rstd) @ _dequant(wq, nw).t()
    assert rel(y, y_ref) < 1e-2
    gu = (s.float() * rstd) @ _dequant(wgu, nw).t()
    m_ref = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
    assert rel(mm, m_ref) < 1e-2
    assert rel(y, y16) < 0.06 and rel(mm, m16) < 0.08
    assert rel(y16, h_ref @ wq.float().t()) < 1e-2  # (the bf16 reference itself)


@pytest.mark.parametrize("B", [8, 40])
def test_fp8_generation_graph_matches_eager_and_tracks_bf16(B):
    """generate(weight_dtype="fp8") on the fused decode layer (B 8: csrc/skinny.hip F8 kernels,
    B 40: csrc/skinny64.hip F8): graph == eager (greedy, bitwise), the fp8 copies are refreshed
    when the weights move, and the first decode step's logits stay within quantisation error of
    the bf16 decode."""
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, generate
    from distributed_llm_alignment_amd.models.generation import KVCache, clear_graph_cache

    cfg = _fused_cfg()
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=4).eval()
    g = torch.Generator(device=DEV).manual_seed(9)
    ids = torch.randint(3, cfg.vocab_size, (B, 40), device=DEV, generator=g)
    nxt = torch.randint(3, cfg.vocab_size, (B, 1), device=DEV, generator=g)
    logits = {}
    with torch.no_grad():
        for dt in ("bf16", "fp8"):
            with ops.decode.fp8_weights(dt == "fp8"):
                cache = KVCache(m, B, 48, None)
                m(ids, cache=cache)
                logits[dt] = m.logits(m(nxt, cache=cache)[:, -1]).float()
    rel = float((logits["fp8"] - logits["bf16"]).norm() / logits["bf16"].norm())
    assert rel < 0.1, rel
    assert getattr(m.layers[0].mlp.down_proj, "_dla_f8", None) is not None  # the fp8 path ran
    clear_graph_cache()
    a = generate(m, ids, max_new_tokens=12, do_sample=False, eos_token_id=-1, use_graph=False, weight_dtype="fp8")
    # after the prefill's fp8 inference scope the marking is undone and its e4m3 weight copy is
    # dropped (not left resident on a trainable policy between rollouts)
    w0 = m.layers[0].mlp.up_proj
    assert getattr(w0, "_dla_fp8", None) is None and not getattr(w0, "_dla_fp8_infer", False)
    b = generate(m, ids, max_new_tokens=12, do_sample=False, eos_token_id=-1, use_graph=True, weight_dtype="fp8")
    assert torch.equal(a, b)
    # weights move (an optimizer step): the in-place refreshed fp8 copies follow, graph reused
    with torch.no_grad():
        for p in m.parameters():
            p.mul_(1.01)
    c = generate(m, ids, max_new_tokens=12, do_sample=False, eos_token_id=-1, use_graph=True, weight_dtype="fp8")
    d = generate(m, ids, max_new_tokens=12, do_sample=False, eos_token_id=-1, use_graph=False, weight_dtype="fp8")
    clear_graph_cache()
    assert torch.equal(c, d)


def test_quant_tile_f8_kernel_matches_torch_reference():
    """The one-pass HIP quantiser (csrc/skinny64.hip quant_tile_f8_kernel) against the torch
    quantise + tile reference: plain, norm-folded and gate / up interleaved."""
    from distributed_llm_alignment_amd import ops

    C = ops._ext.require()
    g = torch.Generator(device=DEV).manual_seed(11)
    for N, K, fold, glu in ((64, 1024, False, False), (96, 2048, True, False), (128, 1024, True, True)):
        w = (torch.randn(N, K, device=DEV, generator=g) * torch.rand(N, 1, device=DEV, generator=g) * 3).to(torch.bfloat16)
        nw = (1 + 0.2 * torch.randn(K, device=DEV, generator=g)).to(torch.bfloat16) if fold else None
        t = torch.empty(N // 16, K // 64, 64, 16, dtype=torch.uint8, device=DEV)
        sc = torch.empty(N, dtype=torch.float32, device=DEV)
        C.quant_tile_f8(w, nw, t, sc, glu)
        src = w if nw is None else w * nw.view(1, -1)
        if glu:
            src = ops.decode._glu_interleave(src)
        q_ref, sc_ref = ops.decode.quantize_rows_f8(src)
        assert torch.allclose(sc, sc_ref, rtol=1e-6, atol=0)
        t_ref = ops.decode.tile_f8(q_ref)
        mismatch = (t != t_ref).float().mean().item()
        assert mismatch < 1e-2, mismatch  # rounding of values within an ulp of a tie only
        # any difference is one e4m3 code step (same sign: adjacent byte values)
        assert int((t.int() - t_ref.int()).abs().max()) <= 1
