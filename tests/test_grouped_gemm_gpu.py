"""MI355X numerics of the device-driven grouped expert GEMM (csrc/grouped_gemm.hip) against
plain PyTorch fp32 references: forward (bf16 and block-scaled fp8), the SwiGLU epilogues, input
and weight gradients (bf16 / fp32 accumulate), uneven and empty expert groups, partial tiles,
and hipGraph capture of a whole MoE layer (no host sync)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _native():
    from distributed_llm_alignment_amd.ops import _ext

    _ext.require()


def _C():
    from distributed_llm_alignment_amd.ops import _ext

    return _ext.require()


def _offs(counts):
    c = torch.tensor(counts, device=DEV)
    o = torch.zeros(len(counts) + 1, dtype=torch.int32, device=DEV)
    o[1:] = torch.cumsum(c, 0).to(torch.int32)
    return o


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


COUNTS = [300, 0, 17, 520, 256, 1]  # empty group, partial tiles, exact tile, single row


def _rand(*shape, g, scale=1.0):
    return (torch.randn(*shape, device=DEV, generator=g) * scale).to(torch.bfloat16)


@pytest.fixture(params=["default", "0", "3", "4"])
def gg_sched(request):
    """every K-step schedule: the per-layout default, the plain 2-phase step (0), the ping-pong
    phases (3) and the counted 4-phase step (4); switched in-process (torch.ops.dla.gg_set_sched)"""
    prev = _C().gg_set_sched(-1 if request.param == "default" else int(request.param))
    yield request.param
    _C().gg_set_sched(prev)


@pytest.mark.parametrize("N,K", [(384, 256), (264, 136)])
def test_grouped_fwd_vs_fp32(N, K, gg_sched):
    g = torch.Generator(device=DEV).manual_seed(0)
    M, G = sum(COUNTS), len(COUNTS)
    x = _rand(M, K, g=g)
    w = _rand(G, N, K, g=g, scale=0.05)
    y = _C().gg_fwd(x, w, _offs(COUNTS), None, None)
    ref = torch.empty(M, N, device=DEV)
    s = 0
    for e, c in enumerate(COUNTS):
        ref[s:s + c] = x[s:s + c].float() @ w[e].float().t()
        s += c
    assert _rel(y, ref) < 1e-2
    # asymmetric check of the row/column mapping: exact small-integer data
    xi = torch.randint(-3, 4, (M, K), device=DEV, generator=g).to(torch.bfloat16)
    wi = torch.randint(-3, 4, (G, N, K), device=DEV, generator=g).to(torch.bfloat16)
    yi = _C().gg_fwd(xi, wi, _offs(COUNTS), None, None)
    s = 0
    for e, c in enumerate(COUNTS):
        r = xi[s:s + c].float() @ wi[e].float().t()
        assert torch.equal(yi[s:s + c].float(), r.bfloat16().float()), e
        s += c


def test_grouped_fwd_swiglu_epilogue(gg_sched):
    g = torch.Generator(device=DEV).manual_seed(1)
    M, G, K, Fd = sum(COUNTS), len(COUNTS), 192, 256
    x = _rand(M, K, g=g)
    w = _rand(G, 2 * Fd, K, g=g, scale=0.08)
    gu, a = _C().gg_fwd_swiglu(x, w, _offs(COUNTS), None, None)
    s = 0
    for e, c in enumerate(COUNTS):
        r = x[s:s + c].float() @ w[e].float().t()
        if c:
            assert _rel(gu[s:s + c], r) < 1e-2, e
            rg = gu[s:s + c].float()
            ra = F.silu(rg[:, :Fd]) * rg[:, Fd:]
            assert _rel(a[s:s + c], ra) < 1e-2, e
        s += c


@pytest.mark.parametrize("kind", ["fwd", "fwd_swiglu", "dgrad", "dgrad_swiglu", "wgrad"])
def test_grouped_counted_schedule_bitwise(monkeypatch, kind):
    """DLA_GG_SCHED=4 (4 phases per K step, quarter tiles staged 2-6 phases ahead, counted
    vmcnt) sums every output in the same k order as the 2-phase step (0): bitwise equal outputs
    over ragged and empty groups, K tails and >= 16 K steps, for every operand layout."""
    g = torch.Generator(device=DEV).manual_seed(5)
    counts = [700, 0, 1, 256, 333, 1024, 90]
    M, G, K, N = sum(counts), len(counts), 1000, 768
    offs = _offs(counts)
    if kind.startswith("fwd"):
        x = _rand(M, K, g=g)
        w = _rand(G, N, K, g=g, scale=0.05)
        run = (lambda: _C().gg_fwd_swiglu(x, w, offs, None, None)) if kind == "fwd_swiglu" else \
              (lambda: (_C().gg_fwd(x, w, offs, None, None),))
    elif kind == "dgrad":
        dy = _rand(M, N, g=g)
        w = _rand(G, N, K, g=g, scale=0.05)
        run = lambda: (_C().gg_dgrad(dy, w, offs),)
    elif kind == "dgrad_swiglu":
        dy = _rand(M, K, g=g)
        w_down = _rand(G, K, N // 2, g=g, scale=0.05)
        gu = _rand(M, N, g=g)
        run = lambda: _C().gg_dgrad_swiglu(dy, w_down, offs, gu)
    else:
        dy = _rand(M, 264, g=g)
        x = _rand(M, 520, g=g)

        def run():
            out = torch.zeros(G, 264, 520, device=DEV)
            _C().gg_wgrad(dy, x, offs, out, True)
            return (out,)
    outs = []
    prev = _C().gg_set_sched(0)
    try:
        for sc in (0, 4):
            _C().gg_set_sched(sc)
            outs.append(run())
    finally:
        _C().gg_set_sched(prev)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_grouped_dgrad_and_swiglu_bwd_epilogue(gg_sched):
    g = torch.Generator(device=DEV).manual_seed(2)
    M, G, H, Fd = sum(COUNTS), len(COUNTS), 256, 384
    dy = _rand(M, 2 * Fd, g=g)
    w_up = _rand(G, 2 * Fd, H, g=g, scale=0.05)
    dx = _C().gg_dgrad(dy, w_up, _offs(COUNTS))
    s = 0
    for e, c in enumerate(COUNTS):
        if c:
            assert _rel(dx[s:s + c], dy[s:s + c].float() @ w_up[e].float()) < 1e-2, e
        s += c
    dyo = _rand(M, H, g=g)
    w_down = _rand(G, H, Fd, g=g, scale=0.05)
    gu = _rand(M, 2 * Fd, g=g)
    dgu, a = _C().gg_dgrad_swiglu(dyo, w_down, _offs(COUNTS), gu)
    s = 0
    for e, c in enumerate(COUNTS):
        if c:
            da = dyo[s:s + c].float() @ w_down[e].float()
            gg = gu[s:s + c, :Fd].float().requires_grad_(True)
            uu = gu[s:s + c, Fd:].float().requires_grad_(True)
            ra = F.silu(gg) * uu
            dg_, du_ = torch.autograd.grad(ra, [gg, uu], da)
            assert _rel(dgu[s:s + c, :Fd], dg_) < 2e-2, e
            assert _rel(dgu[s:s + c, Fd:], du_) < 2e-2, e
            assert _rel(a[s:s + c], ra.detach()) < 1e-2, e
        s += c


@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_grouped_wgrad_accumulate(out_dtype, gg_sched):
    g = torch.Generator(device=DEV).manual_seed(3)
    M, G, N1, N2 = sum(COUNTS), len(COUNTS), 264, 512
    dy = _rand(M, N1, g=g)
    x = _rand(M, N2, g=g)
    base = torch.randn(G, N1, N2, device=DEV, generator=g).to(out_dtype)
    out = base.clone()
    _C().gg_wgrad(dy, x, _offs(COUNTS), out, True)
    fresh = torch.full_like(base, 7.0)
    _C().gg_wgrad(dy, x, _offs(COUNTS), fresh, False)
    s = 0
    for e, c in enumerate(COUNTS):
        r = dy[s:s + c].float().t() @ x[s:s + c].float()
        assert _rel(out[e].float() - base[e].float(), r) < 2e-2 if c else torch.equal(out[e], base[e])
        if c:
            assert _rel(fresh[e], r) < 1e-2, e
        else:
            assert (fresh[e] == 0).all(), "empty group without accumulate must write zeros"
        s += c


def test_grouped_fp8_forward_vs_dequantized_reference():
    from distributed_llm_alignment_amd import ops

    g = torch.Generator(device=DEV).manual_seed(4)
    M, G, K, N = sum(COUNTS), len(COUNTS), 512, 256
    x = _rand(M, K, g=g, scale=2.0)
    w = _rand(G, N, K, g=g, scale=0.05)
    xq, sx = ops.moe.quant_fp8_rows(x)
    wq, sw = ops.moe.quant_fp8_rows(w.reshape(-1, K))
    wq, sw = wq.view(G, N, K), sw.view(G, N, 1)
    y = _C().gg_fwd(xq, wq, _offs(COUNTS), sx, sw)
    xd = xq.float() * sx
    wd = wq.float() * sw
    s = 0
    for e, c in enumerate(COUNTS):
        if c:
            # same quantised operands in fp32: only accumulation order and bf16 output differ
            assert _rel(y[s:s + c], xd[s:s + c] @ wd[e].t()) < 1e-2, e
        s += c
    gu, a = _C().gg_fwd_swiglu(xq, torch.cat([wq, wq], 1).contiguous(), _offs(COUNTS), sx,
                               torch.cat([sw, sw], 1).contiguous())
    s = 0
    for e, c in enumerate(COUNTS):
        if c:
            r = xd[s:s + c] @ wd[e].t()
            assert _rel(gu[s:s + c, :N], r) < 1e-2 and _rel(gu[s:s + c, N:], r) < 1e-2, e
        s += c


def test_moe_layer_grouped_matches_loop_and_captures():
    import os

    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, get_config

    cfg = get_config("tiny-mixtral", hidden_size=256, intermediate_size=512, num_experts=8)
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=2)
    moe = m.layers[0].mlp
    g = torch.Generator(device=DEV).manual_seed(5)
    h = _rand(4, 200, cfg.hidden_size, g=g).requires_grad_(True)
    os.environ["DLA_MOE_GEMM"] = "grouped"
    try:
        out = moe(h)
        go = _rand(*out.shape, g=g)
        grads = torch.autograd.grad(out, [h, moe.router, moe.expert_up, moe.expert_down], go)
    finally:
        os.environ.pop("DLA_MOE_GEMM")
    os.environ["DLA_MOE_GEMM"] = "loop"
    try:
        out_l = moe(h)
        grads_l = torch.autograd.grad(out_l, [h, moe.router, moe.expert_up, moe.expert_down], go)
    finally:
        os.environ.pop("DLA_MOE_GEMM")
    assert _rel(out, out_l) < 1e-2
    for a, b in zip(grads, grads_l):
        assert _rel(a, b) < 3e-2
    ref = ops.moe.ref_moe(h.detach().reshape(-1, cfg.hidden_size), moe.router, moe.expert_up,
                          moe.expert_down, cfg.num_experts_per_tok).view_as(h)
    assert _rel(out, ref) < 2e-2
    # the whole routed layer (router, sort, dispatch, grouped GEMMs, combine) captures: no host sync
    assert m.moe_device_dispatch
    hs = h.detach().clone()
    with torch.no_grad():
        moe(hs)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            yg = moe(hs)
        hs.copy_(_rand(*hs.shape, g=g))
        graph.replay()
        torch.cuda.synchronize()
        assert _rel(yg, moe(hs)) < 1e-6
