"""MI355X numerics of the MoE HIP kernels (router top-k fwd/bwd, dispatch, combine fwd/bwd)
and the Mixtral layer built on them, against plain PyTorch fp32 references."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module", autouse=True)
def _native():
    from distributed_llm_alignment_amd.ops import _ext

    _ext.require()


def test_topk_kernel_fwd_bwd():
    from distributed_llm_alignment_amd import ops

    g = torch.Generator(device=DEV).manual_seed(0)
    # distinct logits per row (bf16 ties would make the top-k order implementation-defined)
    perm = torch.argsort(torch.rand(4099, 8, device=DEV, generator=g), -1).float()
    logits = (perm * 0.375 - 1.3).to(torch.bfloat16).requires_grad_(True)
    v, i = ops.moe.route_topk(logits, 2)
    lf = logits.detach().float().requires_grad_(True)
    rv, ri = torch.topk(torch.softmax(lf, -1), 2, -1)
    rv = rv / rv.sum(-1, keepdim=True)
    assert torch.equal(i.long(), ri)
    assert torch.allclose(v, rv, atol=1e-5)
    gv = torch.randn_like(v)
    (dl,) = torch.autograd.grad(v, logits, gv)
    (rdl,) = torch.autograd.grad(rv, lf, gv)
    assert torch.allclose(dl.float(), rdl, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("N,H,k,E", [(1000, 4096, 2, 8), (77, 136, 3, 5)])
def test_dispatch_combine_kernels(N, H, k, E):
    from distributed_llm_alignment_amd import ops

    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(N, H, device=DEV, generator=g).to(torch.bfloat16)
    topi = torch.stack([torch.randperm(E, device=DEV, generator=g)[:k] for _ in range(N)]).to(torch.int32)
    pos, counts = ops.moe.expert_positions(topi, E)
    xs = ops.moe.dispatch(x, pos)
    assert torch.equal(xs, ops.moe._ref_dispatch(x, pos))
    w = torch.rand(N, k, device=DEV, generator=g).requires_grad_(True)
    ys = torch.randn(N * k, H, device=DEV, generator=g).to(torch.bfloat16).requires_grad_(True)
    out = ops.moe.combine(ys, pos, w)
    ysf = ys.detach().float().requires_grad_(True)
    wf = w.detach().clone().requires_grad_(True)
    ref = ops.moe._ref_combine(ysf, pos, wf)
    assert torch.allclose(out.float(), ref, atol=2e-2, rtol=1e-2)
    go = torch.randn(N, H, device=DEV, generator=g).to(torch.bfloat16)
    dys, dw = torch.autograd.grad(out, [ys, w], go)
    rdys, rdw = torch.autograd.grad(ref, [ysf, wf], go.float())
    assert torch.allclose(dys.float(), rdys, atol=2e-2, rtol=1e-2)
    assert torch.allclose(dw, rdw, atol=1e-1, rtol=1e-2)


def test_combine_capacity_layout_kernels():
    """The EP capacity path combines from a padded slot buffer (parallel/expert.py): pos indexes a
    [R, H] buffer with R > N*k, unused rows, and every dropped slot on one appended zero row."""
    from distributed_llm_alignment_amd import ops

    g = torch.Generator(device=DEV).manual_seed(4)
    N, k, H, R = 300, 2, 512, 1000
    pos = torch.randperm(R - 1, device=DEV, generator=g)[:N * k].view(N, k).to(torch.int32)
    pos[::7, 1] = R - 1  # dropped slots on an explicit zero row
    pos[3::11, 0] = R  # and one past the buffer (read as zero by the kernels)
    ys = torch.randn(R, H, device=DEV, generator=g).to(torch.bfloat16)
    ys[-1] = 0
    ys.requires_grad_(True)
    w = torch.rand(N, k, device=DEV, generator=g).requires_grad_(True)
    out = ops.moe.combine(ys, pos, w)
    ysf = ys.detach().float().requires_grad_(True)
    wf = w.detach().clone().requires_grad_(True)
    ref = ops.moe._ref_combine(torch.cat([ysf, ysf.new_zeros(1, H)]), pos, wf)
    assert torch.allclose(out.float(), ref, atol=2e-2, rtol=1e-2)
    go = torch.randn(N, H, device=DEV, generator=g).to(torch.bfloat16)
    dys, dw = torch.autograd.grad(out, [ys, w], go)
    rdys, rdw = torch.autograd.grad(ref, [ysf, wf], go.float())
    assert torch.allclose(dys[:-1].float(), rdys[:-1], atol=2e-2, rtol=1e-2)  # unread rows: zero
    assert torch.allclose(dw, rdw, atol=1e-1, rtol=1e-2)


@pytest.mark.parametrize("shape_ep", [4, 8])  # 2 local experts: grouped kernels; 1: the hipBLASLt path
def test_expert_parallel_shape_mode_layer_matches_fp32(shape_ep):
    """bench.py --ep-shape on the GPU: the capacity dispatch (identity all-to-alls, device-built
    expert order, grouped expert kernels, padded combine) of one EP rank's experts, forward and
    backward, against the same layer in fp32 on the CPU."""
    import copy

    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.parallel.expert import apply_expert_parallel

    cfg = get_config("tiny-mixtral", hidden_size=256, intermediate_size=512, num_experts=8)
    m = build_model(cfg, device="cpu", dtype=torch.float32, seed=2)
    apply_expert_parallel(m, None, capacity_factor=2.0, shape_ep=shape_ep)
    mg = copy.deepcopy(m).to(DEV, torch.bfloat16)
    m = m.to(torch.bfloat16).to(torch.float32)  # the reference sees the same (rounded) weights
    for w in (mg.layers[0].mlp.expert_up, mg.layers[0].mlp.expert_down):  # as a training engine does
        w.main_grad = torch.zeros(w.shape, dtype=torch.float32, device=DEV)
    g = torch.Generator().manual_seed(5)
    h = torch.randn(2, 256, cfg.hidden_size, generator=g).to(torch.bfloat16).float()
    outs = []
    for mod, x in ((m.layers[0].mlp, h.clone()), (mg.layers[0].mlp, h.to(DEV, torch.bfloat16))):
        x.requires_grad_(True)
        y = mod(x)
        y.float().pow(2).sum().backward()
        gu = mod.expert_up.main_grad if x.is_cuda else mod.expert_up.grad
        outs.append((y.detach().float().cpu(), x.grad.float().cpu(), gu.float().cpu()))
    (y0, dx0, du0), (y1, dx1, du1) = outs
    # a token whose top-2 router logits nearly tie may pick another expert in bf16 than in fp32:
    # per-token rows are compared with a small allowance for such flips, the expert grads as a whole
    for name, a, b in (("y", y0, y1), ("dx", dx0, dx1)):
        assert torch.isfinite(b).all(), name
        a2, b2 = a.reshape(-1, a.shape[-1]), b.reshape(-1, b.shape[-1])
        rel = (a2 - b2).norm(dim=-1) / a2.norm(dim=-1).clamp_min(1e-12)
        assert (rel > 3e-2).float().mean() < 0.03, (name, rel.sort().values[-20:])
    assert torch.isfinite(du1).all()
    assert (du0 - du1).norm() / du0.norm() < 5e-2


def test_mixtral_layer_bf16_vs_fp32_reference():
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, get_config

    cfg = get_config("tiny-mixtral", hidden_size=256, intermediate_size=512, num_experts=8)
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=2)
    moe = m.layers[0].mlp
    g = torch.Generator(device=DEV).manual_seed(3)
    h = (torch.randn(4, 256, cfg.hidden_size, device=DEV, generator=g)).to(torch.bfloat16).requires_grad_(True)
    out = moe(h)
    ref = ops.moe.ref_moe(h.detach().reshape(-1, cfg.hidden_size), moe.router, moe.expert_up,
                          moe.expert_down, cfg.num_experts_per_tok).view_as(h)
    err = (out.float() - ref).abs().max() / ref.abs().max()
    assert err < 3e-2, err
    out.float().pow(2).sum().backward()
    for p in (h, moe.router, moe.expert_up, moe.expert_down):
        assert p.grad is not None and torch.isfinite(p.grad.float()).all()


def test_fp8_expert_forward_close_to_bf16():
    from distributed_llm_alignment_amd import ops

    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn(512, 1024, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(2048, 1024, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    y8 = ops.moe.fp8_linear(x, w)
    y = x.float() @ w.float().t()
    rel = (y8.float() - y).norm() / y.norm()
    assert rel < 6e-2, rel


def test_fp8_rowwise_quant_kernel_and_moe_layer():
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, get_config

    g = torch.Generator(device=DEV).manual_seed(5)
    x = (torch.randn(333, 4096, device=DEV, generator=g) * 3).to(torch.bfloat16)
    q, inv = ops.moe.quant_fp8_rows(x)
    assert q.dtype == torch.float8_e4m3fn and inv.shape == (333, 1)
    deq = q.float() * inv
    assert ((deq - x.float()).abs() / x.float().abs().amax(1, keepdim=True)).max() < 0.07
    assert torch.allclose(inv, x.float().abs().amax(1, keepdim=True) / 448.0, rtol=1e-6)
    cfg = get_config("tiny-mixtral", hidden_size=256, intermediate_size=512, num_experts=8)
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=2)
    moe = m.layers[0].mlp
    h = torch.randn(3, 171, cfg.hidden_size, device=DEV, generator=g).to(torch.bfloat16)
    ref = moe(h).float()
    moe.fp8 = True
    out = moe(h).float()
    assert (out - ref).norm() / ref.norm() < 0.08


@pytest.mark.parametrize("gemm", ["grouped", "auto"])
@pytest.mark.parametrize("policy", ["full", "mlp"])
def test_moe_recompute_keeps_expert_grads(policy, gemm, monkeypatch):
    """Expert weights accumulate into the engine's main_grad from the expert autograd node
    (grouped GEMM, or the per-expert loop that `auto` takes for bf16 training); under activation
    recompute (whole layer or MLP block) that node must still see the real parameters (weights
    ride on ctx): one DPO step's gradients equal the no-recompute step's."""
    monkeypatch.setenv("DLA_MOE_GEMM", gemm)
    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.objectives import dpo_step_loss
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine

    cfg = get_config("tiny-mixtral", hidden_size=256, head_dim=64, intermediate_size=512, num_experts=8)
    grads = []
    for pol in (None, policy):
        m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=3)
        ref = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=3).requires_grad_(False)
        if pol is not None:
            m.gradient_checkpointing_enable(pol)
        eng = DataParallelEngine(m, lr=1e-3, weight_decay=0.0, max_grad_norm=1.0)
        b = synthetic_preference_batch(2, 128, cfg.vocab_size, device=DEV, generator=torch.Generator().manual_seed(1))
        loss, _ = dpo_step_loss(m, ref, b)
        loss.backward()
        eng.finish_grad_sync()
        grads.append({n: (p.main_grad if getattr(p, "main_grad", None) is not None else p.grad).float().clone()
                      for n, p in m.named_parameters()})
    for n, a in grads[0].items():
        assert a.abs().max() > 0, n
        torch.testing.assert_close(grads[1][n], a, rtol=2e-2, atol=2e-4, msg=n)


def test_moe_fp8_hybrid_backward_matches_grouped(monkeypatch):
    """fp8 experts: `auto` with DLA_MOE_BWD=loop runs the forward on the grouped fp8 kernel and
    the backward on the per-expert hipBLASLt loop; its input / weight gradients match the
    all-grouped backward (the default)."""
    from distributed_llm_alignment_amd.models import build_model, get_config

    cfg = get_config("tiny-mixtral", hidden_size=256, intermediate_size=512, num_experts=8)
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=4)
    moe = m.layers[0].mlp
    moe.fp8 = True
    g = torch.Generator(device=DEV).manual_seed(8)
    h = torch.randn(2, 160, cfg.hidden_size, device=DEV, generator=g).to(torch.bfloat16).requires_grad_(True)
    go = torch.randn(2, 160, cfg.hidden_size, device=DEV, generator=g).to(torch.bfloat16)
    res = {}
    monkeypatch.setenv("DLA_MOE_BWD", "loop")
    for mode in ("auto", "grouped"):
        monkeypatch.setenv("DLA_MOE_GEMM", mode)
        out = moe(h)
        res[mode] = (out.float(),) + tuple(
            t.float() for t in torch.autograd.grad(out, [h, moe.expert_up, moe.expert_down], go))
    for a, b in zip(res["auto"], res["grouped"]):
        assert (a - b).norm() / b.norm().clamp(min=1e-6) < 2e-2


@pytest.mark.parametrize("K", [1024, 4096, 14336, 20480])
def test_fp8_row_quant_matches_torch_conversion(K):
    """Row-wise e4m3 quantiser (single-pass register form up to K = 16384, two-pass above):
    scale = amax / 448, codes equal torch's float8_e4m3fn conversion of x * 448 / amax (up to
    the last bits of the kernel's scale and the hardware conversion: ~0.2 % of codes one step away)."""
    from distributed_llm_alignment_amd import ops

    g = torch.Generator(device=DEV).manual_seed(K)
    x = (torch.randn(67, K, device=DEV, generator=g) * 2).to(torch.bfloat16)
    q, inv = ops.moe.quant_fp8_rows(x)
    amax = x.float().abs().amax(1, keepdim=True).clamp(min=1e-12)
    assert torch.allclose(inv, amax / 448.0, rtol=1e-6, atol=0)
    ref = (x.float() * (448.0 / amax)).to(torch.float8_e4m3fn)
    a, b = q.view(torch.uint8).int(), ref.view(torch.uint8).int()
    diff = (a - b).abs()
    assert int(diff.max()) <= 1 and float((diff > 0).float().mean()) < 1e-2


def test_moe_transposed_dgrad_matches_nn_and_follows_steps(monkeypatch):
    """Per-expert backward through the cached transposed expert weights (TN input-gradient GEMMs)
    equals the NN-layout backward, also after the weights changed (the copy is re-made)."""
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine

    monkeypatch.setenv("DLA_MOE_GEMM", "loop")
    cfg = get_config("tiny-mixtral", hidden_size=256, intermediate_size=512, num_experts=8)
    m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=6)
    eng = DataParallelEngine(m, lr=1e-2, weight_decay=0.0, max_grad_norm=1.0)
    moe = m.layers[0].mlp
    g = torch.Generator(device=DEV).manual_seed(2)
    h = torch.randn(2, 150, cfg.hidden_size, device=DEV, generator=g).to(torch.bfloat16)
    go = torch.randn(2, 150, cfg.hidden_size, device=DEV, generator=g).to(torch.bfloat16)
    for step in range(2):
        res = {}
        for tn in (True, False):
            monkeypatch.setattr(ops.moe, "MOE_TRANSPOSED_DGRAD", tn)
            for p in (moe.expert_up, moe.expert_down):
                p.main_grad.zero_()
            x = h.clone().requires_grad_(True)
            moe(x).backward(go)
            res[tn] = [x.grad.float()] + [p.main_grad.float().clone() for p in (moe.expert_up, moe.expert_down)]
        for a, b in zip(res[True], res[False]):
            assert (a - b).norm() / b.norm().clamp(min=1e-6) < 1e-2, step
        with torch.no_grad():  # new weights: the cached transposes must follow
            moe.expert_up.mul_(1.25)
            moe.expert_down.mul_(0.8)
    assert eng is not None


def test_mixtral_layer_fwd_bwd_graph_captured_matches_fp32():
    """The whole Mixtral MoE layer -- router top-k, device-side expert offsets, dispatch, grouped
    expert GEMMs (SwiGLU fused), combine -- forward AND backward captured in ONE hipGraph (no host
    sync anywhere) and replayed; outputs and every gradient against an fp32 autograd reference
    (HF Mixtral semantics, ops.moe.ref_moe) on the same bf16 weights; a second replay with new
    inputs written into the static buffers follows them."""
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, get_config

    cfg = get_config("tiny-mixtral", hidden_size=256, intermediate_size=512, num_experts=8)
    moe = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=5).layers[0].mlp
    g = torch.Generator(device=DEV).manual_seed(9)
    x = torch.randn(512, cfg.hidden_size, device=DEV, generator=g).to(torch.bfloat16).requires_grad_(True)
    gy = torch.randn(512, cfg.hidden_size, device=DEV, generator=g).to(torch.bfloat16)
    params = [x, moe.router, moe.expert_up, moe.expert_down]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up: allocates .grad and every lazily created buffer
        for _ in range(2):
            moe(x).backward(gy)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        y = moe(x)
        y.backward(gy)

    def check():
        for p in params:
            p.grad.zero_()
        graph.replay()
        torch.cuda.synchronize()
        xr, rr, ur, dr = (p.detach().float().requires_grad_(True) for p in params)
        # fp32 Mixtral math with the routing the bf16 router logits select (as the kernel does:
        # near-ties between experts may order differently in fp32)
        with torch.no_grad():
            topi = torch.topk(torch.nn.functional.linear(x.detach(), moe.router.detach()).float(),
                              cfg.num_experts_per_tok, -1).indices
        logits = xr @ rr.t()
        w = torch.softmax(logits.gather(1, topi), -1)
        yr = torch.zeros_like(xr)
        for j in range(topi.shape[1]):
            for e in range(cfg.num_experts):
                sel = topi[:, j] == e
                gu = xr[sel] @ ur[e].t()
                a = torch.nn.functional.silu(gu[:, :gu.shape[1] // 2]) * gu[:, gu.shape[1] // 2:]
                yr = yr.index_add(0, sel.nonzero().squeeze(1), w[sel, j:j + 1] * (a @ dr[e].t()))
        yr.backward(gy.float())
        err = lambda a, b: float((a.float() - b).norm() / (b.norm() + 1e-12))
        assert err(y, yr) < 2e-2
        for p, r in zip(params, (xr, rr, ur, dr)):
            assert err(p.grad, r.grad) < 5e-2, (p.shape, err(p.grad, r.grad))

    check()
    with torch.no_grad():  # new routing: the captured graph must follow the device-side offsets
        x.copy_(torch.randn(x.shape, device=DEV, generator=g).to(torch.bfloat16))
    check()


@pytest.mark.parametrize("E,ep,n,k,cf", [(8, 8, 2048, 2, 1.25), (8, 4, 1000, 2, 1.0), (8, 2, 777, 2, 0.6),
                                         (16, 8, 4096, 2, 2.0), (64, 8, 333, 4, 1.0), (8, 1, 64, 1, 1.0)])
def test_native_ep_route_matches_torch(E, ep, n, k, cf, monkeypatch):
    """csrc/moe.hip ep_route / ep_expert_order == parallel/expert.py's torch forms, bit for bit:
    send rows, slot positions, sent counts, dropped slots (capacity factors that drop), and the
    receiver's expert-major order and offsets."""
    from distributed_llm_alignment_amd.parallel import expert as epm

    g = torch.Generator(device=DEV).manual_seed(E * 131 + ep + n)
    # skewed routing so some destinations overflow their capacity
    w = torch.rand(E, device=DEV, generator=g) ** 3 + 0.05
    topi = torch.multinomial(w.expand(n, E), k, replacement=False, generator=g).to(torch.int32)
    xp = epm.ExpertParallel(None, E, capacity_factor=cf, shape_ep=ep) if ep > 1 else None
    if xp is None:  # ep == 1: shape mode needs ep > 1; build the object by hand
        xp = epm.ExpertParallel.__new__(epm.ExpertParallel)
        xp.shape, xp.group, xp.ep, xp.rank, xp.E, xp.El = True, None, 1, 0, E, E
        xp.capacity_factor, xp.chunks, xp._dropped = cf, 1, None
    C = xp.capacity(n, k)
    got = xp._route_chunk(topi, C)
    nd_native = int(xp._dropped.item())
    monkeypatch.setattr(epm, "_NATIVE_ROUTE", False)
    want = xp._route_chunk(topi, C)
    assert torch.equal(got[0], want[0])
    assert torch.equal(got[1].long(), want[1].long())
    assert torch.equal(got[2].long(), want[2].long())
    assert nd_native == int(want[3].item())
    # receiver order for a few received-count patterns (the shape mode's rc = sent)
    for rc in (want[2].to(torch.int32), torch.randint(0, C // max(1, E // ep) + 1, (ep, E // ep), device=DEV,
                                                       generator=g).to(torch.int32)):
        rc = torch.minimum(rc, torch.full_like(rc, C // (E // ep)))
        ref = xp._expert_order(rc, C)
        monkeypatch.setattr(epm, "_NATIVE_ROUTE", True)
        nat = xp._expert_order(rc, C)
        monkeypatch.setattr(epm, "_NATIVE_ROUTE", False)
        for a, b in zip(nat, ref):
            assert torch.equal(a.long(), b.long())


def test_native_gather_rows_fwd_bwd(monkeypatch):
    """parallel/expert.py _gather_rows on the HIP kernels (gather with holes, adjoint scatter)
    equals its torch form forward and backward, bitwise."""
    from distributed_llm_alignment_amd.parallel import expert as epm

    g = torch.Generator(device=DEV).manual_seed(9)
    R, n, H = 300, 500, 264
    x = torch.randn(R, H, device=DEV, generator=g).to(torch.bfloat16)
    idx = torch.full((n,), -1, dtype=torch.long, device=DEV)
    sel = torch.randperm(n, device=DEV, generator=g)[:R - 20]
    idx[sel] = torch.randperm(R, device=DEV, generator=g)[:R - 20]  # injective, some rows unread
    go = torch.randn(n, H, device=DEV, generator=g).to(torch.bfloat16)
    dup = idx.clone()
    dup[: n // 2] = torch.randint(0, R, (n // 2,), device=DEV, generator=g)  # rows read twice or more
    for ix, inj in ((idx, True), (dup, False)):
        res = []
        for native in (True, False):
            monkeypatch.setattr(epm, "_NATIVE_ROUTE", native)
            xx = x.clone().requires_grad_(True)
            y = epm._gather_rows(xx, ix, injective=inj)
            (dx,) = torch.autograd.grad(y, [xx], go)
            res.append((y, dx.float()))
        assert torch.equal(res[0][0], res[1][0])
        # the adjoint against an fp32 scatter-add (the torch form sums in bf16)
        ref = torch.zeros(R, H, device=DEV).index_add_(0, ix.clamp(min=0), go.float() * (ix >= 0).unsqueeze(-1))
        if inj:
            assert torch.equal(res[0][1], res[1][1])
        assert (res[0][1] - ref).abs().max() <= 1e-2 * ref.abs().max()


@pytest.mark.gpu
def test_native_gather_rows_bwd_through_inverse_map():
    """The token -> slot gather's backward as a gather-sum through the slot positions (the
    combine kernel with unit weights, parallel/expert.py `inv`) equals the fp32 scatter-add,
    including tokens with dropped slots (position >= the slot count)."""
    from distributed_llm_alignment_amd.parallel import expert as epm

    g = torch.Generator(device=DEV).manual_seed(11)
    N, k, H, S = 257, 2, 264, 400  # tokens, top-k, width, slots (some tokens' slots dropped)
    x = torch.randn(N, H, device=DEV, generator=g).to(torch.bfloat16)
    perm = torch.randperm(N * k, device=DEV, generator=g)
    pos = torch.full((N * k,), S, dtype=torch.long, device=DEV)
    pos[perm[:S]] = torch.arange(S, device=DEV)  # slot s <- (token, choice) perm[s]
    src = torch.full((S,), -1, dtype=torch.long, device=DEV)
    src[pos[pos < S]] = (torch.arange(N * k, device=DEV) // k)[pos < S]
    pos = pos.view(N, k)
    go = torch.randn(S, H, device=DEV, generator=g).to(torch.bfloat16)
    out = []
    for inv in (pos, None):
        xx = x.clone().requires_grad_(True)
        y = epm._gather_rows(xx, src, injective=False, inv=inv)
        (dx,) = torch.autograd.grad(y, [xx], go)
        out.append((y, dx))
    assert torch.equal(out[0][0], out[1][0])
    ref = torch.zeros(N, H, device=DEV).index_add_(0, src.clamp(min=0), go.float() * (src >= 0).unsqueeze(-1))
    assert torch.equal(out[0][1], ref.to(torch.bfloat16))  # k = 2: both sums are exact-order fp32
    assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("main", [512, 768, 1024])
def test_single_expert_main_overflow_split_matches_whole_buffer(main):
    """One local expert over a capacity buffer with the library GEMMs on the first `main` rows and
    the overflow rows [main, offs[-1]) on the grouped kernels (ops.moe.MOE_MAIN_ROWS): forward,
    input gradient and the main-grad weight gradients against the same node over the whole buffer
    (main 1024 = every row on the library). Rows past offs[-1] stay zero."""
    from distributed_llm_alignment_amd import ops

    g = torch.Generator(device=DEV).manual_seed(21)
    rows, H, F, valid = 1024, 512, 512, 900
    xs = (torch.randn(rows, H, device=DEV, generator=g)).to(torch.bfloat16)
    xs[valid:] = 0
    w_up = (torch.randn(1, 2 * F, H, device=DEV, generator=g) * H ** -0.5).to(torch.bfloat16)
    w_down = (torch.randn(1, H, F, device=DEV, generator=g) * F ** -0.5).to(torch.bfloat16)
    offs = torch.tensor([0, valid], dtype=torch.int32, device=DEV)
    dy = torch.randn(rows, H, device=DEV, generator=g).to(torch.bfloat16)
    dy[valid:] = 0
    res = {}
    for m in (main, 0):
        wu, wd = w_up.clone(), w_down.clone()
        wu.main_grad = torch.zeros(wu.shape, dtype=torch.float32, device=DEV)
        wd.main_grad = torch.zeros(wd.shape, dtype=torch.float32, device=DEV)
        x = xs.clone().requires_grad_(True)
        y = ops.moe.experts_swiglu_offsets(x, wu, wd, offs, main_rows=m)
        (dx,) = torch.autograd.grad(y, [x], dy)
        res[m] = (y.float(), dx.float(), wu.main_grad.clone(), wd.main_grad.clone())
    rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-12))
    for a, b in zip(res[main], res[0]):
        assert rel(a, b) < 1e-2
    assert float(res[main][0][valid:].abs().max()) == 0.0
    assert float(res[main][1][valid:].abs().max()) == 0.0


def test_expert_parallel_adaptive_main_rows(monkeypatch):
    """parallel.expert ADAPTIVE_MAIN: the rank of a hot expert (EP shape mode, every source at
    capacity) starts with the library GEMMs on the expected n * k rows and, from the next call of
    the same layer on, on every row its expert received (the count copied to a pinned host word
    without a sync); outputs equal the static split's."""
    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.parallel import expert as epmod

    cfg = get_config("tiny-mixtral", hidden_size=256, intermediate_size=512, num_experts=8)
    E = cfg.num_experts
    seen = []
    real = ops.moe.experts_swiglu_offsets

    def spy(xe, w_up, w_down, offs, **kw):
        seen.append((xe.shape[0], kw.get("main_rows", 0)))
        return real(xe, w_up, w_down, offs, **kw)

    monkeypatch.setattr(ops.moe, "experts_swiglu_offsets", spy)
    h = torch.randn(2, 512, cfg.hidden_size, device=DEV).to(torch.bfloat16)
    outs = {}
    for adaptive in (False, True):
        monkeypatch.setattr(epmod, "ADAPTIVE_MAIN", adaptive)
        m = build_model(cfg, device=DEV, dtype=torch.bfloat16, seed=0)
        epmod.apply_expert_parallel(m, None, capacity_factor=1.5, shape_ep=E, shape_hot=True)
        seen.clear()
        with torch.no_grad():
            y0 = m.layers[0].mlp(h)
            torch.cuda.synchronize()
            y1 = m.layers[0].mlp(h)
        (r0, m0), (r1, m1) = seen[0], seen[-1]
        assert m0 < r0
        assert (m1 == r1) if adaptive else (m1 == m0)
        outs[adaptive] = (y0.float(), y1.float())
    rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-12))
    assert rel(outs[True][0], outs[False][0]) == 0.0
    assert rel(outs[True][1], outs[False][1]) < 1e-2
