"""CPU tier: the pure-PyTorch reference ops (the numerics oracles of the HIP kernels) against
literal re-statements of the reference formulas."""
import math

import pytest
import torch
import torch.nn.functional as F

from distributed_llm_alignment_amd import ops
from distributed_llm_alignment_amd.ops.attention import RotaryCache, ref_attention
from distributed_llm_alignment_amd.optim.adamw import adamw_update, clip_coefficient, grad_sumsq


def _naive_attention(q, k, v, scale, causal, off, window, ks, ke):
    B, Tq, Hq, D = q.shape
    Tk, Hkv = k.shape[1], k.shape[2]
    out = torch.zeros(B, Tq, Hq, D, dtype=torch.float64)
    for b in range(B):
        for h in range(Hq):
            hk = h // (Hq // Hkv)
            for i in range(Tq):
                s = []
                idx = []
                for j in range(Tk):
                    ok = True
                    if ks is not None and j < ks[b]:
                        ok = False
                    if ke is not None and j >= ke[b]:
                        ok = False
                    if causal and j > i + off:
                        ok = False
                    if causal and window and j <= i + off - window:
                        ok = False
                    if ok:
                        s.append(float((q[b, i, h].double() * k[b, j, hk].double()).sum()) * scale)
                        idx.append(j)
                if not s:
                    continue
                p = torch.softmax(torch.tensor(s, dtype=torch.float64), 0)
                out[b, i, h] = sum(p[n] * v[b, idx[n], hk].double() for n in range(len(idx)))
    return out


@pytest.mark.parametrize("causal,off,window,pad", [(True, 0, 0, None), (True, 3, 0, None), (True, 0, 4, None),
                                                   (True, 0, 0, "left"), (False, 0, 0, "right")])
def test_ref_attention_matches_naive(causal, off, window, pad):
    torch.manual_seed(0)
    B, Tq, Hq, Hkv, D = 2, 7, 4, 2, 8
    Tk = Tq + off
    q, k, v = torch.randn(B, Tq, Hq, D), torch.randn(B, Tk, Hkv, D), torch.randn(B, Tk, Hkv, D)
    ks = ke = None
    if pad == "left":
        ks = torch.tensor([0, 3])
    if pad == "right":
        ke = torch.tensor([Tk, 4])
    o = ref_attention(q, k, v, 0.3, causal, off, window, ks, ke)
    n = _naive_attention(q, k, v, 0.3, causal, off, window, ks, ke)
    assert torch.allclose(o.double(), n, atol=1e-5)


def test_rope_rotate_half_and_partial():
    cache = RotaryCache(8, 10000.0, 32)
    x = torch.randn(1, 5, 2, 12)
    pos = torch.arange(5).unsqueeze(0)
    y = ops.attention.apply_rope(x, cache, pos)
    # explicit HF rotate_half formula on the first 8 dims, pass-through on the rest
    inv = 1.0 / (10000.0 ** (torch.arange(0, 8, 2, dtype=torch.float64) / 8))
    fr = torch.outer(torch.arange(5, dtype=torch.float64), inv)
    emb = torch.cat([fr, fr], -1)
    cos, sin = emb.cos().float()[None, :, None], emb.sin().float()[None, :, None]
    xr = x[..., :8]
    rot = torch.cat([-xr[..., 4:], xr[..., :4]], -1)
    ref = xr * cos + rot * sin
    assert torch.allclose(y[..., :8], ref, atol=1e-5)
    assert torch.equal(y[..., 8:], x[..., 8:])


def test_norms_match_torch():
    x = torch.randn(6, 32)
    r = torch.randn(6, 32)
    w = torch.rand(32) + 0.5
    b = torch.randn(32)
    y, s = ops.add_norm(x, r, w, None, 1e-6, True)
    s_ref = x + r
    y_ref = s_ref * torch.rsqrt(s_ref.pow(2).mean(-1, keepdim=True) + 1e-6) * w
    assert torch.allclose(s, s_ref) and torch.allclose(y, y_ref, atol=1e-5)
    y2, _ = ops.add_norm(x, None, w, b, 1e-5, False)
    assert torch.allclose(y2, F.layer_norm(x, (32,), w, b, 1e-5), atol=1e-5)


def test_linear_add_grads_without_main_grad():
    """ops.linear_add (the residual add inside the projection GEMM) must be differentiable on
    plain .grad weights too: its GPU custom op has no autograd kernel of its own."""
    x = torch.randn(5, 8, requires_grad=True)
    w = torch.randn(6, 8, requires_grad=True)
    r = torch.randn(5, 6, requires_grad=True)
    y = ops.linear_add(x, w, r)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    assert torch.allclose(y, r + x @ w.t(), atol=1e-5)
    assert torch.allclose(x.grad, g @ w, atol=1e-5)
    assert torch.allclose(w.grad, g.t() @ x, atol=1e-5)
    assert torch.allclose(r.grad, g)


def test_linear_logprob_matches_compute_logprobs():
    """Reference compute_logprobs (train_dpo.py:31-39) on explicit logits."""
    torch.manual_seed(1)
    S, T, H, V = 3, 9, 16, 40
    h = torch.randn(S, T, H)
    W = torch.randn(V, H)
    ids = torch.randint(0, V, (S, T))
    mask = torch.ones(S, T, dtype=torch.long)
    mask[1, 6:] = 0
    mine = ops.sequence_logprob(h, W, ids, mask, "mean")
    logits = (h @ W.t())[:, :-1]
    lab = ids[:, 1:]
    m = mask[:, 1:]
    lp = torch.log_softmax(logits, -1).gather(2, lab.unsqueeze(-1)).squeeze(-1)
    ref = (lp * m).sum(1) / m.sum(1).clamp(min=1)
    assert torch.allclose(mine, ref, atol=1e-5)
    summed = ops.sequence_logprob(h, W, ids, mask, "sum")
    assert torch.allclose(summed, (lp * m).sum(1), atol=1e-4)


def test_token_nll_matches_hf_causal_lm_loss():
    torch.manual_seed(2)
    S, T, H, V = 2, 8, 8, 30
    h = torch.randn(S, T, H)
    W = torch.randn(V, H)
    labels = torch.randint(0, V, (S, T))
    labels[0, :3] = -100
    mine = ops.token_nll(h, W, labels)
    logits = h @ W.t()
    ref = F.cross_entropy(logits[:, :-1].reshape(-1, V), labels[:, 1:].reshape(-1), ignore_index=-100)
    assert torch.allclose(mine, ref, atol=1e-5)


def test_dpo_loss_formula():
    pc, pr, rc, rr = torch.randn(5), torch.randn(5), torch.randn(5), torch.randn(5)
    loss, m = ops.dpo_loss(pc, pr, rc, rr, beta=0.2)
    ref = -F.logsigmoid(0.2 * ((pc - pr) - (rc - rr))).mean()
    assert torch.allclose(loss, ref, atol=1e-6)
    assert torch.allclose(m["rewards/accuracy"], ((pc - rc) > (pr - rr)).float().mean())


def test_pairwise_and_reinforce_kl_formulas():
    sc, sr = torch.randn(4), torch.randn(4)
    assert torch.allclose(ops.pairwise_loss(sc, sr), -F.logsigmoid(sc - sr).mean())
    lp = torch.randn(6, requires_grad=True)
    lr, r = torch.randn(6), torch.randn(6)
    loss, kl, adv = ops.kl_penalty_pg(lp, lr, r, 0.1)
    # literal reference train_rlhf.py:149-153
    kl_ref = lp - lr
    rewards = r - 0.1 * kl_ref
    adv_ref = rewards - rewards.mean()
    loss_ref = -(adv_ref.detach() * lp).mean()
    assert torch.allclose(loss, loss_ref) and torch.allclose(kl, kl_ref.mean())
    g1, = torch.autograd.grad(loss, lp)
    g2, = torch.autograd.grad(loss_ref, lp)
    assert torch.allclose(g1, g2)


def test_ensemble_kl_matches_reference_formula():
    s = torch.randn(5, 11)
    t = torch.randn(3, 5, 11)
    mine = ops.ensemble_kl(s, t)
    logq = F.log_softmax(s, -1)
    pbar = torch.stack([F.softmax(t[k], -1) for k in range(3)]).mean(0)
    assert torch.allclose(mine, F.kl_div(logq, pbar, reduction="none").sum(-1), atol=1e-6)


def test_adamw_update_matches_torch_adamw():
    torch.manual_seed(3)
    p0 = torch.randn(64)
    g = torch.randn(64)
    p = p0.clone()
    m, v = torch.zeros(64), torch.zeros(64)
    master = p.clone()
    for step in (1, 2, 3):
        adamw_update(None, master, g, m, v, 1e-2, 0.9, 0.95, 1e-8, 0.1, step)
    ref = p0.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for _ in range(3):
        ref.grad = g.clone()
        opt.step()
    assert torch.allclose(master, ref.detach(), atol=1e-6)


def test_clip_coefficient_matches_clip_grad_norm():
    g = torch.randn(100) * 3
    out = torch.zeros(1)
    grad_sumsq(g, out)
    norm, coef = clip_coefficient(out, 1.0)
    p = torch.nn.Parameter(torch.zeros(100))
    p.grad = g.clone()
    tn = torch.nn.utils.clip_grad_norm_([p], 1.0)
    assert torch.allclose(norm, tn, atol=1e-4)
    assert torch.allclose(g * coef, p.grad, atol=1e-5)


def test_gae_matches_per_sequence_loop():
    from distributed_llm_alignment_amd.ops import gae

    torch.manual_seed(0)
    S, T, gamma, lam = 3, 37, 0.99, 0.9
    r, v = torch.randn(S, T), torch.randn(S, T)
    m = torch.zeros(S, T)
    m[0, 5:30] = 1
    m[1, :] = 1
    m[2, 10:11] = 1
    adv, ret = gae(r, v, m, gamma, lam)
    for s in range(S):
        a_next = 0.0
        for t in range(T - 1, -1, -1):
            mn = m[s, t + 1].item() if t + 1 < T else 0.0
            vn = v[s, t + 1].item() if t + 1 < T else 0.0
            delta = r[s, t].item() + gamma * mn * vn - v[s, t].item()
            a = m[s, t].item() * (delta + gamma * lam * mn * a_next)
            assert abs(adv[s, t].item() - a) < 1e-4
            a_next = a
    assert torch.allclose(ret, adv + v)


def test_ppo_losses_match_clipped_formulas():
    from distributed_llm_alignment_amd.ops import ppo_policy_loss, ppo_value_loss

    torch.manual_seed(1)
    N = 64
    lp = torch.randn(N, dtype=torch.float64).mul(0.3).requires_grad_()
    old = lp.detach() + torch.randn(N, dtype=torch.float64) * 0.3
    adv, m = torch.randn(N, dtype=torch.float64), (torch.rand(N) > 0.3).double()
    loss, met = ppo_policy_loss(lp, old, adv, m, 0.2)
    loss.backward()
    rho = torch.exp(lp.detach().float() - old.float())
    per = torch.maximum(-adv.float() * rho, -adv.float() * rho.clamp(0.8, 1.2))
    assert abs(loss.item() - ((per * m.float()).sum() / m.sum()).item()) < 1e-5
    unclipped = (-adv.float() * rho) >= (-adv.float() * rho.clamp(0.8, 1.2))
    g = torch.where(unclipped, -adv.float() * rho, torch.zeros_like(rho)) * m.float() / m.sum()
    assert torch.allclose(lp.grad.float(), g, atol=1e-5)
    v = torch.randn(N).requires_grad_()
    ov, R = v.detach() + torch.randn(N) * 0.5, torch.randn(N)
    vl = ppo_value_loss(v, ov, R, m.float(), 0.2)
    vc = ov + (v.detach() - ov).clamp(-0.2, 0.2)
    ref = 0.5 * (torch.maximum((v.detach() - R) ** 2, (vc - R) ** 2) * m.float()).sum() / m.sum()
    assert abs(vl.item() - ref.item()) < 1e-5


def test_chunked_ensemble_kl_matches_unchunked():
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.objectives import chunked_ensemble_kl

    cfg = get_config("tiny-llama")
    st = build_model(cfg, device="cpu", seed=0)
    ts = [build_model(cfg, device="cpu", seed=s).requires_grad_(False) for s in (1, 2)]
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (3, 21), generator=g)
    mask = torch.ones_like(ids)
    outs = []
    for chunk in (10_000, 16):
        st.zero_grad(set_to_none=True)
        hs = st(ids, mask).reshape(63, -1)
        with torch.no_grad():
            th = [t(ids, mask).reshape(63, -1) for t in ts]
        kl = chunked_ensemble_kl(st, ts, hs, th, chunk=chunk)
        kl.sum().backward()
        outs.append((kl.detach(), [p.grad.clone() for p in st.parameters()]))
    (k1, g1), (k2, g2) = outs
    assert torch.allclose(k1, k2, atol=1e-6)
    for a, b in zip(g1, g2):
        assert torch.allclose(a, b, atol=1e-5, rtol=1e-4)
