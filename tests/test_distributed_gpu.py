"""GPU tier, multi-process over RCCL (torch backend "nccl" on ROCm), one rank per MI355X.

Skipped on a box with fewer than 2 GPUs; on an 8-GPU node each test runs world = min(#GPUs, 8)
(TP/SP/EP tests use 2-rank groups inside that world). This is the hardware counterpart of the
gloo tier (tests/test_distributed_cpu.py): same engines, HIP kernels, bf16 weights, RCCL
collectives over xGMI (reference: DDP/NCCL via accelerate, src/training/utils.py:66-75).

  * raw collectives (all-reduce / reduce-scatter / all-gather / all-to-all) are exact;
  * ZeRO-1 DP over N ranks == one rank on the concatenated batch (loss + grad-norm trajectory);
  * ZeRO-3 (FSDP per-layer gather / reduce-scatter) == ZeRO-1;
  * TP=2 sequence log-probs + grads == dense; Ulysses SP=2 == dense; EP=2 == replicated experts;
  * after an overlapped ZeRO-1 step (all-gathers in flight), graph-replayed generation equals
    the eager loop: the eager prefill's module pre-hooks order the replays after the gathers.
"""
import dataclasses
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

# per-test wall budget: a first-contact RCCL hang costs at most this, not the driver's round
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(120, method="thread")]
_INIT_TIMEOUT_S = 90  # collective / rendezvous timeout inside each rank
_RANK_DEADLINE_S = 110  # the parent waits at most this long for ALL ranks of one test


# DLA_RANKS_ON_CPU=N: host dry run of this file's rank logic on N gloo ranks (torch fallbacks
# instead of the HIP kernels) -- used to check the tests themselves without a multi-GPU box
_CPU_RANKS = int(os.environ.get("DLA_RANKS_ON_CPU", "0"))


def _n_gpus():
    return _CPU_RANKS or torch.cuda.device_count()


needs2 = pytest.mark.skipif(_n_gpus() < 2, reason="needs >= 2 GPUs for RCCL multi-rank tests")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    try:
        import torch.distributed as dist

        from distributed_llm_alignment_amd.ops import _ext
        from distributed_llm_alignment_amd.parallel.dist import destroy, init_distributed

        if _CPU_RANKS:
            st = init_distributed(backend="gloo", device="cpu", timeout_s=_INIT_TIMEOUT_S)
        else:
            _ext.require()
            st = init_distributed(timeout_s=_INIT_TIMEOUT_S)
            if world > 1:
                assert dist.get_backend() == "nccl", dist.get_backend()
        res = fn(rank, world, st.device, *args)
        if st.device.type == "cuda":
            torch.cuda.synchronize()
        q.put((rank, "ok", _cpu(res)))
        destroy()
    except Exception:  # report to the parent instead of hanging it
        import traceback

        q.put((rank, "err", traceback.format_exc()))


def _cpu(x):
    if isinstance(x, torch.Tensor):
        return x.detach().float().cpu().numpy()
    if isinstance(x, dict):
        return {k: _cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_cpu(v) for v in x)
    return x


def run_ranks(fn, world, args=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    import time

    deadline = time.monotonic() + _RANK_DEADLINE_S
    try:
        for _ in procs:
            rank, status, res = q.get(timeout=max(1.0, deadline - time.monotonic()))
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{res}")
            out[rank] = res
    finally:
        for p in procs:
            p.join(max(1.0, min(15.0, deadline + 15 - time.monotonic())))
            if p.is_alive():
                p.kill()
    return out


def _world():
    return min(_n_gpus(), 8)


# ------------------------------------------------------------------------------ raw collectives
def _collectives(rank, world, dev):
    import torch.distributed as dist

    n = 1 << 20
    x = torch.full((n,), float(rank + 1), device=dev, dtype=torch.float32)
    dist.all_reduce(x)
    ok_ar = bool((x == world * (world + 1) / 2).all())
    src = torch.arange(world * 1024, device=dev, dtype=torch.float32) + rank
    rs = torch.empty(1024, device=dev)
    dist.reduce_scatter_tensor(rs, src)
    want_rs = (torch.arange(rank * 1024, (rank + 1) * 1024, device=dev, dtype=torch.float32) * world
               + world * (world - 1) / 2)
    ok_rs = bool(torch.equal(rs, want_rs))
    ag = torch.empty(world * 8, device=dev, dtype=torch.bfloat16)
    dist.all_gather_into_tensor(ag, torch.full((8,), float(rank), device=dev, dtype=torch.bfloat16))
    ok_ag = bool(torch.equal(ag.float(), torch.arange(world, device=dev).repeat_interleave(8).float()))
    a2a_in = torch.arange(world, device=dev, dtype=torch.float32) + 100 * rank
    a2a_out = torch.empty_like(a2a_in)
    dist.all_to_all_single(a2a_out, a2a_in)
    ok_a2a = bool(torch.equal(a2a_out, torch.arange(world, device=dev).float() * 100 + rank))
    return ok_ar, ok_rs, ok_ag, ok_a2a


@needs2
def test_rccl_collectives_exact():
    res = run_ranks(_collectives, _world())
    for r, oks in res.items():
        assert all(oks), (r, oks)


# ------------------------------------------------------------------------------ DP / ZeRO
def _cfg():
    from distributed_llm_alignment_amd.models import get_config

    return get_config("tiny-llama-d128")


def _dp_run(rank, world, dev, mode, rows_total, steps):
    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.models import build_model
    from distributed_llm_alignment_amd.objectives import dpo_step_loss
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine
    from distributed_llm_alignment_amd.parallel.fsdp import FullyShardedEngine, ShardedInference

    cfg = _cfg()
    pol = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    ref = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0).requires_grad_(False)
    kw = dict(lr=1e-3, weight_decay=0.01, max_grad_norm=1.0)
    if mode == "fsdp":
        eng = FullyShardedEngine(pol, **kw)
        ShardedInference(ref)
    else:
        eng = DataParallelEngine(pol, zero_stage=1 if world > 1 else 0, bucket_mb=1.0, **kw)
    g = torch.Generator().manual_seed(7)
    full = synthetic_preference_batch(rows_total, 128, cfg.vocab_size, generator=g, min_len=100)
    per = rows_total // world
    mine = {s: {k: v[rank * per:(rank + 1) * per].to(dev) for k, v in full[s].items()} for s in full}
    losses, norms = [], []
    for _ in range(steps):
        loss, _ = dpo_step_loss(pol, ref, mine, beta=0.1)
        loss.backward()
        norms.append(float(eng.step()))
        losses.append(float(loss.detach()))
    # mean over ranks of the next-step loss == loss of the full batch on one rank
    nxt = dpo_step_loss(pol, ref, mine, beta=0.1)[0].detach().reshape(1)
    if world > 1:
        import torch.distributed as dist

        dist.all_reduce(nxt)
        nxt /= world
    cks = None if mode == "fsdp" else torch.stack([p.detach().float().sum() for p in pol.parameters()])
    return norms, float(nxt), cks


@needs2
def test_rccl_zero1_matches_single_rank():
    W = _world()
    multi = run_ranks(_dp_run, W, ("zero1", 2 * W, 3))
    single = run_ranks(_dp_run, 1, ("zero1", 2 * W, 3))
    import numpy as np

    for r in range(1, W):  # replicas stay bitwise in sync
        assert np.array_equal(multi[r][2], multi[0][2]), r
    assert multi[0][0] == pytest.approx(single[0][0], rel=3e-2)
    assert multi[0][1] == pytest.approx(single[0][1], abs=2e-2)


@needs2
def test_rccl_fsdp_matches_zero1():
    W = _world()
    a = run_ranks(_dp_run, W, ("zero1", 2 * W, 3))
    b = run_ranks(_dp_run, W, ("fsdp", 2 * W, 3))
    assert a[0][0] == pytest.approx(b[0][0], rel=3e-2)
    assert a[0][1] == pytest.approx(b[0][1], abs=2e-2)


# ------------------------------------------------------------------------------ TP / SP / EP
def _pairs_mesh(kind):
    from distributed_llm_alignment_amd.parallel.mesh import build_mesh

    return build_mesh(**{("tp" if kind == "tpseq" else kind): 2})


def _logprob_vs_dense(rank, world, dev, kind):
    from distributed_llm_alignment_amd.models import build_model, get_config

    cfg = _cfg()
    if kind == "ep":
        cfg = dataclasses.replace(get_config("tiny-mixtral"), hidden_size=256, num_heads=2,
                                  num_kv_heads=1, head_dim=128, intermediate_size=256)
    mesh = _pairs_mesh(kind)
    dense = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    par = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    if kind in ("tp", "tpseq"):
        from distributed_llm_alignment_amd.parallel.tensor_parallel import apply_tensor_parallel

        apply_tensor_parallel(par, mesh.tp_group, sequence_parallel=kind == "tpseq")
    elif kind == "sp":
        from distributed_llm_alignment_amd.parallel.sequence import apply_sequence_parallel

        apply_sequence_parallel(par, mesh.sp_group)
    else:
        from distributed_llm_alignment_amd.parallel.expert import apply_expert_parallel

        apply_expert_parallel(par, mesh)
    g = torch.Generator().manual_seed(3 + (mesh.dp_rank if kind == "ep" else 0))
    ids = torch.randint(3, cfg.vocab_size, (4, 200), generator=g).to(dev)
    mask = torch.ones_like(ids)
    mask[1, 150:] = 0
    mask[2, :20] = 0
    a = dense.sequence_logprob(ids, mask)
    b = par.sequence_logprob(ids, mask)
    a.sum().backward()
    b.sum().backward()
    gn_dense = dense.norm_w.grad.float()
    gn_par = par.norm_w.grad.float().clone()
    if kind == "sp":  # each SP rank holds a partial gradient of the replicated norm weight
        import torch.distributed as dist

        dist.all_reduce(gn_par, group=mesh.sp_group)
    err_g = float((gn_dense - gn_par).abs().max() / (gn_dense.abs().max() + 1e-12))
    return a.float(), b.float(), err_g


@needs2
@pytest.mark.parametrize("kind", ["tp", "tpseq", "sp", "ep"])
def test_rccl_parallel_logprob_matches_dense(kind):
    import numpy as np

    res = run_ranks(_logprob_vs_dense, 2 if kind != "ep" else _world() - _world() % 2, (kind,))
    for r, (a, b, err_g) in res.items():
        assert np.allclose(a, b, atol=3e-2, rtol=1e-2), (r, a, b)
        assert err_g < 5e-2, (r, err_g)


def _tp_fused_mlp(rank, world, dev):
    """The fused Megatron MLP node with overlapped collectives (chunked row-parallel forward,
    async column-parallel input-grad all-reduce behind the weight-grad GEMM) == the dense MLP."""
    import torch.distributed as dist

    from distributed_llm_alignment_amd import ops
    from distributed_llm_alignment_amd.parallel.tensor_parallel import shard_tensor

    if not dist.is_initialized():  # world 1: a one-rank RCCL group still runs the async path
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    group = dist.group.WORLD
    H, F_, M = 256, 512, 264
    g = torch.Generator().manual_seed(1)
    h = (torch.randn(M, H, generator=g) * 0.5).to(dev, torch.bfloat16)
    w_up = (torch.randn(2 * F_, H, generator=g) / H ** 0.5).to(dev, torch.bfloat16)
    w_dn = (torch.randn(H, F_, generator=g) / F_ ** 0.5).to(dev, torch.bfloat16)
    gy = torch.randn(M, H, generator=g).to(dev, torch.bfloat16)
    out = {}
    for name, (wu, wd, grp) in {
        "dense": (w_up, w_dn, None),
        "tp": (shard_tensor(w_up, (0, [F_, F_]), rank, world), shard_tensor(w_dn, (1, [F_]), rank, world), group),
    }.items():
        wu = wu.clone().requires_grad_(True)
        wd = wd.clone().requires_grad_(True)
        for w in (wu, wd):
            w.main_grad = torch.zeros(w.shape, dtype=torch.float32, device=dev)
        x = h.clone().requires_grad_(True)
        assert ops.swiglu_mlp_ok(x, wu, wd)
        y = ops.swiglu_mlp(x, wu, wd, tp_group=grp, chunks=3)
        y.backward(gy)
        torch.cuda.synchronize()
        out[name] = (y.float(), x.grad.float(), wu.main_grad, wd.main_grad)
    d, t = out["dense"], out["tp"]
    err = lambda a, b: float((a - b).norm() / (b.norm() + 1e-12))
    wu_full = shard_tensor(d[2], (0, [F_, F_]), rank, world)
    wd_full = shard_tensor(d[3], (1, [F_]), rank, world)
    return err(t[0], d[0]), err(t[1], d[1]), err(t[2], wu_full), err(t[3], wd_full)


@pytest.mark.parametrize("world", [1, 2])
def test_rccl_tp_fused_mlp_overlapped_collectives(world):
    if world > _n_gpus() or _CPU_RANKS:
        pytest.skip("needs that many GPUs (the fused node is GPU-only)")
    res = run_ranks(_tp_fused_mlp, world)
    for r, errs in res.items():
        assert max(errs) < 2e-2, (r, errs)


# ------------------------------------------------------------------------------ overlap + graphs
def _overlap_then_generate(rank, world, dev):
    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.models import build_model, generate
    from distributed_llm_alignment_amd.models.generation import clear_graph_cache
    from distributed_llm_alignment_amd.objectives import dpo_step_loss
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine

    cfg = _cfg()
    pol = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0)
    ref = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=0).requires_grad_(False)
    eng = DataParallelEngine(pol, lr=1e-2, zero_stage=1, bucket_mb=0.5)
    g = torch.Generator().manual_seed(rank)
    b = synthetic_preference_batch(2, 128, cfg.vocab_size, device=dev, generator=g)
    prompts = torch.randint(3, cfg.vocab_size, (4, 40), generator=torch.Generator().manual_seed(9)).to(dev)
    clear_graph_cache()
    same, last = True, None
    for _ in range(3):  # step 1 captures the decode graph, steps 2-3 replay the cached one
        loss, _ = dpo_step_loss(pol, ref, b)
        loss.backward()
        eng.step()  # ZeRO-1 all-gathers are still in flight when generate() starts
        graph = generate(pol, prompts, max_new_tokens=24, do_sample=False, use_graph=True)
        eng.wait_params()
        eager = generate(pol, prompts, max_new_tokens=24, do_sample=False, use_graph=False)
        same = same and bool(torch.equal(graph, eager))
        last = graph
    clear_graph_cache()
    return same, last


@needs2
def test_rccl_overlapped_allgather_then_graph_decode_is_race_free():
    import numpy as np

    res = run_ranks(_overlap_then_generate, 2)
    for r in res:
        assert res[r][0], f"rank {r}: graph replay after overlapped all-gather != eager"
    assert np.array_equal(res[0][1], res[1][1])  # replicas generate identically


# ------------------------------------------------------------------------------ xGMI bandwidth
@needs2
def test_rccl_bus_bandwidth_recorded():
    """tools/comm_bench.py over all visible GPUs; rows land in gpurun_out/ (copied to profiles/).
    A bus bandwidth floor of 20 GB/s at 64 MB catches a host-staged (non-xGMI) fallback."""
    import json
    import subprocess
    import sys

    if _CPU_RANKS:
        pytest.skip("bandwidth is meaningless on the host dry run")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    W = _world()
    out = os.path.join(root, "gpurun_out", f"rccl_busbw_w{W}.jsonl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={W}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(root, "tools", "comm_bench.py"), "--sizes-mb", "16,64,256", "--out", out]
    p = subprocess.run(cmd, cwd=root, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=100)
    assert p.returncode == 0, p.stdout[-3000:]
    rows = [json.loads(ln) for ln in open(out)]
    assert {r["op"] for r in rows} == {"all_reduce", "reduce_scatter", "all_gather", "all_to_all"}
    for r in rows:
        assert r["world"] == W and r["backend"] == "nccl"
        if r["size_mb"] >= 64:
            assert r["busbw_GBps"] > 20.0, r
