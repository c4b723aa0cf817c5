"""CPU tier, multi-process: gloo world_size=2.

  * DP (ZeRO-0 all-reduce and ZeRO-1 reduce-scatter) gives the same update as one process on
    the concatenated batch;
  * gradient accumulation with no_sync == one big batch;
  * checkpoint save -> resume reproduces the next step exactly.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from distributed_llm_alignment_amd.parallel.dist import destroy, init_distributed

        init_distributed(backend="gloo", device="cpu")
        res = _to_numpy(fn(rank, world, *args))
        q.put((rank, "ok", res))
        destroy()
    except Exception as e:  # report to parent
        import traceback

        q.put((rank, "err", traceback.format_exc()))


def _to_numpy(x):
    # tensors cross the queue by value (shared-memory handles die with the child process)
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    if isinstance(x, dict):
        return {k: _to_numpy(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_numpy(v) for v in x)
    return x


def _to_torch(x):
    import numpy as np

    if isinstance(x, np.ndarray):
        return torch.from_numpy(x)
    if isinstance(x, dict):
        return {k: _to_torch(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_torch(v) for v in x)
    return x


def run_ranks(fn, world=2, args=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        rank, status, res = q.get(timeout=300)
        if status != "ok":
            raise AssertionError(f"rank {rank} failed:\n{res}")
        out[rank] = _to_torch(res)
    for p in procs:
        p.join(60)
    return out


def _train_dp(rank, world, zero, accum):
    import torch

    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.objectives import dpo_step_loss
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine

    cfg = get_config("tiny-llama")
    pol = build_model(cfg, device="cpu", seed=0)
    ref = build_model(cfg, device="cpu", seed=0).requires_grad_(False)
    eng = DataParallelEngine(pol, lr=1e-2, weight_decay=0.01, max_grad_norm=1.0, zero_stage=zero,
                             bucket_mb=0.05)
    g = torch.Generator().manual_seed(123)
    full = [synthetic_preference_batch(4, 16, cfg.vocab_size, generator=g) for _ in range(accum)]
    for a in range(accum):
        b = full[a]
        per = 4 // world
        mine = {s: {k: v[rank * per:(rank + 1) * per] for k, v in b[s].items()} for s in b}
        ctxm = eng.no_sync() if a < accum - 1 else _Null()
        with ctxm:
            loss, _ = dpo_step_loss(pol, ref, mine, beta=0.1)
            (loss / accum).backward()
    eng.step()
    return {n: p.detach().clone() for n, p in pol.named_parameters()}, len(eng.buckets)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _single(accum):
    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.objectives import dpo_step_loss
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine

    cfg = get_config("tiny-llama")
    pol = build_model(cfg, device="cpu", seed=0)
    ref = build_model(cfg, device="cpu", seed=0).requires_grad_(False)
    eng = DataParallelEngine(pol, lr=1e-2, weight_decay=0.01, max_grad_norm=1.0)
    g = torch.Generator().manual_seed(123)
    full = [synthetic_preference_batch(4, 16, cfg.vocab_size, generator=g) for _ in range(accum)]
    for a in range(accum):
        # DP mean over ranks == mean of the two halves' means
        for half in range(2):
            mine = {s: {k: v[half * 2:(half + 1) * 2] for k, v in full[a][s].items()} for s in full[a]}
            loss, _ = dpo_step_loss(pol, ref, mine, beta=0.1)
            (loss / (2 * accum)).backward()
    eng.step()
    return {n: p.detach().clone() for n, p in pol.named_parameters()}


@pytest.mark.parametrize("zero", [0, 1])
@pytest.mark.parametrize("accum", [1, 2])
def test_dp_matches_single_process(zero, accum):
    res = run_ranks(_train_dp, 2, (zero, accum))
    ref = _single(accum)
    (p0, nb), (p1, _) = res[0], res[1]
    assert nb > 1, "test must exercise several buckets"
    for n in ref:
        assert torch.allclose(p0[n], p1[n], atol=0, rtol=0), f"ranks diverged on {n}"
        assert torch.allclose(p0[n], ref[n], atol=2e-5), f"{n}: {(p0[n] - ref[n]).abs().max()}"


def _ckpt_resume(rank, world, d):
    import torch

    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.objectives import dpo_step_loss
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine
    from distributed_llm_alignment_amd.utils.checkpoint import load_state, save_state

    cfg = get_config("tiny-llama")

    def make():
        pol = build_model(cfg, device="cpu", seed=0)
        ref = build_model(cfg, device="cpu", seed=0).requires_grad_(False)
        return pol, ref, DataParallelEngine(pol, lr=1e-2, weight_decay=0.0, zero_stage=1, bucket_mb=0.05)

    g = torch.Generator().manual_seed(7 + rank)
    batches = [synthetic_preference_batch(2, 16, cfg.vocab_size, generator=g) for _ in range(3)]
    pol, ref, eng = make()
    losses = []
    for i, b in enumerate(batches):
        if i == 2:
            save_state(d, [pol, ref], eng, None, step=2)
        loss, _ = dpo_step_loss(pol, ref, b)
        loss.backward()
        eng.step()
        losses.append(loss.item())
    pol2, ref2, eng2 = make()
    step = load_state(d, [pol2, ref2], eng2)
    loss, _ = dpo_step_loss(pol2, ref2, batches[2])
    loss.backward()
    eng2.step()
    same = all(torch.equal(a, b) for a, b in zip(pol.parameters(), pol2.parameters()))
    return step, losses[2], loss.item(), same


def test_checkpoint_resume_exact_zero1():
    d = tempfile.mkdtemp()
    res = run_ranks(_ckpt_resume, 2, (os.path.join(d, "step_2"),))
    for r in (0, 1):
        step, l_orig, l_res, same = res[r]
        assert step == 2
        assert l_orig == pytest.approx(l_res, abs=1e-6)
        assert same
    files = set(os.listdir(os.path.join(d, "step_2")))
    for f in ("model.safetensors", "model_1.safetensors", "optimizer.bin", "random_states_0.pkl",
              "random_states_1.pkl", "optimizer_shard_0.pt", "optimizer_shard_1.pt"):
        assert f in files, f
