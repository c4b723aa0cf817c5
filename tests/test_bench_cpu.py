"""bench.py launch contract on the host: `--gpus N` must really run N ranks (gloo here, RCCL on
the GPU node), and a request for more GPUs than are visible must fail instead of silently timing
one (VERDICT r1 "next round" #1; reference launch contract config/accelerate_config.yaml:12)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                          env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                          timeout=timeout)


def _record(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout  # exactly one JSON line, from rank 0 only
    return json.loads(lines[0])


def test_bench_spawns_n_gloo_ranks():
    p = _run(["--gpus", "2", "--device", "cpu", "--model", "tiny-llama", "--steps", "3",
              "--warmup", "1", "--seq-len", "64", "--micro-pairs", "2", "--accum", "2"])
    assert p.returncode == 0, p.stderr[-3000:]
    rec = _record(p.stdout)
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["config"]["backend"] == "gloo"
    assert rec["config"]["parallelism"].startswith("dp2")
    assert rec["config"]["global_batch"] == 2 * 2 * 2  # micro x accum x dp
    assert rec["value"] > 0 and rec["ms_per_step"] > 0


def test_bench_refuses_more_gpus_than_visible():
    # no GPU in the container: asking for GPUs must exit non-zero before any rank starts
    p = _run(["--gpus", "2", "--model", "tiny-llama", "--steps", "1", "--warmup", "0"],
             env_extra={"HIP_VISIBLE_DEVICES": ""} if not _has_gpu() else {"HIP_VISIBLE_DEVICES": "0"})
    assert p.returncode != 0
    assert "refusing" in p.stderr or "GPU" in p.stderr


def test_bench_world_mismatch_is_an_error():
    p = _run(["--gpus", "2", "--device", "cpu", "--model", "tiny-llama", "--steps", "1"],
             env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr


def _has_gpu():
    import torch

    return torch.cuda.device_count() > 0


def test_bench_rank_failure_ends_the_whole_run_fast():
    """One rank dying mid-step (no cleanup) must make the whole command exit non-zero quickly:
    torchrun tears down the surviving rank, which is otherwise blocked in a collective."""
    import time

    t0 = time.perf_counter()
    p = _run(["--gpus", "2", "--device", "cpu", "--model", "tiny-llama", "--steps", "50",
              "--warmup", "1", "--seq-len", "64", "--micro-pairs", "2", "--accum", "2"],
             env_extra={"DLA_BENCH_FAIL_RANK": "1", "DLA_BENCH_FAIL_STEP": "2"}, timeout=240)
    dt = time.perf_counter() - t0
    assert p.returncode != 0
    assert "injected failure on rank 1" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert dt < 90, dt  # includes two interpreter + torch start-ups


def test_bench_preflight_line_per_rank():
    p = _run(["--gpus", "2", "--device", "cpu", "--model", "tiny-llama", "--steps", "1",
              "--warmup", "0", "--seq-len", "64", "--micro-pairs", "2", "--accum", "1"])
    assert p.returncode == 0, p.stderr[-3000:]
    import re

    ranks = sorted(int(m) for m in re.findall(r"\[preflight\] rank (\d+)/2 .*?all_reduce16MB ok", p.stderr))
    assert ranks == [0, 1], p.stderr[-2000:]


def test_launcher_counts_gpus_without_hip(monkeypatch):
    import importlib.util

    spec = importlib.util.spec_from_file_location("benchmod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2")
    assert mod._visible_list(8) == 3
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "")
    assert mod._visible_list(8) == 0
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    assert mod._visible_list(4) == 4
    import torch

    n = mod.visible_gpu_count()  # sysfs here (or the child-process count): never HIP in-process
    assert n >= 0
    assert not torch.cuda.is_initialized()


def test_bench_records_collective_bandwidth():
    """Multi-rank result lines carry the run's own collective bus bandwidth (`config.rccl`,
    measured before the timed window; on the GPU node RCCL all-reduce and reduce-scatter over
    xGMI). Here on gloo: the all-reduce is measured; gloo's missing reduce-scatter is skipped
    without failing the run."""
    p = _run(["--gpus", "2", "--device", "cpu", "--model", "tiny-llama", "--steps", "1",
              "--warmup", "0", "--seq-len", "64", "--micro-pairs", "2", "--accum", "1"],
             {"DLA_BENCH_COLLBW": "1", "DLA_BENCH_COLLBW_MB": "2"})
    assert p.returncode == 0, p.stderr[-3000:]
    rec = _record(p.stdout)
    bw = rec["config"]["rccl"]
    assert bw["allreduce_2MB_busbw_GBps"] > 0, bw


import pytest  # noqa: E402


@pytest.mark.parametrize("flags,mesh,gpus", [
    (["--tp-shape", "2"], "tp2", 2),
    (["--tp-shape", "2", "--tp-seq"], "tp2", 2),
    (["--zero", "3", "--fsdp-shape", "2"], "fsdp2", 2),
    (["--zero", "3", "--fsdp-shape", "2", "--tp-shape", "2"], "fsdp2xtp2", 4),
    (["--model", "tiny-mixtral", "--ep-shape", "2", "--edp-shape", "2"], "ep2xedp2", 4),
])
def test_bench_shape_meshes_run_one_rank(flags, mesh, gpus):
    """One rank of an FSDP x TP / EP x EDP mesh on one device (parallel.collectives.ShapeGroup
    stand-ins): the step runs, the loss is finite and the record carries the mesh's per-rank
    collective bytes (profiles/r5_70b_meshes.md)."""
    args = ["--device", "cpu", "--model", "tiny-llama", "--steps", "1", "--warmup", "1",
            "--seq-len", "64", "--micro-pairs", "2", "--accum", "2"]
    if "--model" in flags:
        i = args.index("--model")
        del args[i:i + 2]
    p = _run(args + flags)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = _record(p.stdout)
    shape = rec["config"]["shape"]
    assert shape["mesh"] == mesh and shape["job_gpus"] == gpus
    assert rec["config"]["final_loss"] == rec["config"]["final_loss"]  # not NaN
    if "--tp-shape" in flags:
        assert "tp_allreduce" in shape["comm_gb_per_step_per_rank"]


def test_shape_group_collectives():
    import torch

    from distributed_llm_alignment_amd.parallel import collectives as coll

    g = coll.ShapeGroup(4)
    x = torch.arange(6.0)
    out = torch.empty(24)
    coll.all_gather_into_tensor(out, x, group=g)
    assert torch.equal(out.view(4, 6), x.expand(4, 6))
    rs = torch.empty(6)
    assert coll.reduce_scatter_tensor(rs, out, group=g, async_op=True).wait()
    assert torch.equal(rs, x)  # this rank's slot, not a sum: values stay at one rank's scale
    y = x.clone()
    coll.all_reduce(y, group=g)
    assert torch.equal(y, x) and coll.world_size(g) == 4 and coll.rank(g) == 0
