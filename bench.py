#!/usr/bin/env python
"""Headline benchmark: Llama-3-8B DPO preference-pairs/s (whole job), BASELINE.json config 2.

One process per GPU (torchrun / torch.distributed.run launches N ranks over RCCL). Each rank:
policy (trainable, bf16 weights, fp32 master + Adam moments, ZeRO-1 sharded across ranks) and a
frozen reference model co-resident on its MI355X; every optimizer step consumes
`--micro-pairs x --accum` synthetic preference pairs of `--seq-len` tokens per side on each rank
(weak scaling). The timed region is K full optimizer steps: policy fwd+bwd on chosen+rejected,
reference fwd, fused DPO loss, bucketed RCCL reduce-scatter overlapped with backward, clip,
fused AdamW, all-gather. Data: synthetic token ids, random-init weights (no network).

    python bench.py [--gpus N] [--steps K] [--warmup W]

Launch contract: under torchrun (WORLD_SIZE set) every process is one rank and the world size
must equal --gpus. Invoked bare with --gpus N > 1, this process is only a launcher: it never
initialises HIP (counting devices does not), starts `torch.distributed.run` with N ranks on
127.0.0.1 as a CHILD process and exits with its return code (reference launch contract:
config/accelerate_config.yaml:12, 8 processes on one node).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch


HF_STACK_PAIRS_PER_S_1GPU = 5.2648  # BASELINE.md, measured on MI355X
PEAK_DENSE_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA peak (no sparsity)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--device", choices=("auto", "cpu"), default="auto",
                    help="cpu: gloo ranks on the host (plumbing test of the launch path only)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--micro-pairs", type=int, default=None,
                    help="pairs per micro-batch (default 4; 2 with --ep-shape, whose capacity-padded "
                         "expert activations do not fit 4 at full depth)")
    ap.add_argument("--accum", type=int, default=None,
                    help="micro-batches per step (default: 16 pairs per step in total)")
    ap.add_argument("--beta", type=float, default=0.1)
    ap.add_argument("--zero", type=int, default=None)
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree (dp = gpus / tp)")
    ap.add_argument("--tp-seq", action="store_true",
                    help="Megatron sequence parallel inside the TP group (reduce-scatter/all-gather)")
    ap.add_argument("--ep", type=int, default=1, help="expert-parallel degree for MoE models")
    ap.add_argument("--ep-capacity", type=float, default=None,
                    help="EP dispatch capacity factor (sync-free fixed blocks); 0 = exact, host splits "
                         "(default 2.0; 1.25 with --ep-shape)")
    ap.add_argument("--sp", type=int, default=1, help="Ulysses sequence-parallel degree (long context)")
    ap.add_argument("--fp8", action="store_true", help="MoE: e4m3 expert GEMMs in the forward")
    ap.add_argument("--grad-ckpt", nargs="?", const="full", default=None, choices=("full", "mlp", "attention"),
                    help="activation recompute on the policy: full layers (bare flag) or selective")
    ap.add_argument("--bucket-mb", type=float, default=256.0)
    ap.add_argument("--ref-stream", type=int, default=0,
                    help="1: frozen reference forward on a second HIP stream, overlapping the policy "
                         "(measured 1.2 %% slower on 1x MI355X: the GEMMs are power-bound, so the "
                         "two streams only contend)")
    ap.add_argument("--profile-dir", default=None, help="write a torch.profiler trace of 1 step")
    ap.add_argument("--tp-shape", type=int, default=1,
                    help="debug: time ONE tensor-parallel rank of a TP=N group at world 1: the full "
                         "model built on the meta device, TP-sharded for rank 0 of a "
                         "parallel.collectives.ShapeGroup(N) and materialised, the overlapped TP layers "
                         "(token-chunked GEMMs, vocab-parallel log-prob) with local stand-in collectives")
    ap.add_argument("--fsdp-shape", type=int, default=1,
                    help="debug (with --zero 3): time ONE rank of an N-way ZeRO-3 / FSDP group at "
                         "world 1 (1/N shards, per-unit gathers / reduce-scatters as local stand-ins); "
                         "with --tp-shape M: one rank of an N x M (FSDP x TP) mesh")
    ap.add_argument("--ep-shape", type=int, default=1,
                    help="debug: time ONE expert-parallel rank of an N-GPU MoE job at world 1: E/N "
                         "local experts per layer, the capacity-padded sync-free dispatch with the "
                         "all-to-alls as local copies, ZeRO-1 optimizer state of one of N ranks")
    ap.add_argument("--ep-hot", action="store_true",
                    help="debug (with --ep-shape = num_experts): the timed rank hosts a HOT expert, "
                         "every source sending its full capacity (ep-capacity x the balanced rows; "
                         "the rows past the expected ones run on the overflow grouped kernels)")
    ap.add_argument("--edp-shape", type=int, default=1,
                    help="debug (with --ep-shape N): the job has M expert-data-parallel replicas of "
                         "each EP group (N x M GPUs): dense ZeRO-1 state over N*M ranks, expert "
                         "optimizer state over the M replicas")
    ap.add_argument("--sharded-init", choices=("auto", "on", "off"), default="auto",
                    help="build on the meta device and materialise only this rank's TP / FSDP "
                         "shards (auto: with --tp > 1 or --zero 3)")
    ap.add_argument("--ref-fp8", action="store_true", default=os.environ.get("DLA_REF_FP8") == "1",
                    help="the frozen reference's layer GEMMs on e4m3 weights + activations (row scales, "
                         "hipBLASLt fp8); an opt-in configuration, not the bf16 headline")
    ap.add_argument("--force-pg", action="store_true",
                    help="one GPU: create a real ONE-rank RCCL process group before any GPU work and "
                         "run the N-GPU engine path on it (ZeRO-1 bucket hooks, reduce-scatter on "
                         "RCCL's stream during backward, shard AdamW, overlapped all-gather)")
    ap.add_argument("--layers", type=int, default=None, help="debug only: override layer count "
                    "(a reduced model is NOT the benchmark config)")
    a = ap.parse_args(argv)
    if a.edp_shape > 1 and a.ep_shape <= 1:
        ap.error("--edp-shape needs --ep-shape")
    if a.ep_hot and a.ep_shape <= 1:
        ap.error("--ep-hot needs --ep-shape")
    if a.fsdp_shape > 1 and a.zero != 3:
        ap.error("--fsdp-shape needs --zero 3")
    shape = a.ep_shape > 1
    if a.micro_pairs is None:
        a.micro_pairs = 2 if shape else 4
    if a.accum is None:
        a.accum = max(1, 16 // a.micro_pairs)
    if a.ep_capacity is None:
        a.ep_capacity = 1.25 if shape else 2.0
    return a


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _visible_list(n_phys: int):
    """Apply ROCR/HIP/CUDA_VISIBLE_DEVICES (innermost wins the count) to n_phys devices."""
    n = n_phys
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def visible_gpu_count() -> int:
    """GPUs this process could use, WITHOUT initialising HIP in this process (the launcher later
    forks/execs torchrun, which must never happen from a HIP-initialised process): KFD topology
    nodes with SIMDs whose DRM render node exists and is accessible here, narrowed by the
    *_VISIBLE_DEVICES variables. If sysfs cannot be read, a throw-away child process counts."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = os.listdir(root)
    except OSError:
        nodes = None
    if nodes is not None:
        n = 0
        for nd in nodes:
            try:
                with open(os.path.join(root, nd, "properties")) as fh:
                    props = dict(ln.split(None, 1) for ln in fh.read().splitlines() if " " in ln)
            except OSError:
                continue
            if int(props.get("simd_count", "0")) <= 0:
                continue  # CPU node
            minor = props.get("drm_render_minor", "").strip()
            dev = f"/dev/dri/renderD{minor}"
            if minor and os.path.exists(dev) and os.access(dev, os.R_OK | os.W_OK):
                n += 1
        return _visible_list(n)
    code = "import torch; print(torch.cuda.device_count())"
    try:
        out = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE,
                             stderr=subprocess.DEVNULL, text=True, timeout=300)
        return int(out.stdout.strip().splitlines()[-1])
    except Exception:
        return 0


def launch_ranks(args, argv) -> int:
    """Parent-side launcher for `--gpus N` without torchrun. Touches no GPU (device count from
    sysfs or a child process), and the ranks run in a child process tree: torchrun tears every
    rank down as soon as one exits non-zero, and its exit code is returned."""
    if args.device != "cpu":
        n_dev = visible_gpu_count()
        if args.gpus > n_dev:
            print(f"bench.py: --gpus {args.gpus} but only {n_dev} GPU(s) visible; refusing to "
                  f"run fewer ranks than requested", file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def preflight(st, dev) -> None:
    """Per-rank first-contact check before anything is timed (stderr, one line per rank): rank,
    device, RCCL version, world, and a 16 MB all-reduce of known values verified element-wise.
    A wrong sum or a hang (collective timeout) ends the run before the benchmark starts."""
    import torch.distributed as dist

    name = torch.cuda.get_device_name(dev) if dev.type == "cuda" else "cpu"
    try:
        rccl = ".".join(map(str, torch.cuda.nccl.version())) if dev.type == "cuda" else "-"
    except Exception:  # pragma: no cover - version query unsupported
        rccl = "?"
    n = 4 * 1024 * 1024  # 16 MB of fp32
    x = torch.full((n,), float(st.rank + 1), dtype=torch.float32, device=dev)
    t0 = time.perf_counter()
    if st.initialized:
        dist.all_reduce(x)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    want = st.world_size * (st.world_size + 1) / 2
    ok = bool(torch.all(x == want).item())
    sys.stderr.write(f"[preflight] rank {st.rank}/{st.world_size} local {st.local_rank} device {dev} "
                     f"({name}) backend {st.backend or 'single-process'} rccl {rccl} all_reduce16MB "
                     f"{'ok' if ok else 'WRONG'} {dt * 1e3:.1f} ms\n")  # one write: no interleaving
    sys.stderr.flush()
    if not ok:
        raise SystemExit(f"bench.py: preflight all-reduce returned wrong values on rank {st.rank}")


def collective_bandwidth(st, dev, mb: int = 256, iters: int = 5) -> dict:
    """RCCL bus bandwidth over this run's ranks, measured before the timed window: a `mb` MB bf16
    all-reduce and reduce-scatter (the collectives of the DDP / ZeRO-1 gradient sync), 2 warm-up +
    `iters` timed calls each, slowest rank's time (nccl-tests' busbw convention:
    all-reduce algbw x 2(n-1)/n, reduce-scatter algbw x (n-1)/n). Recorded in the result line so a
    multi-GPU run carries its own xGMI evidence."""
    import torch.distributed as dist

    n = st.world_size
    if n < 2 or not st.initialized:
        return {}
    numel = mb * 1024 * 1024 // 2
    x = torch.ones(numel, dtype=torch.bfloat16, device=dev)
    out = torch.empty(numel // n, dtype=torch.bfloat16, device=dev)
    res = {}
    for name, fn, factor in (("allreduce", lambda: dist.all_reduce(x), 2 * (n - 1) / n),
                             ("reduce_scatter", lambda: dist.reduce_scatter_tensor(out, x), (n - 1) / n)):
        try:
            res[f"{name}_{mb}MB_busbw_GBps"] = _time_collective(st, dev, fn, mb, iters, factor)
        except Exception as e:  # informational only: never fails the benchmark (gloo has no RS)
            sys.stderr.write(f"[preflight] {name} bandwidth probe skipped: {e}\n")
    del x, out
    return res


def _time_collective(st, dev, fn, mb: int, iters: int, factor: float) -> float:
    import torch.distributed as dist

    for _ in range(2):
        fn()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dt = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=dev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    return round(mb * 2 ** 20 / float(dt.item()) * factor / 1e9, 1)


def _maybe_fail(step: int, rank: int) -> None:
    """Fault injection for the launcher test: DLA_BENCH_FAIL_RANK / DLA_BENCH_FAIL_STEP make that
    rank die abruptly (no cleanup) at that step; the whole command must still exit non-zero."""
    r = os.environ.get("DLA_BENCH_FAIL_RANK")
    if r is not None and int(r) == rank and step == int(os.environ.get("DLA_BENCH_FAIL_STEP", "0")):
        print(f"bench.py: injected failure on rank {rank} at step {step}", file=sys.stderr, flush=True)
        os._exit(17)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, argv)
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}")
    import distributed_llm_alignment_amd as dla  # noqa: F401  (loads the HIP extension)
    from distributed_llm_alignment_amd.data.synthetic import synthetic_preference_batch
    from distributed_llm_alignment_amd.models import build_model, get_config
    from distributed_llm_alignment_amd.objectives import RefLogpsStream, dpo_step_loss
    from distributed_llm_alignment_amd.ops import _ext
    from distributed_llm_alignment_amd.parallel.data_parallel import DataParallelEngine
    from distributed_llm_alignment_amd.parallel.dist import barrier, init_distributed
    from distributed_llm_alignment_amd.parallel.mesh import build_mesh
    from distributed_llm_alignment_amd.parallel.tensor_parallel import apply_tensor_parallel

    from distributed_llm_alignment_amd.utils.tuning import enable_gemm_tuning

    # a dead peer must end the run in bounded time, not after the 30 min default
    st = init_distributed(device="cpu" if args.device == "cpu" else None,
                          timeout_s=int(os.environ.get("DLA_BENCH_COLLECTIVE_TIMEOUT_S", "300")),
                          force_pg=args.force_pg or None)
    if args.force_pg and not st.forced and st.world_size == 1:
        raise SystemExit("bench.py: --force-pg could not create the one-rank process group")
    dev = st.device
    if st.world_size != args.gpus:
        raise SystemExit(f"bench.py: running {st.world_size} rank(s) for --gpus {args.gpus}")
    if st.world_size > 1:
        import torch.distributed as dist

        want = "gloo" if dev.type == "cpu" else "nccl"  # nccl == RCCL on ROCm
        got = dist.get_backend()
        if got != want or dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: backend {got} world {dist.get_world_size()}, "
                             f"expected {want} x {args.gpus}")
    if args.device != "cpu" and not torch.cuda.is_available():
        raise SystemExit("bench.py: no GPU visible (use --device cpu for the host plumbing run)")
    gemm_mode = "off"
    if dev.type == "cuda":
        _ext.require()
        gemm_mode = enable_gemm_tuning(dev.index)
    coll_bw = {}
    if st.world_size > 1 or st.forced or os.environ.get("DLA_BENCH_PREFLIGHT") == "1":
        preflight(st, dev)
        if dev.type == "cuda" or os.environ.get("DLA_BENCH_COLLBW") == "1":
            coll_bw = collective_bandwidth(st, dev, mb=int(os.environ.get("DLA_BENCH_COLLBW_MB", "256")))
    world = st.world_size
    mesh = build_mesh(tp=args.tp, ep=args.ep, sp=args.sp)
    overrides = {} if args.layers is None else {"num_layers": args.layers}
    from distributed_llm_alignment_amd.parallel.collectives import ShapeGroup

    shape_mode = args.tp_shape > 1 or args.fsdp_shape > 1 or args.ep_shape > 1
    # --tp-shape N with --force-pg: rank 0's TP shards of an N-way group (per-rank GEMM shapes),
    # but the TP collectives run on the real one-rank RCCL communicator (RCCL's stream, its
    # kernels in the trace) instead of a ShapeGroup stand-in
    tp_forced = args.tp_shape > 1 and st.forced
    if shape_mode and (world != 1 or args.tp != 1 or args.ep != 1 or args.sp != 1
                       or (st.forced and (args.fsdp_shape > 1 or args.ep_shape > 1))):
        raise SystemExit("bench.py: the --*-shape modes are one-GPU debug modes (world 1, no --tp/--ep/--sp; "
                         "--force-pg only with --tp-shape)")
    # one rank of a TP group / FSDP group that does not exist: ShapeGroup stand-ins
    if tp_forced:
        import torch.distributed as dist

        tp_group = dist.group.WORLD
    else:
        tp_group = ShapeGroup(args.tp_shape) if args.tp_shape > 1 else mesh.tp_group
    fsdp_group = ShapeGroup(args.fsdp_shape) if args.fsdp_shape > 1 else mesh.dp_group
    cfg = get_config(args.model, **overrides)
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32

    meta = args.sharded_init == "on" or (args.sharded_init == "auto" and (
        args.tp > 1 or args.zero == 3 or args.tp_shape > 1))
    policy = build_model(cfg, device=dev, dtype=dtype, seed=1234, meta=meta)
    ref = build_model(cfg, device=dev, dtype=dtype, seed=1234, meta=meta)
    ref.eval()
    for p in ref.parameters():
        p.requires_grad_(False)
    if args.ref_fp8:
        from distributed_llm_alignment_amd.ops import enable_fp8_inference

        enable_fp8_inference(ref)
    if mesh.tp > 1 or args.tp_shape > 1:
        kw = dict(tp_rank=0, tp_size=args.tp_shape, force=True) if tp_forced else {}
        apply_tensor_parallel(policy, tp_group, sequence_parallel=args.tp_seq, **kw)
        apply_tensor_parallel(ref, tp_group, sequence_parallel=args.tp_seq, **kw)
    if mesh.sp > 1:
        from distributed_llm_alignment_amd.parallel.sequence import apply_sequence_parallel

        apply_sequence_parallel(policy, mesh.sp_group)
        apply_sequence_parallel(ref, mesh.sp_group)
    if mesh.ep > 1:
        from distributed_llm_alignment_amd.parallel.expert import apply_expert_parallel

        apply_expert_parallel(policy, mesh, capacity_factor=args.ep_capacity)
        apply_expert_parallel(ref, mesh, capacity_factor=args.ep_capacity)
    if args.ep_shape > 1:
        if world != 1 or args.ep != 1 or not cfg.is_moe:
            raise SystemExit("bench.py: --ep-shape is a one-GPU debug mode for MoE models (world 1, --ep 1)")
        from distributed_llm_alignment_amd.parallel.expert import apply_expert_parallel

        for m in (policy, ref):
            apply_expert_parallel(m, None, capacity_factor=args.ep_capacity or 2.0, shape_ep=args.ep_shape,
                                  shape_hot=args.ep_hot)
    if cfg.is_moe and args.fp8:
        for m in (policy, ref):
            for layer in m.layers:
                layer.mlp.fp8 = True
    if args.grad_ckpt:
        policy.gradient_checkpointing_enable(args.grad_ckpt)
    if args.zero == 3:  # ZeRO-3 / FSDP: per-layer gather, sharded frozen reference
        from distributed_llm_alignment_amd.parallel.fsdp import FullyShardedEngine, ShardedInference

        engine = FullyShardedEngine(policy, lr=1e-6, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                                    max_grad_norm=1.0, group=fsdp_group, tp_group=tp_group)
        ShardedInference(ref, group=fsdp_group)  # (materialises the meta ref unit by unit)
    else:
        if meta:  # this rank's TP / EP shards only, one parameter at a time
            from distributed_llm_alignment_amd.models.materialize import materialize

            materialize(policy, dev)
            materialize(ref, dev)
        edp_group = (ShapeGroup(args.edp_shape) if args.edp_shape > 1
                     else (mesh.edp_group if mesh.ep > 1 else None))
        engine = DataParallelEngine(policy, lr=1e-6, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                                    max_grad_norm=1.0, zero_stage=args.zero, bucket_mb=args.bucket_mb,
                                    group=mesh.grad_group, tp_group=tp_group,
                                    expert_group=edp_group, sp_size=mesh.sp,
                                    shape_world=args.ep_shape * args.edp_shape)
    policy.train()

    gen = torch.Generator().manual_seed(17 + mesh.dp_rank)  # TP ranks share a batch
    n_batches = 4
    batches = [synthetic_preference_batch(args.micro_pairs, args.seq_len, cfg.vocab_size, device=dev,
                                          generator=gen) for _ in range(n_batches)]
    state = {"i": 0, "loss": None, "step": 0}

    # only when the ref forward issues no collectives (TP / EP / ZeRO-3 gathers would race the
    # policy's on the same communicators from two streams)
    ref_stream = bool(args.ref_stream) and args.tp == 1 and args.ep == 1 and args.sp == 1 and args.zero != 3
    refs = RefLogpsStream(ref, enabled=ref_stream)
    ref_stream = refs.stream is not None

    def train_step():
        # the ref pass of micro-batch a+1 is queued on its own stream before micro-batch a's
        # backward, so it runs alongside the policy backward
        _maybe_fail(state["step"], st.rank)
        state["step"] += 1
        pending = refs.submit(batches[state["i"] % n_batches])
        for a in range(args.accum):
            b = batches[state["i"] % n_batches]
            state["i"] += 1
            ctx = engine.no_sync() if a < args.accum - 1 else _null()
            with ctx:
                loss, _ = dpo_step_loss(policy, ref, b, beta=args.beta, ref_logps=refs.result(pending))
                if a + 1 < args.accum:
                    pending = refs.submit(batches[state["i"] % n_batches])
                (loss / args.accum).backward()
            state["loss"] = loss
        engine.step()

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        train_step()
    sync()
    barrier()
    sync()
    engine.comm_timer.reset()
    t0 = time.perf_counter()
    if args.profile_dir:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
            for _ in range(args.steps):
                train_step()
            sync()
    else:
        for _ in range(args.steps):
            train_step()
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if st.initialized:
        import torch.distributed as dist

        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    elapsed = float(t_max.item())
    # gradient-comm time the step did NOT hide: the compute stream's wait on RCCL at the step
    # boundary (0 without collectives), averaged over the timed steps, max over ranks
    exposed = torch.tensor([engine.comm_timer.total_ms() / args.steps], dtype=torch.float64, device=dev)
    if st.initialized:
        dist.all_reduce(exposed, op=dist.ReduceOp.MAX)
    exposed_ms = float(exposed.item())
    if args.profile_dir and st.rank == 0:
        os.makedirs(args.profile_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(args.profile_dir, "trace.json"))
        with open(os.path.join(args.profile_dir, "kernels.txt"), "w") as fh:
            fh.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
        with open(os.path.join(args.profile_dir, "ops_by_shape.txt"), "w") as fh:
            fh.write(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total",
                                                                         row_limit=100, max_name_column_width=60,
                                                                         max_shapes_column_width=120))

    pairs_per_step = args.micro_pairs * args.accum * mesh.dp
    ms = elapsed / args.steps * 1000.0
    value = pairs_per_step * args.steps / elapsed
    # model FLOPs: policy fwd+bwd (3x) + ref fwd (1x) over 2*seq tokens per pair
    tokens_per_pair = 2 * args.seq_len
    flops_pair = 4 * cfg.flops_per_token(args.seq_len) * tokens_per_pair
    # a TP group of G ranks shares each micro-batch: one rank does 1/G of the replica's FLOPs
    per_replica_gpus = max(1, args.tp_shape) * mesh.tp
    tflops_gpu = value * flops_pair / world / per_replica_gpus / 1e12
    shape_info = None
    if shape_mode:
        from distributed_llm_alignment_amd.parallel.comm_model import dpo_comm_bytes

        g_tp, g_fs, g_ep, g_edp = args.tp_shape, args.fsdp_shape, args.ep_shape, args.edp_shape
        gpus = g_tp * g_fs * g_ep * g_edp
        replicas = gpus // g_tp
        cb = dpo_comm_bytes(cfg, args.seq_len, args.micro_pairs, args.accum, tp=g_tp, fsdp=g_fs,
                            ep=g_ep, edp=g_edp, ep_capacity=args.ep_capacity, tp_seq=args.tp_seq)
        shape_info = {
            "mesh": "x".join(f"{n}{g}" for n, g in (("fsdp", g_fs), ("tp", g_tp), ("ep", g_ep),
                                                      ("edp", g_edp)) if g > 1),
            "job_gpus": gpus, "data_replicas": replicas,
            "job_pairs_per_s_if_comm_hidden": round(value * replicas, 3),
            "peak_gib": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1) if dev.type == "cuda" else None,
            "comm_gb_per_step_per_rank": {k: round(v / 1e9, 2) for k, v in cb.items()},
        }
    if st.rank == 0:
        rec = {
            "metric": "preference-samples/sec (whole node), Llama-3-8B DPO at 1/2/4/8 MI355X" if cfg.name == "llama3-8b"
                      else f"preference-samples/sec (whole node), {cfg.name} DPO",
            "value": round(value, 4),
            "unit": "preference_pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            # BASELINE.md comparison point: the reference's DPO step on stock PyTorch-ROCm + HF
            # (tools/hf_stack_dpo_bench.py, same shapes, 1x MI355X) = 5.2648 pairs/s per GPU,
            # scaled ideally (x N) for N GPUs
            "vs_baseline": round(value / (HF_STACK_PAIRS_PER_S_1GPU * world), 3) if cfg.name == "llama3-8b" else None,
            "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
            "data": "synthetic preference pairs (random token ids), random-init weights",
            "config": {
                "model": (cfg.name if args.layers is None else f"{cfg.name}-L{args.layers}(debug)")
                         + (f"(one rank of a {shape_info['mesh']} mesh, "
                            + ("TP collectives on a one-rank RCCL group" if tp_forced else "local stand-in collectives")
                            + ", debug)" if shape_mode and args.ep_shape <= 1 else "")
                         + (f"(one EP rank of ep{args.ep_shape}: {cfg.num_experts // args.ep_shape} "
                            "local experts/layer, a2a as local copies, debug)" if args.ep_shape > 1 else "")
                         + (f"(hot expert: every source at capacity {args.ep_capacity})" if args.ep_hot else ""),
                "global_batch": pairs_per_step,
                "seq_len": args.seq_len,
                "parallelism": f"dp{mesh.dp}" + (f"-tp{mesh.tp}" if mesh.tp > 1 else "")
                               + (f"-ep{mesh.ep}" if mesh.ep > 1 else "")
                               + (f"-sp{mesh.sp}" if mesh.sp > 1 else "")
                               + (f"-zero{engine.zero}" if mesh.dp * mesh.sp > 1 or engine.zero == 3
                                  or st.forced else "")
                               + ("(one-rank RCCL group, forced comm)" if st.forced else ""),
                "micro_batch_pairs": args.micro_pairs,
                "grad_accum": args.accum,
                "ref_model": "frozen, co-resident" + (", own HIP stream" if ref_stream else "")
                             + (", fp8 layer GEMMs (e4m3 weights + activations, row scales)" if args.ref_fp8 else ""),
                "model_tflops_per_gpu": round(tflops_gpu, 1),
                "mfu": round(tflops_gpu / PEAK_DENSE_BF16_TFLOPS, 4) if dev.type == "cuda" else None,
                "backend": st.backend or "single-process",
                "final_loss": round(float(state["loss"].item()), 5),
                "comm_exposed_ms_per_step": round(exposed_ms, 2),
                **({"shape": shape_info} if shape_info else {}),
                "gemm_selection": "tunableop:" + gemm_mode,
                **({"rccl": coll_bw} if coll_bw else {}),
            },
        }
        print(json.dumps(rec), flush=True)
    if st.initialized:  # orderly teardown: no communicator threads left running at exit
        if hasattr(engine, "wait_params"):
            engine.wait_params()  # the last step's overlapped all-gathers (never waited otherwise)
        barrier()
        from distributed_llm_alignment_amd.parallel.dist import destroy

        destroy()
    return 0


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


if __name__ == "__main__":
    sys.exit(main())
