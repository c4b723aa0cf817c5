"""Collective bandwidth microbenchmark over the process group (RCCL over xGMI on MI355X, gloo on
CPU): all-reduce, reduce-scatter, all-gather and all-to-all at a sweep of message sizes, reporting
algorithm and bus bandwidth (nccl-tests conventions). SURVEY §5.8 #2: checks that bucketed DP /
ZeRO collectives reach multi-link xGMI rates at world sizes 2/4/8 and picks the bucket size.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/comm_bench.py --sizes-mb 16,64,256,1024
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def bus_factor(op: str, n: int) -> float:
    if op == "all_reduce":
        return 2.0 * (n - 1) / n
    return (n - 1) / n  # reduce_scatter, all_gather, all_to_all


def run(op: str, nbytes: int, dev, dtype, iters: int, warmup: int) -> float:
    n = dist.get_world_size()
    numel = max(n, nbytes // torch.tensor([], dtype=dtype).element_size() // n * n)
    x = torch.ones(numel, dtype=dtype, device=dev)
    if op == "all_reduce":
        fn = lambda: dist.all_reduce(x)  # noqa: E731
    elif op == "reduce_scatter":
        y = torch.empty(numel // n, dtype=dtype, device=dev)
        fn = lambda: dist.reduce_scatter_tensor(y, x)  # noqa: E731
    elif op == "all_gather":
        y = torch.empty(numel // n, dtype=dtype, device=dev)
        fn = lambda: dist.all_gather_into_tensor(x, y)  # noqa: E731
    else:
        y = torch.empty_like(x)
        fn = lambda: dist.all_to_all_single(y, x)  # noqa: E731
    for _ in range(warmup):
        fn()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dist.barrier()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = torch.tensor([(time.perf_counter() - t) / iters], dtype=torch.float64)
    if dev.type == "cuda":
        dt = dt.to(dev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    return float(dt.item())


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,16,64,256")
    ap.add_argument("--ops", default="all_reduce,reduce_scatter,all_gather,all_to_all")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--backend", default=None)
    ap.add_argument("--out", default=None, help="rank 0 also writes the rows (JSON lines) here")
    args = ap.parse_args(argv)
    gpu = torch.cuda.is_available() and args.backend != "gloo"
    backend = args.backend or ("nccl" if gpu else "gloo")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if gpu:
        torch.cuda.set_device(local)
    dist.init_process_group(backend)
    dev = torch.device("cuda", local) if gpu else torch.device("cpu")
    dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[args.dtype]
    if not gpu and dtype == torch.bfloat16:
        dtype = torch.float32  # gloo reduces fp32
    n = dist.get_world_size()
    rows = []
    for op in args.ops.split(","):
        for mb in (float(s) for s in args.sizes_mb.split(",")):
            nbytes = int(mb * 2 ** 20)
            dt = run(op, nbytes, dev, dtype, args.iters, args.warmup)
            algbw = nbytes / dt / 1e9
            rows.append({"op": op, "size_mb": mb, "ms": round(dt * 1e3, 3), "algbw_GBps": round(algbw, 2),
                         "busbw_GBps": round(algbw * bus_factor(op, n), 2), "world": n, "backend": backend})
    if dist.get_rank() == 0:
        for r in rows:
            print(json.dumps(r), flush=True)
        if args.out:
            Path(args.out).parent.mkdir(parents=True, exist_ok=True)
            Path(args.out).write_text("".join(json.dumps(r) + "\n" for r in rows))
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
