#!/usr/bin/env python
"""One parametrised GPU A/B runner (replaces the round-1/2 one-off `tools/gpu_*.sh` scripts).

Runs, in ONE gpurun call and in this order, stopping at the first failure (no retries, no GPU
step after a fault, abort or time limit):
  1. an optional pytest selection (`--tests`),
  2. `--rounds` interleaved repetitions of every arm of `--cmd` (arms differ only by environment
     variables, e.g. a flag or `DLA_EXT_PATH` of an alternative `_C.so`): box-to-box clock
     variance is larger than most single optimisations, so A and B always run on the same box,
     alternating,
  3. an optional `rocprofv3 --kernel-trace --stats` pass of the first arm (`--prof NAME`).
Every step runs under its own `timeout -k 10`. The last JSON line (or a `--metric-re` match) of
each run is parsed; one JSON record per run goes to `--out` (default gpurun_out/ab.jsonl) and a
summary table (median per arm) is printed. This parent process never touches the GPU.

    python tools/gpu_ab.py --cmd "python -u bench.py --steps 8 --warmup 3" \\
        --arm base: --arm tn:DLA_TN_WGRAD=0 --rounds 2 --tests "tests/test_kernels_gpu.py -k norm"
    python tools/gpu_ab.py --cmd "python -u tools/attn_bench.py --iters 30" \\
        --arm old:DLA_EXT_PATH=$PWD/_C_old.so --arm new: --metric-re "attn.*?([0-9.]+) TFLOP"
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shlex
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FATAL = {124, 134, 137, 139, -6, -9, -11}  # time limit, abort, kill, segfault: stop the GPU work


def _arm(spec: str):
    name, _, env = spec.partition(":")
    kv = {}
    for item in filter(None, (x.strip() for x in env.split(","))):
        k, _, v = item.partition("=")
        kv[k] = os.path.expandvars(v)
    return name or "arm", kv


def _run(cmd, env_extra, timeout_s, log):
    env = dict(os.environ, PYTHONUNBUFFERED="1", **env_extra)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    full = ["timeout", "-k", "10", str(timeout_s), *cmd]
    t0 = time.perf_counter()
    with open(log, "w") as fh:
        rc = subprocess.call(full, cwd=ROOT, env=env, stdout=fh, stderr=subprocess.STDOUT)
    return rc, time.perf_counter() - t0


def _metric(log, rx):
    text = open(log, errors="replace").read()
    if rx:
        m = re.findall(rx, text)
        return {"value": float(m[-1] if isinstance(m[-1], str) else m[-1][0])} if m else None
    for ln in reversed(text.splitlines()):
        ln = ln.strip()
        if ln.startswith("{"):
            try:
                return json.loads(ln)
            except json.JSONDecodeError:
                continue
    return None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--cmd", required=True, help="command of every arm (shell-split)")
    ap.add_argument("--arm", action="append", default=[], help="NAME:VAR=V,VAR2=V2 (repeatable)")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--timeout", type=int, default=400, help="seconds per run")
    ap.add_argument("--tests", default=None, help="pytest args run first, e.g. 'tests -m gpu'")
    ap.add_argument("--tests-timeout", type=int, default=600)
    ap.add_argument("--metric-re", default=None, help="regex with one group; default: last JSON line")
    ap.add_argument("--key", default="value", help="JSON key summarised per arm")
    ap.add_argument("--prof", default=None, help="rocprofv3 --kernel-trace --stats of arm 1 into gpurun_out/NAME")
    ap.add_argument("--out", default=os.path.join("gpurun_out", "ab.jsonl"))
    a = ap.parse_args(argv)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    arms = [_arm(s) for s in (a.arm or ["base:"])]
    cmd = shlex.split(a.cmd)
    out = open(os.path.join(ROOT, a.out), "a")
    if a.tests:
        log = os.path.join(ROOT, "gpurun_out", "ab_tests.log")
        rc, dt = _run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "--timeout", "120",
                       "--timeout-method", "thread", "-p", "no:cacheprovider", *shlex.split(a.tests)],
                      {}, a.tests_timeout, log)
        tail = open(log, errors="replace").read().splitlines()[-3:]
        print(f"[tests] rc={rc} {dt:.0f}s :: " + " | ".join(tail), flush=True)
        if rc != 0:
            return rc
    res = {n: [] for n, _ in arms}
    for r in range(a.rounds):
        for name, env in arms:
            log = os.path.join(ROOT, "gpurun_out", f"ab_{name}_{r}.log")
            rc, dt = _run(cmd, env, a.timeout, log)
            rec = _metric(log, a.metric_re) if rc == 0 else None
            v = rec.get(a.key) if isinstance(rec, dict) else None
            out.write(json.dumps({"arm": name, "env": env, "round": r, "rc": rc, "wall_s": round(dt, 1),
                                  "cmd": a.cmd, "record": rec}) + "\n")
            out.flush()
            print(f"[{name} r{r}] rc={rc} {dt:.0f}s {a.key}={v}", flush=True)
            if rc != 0:
                print(open(log, errors="replace").read()[-2000:], flush=True)
                return rc if rc in FATAL else 1
            if v is not None:
                res[name].append(float(v))
    print("arm\tmedian\truns")
    for name, _ in arms:
        vals = res[name]
        print(f"{name}\t{statistics.median(vals) if vals else float('nan'):.4f}\t{vals}")
    if a.prof:
        d = os.path.join("gpurun_out", a.prof)
        log = os.path.join(ROOT, "gpurun_out", f"{a.prof}.log")
        env = dict(arms[0][1], TMPDIR="/tmp")
        rc, dt = _run(["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", d,
                       "-o", a.prof, "--", *cmd], env, a.timeout + 120, log)
        print(f"[prof {a.prof}] rc={rc} {dt:.0f}s", flush=True)
        if rc != 0:
            return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
