#!/usr/bin/env python
"""Summarise a rocprofv3 SQLite results DB (ROCm 7.2 default output of `--kernel-trace`):
top kernels by total GPU time (from per-dispatch start/end, ns), markdown table.
Usage: prof_summary_db.py <results.db> [top] [name-substring-to-restrict-window]"""
import sqlite3
import sys
from collections import defaultdict

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
c = sqlite3.connect(path)
agg = defaultdict(lambda: [0, 0.0])
for name, dur in c.execute("select name, end - start from kernels"):
    a = agg[name]
    a[0] += 1
    a[1] += dur
tot = sum(v[1] for v in agg.values())
print(f"total kernel time {tot / 1e6:.1f} ms over {sum(v[0] for v in agg.values())} dispatches")
print("| total ms | % | calls | avg us | kernel |\n|---|---|---|---|---|")
for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"| {t / 1e6:.1f} | {100 * t / tot:.1f} | {n} | {t / n / 1e3:.1f} | `{name[:100]}` |")
