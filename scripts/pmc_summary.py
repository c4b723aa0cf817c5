#!/usr/bin/env python
"""Per-kernel PMC counter table from a rocprofv3 --pmc SQLite DB (sum of per-dispatch values
over dispatches of the same kernel, plus dispatch count and mean duration).
Usage: pmc_summary.py <results.db> [kernel-substring ...]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
filt = sys.argv[2:]
c = sqlite3.connect(db)
vals = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
dur = defaultdict(float)
for name, cname, v, did, d in c.execute(
        "select kernel_name, counter_name, value, dispatch_id, duration from counters_collection"):
    short = name.split("(")[0][:60]
    if filt and not any(f in name for f in filt):
        continue
    vals[short][cname] += v
    if did not in disp[short]:
        disp[short].add(did)
        dur[short] += d
for k in vals:
    n = len(disp[k])
    print(f"## {k}  dispatches={n} mean_dur_us={dur[k] / max(n, 1) / 1e3:.1f}")
    for cname, v in sorted(vals[k].items()):
        print(f"  {cname:28s} {v / max(n, 1):.4g} per dispatch")
