#!/usr/bin/env python
"""Summarise rocprofv3 `--pmc` output: per kernel, the mean of every counter over its
dispatches (rows of one dispatch and counter are summed first), plus the dispatch geometry and
register / LDS / scratch allocation. Usage:

    rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES ... -d gpurun_out/pmc1 -o run --output-format csv -- python ...
    python tools/pmc_summary.py gpurun_out/pmc1 [--filter attn_bwd]
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import sys
from collections import defaultdict


def summarise(root: str, filt: str = "") -> str:
    files = sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True))
    if not files:
        return f"no *counter_collection.csv under {root}\n"
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    geo = {}
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "?")
                if filt and filt not in name:
                    continue
                key = (name, f, row.get("Dispatch_Id", row.get("Correlation_Id", "0")))
                per[key][row["Counter_Name"]] += float(row["Counter_Value"])
                geo.setdefault(name, (row.get("Grid_Size"), row.get("Workgroup_Size"), row.get("LDS_Block_Size"),
                                      row.get("VGPR_Count"), row.get("Accum_VGPR_Count"), row.get("Scratch_Size")))
    kern = defaultdict(lambda: defaultdict(list))
    for (name, _, _), counters in per.items():
        for c, v in counters.items():
            kern[name][c].append(v)
    out = []
    for name in sorted(kern):
        g = geo[name]
        out.append(f"## {name[:110]}")
        out.append(f"grid {g[0]} wg {g[1]} lds {g[2]} vgpr {g[3]} agpr {g[4]} scratch {g[5]}")
        for c in sorted(kern[name]):
            vals = kern[name][c]
            out.append(f"  {c:<32s} {sum(vals) / len(vals):>12.4g}  (n={len(vals)})")
    return "\n".join(out) + "\n"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("roots", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    for r in a.roots:
        sys.stdout.write(summarise(r, a.filter))
    return 0


if __name__ == "__main__":
    sys.exit(main())
