#!/usr/bin/env python
"""Per-kernel PMC table from rocprofv3 --pmc CSV output(s) (counter_collection.csv): mean
counter value per dispatch for every kernel whose name contains one of the filters.
Usage: pmc_summary_csv.py <counter_collection.csv> [more.csv ...] [--by-grid] [-k substr ...]
--by-grid keys the table by (kernel, grid size): library GEMMs share one kernel name across shapes."""
import csv
import sys
from collections import defaultdict

args = sys.argv[1:]
by_grid = "--by-grid" in args
args = [a for a in args if a != "--by-grid"]
filt = []
if "-k" in args:
    i = args.index("-k")
    filt, args = args[i + 1:], args[:i]
vals = defaultdict(lambda: defaultdict(list))
meta = {}
for path in args:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if filt and not any(f in name for f in filt):
            continue
        short = name.split("(")[0].replace("void ", "")[:70]
        if by_grid:
            short = f"{short} @grid {r['Grid_Size']}"
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta[short] = (r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"],
                       r["Accum_VGPR_Count"], r["Scratch_Size"])
for k, cs in vals.items():
    g, wg, lds, v, a, sc = meta[k]
    print(f"## {k}\ngrid {g} wg {wg} lds {lds} vgpr {v} agpr {a} scratch {sc}")
    for c, xs in sorted(cs.items()):
        print(f"  {c:28s} {sum(xs) / len(xs):14.4g}  (n={len(xs)})")
