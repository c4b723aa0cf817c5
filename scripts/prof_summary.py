#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: top kernels by total time."""
import csv
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms")
print("| total ms | % | calls | avg us | kernel |\n|---|---|---|---|---|")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"| {float(r['TotalDurationNs'])/1e6:.1f} | {float(r['Percentage']):.1f} | {r['Calls']} | "
          f"{float(r['AverageNs'])/1e3:.1f} | `{r['Name'][:90]}` |")
