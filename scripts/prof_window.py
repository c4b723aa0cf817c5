#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace (`*_kernel_trace.csv`) into a small markdown table.

    prof_window.py TRACE.csv [--window adamw|all] [--top N] [--by-grid] [--per N]

--window adamw: only the kernels between the last two fused-AdamW launches (one optimizer step
of bench.py); --by-grid: group by (kernel, grid size) -- GEMM shapes show up as distinct grids;
--per N: divide totals by N (e.g. decode steps x layers) to get per-unit averages;
--seq START:COUNT: instead of the table, list COUNT launches of the window in issue order from
launch START (negative START counts from the end), with their grids and durations -- which GEMM
sits where in a layer's forward / backward, and what each call costs in place."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", default="all", choices=("all", "adamw"))
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--by-grid", action="store_true")
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--match", default=None, help="only kernels whose name contains this")
    ap.add_argument("--seq", default=None, help="START:COUNT launches in issue order")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    if a.window == "adamw":
        ad = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
        rows = rows[ad[-2] + 1:ad[-1] + 1]
    if a.match:
        rows = [r for r in rows if a.match in r["Kernel_Name"]]
    if a.seq:
        st, cnt = (int(x) for x in a.seq.split(":"))
        sel = rows[st:st + cnt] if st >= 0 else rows[len(rows) + st:len(rows) + st + cnt]
        print("| # | us | grid | kernel |")
        print("|---|---|---|---|")
        for i, r in enumerate(sel):
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            g = "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
            print(f"| {i} | {d:.1f} | {g} | `{r['Kernel_Name'][:90]}` |")
        return
    agg = collections.defaultdict(lambda: [0.0, 0])
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        key = r["Kernel_Name"][:100]
        if a.by_grid:
            g = "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
            w = r.get("Workgroup_Size_X", "?")
            key = (key, g, w)
        agg[key][0] += d
        agg[key][1] += 1
    tot = sum(v[0] for v in agg.values())
    wall = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3 if rows else 0.0
    print(f"window: {len(rows)} launches, busy {tot / 1e3:.2f} ms, wall {wall / 1e3:.2f} ms"
          + (f", per unit (/{a.per:g}): busy {tot / a.per:.1f} us" if a.per != 1 else ""))
    hdr = "| total us/unit | % | calls | avg us | kernel |" + (" grid | wg |" if a.by_grid else "")
    print(hdr)
    print("|---" * (hdr.count("|") - 1) + "|")
    for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        name, extra = (k[0], f" {k[1]} | {k[2]} |") if a.by_grid else (k, "")
        print(f"| {t / a.per:.1f} | {100 * t / max(tot, 1e-9):.1f} | {n} | {t / n:.1f} | `{name}` |{extra}")


if __name__ == "__main__":
    main()
