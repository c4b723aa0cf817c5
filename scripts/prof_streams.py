#!/usr/bin/env python
"""Per-stream view of a rocprofv3 kernel trace (`*_kernel_trace.csv`): which HIP streams ran
what, and how much of the communication stream's work overlapped compute.

    prof_streams.py TRACE.csv [--comm-stream ID] [--window adamw]

--window adamw: only the last optimizer step of bench.py (kernels that start after the
second-to-last fused-AdamW launch and up to the last one), i.e. one step's forward, backward
with the bucket collectives, and the AdamW. The communication stream defaults to the non-compute
stream with the most dispatches. Overlap = the part of each comm-stream kernel's interval covered
by some compute-stream kernel (union of intervals)."""
import argparse
import bisect
import collections
import csv


def _union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def _covered(a, b, merged, starts):
    i = max(0, bisect.bisect_right(starts, a) - 1)
    tot = 0
    while i < len(merged) and merged[i][0] < b:
        lo, hi = max(a, merged[i][0]), min(b, merged[i][1])
        if hi > lo:
            tot += hi - lo
        i += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--comm-stream", default=None)
    ap.add_argument("--window", default="all", choices=("all", "adamw"))
    ap.add_argument("--pairs", type=int, default=0, help="pairwise overlap table of the N busiest streams")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    if a.window == "adamw":
        ad = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
        t0, t1 = int(rows[ad[-2]]["End_Timestamp"]), int(rows[ad[-1]]["End_Timestamp"])
        rows = [r for r in rows if t0 <= int(r["Start_Timestamp"]) <= t1]
    by = collections.defaultdict(list)
    for r in rows:
        by[r["Stream_Id"]].append(r)
    comp = max(by, key=lambda s: len(by[s]))
    comm = a.comm_stream or max((s for s in by if s != comp), key=lambda s: len(by[s]), default=None)
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6
    print(f"window: {a.window}, {len(rows)} kernels, {span:.1f} ms wall\n")
    print("| stream | kernels | busy ms | top kernels |\n|---|---|---|---|")
    for s, rs in sorted(by.items(), key=lambda kv: -len(kv[1])):
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e6
        top = collections.Counter(r["Kernel_Name"].split("(")[0][:48] for r in rs).most_common(3)
        tag = " (compute)" if s == comp else (" (comm)" if s == comm else "")
        print(f"| {s}{tag} | {len(rs)} | {busy:.2f} | " + ", ".join(f"`{n}` x{c}" for n, c in top) + " |")
    if a.pairs:  # busy time of each top stream that some kernel of each other stream covers
        top = [s for s, _ in sorted(by.items(), key=lambda kv: -len(kv[1]))][:a.pairs]
        mer = {}
        for s in top:
            m = _union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in by[s]])
            mer[s] = (m, [x[0] for x in m])
        print("\n| stream A | busy ms | % of A concurrent with " + " | ".join(f"stream {t}" for t in top) + " |")
        print("|---|---|" + "---|" * len(top))
        for s in top:
            tot = sum(b - a_ for a_, b in mer[s][0])
            cells = []
            for t in top:
                if t == s:
                    cells.append("—")
                    continue
                ov = sum(_covered(a_, b, *mer[t]) for a_, b in mer[s][0])
                cells.append(f"{100.0 * ov / max(tot, 1):.1f}")
            print(f"| {s} | {tot / 1e6:.2f} | " + " | ".join(cells) + " |")
    if comm is None:
        return
    merged = _union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in by[comp]])
    starts = [m[0] for m in merged]
    cr = by[comm]
    tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in cr)
    ov = sum(_covered(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), merged, starts) for r in cr)
    w0 = int(rows[0]["Start_Timestamp"])
    first, last = (int(cr[0]["Start_Timestamp"]) - w0) / 1e6, (int(cr[-1]["End_Timestamp"]) - w0) / 1e6
    print(f"\ncomm stream {comm}: {len(cr)} kernels, {tot / 1e6:.2f} ms busy, "
          f"{100.0 * ov / max(tot, 1):.1f} % of it concurrent with compute-stream kernels; "
          f"first starts at {first:.1f} ms, last ends at {last:.1f} ms of the {span:.1f} ms window")


if __name__ == "__main__":
    main()
