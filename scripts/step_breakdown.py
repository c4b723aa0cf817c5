"""Per-step kernel-time breakdown from a rocprofv3 kernel trace: the window between the last two
fused-AdamW launches (one full optimizer step), grouped into categories."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ad = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
lo, hi = ad[-2] + 1, ad[-1] + 1
CATS = [("gemm", ("Cijk_",)), ("attention", ("attn_",)), ("swiglu", ("swiglu",)), ("norm", ("norm_",)),
        ("transpose", ("transpose",)), ("adamw", ("adamw",)), ("rope", ("rope_",)),
        ("logprob/loss", ("logprob", "seq_reduce", "dpo_")), ("copy", ("copy", "Copy")),
        ("grad-norm", ("sumsq",))]
agg = collections.Counter()
cnt = collections.Counter()
for r in rows[lo:hi]:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    cat = next((c for c, keys in CATS if any(k in n for k in keys)), "other")
    agg[cat] += d
    cnt[cat] += 1
wall = (int(rows[hi - 1]["End_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e6
tot = sum(agg.values())
print(f"step window: wall {wall:.1f} ms, kernel busy {tot:.1f} ms ({100 * tot / wall:.1f} %)")
print("| category | ms/step | % of busy | launches |\n|---|---|---|---|")
for c, v in agg.most_common():
    print(f"| {c} | {v:.1f} | {100 * v / tot:.1f} | {cnt[c]} |")
