#!/usr/bin/env python
"""Merge TunableOp result tables: rows of NEW tables whose (op, shape) key is not already in the
base table are appended (the base keeps its validator header and existing solutions).

    python tools/merge_tunableop.py BASE.csv NEW.csv [NEW2.csv ...] --out MERGED.csv
"""
from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("base")
    ap.add_argument("new", nargs="+")
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    lines = [ln.rstrip("\n") for ln in open(a.base) if ln.strip()]
    keys = {tuple(ln.split(",")[:2]) for ln in lines if not ln.startswith("Validator")}
    added = 0
    for f in a.new:
        for ln in open(f):
            ln = ln.rstrip("\n")
            if not ln.strip() or ln.startswith("Validator"):
                continue
            k = tuple(ln.split(",")[:2])
            if k not in keys:
                keys.add(k)
                lines.append(ln)
                added += 1
    with open(a.out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print(f"merged {added} new solutions into {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
