#!/bin/bash
# DPO: next step's first ref pass queued beside the optimizer update (DLA_REF_AHEAD) A/B
set -o pipefail
O=gpurun_out/r4_refahead; mkdir -p $O
for r in 1 2 3; do
  for arm in 1 0; do
    DLA_REF_AHEAD=$arm timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $O/dpo_$arm.$r.log 2>&1 || exit 1
    echo "arm=$arm r=$r $(tail -1 $O/dpo_$arm.$r.log | cut -c1-170)"
  done
done
