#!/bin/bash
# TN weight-gradient lower bound (DLA_TN_WGRAD_MIN: 1 Mi elements default vs 0): Mixtral EP-shape A/B
set -o pipefail
O=gpurun_out/r4_tnmin; mkdir -p $O
for r in 1 2; do
  for arm in 1048576 0; do
    DLA_TN_WGRAD_MIN=$arm timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape 8 --steps 3 --warmup 2 > $O/mix_$arm.$r.log 2>&1 || exit 1
    echo "min=$arm r=$r $(tail -1 $O/mix_$arm.$r.log | cut -c1-170)"
  done
done
