#!/bin/bash
# attention reduce-pass grid cap A/B (DLA_ATTN_REDUCE_GRID, read once per process)
set -o pipefail
O=gpurun_out/r4_rgrid; mkdir -p $O
for r in 1 2; do
  for g in 2048 8192 32768 1024; do
    DLA_ATTN_REDUCE_GRID=$g timeout -k 10 200 python -u tools/attn_bench.py --ab DLA_ATTN_DKV_BF16=1,1 --rounds 3 > $O/ab_$g.$r.log 2>&1 || exit 1
    echo "grid=$g r=$r $(grep 'attn-ab\] DLA' $O/ab_$g.$r.log | head -1)"
  done
done
