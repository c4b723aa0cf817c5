#!/bin/bash
# B=8 decode gate|up kernel form A/B (DLA_SKINNY_GLU lds / ks) on the current build
set -o pipefail
O=gpurun_out/r4_glu; mkdir -p $O
for r in 1 2; do
  for arm in lds ks; do
    DLA_SKINNY_GLU=$arm timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > $O/$arm.$r.log 2>&1 || exit 1
    echo "$arm r=$r $(grep -h decode_ms $O/$arm.$r.log | sed 's/.*decode_ms_per_token": \([0-9.]*\).*/\1/')"
  done
done
