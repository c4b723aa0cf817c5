#!/bin/bash
# A/B of two extension builds (build/ab/_C_A.so vs _C_B.so) on the attention microbenchmark,
# interleaved on one box (MI355X devices differ by up to ~12% in clock: never compare boxes).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/ab_attn.log; : > $out
for r in 1 2 3; do
  for v in A B; do
    echo -n "$v: " >> $out
    DLA_EXT_PATH=build/ab/_C_$v.so timeout -k 10 120 python -u tools/attn_bench.py --iters 30 2>/dev/null | grep attn >> $out || exit 1
  done
done
cat $out
