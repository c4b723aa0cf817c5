#!/bin/bash
# rocprofv3 kernel stats of graph decode at B=8 (prompt 1024) and B=64 (prompt 512), +128 tokens.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for cfg in "8 1024" "64 512"; do
  set -- $cfg
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dec_b$1 -o d -- python -u tools/bench_generate.py --modes graph --batch $1 --prompt $2 --new 128 > gpurun_out/prof_dec_b$1.log 2>&1 || { tail -5 gpurun_out/prof_dec_b$1.log; exit 1; }
  grep mode gpurun_out/prof_dec_b$1.log
  python scripts/prof_summary.py gpurun_out/prof_dec_b$1/d_kernel_stats.csv 16
done
# eager-decode A/B against the pre-session tree in ab_old/ (if present): host-side overhead check
if [ -d ab_old ]; then
  for r in 1 2; do
    (cd ab_old && timeout -k 10 300 python -u tools/bench_generate.py --modes eager,graph --batch 8 --prompt 1024 --new 128 > ../gpurun_out/gen_old_$r.log 2>&1) || { tail -5 gpurun_out/gen_old_$r.log; exit 1; }
    echo "old $(grep mode gpurun_out/gen_old_$r.log | tr '\n' ' ')"
    timeout -k 10 300 python -u tools/bench_generate.py --modes eager,graph --batch 8 --prompt 1024 --new 128 > gpurun_out/gen_new_$r.log 2>&1 || { tail -5 gpurun_out/gen_new_$r.log; exit 1; }
    echo "new $(grep mode gpurun_out/gen_new_$r.log | tr '\n' ' ')"
  done
fi
