#!/bin/bash
# Interleaved A/B of bench.py with a flag value on ONE box: tools/ab_bench_flag.sh FLAG A B [steps] [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
FLAG=$1; A=$2; B=$3; STEPS=${4:-8}; ROUNDS=${5:-2}
for r in $(seq $ROUNDS); do
  for v in $A $B; do
    echo -n "$FLAG=$v: "
    timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 3 $FLAG $v > gpurun_out/abf_${v}_$r.log 2>&1 || { tail -5 gpurun_out/abf_${v}_$r.log; exit 1; }
    tail -1 gpurun_out/abf_${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['final_loss'])"
  done
done
