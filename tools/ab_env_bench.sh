#!/bin/bash
# GPU test tier, then an interleaved A/B of the DPO bench with an env toggle on ONE box
# (box-to-box clock variance is larger than most single optimisations).
# usage: tools/ab_env_bench.sh VAR [steps] [rounds]   (A = VAR=0, B = VAR=1)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
VAR=$1; STEPS=${2:-8}; ROUNDS=${3:-2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head -20; exit $rc; }
for r in $(seq $ROUNDS); do
  for v in 0 1; do
    echo -n "$VAR=$v: "
    env $VAR=$v timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 3 > gpurun_out/ab_${VAR}_${v}_$r.log 2>&1 || { tail -5 gpurun_out/ab_${VAR}_${v}_$r.log; exit 1; }
    tail -1 gpurun_out/ab_${VAR}_${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
  done
done
