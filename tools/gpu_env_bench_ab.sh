#!/bin/bash
# Selected GPU tests, then interleaved DPO bench A/B of one env var (separate processes).
# Usage: bash tools/gpu_env_bench_ab.sh NAME v0 v1 "pytest -k expr"
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
NAME=$1; V0=$2; V1=$3; K=$4
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engines_gpu.py tests/test_trainers_gpu.py -x -q --timeout 200 --timeout-method thread -k "$K" -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -1 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/ab_tests.log | head; exit $rc; }
for r in 1 2; do
  for v in $V0 $V1; do
    echo -n "$NAME=$v: "; env $NAME=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 2>/dev/null | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'])" || exit 1
  done
done
