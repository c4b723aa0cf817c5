#!/bin/bash
# Attention numerics + interleaved A/B of one env var across separate processes (kernels read
# their env knobs once per process). Usage: bash tools/gpu_attn_env_ab.sh NAME v0 v1
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
NAME=$1; V0=$2; V1=$3
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or prefill or generation" -p no:cacheprovider > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in $V0 $V1; do
    for args in "" "--T 4096 --B 2" "--noncausal"; do
      echo -n "$NAME=$v $args: "
      env $NAME=$v timeout -k 10 120 python -u tools/attn_bench.py --iters 30 $args 2>/dev/null | grep attn || exit 1
    done
  done
done
