#!/bin/bash
# GPU pipeline tier: reward, teacher rollouts, distillation, RLHF (REINFORCE / PPO), eval CLIs.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pipeline_gpu.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pipeline_gpu.log | tail -12
[ $rc -ne 0 ] && tail -40 gpurun_out/pipeline_gpu.log
exit $rc
