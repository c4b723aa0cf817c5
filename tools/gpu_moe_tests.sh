#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_moe_gpu.py tests/test_grouped_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/moe_tests6.log 2>&1 || { tail -40 gpurun_out/moe_tests6.log; exit 1; }
tail -1 gpurun_out/moe_tests6.log
