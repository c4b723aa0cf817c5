#!/bin/bash
# New GPU tests (layer split, fused MLP), then a rocprofv3 kernel-stats profile of the DPO step.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "layer_split or swiglu or fused" > gpurun_out/new_tests.log 2>&1 || { tail -30 gpurun_out/new_tests.log; exit 1; }
tail -1 gpurun_out/new_tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step -o b -- python -u bench.py --steps 2 --warmup 1 > gpurun_out/prof_step.log 2>&1
echo "rc=$?"; tail -1 gpurun_out/prof_step.log
