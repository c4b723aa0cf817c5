#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k skinny > gpurun_out/skinny_tests.log 2>&1 || { tail -40 gpurun_out/skinny_tests.log; exit 1; }
tail -1 gpurun_out/skinny_tests.log
timeout -k 10 200 python -u tools/skinny_bench.py > gpurun_out/skinny_bench.log 2>&1; rc=$?; grep gemm gpurun_out/skinny_bench.log; exit $rc
