#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "norm or decode or graph or generation" 2>&1 | tail -1 || exit 1
for i in 1 2; do timeout -k 10 200 python -u tools/bench_generate.py --modes graph --new 128 2>/dev/null | grep mode || exit 1; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_decode -o d -- python -u tools/bench_generate.py --modes graph --new 128 > gpurun_out/prof_decode.log 2>&1
