#!/bin/bash
# Attention numerics + microbenchmark only (fast iteration loop on the GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" -p no:cacheprovider > gpurun_out/attn_tests.log 2>&1 \
 && timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 \
 && timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 > gpurun_out/bench.log 2>&1
echo "rc=$?"
tail -2 gpurun_out/attn_tests.log; cat gpurun_out/attn_bench.log 2>/dev/null; tail -1 gpurun_out/bench.log 2>/dev/null; true
