#!/bin/bash
# Transpose tests, then transpose / SwiGLU bandwidth with build A vs B (one box).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "transpose or swiglu" > gpurun_out/tr_tests.log 2>&1 || { tail -30 gpurun_out/tr_tests.log; exit 1; }
tail -1 gpurun_out/tr_tests.log
for v in A B; do
  echo "== $v"; DLA_EXT_PATH=build/ab/_C_$v.so timeout -k 10 120 python -u tools/transpose_bench.py || exit 1
done
