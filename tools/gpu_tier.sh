#!/bin/bash
# Full GPU test tier (+ optional attention microbench with a forced backward head split).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head -20; exit $rc; }
for hs in 0 4; do
  echo -n "hsplit=$hs: "; DLA_ATTN_BWD_HSPLIT=$hs timeout -k 10 120 python -u tools/attn_bench.py --iters 30 2>/dev/null | grep attn || exit 1
done
