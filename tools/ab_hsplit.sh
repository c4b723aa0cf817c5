#!/bin/bash
# Attention numerics, then the backward with forced GQA head split 1 vs automatic (one box).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" -p no:cacheprovider > gpurun_out/attn_tests.log 2>&1 || { tail -20 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
for r in 1 2; do
  for hs in 0 1; do
    echo -n "hsplit=$hs: "; DLA_ATTN_BWD_HSPLIT=$hs timeout -k 10 120 python -u tools/attn_bench.py --iters 30 2>/dev/null | grep attn || exit 1
  done
done
