#!/bin/bash
# Attention numerics (new build) + interleaved old/new microbenchmark on one box.
# Usage: bash tools/gpu_attn_ab.sh OLD_SO   (the in-tree _C.so is the new build)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
OLD=${1:-_C_old.so}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" -p no:cacheprovider > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for so in "$OLD" distributed_llm_alignment_amd/_C.so; do
    for args in "" "--T 4096 --B 2" "--noncausal"; do
      echo -n "$so $args: "
      DLA_EXT_PATH=$PWD/$so timeout -k 10 120 python -u tools/attn_bench.py --iters 30 $args 2>/dev/null | grep attn || exit 1
    done
  done
done
