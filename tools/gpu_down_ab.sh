#!/bin/bash
# Decode down projection (K = 14336) on the skinny split-K kernel (2- or 4-deep ring) vs hipBLASLt.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k skinny > gpurun_out/down_tests.log 2>&1 || { tail -40 gpurun_out/down_tests.log; exit 1; }
tail -1 gpurun_out/down_tests.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u tools/bench_generate.py --modes graph --batch 8 --prompt 1024 --new 128 > gpurun_out/gen_$lab.log 2>&1 || { tail -20 gpurun_out/gen_$lab.log; exit 1; }
  echo "$lab $(grep mode gpurun_out/gen_$lab.log)"
}
for r in 1 2; do
run lib$r
run ks4_$r DLA_SKINNY_MAX_NARROW_K=16384
run ks2_$r DLA_SKINNY_MAX_NARROW_K=16384 DLA_SKINNY_DEEP_K=1000000
done
