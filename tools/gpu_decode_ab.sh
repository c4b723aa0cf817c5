#!/bin/bash
# Decode A/B: skinny GEMM variants (nt weight loads, split-K gate|up, split-K down) by env, each
# config in its own process (the switches are read once). Numerics tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dec_tests.log 2>&1 || { tail -40 gpurun_out/dec_tests.log; exit 1; }
tail -1 gpurun_out/dec_tests.log
for nt in 0 1; do
  DLA_SKINNY_NT=$nt timeout -k 10 200 python -u tools/skinny_bench.py > gpurun_out/skb_nt$nt.log 2>&1 || { tail -20 gpurun_out/skb_nt$nt.log; exit 1; }
  echo "nt=$nt"; cat gpurun_out/skb_nt$nt.log | grep gemm
done
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > gpurun_out/gen_$lab.log 2>&1 || { tail -20 gpurun_out/gen_$lab.log; exit 1; }
  echo "$lab $(grep mode gpurun_out/gen_$lab.log)"
}
run base DLA_SKINNY_NT=0
run nt DLA_SKINNY_NT=1
run ks DLA_SKINNY_GLU=ks
run ks_nt DLA_SKINNY_GLU=ks DLA_SKINNY_NT=1
run ks_nt_down DLA_SKINNY_GLU=ks DLA_SKINNY_NT=1 DLA_SKINNY_MAX_NARROW_K=16384
run base2 DLA_SKINNY_NT=0
