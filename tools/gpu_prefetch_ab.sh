#!/bin/bash
# Decode A/B: Infinity-Cache weight prefetch on a side stream, by gate|up K fraction / workgroups.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "prefetch or graph" > gpurun_out/pf_tests.log 2>&1 || { tail -40 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > gpurun_out/gen_$lab.log 2>&1 || { tail -20 gpurun_out/gen_$lab.log; exit 1; }
  echo "$lab $(grep mode gpurun_out/gen_$lab.log)"
}
run base DLA_DECODE_PREFETCH=0
run pf0.01 DLA_DECODE_PREFETCH=0.01
run pf0.25 DLA_DECODE_PREFETCH=0.25
run pf0.5 DLA_DECODE_PREFETCH=0.5
run pf0.25w128 DLA_DECODE_PREFETCH=0.25 DLA_PREFETCH_WGS=128
run pf0.25w32 DLA_DECODE_PREFETCH=0.25 DLA_PREFETCH_WGS=32
run base2 DLA_DECODE_PREFETCH=0
