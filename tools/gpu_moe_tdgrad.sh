#!/bin/bash
# MoE per-expert backward: input-gradient GEMMs through transposed expert weights (TN, copy by
# the HIP tiled transpose once per step) vs the NN layout.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
DLA_MOE_TRANSPOSED_DGRAD=1 timeout -k 10 400 python -u -m pytest tests/test_moe_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/moe_tests5.log 2>&1 || { tail -40 gpurun_out/moe_tests5.log; exit 1; }
tail -1 gpurun_out/moe_tests5.log
run() {  # label, env, args...
  local lab=$1; shift
  env $1 timeout -k 10 400 python -u bench.py --model mixtral-8x7b --layers 2 --steps 4 --warmup 2 ${@:2} > gpurun_out/mix_$lab.log 2>&1 || { tail -20 gpurun_out/mix_$lab.log; exit 1; }
  echo "$lab $(tail -1 gpurun_out/mix_$lab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["mfu"])')"
}
for r in 1 2; do
run tn_bf16_$r DLA_MOE_TRANSPOSED_DGRAD=1
run nn_bf16_$r DLA_MOE_TRANSPOSED_DGRAD=0
run tn_fp8_$r DLA_MOE_TRANSPOSED_DGRAD=1 --fp8
run nn_fp8_$r DLA_MOE_TRANSPOSED_DGRAD=0 --fp8
done
