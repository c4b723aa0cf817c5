#!/bin/bash
# fp8 row quantiser: single-pass register form vs the two-pass kernel (tests + Mixtral fp8 bench).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_moe_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fp8q_tests.log 2>&1 || { tail -40 gpurun_out/fp8q_tests.log; exit 1; }
tail -1 gpurun_out/fp8q_tests.log
run() {  # label, env, args...
  local lab=$1; shift
  env $1 timeout -k 10 400 python -u bench.py --model mixtral-8x7b --layers 2 --steps 4 --warmup 2 ${@:2} > gpurun_out/mix_$lab.log 2>&1 || { tail -20 gpurun_out/mix_$lab.log; exit 1; }
  echo "$lab $(tail -1 gpurun_out/mix_$lab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["mfu"])')"
}
for r in 1 2; do
run reg_fp8_$r DLA_FP8_QUANT_2PASS=0 --fp8
run twopass_fp8_$r DLA_FP8_QUANT_2PASS=1 --fp8
done
