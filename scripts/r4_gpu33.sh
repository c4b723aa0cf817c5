#!/bin/bash
# EP chunk views by one split: MoE GPU tests + Mixtral EP-shape run
set -o pipefail
O=gpurun_out/r4_split; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape 8 --steps 3 --warmup 2 > $O/mix.$r.log 2>&1 || exit 1
  echo "r=$r $(tail -1 $O/mix.$r.log | cut -c1-200)"
done
