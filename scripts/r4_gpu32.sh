#!/bin/bash
# MoE capacity-buffer tails zeroed in place (DLA_MOE_TAIL_INPLACE): MoE GPU tests + Mixtral EP-shape A/B
set -o pipefail
O=gpurun_out/r4_tail; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
DLA_MOE_TAIL_INPLACE=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe_gpu.py -k "shape_mode" > $O/tests0.log 2>&1 || { tail -30 $O/tests0.log; exit 1; }
tail -1 $O/tests0.log
for r in 1 2; do
  for arm in 1 0; do
    DLA_MOE_TAIL_INPLACE=$arm timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape 8 --steps 3 --warmup 2 > $O/mix_$arm.$r.log 2>&1 || exit 1
    echo "arm=$arm r=$r $(tail -1 $O/mix_$arm.$r.log | cut -c1-200)"
  done
done
