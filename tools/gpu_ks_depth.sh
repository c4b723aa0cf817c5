#!/bin/bash
# qkv / o skinny split-K ring depth 2 / 3 / 4 (graph decode, B = 8), two interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k skinny > gpurun_out/ksd_tests.log 2>&1 || { tail -30 gpurun_out/ksd_tests.log; exit 1; }
tail -1 gpurun_out/ksd_tests.log
for r in 1 2; do
for d in 2 3 4; do
  DLA_SKINNY_KS_DEPTH=$d timeout -k 10 300 python -u tools/bench_generate.py --modes graph --batch 8 --prompt 1024 --new 128 > gpurun_out/gen_ksd$d.log 2>&1 || { tail -20 gpurun_out/gen_ksd$d.log; exit 1; }
  echo "depth $d $(grep -o '"decode_ms_per_token": [0-9.]*' gpurun_out/gen_ksd$d.log)"
done
done
