#!/bin/bash
# m64 weight-chunk depth A/B (DLA_M64_DEPTH 2 / 3 / 4): probe + B=64 graph decode
set -o pipefail
O=gpurun_out/r4_m64depth; mkdir -p $O
for d in 2 3 4; do
  DLA_M64_DEPTH=$d timeout -k 10 120 python -u tools/m64_probe.py > $O/probe_d$d.jsonl 2>&1 || exit 1
done
for r in 1 2; do
  for d in 2 3 4; do
    DLA_M64_DEPTH=$d timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 --batch 64 --prompt 512 > $O/gen64_d$d.$r.log 2>&1 || exit 1
  done
done
DLA_M64_DEPTH=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decode_gpu.py -k "m64 or 64 or slab" > $O/tests.log 2>&1 || exit 1
tail -2 $O/tests.log
for d in 2 3 4; do echo "d=$d"; grep -h rows $O/probe_d$d.jsonl; grep -h decode_ms $O/gen64_d$d.*.log; done
