#!/bin/bash
# m64 split rule A/B in graph decode: default (<= one workgroup per CU) vs DLA_M64_WG=256 (round 3)
set -o pipefail
O=gpurun_out/r4_m64split; mkdir -p $O
timeout -k 10 120 python -u tools/m64_probe.py > $O/probe_new.jsonl 2>&1 || exit 1
timeout -k 10 120 python -u tools/m64_probe.py --rows 32 > $O/probe_new32.jsonl 2>&1 || exit 1
DLA_M64_WG=256 timeout -k 10 120 python -u tools/m64_probe.py --rows 32 > $O/probe_old32.jsonl 2>&1 || exit 1
for r in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export DLA_M64_WG=256; else unset DLA_M64_WG; fi
    timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 --batch 64 --prompt 512 > $O/gen64_$arm$r.log 2>&1 || exit 1
  done
done
unset DLA_M64_WG
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decode_gpu.py -k "m64 or 64 or slab" > $O/tests.log 2>&1 || exit 1
tail -2 $O/tests.log
cat $O/probe_*.jsonl
grep -h "ms_per_token\|ms/token" $O/gen64_*.log
