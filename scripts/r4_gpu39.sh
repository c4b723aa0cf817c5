#!/bin/bash
# head-major KV cache (DLA_KV_HEAD_MAJOR=1): whole GPU tier on it, then a decode A/B
set -o pipefail
O=gpurun_out/r4_khm; mkdir -p $O
DLA_KV_HEAD_MAJOR=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tier.log 2>&1 || { tail -30 $O/gpu_tier.log; exit 1; }
tail -1 $O/gpu_tier.log
for r in 1 2; do
  for arm in 1 0; do
    DLA_KV_HEAD_MAJOR=$arm timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 --batch 64 --prompt 512 > $O/g64_$arm.$r.log 2>&1 || exit 1
    DLA_KV_HEAD_MAJOR=$arm timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > $O/g8_$arm.$r.log 2>&1 || exit 1
    echo "hm=$arm r=$r B64 $(grep -h decode_ms $O/g64_$arm.$r.log | sed 's/.*decode_ms_per_token": \([0-9.]*\).*/\1/') B8 $(grep -h decode_ms $O/g8_$arm.$r.log | sed 's/.*decode_ms_per_token": \([0-9.]*\).*/\1/')"
  done
done
