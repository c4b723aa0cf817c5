#!/bin/bash
# bf16 dK / dV head-split partials: attention tests, attn_bench A/B, DPO bench A/B
set -o pipefail
O=gpurun_out/r4_dkv16; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/attn_bench.py --ab DLA_ATTN_DKV_BF16=1,0 --rounds 3 > $O/attn_ab.log 2>&1 || exit 1
tail -8 $O/attn_ab.log
timeout -k 10 300 python -u tools/attn_bench.py --noncausal --ab DLA_ATTN_DKV_BF16=1,0 --rounds 2 > $O/attn_ab_nc.log 2>&1 || exit 1
tail -4 $O/attn_ab_nc.log
for r in 1 2; do
  for arm in 1 0; do
    DLA_ATTN_DKV_BF16=$arm timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 > $O/dpo_$arm.$r.log 2>&1 || exit 1
    echo "arm=$arm r=$r $(tail -1 $O/dpo_$arm.$r.log | cut -c1-200)"
  done
done
