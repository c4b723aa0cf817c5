#!/bin/bash
# TunableOp tuning pass over the Mixtral EP-shape step's GEMM shapes (M = 4096-token micro-batches,
# capacity-padded single-expert GEMMs), merged into the shipped table, then A/B
set -o pipefail
O=gpurun_out/r4_mixtune; mkdir -p $O
DLA_GEMM_TUNE=1 DLA_GEMM_TABLE=$PWD/$O/mix_tune.csv timeout -k 10 900 python -u bench.py --model mixtral-8x7b --ep-shape 8 --steps 1 --warmup 1 > $O/tune_run.log 2>&1 || { tail -20 $O/tune_run.log; exit 1; }
ls -la $O
python tools/merge_tunableop.py distributed_llm_alignment_amd/tuning/tunableop_gfx950.csv $O/mix_tune0.csv --out $O/merged.csv || exit 1
for r in 1 2; do
  for arm in merged shipped; do
    if [ $arm = merged ]; then export DLA_GEMM_TABLE=$PWD/$O/merged.csv; else unset DLA_GEMM_TABLE; fi
    timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape 8 --steps 3 --warmup 2 > $O/mix_$arm.$r.log 2>&1 || exit 1
    echo "arm=$arm r=$r $(tail -1 $O/mix_$arm.$r.log | cut -c1-200)"
  done
done
