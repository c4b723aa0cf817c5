#!/bin/bash
# Decode attention A/B: current tree vs a saved .so (DLA_EXT_PATH), decode tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/da_tests.log 2>&1 || { tail -40 gpurun_out/da_tests.log; exit 1; }
tail -1 gpurun_out/da_tests.log
for r in 1 2; do
for v in old new; do
  ext=""; [ $v = old ] && ext="DLA_EXT_PATH=$PWD/ab_so/_C_old.so"
  for B in 8 64; do
    env $ext timeout -k 10 200 python -u tools/decode_attn_bench.py --B $B --lens 640,1152 > gpurun_out/dab_${v}_$B.log 2>&1 || { tail -20 gpurun_out/dab_${v}_$B.log; exit 1; }
    echo "$v B=$B $(grep kv_len gpurun_out/dab_${v}_$B.log | tr '\n' ' ')"
  done
done
done
for v in old new; do
  ext=""; [ $v = old ] && ext="DLA_EXT_PATH=$PWD/ab_so/_C_old.so"
  env $ext timeout -k 10 300 python -u tools/bench_generate.py --modes graph --batch 8 --prompt 1024 --new 128 > gpurun_out/gen_da_$v.log 2>&1 || { tail -20 gpurun_out/gen_da_$v.log; exit 1; }
  echo "$v $(grep mode gpurun_out/gen_da_$v.log)"
done
