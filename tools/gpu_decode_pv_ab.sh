#!/bin/bash
# Decode attention P.V on MFMA (default) vs the VALU form (DLA_DECODE_PV=valu): numerics tests,
# microbench, generation at B = 8 and 64.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pv_tests.log 2>&1 || { tail -40 gpurun_out/pv_tests.log; exit 1; }
tail -1 gpurun_out/pv_tests.log
DLA_DECODE_PV=valu timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "decode_attn or rope or graph" > gpurun_out/pv_tests_valu.log 2>&1 || { tail -40 gpurun_out/pv_tests_valu.log; exit 1; }
tail -1 gpurun_out/pv_tests_valu.log
for pv in valu mfma; do
  for B in 8 64; do
    DLA_DECODE_PV=$pv timeout -k 10 200 python -u tools/decode_attn_bench.py --B $B --lens 640,1152 > gpurun_out/dab_${pv}_$B.log 2>&1 || { tail -20 gpurun_out/dab_${pv}_$B.log; exit 1; }
    echo "$pv B=$B"; grep -v "^/opt" gpurun_out/dab_${pv}_$B.log | tail -3
  done
done
run() {  # label, batch, prompt, env...
  local lab=$1 b=$2 pr=$3; shift 3
  env "$@" timeout -k 10 300 python -u tools/bench_generate.py --modes graph --batch $b --prompt $pr --new 128 > gpurun_out/gen_$lab.log 2>&1 || { tail -20 gpurun_out/gen_$lab.log; exit 1; }
  echo "$lab $(grep mode gpurun_out/gen_$lab.log)"
}
run b8_valu 8 1024 DLA_DECODE_PV=valu
run b8_mfma 8 1024 DLA_DECODE_PV=mfma
run b64_valu 64 512 DLA_DECODE_PV=valu
run b64_mfma 64 512 DLA_DECODE_PV=mfma
run b8_valu2 8 1024 DLA_DECODE_PV=valu
run b8_mfma2 8 1024 DLA_DECODE_PV=mfma
