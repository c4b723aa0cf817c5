#!/bin/bash
# Tune the decode GEMMs left on hipBLASLt, then A/B generation with the merged table.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 python -u tools/tune_decode_gemms.py --out gpurun_out/decode_tune.csv > gpurun_out/tune_decode.log 2>&1 || { tail -20 gpurun_out/tune_decode.log; exit 1; }
grep -c tune gpurun_out/tune_decode.log
T=distributed_llm_alignment_amd/tuning/tunableop_gfx950.csv
{ cat $T; grep "^Gemm" gpurun_out/decode_tune.csv | grep -v -F -f <(grep "^Gemm" $T | cut -d, -f1,2); } > gpurun_out/merged.csv
wc -l gpurun_out/merged.csv
run() {  # label, batch, prompt, env...
  local lab=$1 b=$2 pr=$3; shift 3
  env "$@" timeout -k 10 300 python -u tools/bench_generate.py --modes graph --batch $b --prompt $pr --new 128 > gpurun_out/gen_$lab.log 2>&1 || { tail -20 gpurun_out/gen_$lab.log; exit 1; }
  echo "$lab $(grep mode gpurun_out/gen_$lab.log)"
}
run b64_old 64 512
run b64_new 64 512 DLA_GEMM_TABLE=$PWD/gpurun_out/merged.csv
run b32_old 32 512
run b32_new 32 512 DLA_GEMM_TABLE=$PWD/gpurun_out/merged.csv
run b8_old 8 1024
run b8_new 8 1024 DLA_GEMM_TABLE=$PWD/gpurun_out/merged.csv
