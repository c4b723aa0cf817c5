#!/bin/bash
# 64-row decode: skinny split-K only where x is small next to the weights (qkv, o), hipBLASLt for
# gate|up and the long-K down projection, vs all-hipBLASLt.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() {  # label, batch, prompt, env...
  local lab=$1 b=$2 pr=$3; shift 3
  env "$@" timeout -k 10 300 python -u tools/bench_generate.py --modes graph --batch $b --prompt $pr --new 128 > gpurun_out/gen_$lab.log 2>&1 || { tail -20 gpurun_out/gen_$lab.log; exit 1; }
  echo "$lab $(grep mode gpurun_out/gen_$lab.log)"
}
run b64_lib 64 512
run b64_qkvo 64 512 DLA_SKINNY_MAX_ROWS=64 DLA_SKINNY_GLU_MAX_ROWS=16 DLA_SKINNY_KS_MAX_K=4096
run b32_lib 32 512
run b32_qkvo 32 512 DLA_SKINNY_MAX_ROWS=64 DLA_SKINNY_GLU_MAX_ROWS=16 DLA_SKINNY_KS_MAX_K=4096
run b64_lib2 64 512
