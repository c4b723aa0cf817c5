#!/bin/bash
# Decode at 17..64 rows: split-K skinny kernels with 2/4 row tiles vs hipBLASLt (DLA_SKINNY_MAX_ROWS=16),
# long-K down on either; B = 8 unchanged; then the RLHF step at the reference's 64 rollouts.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mr_tests.log 2>&1 || { tail -40 gpurun_out/mr_tests.log; exit 1; }
tail -1 gpurun_out/mr_tests.log
run() {  # label, batch, env...
  local lab=$1 b=$2; shift 2
  env "$@" timeout -k 10 300 python -u tools/bench_generate.py --modes graph --batch $b --prompt 512 --new 128 > gpurun_out/gen_$lab.log 2>&1 || { tail -20 gpurun_out/gen_$lab.log; exit 1; }
  echo "$lab $(grep mode gpurun_out/gen_$lab.log)"
}
run b64_lib 64 DLA_SKINNY_MAX_ROWS=16
run b64_ks 64 DLA_SKINNY_MAX_ROWS=64
run b64_ks_downlib 64 DLA_SKINNY_KS_MAX_K=8192
run b32_lib 32 DLA_SKINNY_MAX_ROWS=16
run b32_ks 32 DLA_SKINNY_MAX_ROWS=64
run b8 8 DLA_SKINNY_MAX_ROWS=64
timeout -k 10 500 python -u tools/bench_rlhf.py --batch 64 --grad-ckpt full > gpurun_out/rlhf_b64ks.log 2>&1 || { grep -v "^  " gpurun_out/rlhf_b64ks.log | tail -5; exit 1; }
grep bench gpurun_out/rlhf_b64ks.log
