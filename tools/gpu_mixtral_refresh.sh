#!/bin/bash
# Mixtral-8x7B (full width, 2 layers) DPO on one MI355X with the device-driven grouped expert GEMM
# (default) vs the per-expert hipBLASLt loop, bf16 and fp8 expert forward; kernel summary.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # label, env/args...
  local lab=$1; shift
  env $1 timeout -k 10 400 python -u bench.py --model mixtral-8x7b --layers 2 --steps 4 --warmup 2 ${@:2} > gpurun_out/mix_$lab.log 2>&1 || { tail -20 gpurun_out/mix_$lab.log; exit 1; }
  echo "$lab $(tail -1 gpurun_out/mix_$lab.log)"
}
run grouped_bf16 DLA_MOE_GEMM=grouped
run loop_bf16 DLA_MOE_GEMM=loop
run grouped_fp8 DLA_MOE_GEMM=grouped --fp8
run loop_fp8 DLA_MOE_GEMM=loop --fp8
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mix2 -o p -- python -u bench.py --model mixtral-8x7b --layers 2 --fp8 --steps 2 --warmup 1 > gpurun_out/prof_mix2.log 2>&1 || { tail -20 gpurun_out/prof_mix2.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_mix2/p_kernel_stats.csv 20
