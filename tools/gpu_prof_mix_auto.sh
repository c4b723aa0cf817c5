#!/bin/bash
# rocprofv3 kernel stats of the Mixtral 2-layer DPO step, fp8 expert forward, MoE GEMM policy auto.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mix3 -o p -- python -u bench.py --model mixtral-8x7b --layers 2 --fp8 --steps 2 --warmup 1 > gpurun_out/prof_mix3.log 2>&1 || { tail -20 gpurun_out/prof_mix3.log; exit 1; }
tail -1 gpurun_out/prof_mix3.log
python scripts/prof_summary.py gpurun_out/prof_mix3/p_kernel_stats.csv 16
