#!/bin/bash
# Long-context Llama-3-8B DPO on 1x MI355X (the per-GPU shard an SP group would run) .
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --seq-len 4096 --micro-pairs 1 --accum 4 --steps 3 --warmup 1 2>/dev/null | tail -1 > gpurun_out/longctx_4k.log && cat gpurun_out/longctx_4k.log \
 && timeout -k 10 500 python -u bench.py --seq-len 8192 --micro-pairs 1 --accum 2 --steps 3 --warmup 1 2>/dev/null | tail -1 > gpurun_out/longctx_8k.log && cat gpurun_out/longctx_8k.log
