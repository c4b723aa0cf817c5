#!/bin/bash
# Larger decode batches (288 GB per GPU): the RLHF step at the reference's rlhf_config batch_size
# (64 rollouts per step) on one GPU with policy recompute; 32 for comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() {  # label, args...
  local lab=$1; shift
  timeout -k 10 500 python -u tools/bench_rlhf.py "$@" > gpurun_out/rlhf_$lab.log 2>&1 || { grep -v "^  " gpurun_out/rlhf_$lab.log | tail -5; exit 1; }
  grep bench gpurun_out/rlhf_$lab.log
}
run b64full --batch 64 --grad-ckpt full
run b32mlp --batch 32 --grad-ckpt mlp
