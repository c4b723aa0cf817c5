#!/bin/bash
# RLHF at the reference's 64 rollouts per step on one GPU: MLP recompute with expandable
# allocator segments (the plain allocator left 7 GB fragmented and ran out) vs full recompute.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() {  # label, env, args...
  local lab=$1 e=$2; shift 2
  env $e timeout -k 10 500 python -u tools/bench_rlhf.py "$@" > gpurun_out/rlhf_$lab.log 2>&1 || { grep -v "^  " gpurun_out/rlhf_$lab.log | tail -3; return 0; }
  grep bench gpurun_out/rlhf_$lab.log
}
run b64mlp_exp PYTORCH_ALLOC_CONF=expandable_segments:True --batch 64 --grad-ckpt mlp
run b64full_exp PYTORCH_ALLOC_CONF=expandable_segments:True --batch 64 --grad-ckpt full
run b64attn_exp PYTORCH_ALLOC_CONF=expandable_segments:True --batch 64 --grad-ckpt attention
