#!/bin/bash
# Larger decode batches (288 GB per GPU): generation and the RLHF step at the reference's
# rlhf_config batch_size (64 rollouts per step) on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for b in 16 32 64; do
  timeout -k 10 300 python -u tools/bench_generate.py --modes graph,eager --batch $b --new 128 > gpurun_out/gen_b$b.log 2>&1 || { tail -20 gpurun_out/gen_b$b.log; exit 1; }
  grep mode gpurun_out/gen_b$b.log
done
timeout -k 10 400 python -u tools/bench_rlhf.py --batch 64 > gpurun_out/rlhf_b64.log 2>&1 || { tail -20 gpurun_out/rlhf_b64.log; exit 1; }
grep bench gpurun_out/rlhf_b64.log
