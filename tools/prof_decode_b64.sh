#!/bin/bash
# rocprofv3 kernel stats of graph-captured decode at the RLHF rollout shape on one GPU
# (Llama-3-8B, B=64, prompt 512, +128 tokens).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_decode64 -o d -- python -u tools/bench_generate.py --modes graph --batch 64 --prompt 512 --new 128 > gpurun_out/prof_decode64.log 2>&1
echo "rc=$?"
grep mode gpurun_out/prof_decode64.log
f=$(find gpurun_out/prof_decode64 -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py "$f" 30
