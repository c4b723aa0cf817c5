#!/bin/bash
# rocprofv3 kernel stats of graph-captured decode (Llama-3-8B, B=8, prompt 1024, +128 tokens).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/bench_generate.py --modes graph,eager --new 128 > gpurun_out/gen.log 2>&1 && tail -3 gpurun_out/gen.log \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_decode -o d -- python -u tools/bench_generate.py --modes graph --new 128 > gpurun_out/prof_decode.log 2>&1
echo "rc=$?"
