#!/bin/bash
# Bench variants + rocprofv3 kernel stats of the flagship DPO step (1x MI355X).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --micro-pairs 8 --accum 2 > gpurun_out/bench_m8.log 2>&1 \
 && timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --micro-pairs 2 --accum 8 > gpurun_out/bench_m2.log 2>&1 \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o b -- python -u bench.py --steps 2 --warmup 1 > gpurun_out/prof_bench.log 2>&1
echo "rc=$?"
tail -1 gpurun_out/bench_m8.log; tail -1 gpurun_out/bench_m2.log; tail -1 gpurun_out/prof_bench.log
