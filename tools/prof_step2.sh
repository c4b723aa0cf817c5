#!/bin/bash
# rocprofv3 kernel trace of the headline DPO step (2 timed steps) + per-category breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step -o b -- python -u bench.py --steps 2 --warmup 1 > gpurun_out/prof_step.log 2>&1
echo "rc=$?"; tail -1 gpurun_out/prof_step.log
python scripts/step_breakdown.py gpurun_out/prof_step/b_kernel_trace.csv > gpurun_out/step_breakdown.md 2>&1; head -30 gpurun_out/step_breakdown.md
