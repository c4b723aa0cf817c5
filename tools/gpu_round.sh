#!/bin/bash
# Full GPU tier + headline bench + RLHF step bench (1x MI355X).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log \
 && timeout -k 10 300 python -u tools/bench_generate.py --modes graph,eager --new 128 > gpurun_out/gen.log 2>&1 && grep mode gpurun_out/gen.log \
 && timeout -k 10 400 python -u tools/bench_rlhf.py > gpurun_out/bench_rlhf.log 2>&1; rc=$?; tail -3 gpurun_out/bench_rlhf.log; exit $rc
