set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && tail -3 gpurun_out/gpu_tests.log \
 && timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 && tail -2 gpurun_out/bench_default.log
