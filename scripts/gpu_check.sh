#!/usr/bin/env bash
# GPU-box validation: kernel numerics tests, then the 1-GPU headline bench.
# Stops at the first crash / abort / timeout (exit codes other than pytest's 0/1).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import torch; print(torch.cuda.get_device_name(0), torch.version.hip)"
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed rc=$rc; stopping"; exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
brc=$?
tail -20 gpurun_out/bench.log
exit $(( rc != 0 ? rc : brc ))
