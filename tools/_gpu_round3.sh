set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_gpu_tests3.log 2>&1
rc=$?; tail -3 gpurun_out/r3_gpu_tests3.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r3_gpu_tests3.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench1.log 2>&1 || { tail -5 gpurun_out/r3_bench1.log; exit 1; }
tail -1 gpurun_out/r3_bench1.log
timeout -k 10 120 python -u tools/bench_handoff.py > gpurun_out/r3_handoff.log 2>&1 || exit 1
cat gpurun_out/r3_handoff.log
timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 --batch 64 --prompt 512 > gpurun_out/r3_gen64.log 2>&1 || exit 1
tail -1 gpurun_out/r3_gen64.log
