#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_rlhf.py --steps 3 --warmup 1 > gpurun_out/r3_rlhf_serial.log 2>&1 || { tail -20 gpurun_out/r3_rlhf_serial.log; exit 1; }
tail -1 gpurun_out/r3_rlhf_serial.log
timeout -k 10 400 python -u tools/bench_rlhf.py --steps 3 --warmup 1 --overlap > gpurun_out/r3_rlhf_overlap.log 2>&1 || { tail -20 gpurun_out/r3_rlhf_overlap.log; exit 1; }
tail -1 gpurun_out/r3_rlhf_overlap.log
