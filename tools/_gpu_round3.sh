#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "attention or qkv" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_attn_tests.log 2>&1 || { tail -30 gpurun_out/r3_attn_tests.log; exit 1; }
tail -1 gpurun_out/r3_attn_tests.log
timeout -k 10 60 tools/attn_bwd_probe.bin 8 > gpurun_out/probe.log 2>&1 || { cat gpurun_out/probe.log; exit 1; }
grep -v "tile 10" gpurun_out/probe.log
timeout -k 10 200 python -u tools/attn_bench.py --ab DLA_ATTN_BWD_WAVES=4,8 --rounds 3 > gpurun_out/r3_attn_ab.log 2>&1 || { tail -20 gpurun_out/r3_attn_ab.log; exit 1; }
for hs in 1 2 4; do DLA_ATTN_BWD_WAVES=8 DLA_ATTN_BWD_HSPLIT=$hs timeout -k 10 100 python -u tools/attn_bench.py >> gpurun_out/r3_attn_ab.log 2>&1 || exit 1; done
grep attn gpurun_out/r3_attn_ab.log
