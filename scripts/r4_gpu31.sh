#!/bin/bash
# torch.profiler op table (by input shape) of one Mixtral EP-shape step: where the non-GEMM
# elementwise / copy / fill time comes from
set -o pipefail
O=gpurun_out/r4_mixops; mkdir -p $O
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape 8 --steps 1 --warmup 2 --profile-dir /tmp/mixprof > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
cp /tmp/mixprof/kernels.txt /tmp/mixprof/ops_by_shape.txt $O/
tail -1 $O/run.log | cut -c1-150
