#!/bin/bash
# torch.profiler op table (by input shape) of one Llama-3-8B DPO step
set -o pipefail
O=gpurun_out/r4_dpoops; mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 1 --warmup 2 --profile-dir /tmp/dpoprof > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
cp /tmp/dpoprof/kernels.txt /tmp/dpoprof/ops_by_shape.txt $O/
tail -1 $O/run.log | cut -c1-150
