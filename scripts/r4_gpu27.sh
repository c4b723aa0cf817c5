#!/bin/bash
# RLHF 64 rollouts on one GPU: update as 8 micro-batches of 8 (per-micro baseline = the 8-rank DDP
# gradient, no recompute) vs one batch with full recompute
set -o pipefail
O=gpurun_out/r4_rlhf64; mkdir -p $O
timeout -k 10 600 python -u tools/bench_rlhf.py --batch 64 --micro 8 > $O/micro8.log 2>&1 || { tail -20 $O/micro8.log; exit 1; }
tail -1 $O/micro8.log
timeout -k 10 600 python -u tools/bench_rlhf.py --batch 64 --micro 16 > $O/micro16.log 2>&1 || { tail -20 $O/micro16.log; exit 1; }
tail -1 $O/micro16.log
timeout -k 10 600 python -u tools/bench_rlhf.py --batch 64 --grad-ckpt full > $O/full.log 2>&1 || { tail -20 $O/full.log; exit 1; }
tail -1 $O/full.log
