#!/bin/bash
# r2: full GPU test tier + a 2-rank RCCL probe on ONE GPU (tiny model) to exercise the
# multi-rank NCCL/RCCL code path when only one MI355X is available.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
NCCL_DEBUG=WARN timeout -k 10 180 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --model tiny-llama-d128 --steps 3 --warmup 1 --seq-len 256 > gpurun_out/rccl_same_gpu.log 2>&1
echo "same-gpu rccl rc=$?"; tail -5 gpurun_out/rccl_same_gpu.log
