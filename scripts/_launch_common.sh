#!/usr/bin/env bash
# Shared launcher: one process per GPU over RCCL (torch "nccl" backend) on this node.
#   NPROC=<ranks> (default: visible GPUs, or 1 on CPU), MASTER_PORT (default 29500).
set -euo pipefail
export TOKENIZERS_PARALLELISM=false
export HSA_ENABLE_IPC_MODE_LEGACY=0          # dmabuf IPC for RCCL peer buffers
export NCCL_MIN_NCHANNELS=${NCCL_MIN_NCHANNELS:-16}   # keep all 7 xGMI links busy
if [ "${DLA_DEBUG:-0}" = "1" ]; then   # serialised HIP + loud RCCL errors
  export AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 TORCH_NCCL_ASYNC_ERROR_HANDLING=1 NCCL_DEBUG=WARN
fi
REPO="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
export PYTHONPATH="$REPO${PYTHONPATH:+:$PYTHONPATH}"
if [ -z "${NPROC:-}" ]; then
  NPROC=$(python -c "import torch; print(max(1, torch.cuda.device_count()))")
fi
dla_run() {  # dla_run <module> [args...]
  local mod="$1"; shift
  if [ "$NPROC" -gt 1 ]; then
    exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NPROC" \
      --master-addr 127.0.0.1 --master-port "${MASTER_PORT:-29500}" -m "$mod" "$@"
  else
    exec python -m "$mod" "$@"
  fi
}
