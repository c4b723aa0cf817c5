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
ACCEL_CFG="${ACCELERATE_CONFIG:-$REPO/config/accelerate_config.yaml}"
if [ -z "${NPROC:-}" ] || [ -z "${MASTER_PORT:-}" ]; then
  # reference contract: num_processes / main_process_port from the accelerate config, capped at
  # the GPUs actually visible (device_count() does not initialise HIP)
  read -r _NP _PORT < <(python - "$ACCEL_CFG" <<'PY'
import sys, yaml, torch
try:
    c = yaml.safe_load(open(sys.argv[1])) or {}
except OSError:
    c = {}
n = torch.cuda.device_count()
want = int(c.get("num_processes", n or 1))
print(max(1, min(want, n)) if n else 1, int(c.get("main_process_port", 29500)))
PY
)
  NPROC=${NPROC:-$_NP}
  MASTER_PORT=${MASTER_PORT:-$_PORT}
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
