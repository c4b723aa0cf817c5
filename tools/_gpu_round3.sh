#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/probe_var.log
for r in 1 2; do for b in attn_bwd_probe attn_bwd_probe_v1 attn_bwd_probe_v2; do
  echo "== $b" >> gpurun_out/probe_var.log
  timeout -k 10 60 tools/$b.bin 8 >> gpurun_out/probe_var.log 2>&1 || exit 1
done; done
grep -E "==|main kernel|ticks|chains|dV/dK" gpurun_out/probe_var.log
