#!/bin/bash
# m64 decode projections: split-K workgroup target A/B (tools/m64_probe.py), one process per arm
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/m64_probe.jsonl
: > $out
for wg in 256 512 768 128 256; do
  DLA_M64_WG=$wg timeout -k 10 120 python -u tools/m64_probe.py >> $out 2>> gpurun_out/m64_probe.err || exit $?
done
DLA_DECODE_NT=0 timeout -k 10 120 python -u tools/m64_probe.py >> $out 2>> gpurun_out/m64_probe.err || exit $?
cat $out
