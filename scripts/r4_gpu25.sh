#!/bin/bash
# B=8 decode attention: fewer, longer blocks with the 3-deep ring (existing knobs)
set -o pipefail
O=gpurun_out/r4_fewblk; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h decode_ms $O/$n.log | sed 's/.*decode_ms_per_token": \([0-9.]*\).*/\1/')"
}
for r in 1 2; do
  run base$r DLA_DECODE_RING=2
  run b64r3_$r DLA_DECODE_BLOCKS=64 DLA_DECODE_RING=3
  run b128r3_$r DLA_DECODE_BLOCKS=128 DLA_DECODE_RING=3
  run b96r3_$r DLA_DECODE_BLOCKS=96 DLA_DECODE_RING=3
  run b64r2_$r DLA_DECODE_BLOCKS=64 DLA_DECODE_RING=2
done
