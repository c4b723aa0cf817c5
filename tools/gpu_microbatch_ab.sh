#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "--micro-pairs 4 --accum 4" "--micro-pairs 8 --accum 2" "--micro-pairs 16 --accum 1" "--micro-pairs 4 --accum 4"; do
  echo -n "$cfg: "; timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 $cfg 2>/dev/null | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'])" || exit 1
done
for hs in 1 2 4; do echo -n "hsplit=$hs: "; DLA_ATTN_BWD_HSPLIT=$hs timeout -k 10 120 python -u tools/attn_bench.py --iters 30 2>/dev/null | grep attn || exit 1; done
