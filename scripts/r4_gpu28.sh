#!/bin/bash
# full GPU tier + smoke + bench (driver defaults) on the current tree
set -o pipefail
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tier.log 2>&1 || { tail -30 $O/gpu_tier.log; exit 1; }
tail -1 $O/gpu_tier.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
