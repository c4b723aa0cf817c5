#!/bin/bash
# Overlapped optimizer step: GPU equivalence tests, then interleaved A/B of the headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "engine or overlapped or dpo or fsdp" 2>&1 | tail -2 || exit 1
for v in 1 0 1 0; do echo -n "overlap_opt=$v "; DLA_OVERLAP_OPT=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 2>/dev/null | python -c "import json,sys; r=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'], r['config']['final_loss'])" || exit 1; done
