#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in "65536 8192" "999999999 999999" "65536 8192" "999999999 999999"; do set -- $v; echo "max_n=$1 max_narrow_k=$2"; DLA_SKINNY_MAX_N=$1 DLA_SKINNY_MAX_NARROW_K=$2 timeout -k 10 200 python -u tools/bench_generate.py --modes graph,eager --new 128 2>/dev/null | grep mode || exit 1; done
