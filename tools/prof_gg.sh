#!/bin/bash
# PMC passes over the grouped expert GEMM (one counter group per run; gfx950 SQ block: 8 slots).
# usage (on the GPU box): bash tools/prof_gg.sh "<case substring>" <sched>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gg_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CASE=${1:-up+swiglu fwd}
SCHED=${2:-0}
export DLA_GG_SCHED=$SCHED
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- \
    python3 $R/tools/grouped_gemm_bench.py --only "$CASE" --scheds $SCHED --iters 3 --blocks 0 --no-loop > $OUT/p$i.log 2>&1
done
python3 $R/scripts/pmc_summary_csv.py $(find $OUT -name "*counter_collection.csv") -k grouped_gemm > $OUT/summary.md
cat $OUT/summary.md
