#!/bin/bash
# rocprofv3 kernel trace + PMC counter passes over the attention microbenchmark (1x MI355X).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_attn_trace -o t -- python -u tools/attn_bench.py --iters 10 > gpurun_out/prof_attn_trace.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d gpurun_out/prof_attn_pmc1 -o p -- python -u tools/attn_bench.py --iters 2 > gpurun_out/prof_attn_pmc1.log 2>&1 \
 && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/prof_attn_pmc2 -o p -- python -u tools/attn_bench.py --iters 2 > gpurun_out/prof_attn_pmc2.log 2>&1
echo "rc=$?"
find gpurun_out/prof_attn_* -name "*.csv" | head -20
