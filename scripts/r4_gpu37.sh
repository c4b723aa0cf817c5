# PMC counters of the B=64 decode kernels (eager decode, 4 new tokens: the same fused-layer kernels
# as the graph), one counter pass within the per-block limits, summarised on the box.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4pd
mkdir -p $O
cd /tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE FETCH_SIZE"
timeout -s KILL 170 rocprofv3 --pmc $P1 --output-format csv -d /tmp/pmcd -o run -- python3 $R/tools/bench_generate.py --modes eager --new 4 --batch 64 --prompt 512 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
c1=$(find /tmp/pmcd -name '*counter_collection.csv' | head -1)
python3 $R/scripts/pmc_summary_csv.py "$c1" -k m64_gemm m64_reduce decode_attn_loop > $O/decode64_pmc.md
rm -rf /tmp/pmcd
cat $O/decode64_pmc.md
echo ALL_DONE
