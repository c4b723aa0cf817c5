# Round-4 GPU pass 16: PMC counters of the attention kernels (fwd, 8-wave bwd, dQ reduce), two
# counter passes (each within the per-block limits), summarised on the box.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4p
mkdir -p $O
cd /tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS GRBM_COUNT"
timeout -s KILL 150 rocprofv3 --pmc $P1 --output-format csv -d /tmp/pmc1 -o run -- python3 $R/tools/attn_bench.py --iters 3 > $O/pmc1.log 2>&1 || { tail -5 $O/pmc1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $P2 --output-format csv -d /tmp/pmc2 -o run -- python3 $R/tools/attn_bench.py --iters 3 > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
c1=$(find /tmp/pmc1 -name '*counter_collection.csv' | head -1)
c2=$(find /tmp/pmc2 -name '*counter_collection.csv' | head -1)
python3 $R/scripts/pmc_summary_csv.py "$c1" "$c2" -k attn_fwd attn_bwd8 attn_dq_reduce attn_dkv_reduce > $O/attn_pmc.md
rm -rf /tmp/pmc1 /tmp/pmc2
head -60 $O/attn_pmc.md
echo ALL_DONE
