# Round-4 GPU pass 9: Mixtral --ep-shape 8 fp8 expert forward and a kernel profile of the bf16 step
# on the round-4 EP path (hipBLASLt single-expert GEMMs, fused routing).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4i
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8 --ep-capacity 1.25 --fp8 --steps 3 --warmup 2 > $O/mx_fp8.log 2>&1 || { tail -5 $O/mx_fp8.log; exit 1; }
echo "fp8 $(tail -1 $O/mx_fp8.log | cut -c1-300)"
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d /tmp/pmx -o run -- python3 $R/bench.py --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8 --ep-capacity 1.25 --steps 2 --warmup 1 > $R/$O/prof_mixtral.log 2>&1 || exit 1
tr=$(find /tmp/pmx -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/step_breakdown.py "$tr" > $R/$O/mixtral_breakdown.md
python3 $R/scripts/prof_window.py "$tr" --window adamw --top 40 > $R/$O/mixtral_top.md
rm -rf /tmp/pmx
echo ALL_DONE
