# Round-4 GPU pass 3: EP capacity path on the GPU (tests + Mixtral --ep-shape 8 full depth), the
# TP chunk-split probe at 70B per-rank shapes, rocprof kernel tables (csv) of fused / unfused
# graph decode and of the DPO step. Raw traces stay in /tmp on the box; summaries come back.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4c
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() {  # dir out args...
  local tr=$(find "$1" -name '*kernel_trace.csv' | head -1)
  python3 $R/scripts/prof_window.py "$tr" "${@:3}" > "$2" && rm -rf "$1"
}
for v in "" "--fp8"; do
  timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8 --ep-capacity 1.25 $v --steps 3 --warmup 2 > $O/mixtral_ep8$v.log 2>&1 || { echo "MIXTRAL$v rc=$?"; tail -5 $O/mixtral_ep8$v.log; }
  tail -1 $O/mixtral_ep8$v.log
done
timeout -k 10 300 python -u tools/tp_chunk_probe.py > $O/tp_chunks.log 2>&1 || { tail -20 $O/tp_chunks.log; exit 1; }
cat $O/tp_chunks.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/pdec -o run -- python3 $R/tools/bench_generate.py --modes graph --new 128 > $R/$O/prof_dec.log 2>&1 || exit 1
summ /tmp/pdec $R/$O/prof_dec_fused.md --by-grid --top 30 --per 4096
DLA_DECODE_QKV_ATTN=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/pdec0 -o run -- python3 $R/tools/bench_generate.py --modes graph --new 128 > $R/$O/prof_dec0.log 2>&1 || exit 1
summ /tmp/pdec0 $R/$O/prof_dec_unfused.md --by-grid --top 30 --per 4096
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/pdec64 -o run -- python3 $R/tools/bench_generate.py --modes graph --new 128 --batch 64 --prompt 512 > $R/$O/prof_dec64.log 2>&1 || exit 1
summ /tmp/pdec64 $R/$O/prof_dec64.md --by-grid --top 30 --per 4096
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d /tmp/pdpo -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/$O/prof_dpo.log 2>&1 || exit 1
tr=$(find /tmp/pdpo -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/step_breakdown.py "$tr" > $R/$O/dpo_breakdown.md
python3 $R/scripts/prof_window.py "$tr" --window adamw --by-grid --top 60 > $R/$O/dpo_by_grid.md
rm -rf /tmp/pdpo
echo ALL_DONE
