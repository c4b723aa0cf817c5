# Round-4 end-state kernel tables: B=64 graph decode (m64 split rule) and the DPO step (bf16 dK/dV
# partials). Raw traces stay in /tmp on the box; summaries come back.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4e
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() {  # dir out args...
  local tr=$(find "$1" -name '*kernel_trace.csv' | head -1)
  python3 $R/scripts/prof_window.py "$tr" "${@:3}" > "$2" && rm -rf "$1"
}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/pdec64 -o run -- python3 $R/tools/bench_generate.py --modes graph --new 128 --batch 64 --prompt 512 > $R/$O/prof_dec64.log 2>&1 || exit 1
summ /tmp/pdec64 $R/$O/prof_dec64.md --by-grid --top 30 --per 4096
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d /tmp/pdpo -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/$O/prof_dpo.log 2>&1 || exit 1
tr=$(find /tmp/pdpo -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/step_breakdown.py "$tr" > $R/$O/dpo_breakdown.md
python3 $R/scripts/prof_window.py "$tr" --window adamw --by-grid --top 60 > $R/$O/dpo_by_grid.md
rm -rf /tmp/pdpo
echo ALL_DONE
