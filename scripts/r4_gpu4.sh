# Round-4 GPU pass 4: fused qkv+attention with the write-through hand-off (tests, same-box A/B,
# kernel table), RLHF B=8 on the default path, PPO without activation recompute.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4d
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() {  # dir out args...
  local tr=$(find "$1" -name '*kernel_trace.csv' | head -1)
  python3 $R/scripts/prof_window.py "$tr" "${@:3}" > "$2" && rm -rf "$1"
}
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused_qkv or slab or fsdp" > $O/dec_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/dec_tests.log; exit 1; }
tail -2 $O/dec_tests.log
for arm in 1 0 1 0; do
  DLA_DECODE_QKV_ATTN=$arm timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > $O/gen_b8_qa$arm.log 2>&1 || exit 1
  echo "qkv_attn=$arm $(tail -1 $O/gen_b8_qa$arm.log)"
done
cd /tmp
DLA_DECODE_QKV_ATTN=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/pdec -o run -- python3 $R/tools/bench_generate.py --modes graph --new 128 > $R/$O/prof_dec.log 2>&1 || exit 1
summ /tmp/pdec $R/$O/prof_dec_fused.md --by-grid --top 30 --per 4096
cd $R
timeout -k 10 400 python -u tools/bench_rlhf.py --batch 8 > $O/rlhf_b8.log 2>&1 || exit 1
tail -1 $O/rlhf_b8.log
timeout -k 10 600 python -u tools/bench_rlhf.py --algorithm ppo --zero-shape 8 --batch 8 > $O/ppo_z8_nockpt.log 2>&1 || { echo "PPO_NOCKPT rc=$?"; tail -3 $O/ppo_z8_nockpt.log; }
tail -1 $O/ppo_z8_nockpt.log
timeout -k 10 300 python -u tools/grouped_gemm_bench.py --scheds 0,3 --rounds 2 > $O/gg_bench.log 2>&1 || { echo "GG rc=$?"; tail -3 $O/gg_bench.log; }
grep '^{' $O/gg_bench.log | tail -12
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d /tmp/pmx -o run -- python3 $R/bench.py --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8 --ep-capacity 1.25 --steps 2 --warmup 1 > $R/$O/prof_mixtral.log 2>&1 || exit 1
tr=$(find /tmp/pmx -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/step_breakdown.py "$tr" > $R/$O/mixtral_breakdown.md
python3 $R/scripts/prof_window.py "$tr" --window adamw --top 45 > $R/$O/mixtral_top.md
rm -rf /tmp/pmx
echo ALL_DONE
