# Round-4 GPU pass 2: persistent fused qkv+attention decode (tests + A/B + profile), DPO step
# profile by GEMM grid, RLHF/PPO/Mixtral-EP shape benches. Raw rocprof traces are summarised on
# the box (scripts/prof_window.py) and deleted: only small files come back.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r4b
( while true; do date > gpurun_out/r4b/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() {  # dir out args...
  local tr=$(find "$1" -name '*kernel_trace.csv' | head -1)
  python3 $R/scripts/prof_window.py "$tr" "${@:3}" > "$2" && rm -rf "$1"
}
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b/dec_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r4b/dec_tests.log; exit 1; }
tail -2 gpurun_out/r4b/dec_tests.log
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn or attention or flash" > gpurun_out/r4b/attn_tests.log 2>&1 || { echo ATTN_TESTS_FAILED; tail -40 gpurun_out/r4b/attn_tests.log; exit 1; }
tail -2 gpurun_out/r4b/attn_tests.log
for arm in 1 0; do
  DLA_ATTN_DQ_BF16=$arm timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 > gpurun_out/r4b/dpo_dq$arm.log 2>&1 || exit 1
  echo "dq_bf16=$arm $(tail -1 gpurun_out/r4b/dpo_dq$arm.log)"
done
for arm in 1 0 1 0; do
  DLA_DECODE_QKV_ATTN=$arm timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > gpurun_out/r4b/gen_b8_qa$arm.log 2>&1 || exit 1
  echo "qkv_attn=$arm $(tail -1 gpurun_out/r4b/gen_b8_qa$arm.log)"
done
for arm in 1 0; do
  DLA_DECODE_SLAB_ATTN=$arm timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 --batch 64 --prompt 512 > gpurun_out/r4b/gen_b64_sl$arm.log 2>&1 || exit 1
  echo "b64 slab_attn=$arm $(tail -1 gpurun_out/r4b/gen_b64_sl$arm.log)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pdec -o run -- python3 $R/tools/bench_generate.py --modes graph --new 128 > $R/gpurun_out/r4b/prof_dec.log 2>&1 || exit 1
summ /tmp/pdec $R/gpurun_out/r4b/prof_dec_fused.md --by-grid --top 25 --per 4096
DLA_DECODE_QKV_ATTN=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pdec0 -o run -- python3 $R/tools/bench_generate.py --modes graph --new 128 > $R/gpurun_out/r4b/prof_dec0.log 2>&1 || exit 1
summ /tmp/pdec0 $R/gpurun_out/r4b/prof_dec_unfused.md --by-grid --top 25 --per 4096
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d /tmp/pdpo -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/r4b/prof_dpo.log 2>&1 || exit 1
tr=$(find /tmp/pdpo -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/step_breakdown.py "$tr" > $R/gpurun_out/r4b/dpo_breakdown.md
python3 $R/scripts/prof_window.py "$tr" --window adamw --by-grid --top 60 > $R/gpurun_out/r4b/dpo_by_grid.md
rm -rf /tmp/pdpo
cd $R
timeout -k 10 400 python -u tools/bench_rlhf.py --batch 8 > gpurun_out/r4b/rlhf_b8.log 2>&1 || exit 1
tail -1 gpurun_out/r4b/rlhf_b8.log
timeout -k 10 600 python -u tools/bench_rlhf.py --algorithm ppo --zero-shape 8 --batch 8 --grad-ckpt full > gpurun_out/r4b/ppo_z8.log 2>&1 || exit 1
tail -1 gpurun_out/r4b/ppo_z8.log
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape 8 --steps 3 --warmup 2 > gpurun_out/r4b/mixtral_ep8.log 2>&1 || exit 1
tail -1 gpurun_out/r4b/mixtral_ep8.log
echo ALL_DONE
