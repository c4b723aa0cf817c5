# Round-4 validation: decode GPU tests, decode A/B (fused qkv+attention on/off), headline bench,
# rocprofv3 kernel tables of the DPO step and of graph decode.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 500 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_dec_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r4_dec_tests.log; exit 1; }
tail -3 gpurun_out/r4_dec_tests.log
for arm in 1 0 1 0; do
  DLA_DECODE_QKV_ATTN=$arm timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > gpurun_out/r4_gen_b8_qa$arm.log 2>&1 || exit 1
  echo "qkv_attn=$arm $(tail -1 gpurun_out/r4_gen_b8_qa$arm.log)"
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_bench0.log 2>&1 || exit 1
tail -1 gpurun_out/r4_bench0.log
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4_prof_dpo -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/r4_prof_dpo.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4_prof_dec -o run -- python3 $R/tools/bench_generate.py --modes graph --new 128 > $R/gpurun_out/r4_prof_dec.log 2>&1 || exit 1
echo ALL_DONE
