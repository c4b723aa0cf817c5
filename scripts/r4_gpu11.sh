# Round-4 GPU pass 11: decode loop attention with early K refills (DLA_DECODE_EARLYK=1): tests,
# B=8 / B=64 A/B; attention backward A/B of the bf16 dQ slabs.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4k
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
DLA_DECODE_EARLYK=1 timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > $O/dec_tests_earlyk.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/dec_tests_earlyk.log; exit 1; }
tail -1 $O/dec_tests_earlyk.log
for r in 1 2; do
  for arm in 0 1; do
    DLA_DECODE_EARLYK=$arm timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > $O/gen8_ek$arm.log 2>&1 || exit 1
    echo "B8 earlyk=$arm $(tail -1 $O/gen8_ek$arm.log | cut -c1-200)"
    DLA_DECODE_EARLYK=$arm timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 --batch 64 --prompt 512 > $O/gen64_ek$arm.log 2>&1 || exit 1
    echo "B64 earlyk=$arm $(tail -1 $O/gen64_ek$arm.log | cut -c1-200)"
  done
done
timeout -k 10 400 python -u tools/attn_bench.py --ab DLA_ATTN_DQ_BF16=1,0 --rounds 3 > $O/attn_ab.log 2>&1 || exit 1
tail -8 $O/attn_ab.log
echo ALL_DONE
