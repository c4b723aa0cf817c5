# Round-4 GPU pass 10: decode loop attention with all chunks in flight (DLA_DECODE_RING=3):
# decode tests under it, then the B=8 A/B, and the round-4 attention microbench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4j
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
DLA_DECODE_RING=3 timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > $O/dec_tests_ring3.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/dec_tests_ring3.log; exit 1; }
tail -1 $O/dec_tests_ring3.log
for r in 1 2; do
  for arm in 2 3; do
    DLA_DECODE_RING=$arm timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > $O/gen_ring$arm.log 2>&1 || exit 1
    echo "ring=$arm $(tail -1 $O/gen_ring$arm.log)"
  done
done
timeout -k 10 300 python -u tools/attn_bench.py > $O/attn_bench.log 2>&1 || exit 1
tail -6 $O/attn_bench.log
echo ALL_DONE
