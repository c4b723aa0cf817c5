# Round-4 GPU pass 19: persistent attention forward (DLA_ATTN_FWD_PERSIST=1): bitwise check against
# the standard kernel, the attention fp32-oracle tests under it, and a same-box A/B.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4s
mkdir -p $O
DLA_ATTN_FWD_PERSIST=0 timeout -k 10 200 python -u scripts/attn_fwd_bitwise.py /tmp/attn_ref.pt > $O/bitwise0.log 2>&1 || { tail -5 $O/bitwise0.log; exit 1; }
DLA_ATTN_FWD_PERSIST=1 timeout -k 10 200 python -u scripts/attn_fwd_bitwise.py /tmp/attn_ref.pt --compare > $O/bitwise1.log 2>&1; rc=$?
tail -6 $O/bitwise1.log
[ $rc -le 1 ] || exit 1
DLA_ATTN_FWD_PERSIST=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn or attention" > $O/attn_tests.log 2>&1 || { tail -30 $O/attn_tests.log; exit 1; }
tail -1 $O/attn_tests.log
for r in 1 2 3; do
  for arm in 0 1; do
    DLA_ATTN_FWD_PERSIST=$arm timeout -k 10 200 python -u tools/attn_bench.py --ab DLA_ATTN_DQ_BF16=1,1 --rounds 3 > $O/ab_$arm.log 2>&1 || exit 1
    echo "persist=$arm $(grep 'attn-ab' $O/ab_$arm.log | head -1)"
  done
done
DLA_ATTN_FWD_PERSIST=1 timeout -k 10 200 python -u tools/attn_bench.py --noncausal --ab DLA_ATTN_DQ_BF16=1,1 --rounds 3 > $O/ab_nc1.log 2>&1 || exit 1
echo "noncausal persist=1 $(grep 'attn-ab' $O/ab_nc1.log | head -1)"
echo ALL_DONE
