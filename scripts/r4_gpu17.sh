# Round-4 GPU pass 17: attention forward with P.V issued per key sub-tile (VALU exp of sub-tile 1
# beside sub-tile 0's MFMAs) vs the previous build (_C_ab_old.so), separate processes alternating.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn or attention" > $O/attn_tests.log 2>&1 || { tail -30 $O/attn_tests.log; exit 1; }
tail -1 $O/attn_tests.log
for r in 1 2 3; do
  for lib in old new; do
    if [ $lib = old ]; then export DLA_EXT_PATH=$R/distributed_llm_alignment_amd/_C_ab_old.so; else unset DLA_EXT_PATH; fi
    timeout -k 10 200 python -u tools/attn_bench.py --ab DLA_ATTN_DQ_BF16=1,1 --rounds 3 > $O/ab_$lib.log 2>&1 || exit 1
    echo "$lib $(grep 'attn-ab' $O/ab_$lib.log | head -1)"
  done
done
unset DLA_EXT_PATH
timeout -k 10 200 python -u tools/attn_bench.py --noncausal --ab DLA_ATTN_DQ_BF16=1,1 --rounds 3 > $O/ab_nc.log 2>&1 || exit 1
echo "noncausal new $(grep 'attn-ab' $O/ab_nc.log | head -1)"
echo ALL_DONE
