# Round-4 GPU pass 14: attention backward GQA head split A/B (1 vs 2 workgroups per kv head).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4n
mkdir -p $O
for r in 1 2 3; do
  for hs in 2 1; do
    DLA_ATTN_BWD_HSPLIT=$hs timeout -k 10 200 python -u tools/attn_bench.py > $O/attn_hs$hs.log 2>&1 || exit 1
    echo "hsplit=$hs $(grep '\[attn\]' $O/attn_hs$hs.log)"
  done
done
echo ALL_DONE
