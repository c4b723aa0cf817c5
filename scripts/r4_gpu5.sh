# Round-4 GPU pass 5: fused decode qkv+attention tile deal A/B (DLA_QA_TA) vs the two launches.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4e
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for r in 1 2; do
  for arm in "0 -1" "1 1" "1 2"; do
    set -- $arm
    DLA_DECODE_QKV_ATTN=$1 DLA_QA_TA=$2 timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > $O/gen_$1_$2.log 2>&1 || exit 1
    echo "qkv_attn=$1 ta=$2 $(tail -1 $O/gen_$1_$2.log)"
  done
done
echo ALL_DONE
