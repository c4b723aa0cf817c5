# Round-4 GPU pass 12: DPO A/B -- qkv / o weight gradients without the TN transposes.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4l
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for r in 1 2; do
  for arm in 0 50000000; do
    DLA_TN_WGRAD_MIN=$arm timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/dpo_min$arm.log 2>&1 || exit 1
    echo "tn_min=$arm $(tail -1 $O/dpo_min$arm.log | cut -c1-200)"
  done
done
echo ALL_DONE
