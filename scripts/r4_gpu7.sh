# Round-4 GPU pass 7: DPO A/B -- LM-head weight gradient without the TN transposes.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4g
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for r in 1 2; do
  for arm in "" "300000000"; do
    DLA_TN_WGRAD_MAX=${arm:-4611686018427387904} timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/dpo_tn$arm.log 2>&1 || exit 1
    echo "tn_max=${arm:-inf} $(tail -1 $O/dpo_tn$arm.log | cut -c1-200)"
  done
done
echo ALL_DONE
