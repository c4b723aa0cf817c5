# Round-4 GPU pass 13: DPO micro-batch shape A/B at the same 16 pairs/step (4 x 4 vs 2 x 8).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4m
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for r in 1 2; do
  for arm in "4 4" "8 2"; do
    set -- $arm
    timeout -k 10 400 python -u bench.py --micro-pairs $1 --accum $2 --steps 6 --warmup 2 > $O/dpo_mb$1.log 2>&1 || { echo "MB$1 rc=$?"; tail -3 $O/dpo_mb$1.log; continue; }
    echo "micro=$1x$2 $(tail -1 $O/dpo_mb$1.log | cut -c1-200)"
  done
done
echo ALL_DONE
