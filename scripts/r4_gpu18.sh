# Round-4 GPU pass 18: Mixtral per-rank shapes at EP = 4 and 2 (2 / 4 local experts per layer,
# grouped expert kernels with the fused routing).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4r
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for ep in 4 2; do
  timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape $ep --micro-pairs 2 --accum 8 --ep-capacity 1.25 --steps 3 --warmup 2 > $O/mx_ep$ep.log 2>&1 || { echo "EP$ep rc=$?"; tail -3 $O/mx_ep$ep.log; continue; }
  echo "ep=$ep $(tail -1 $O/mx_ep$ep.log | cut -c1-330)"
done
echo ALL_DONE
