# Round-4 GPU pass 8: the whole GPU test tier (as the driver runs it) and smoke().
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tier.log 2>&1
rc=$?
tail -3 $O/gpu_tier.log
grep -E "FAILED|ERROR" $O/gpu_tier.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
