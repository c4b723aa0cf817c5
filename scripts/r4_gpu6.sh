# Round-4 GPU pass 6: EP path on the GPU -- single-local-expert hipBLASLt GEMMs and the fused
# routing kernels (tests + Mixtral --ep-shape 8 A/B).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4f
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -x -q --timeout 120 --timeout-method thread > $O/moe_tests.log 2>&1 || { echo MOE_TESTS_FAILED; tail -30 $O/moe_tests.log; exit 1; }
tail -1 $O/moe_tests.log
for arm in "1 1" "1 0" "0 0" "1 1"; do
  set -- $arm
  DLA_MOE_SINGLE_LIB=$1 DLA_EP_NATIVE_ROUTE=$2 timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape 8 --micro-pairs 2 --accum 8 --ep-capacity 1.25 --steps 3 --warmup 2 > $O/mx_$1$2.log 2>&1 || { echo "MX$1$2 rc=$?"; tail -5 $O/mx_$1$2.log; exit 1; }
  echo "single_lib=$1 native_route=$2 $(tail -1 $O/mx_$1$2.log | cut -c1-260)"
done
echo ALL_DONE
