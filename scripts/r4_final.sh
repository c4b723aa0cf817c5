# Round-4 final validation on one MI355X: the GPU test tier, smoke(), and bench.py as the driver
# runs it (no flags), plus the decode / RLHF / PPO / Mixtral-EP numbers on the same box.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4z
mkdir -p $O
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tier.log 2>&1 || { tail -30 $O/gpu_tier.log; exit 1; }
tail -1 $O/gpu_tier.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 > $O/gen8.log 2>&1 || exit 1
tail -1 $O/gen8.log
timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 --batch 64 --prompt 512 > $O/gen64.log 2>&1 || exit 1
tail -1 $O/gen64.log
timeout -k 10 400 python -u tools/bench_rlhf.py --batch 8 > $O/rlhf8.log 2>&1 || exit 1
tail -1 $O/rlhf8.log
timeout -k 10 600 python -u tools/bench_rlhf.py --batch 64 --grad-ckpt full > $O/rlhf64.log 2>&1 || exit 1
tail -1 $O/rlhf64.log
timeout -k 10 600 python -u tools/bench_rlhf.py --algorithm ppo --zero-shape 8 --batch 8 > $O/ppo.log 2>&1 || exit 1
tail -1 $O/ppo.log | cut -c1-300
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape 8 --steps 3 --warmup 2 > $O/mixtral.log 2>&1 || exit 1
tail -1 $O/mixtral.log | cut -c1-300
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ep-shape 8 --fp8 --steps 3 --warmup 2 > $O/mixtral_fp8.log 2>&1 || exit 1
tail -1 $O/mixtral_fp8.log | cut -c1-300
timeout -k 10 600 python -u tools/bench_rlhf.py --batch 64 --micro 8 > $O/rlhf64_micro8.log 2>&1 || exit 1
tail -1 $O/rlhf64_micro8.log
echo ALL_DONE
