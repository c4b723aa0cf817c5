#!/bin/bash
# Round-2 first GPU pass (1x MI355X): smoke, headline bench (1 GPU), then the 70B and Mixtral
# north-star architectures at full width / reduced depth, with a rocprofv3 kernel summary each.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_8b.log 2>&1 || { tail -20 gpurun_out/bench_8b.log; exit 1; }
tail -1 gpurun_out/bench_8b.log
timeout -k 10 400 python -u bench.py --model llama3-70b --layers 4 --steps 4 --warmup 2 > gpurun_out/bench_70b_l4.log 2>&1 || { tail -20 gpurun_out/bench_70b_l4.log; exit 1; }
tail -1 gpurun_out/bench_70b_l4.log
timeout -k 10 400 python -u bench.py --model mixtral-8x7b --layers 2 --steps 4 --warmup 2 > gpurun_out/bench_mix_l2.log 2>&1 || { tail -20 gpurun_out/bench_mix_l2.log; exit 1; }
tail -1 gpurun_out/bench_mix_l2.log
timeout -k 10 400 python -u bench.py --model mixtral-8x7b --layers 2 --fp8 --steps 4 --warmup 2 > gpurun_out/bench_mix_l2_fp8.log 2>&1 || { tail -20 gpurun_out/bench_mix_l2_fp8.log; exit 1; }
tail -1 gpurun_out/bench_mix_l2_fp8.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_70b -o p -- python -u bench.py --model llama3-70b --layers 4 --steps 2 --warmup 1 > gpurun_out/prof_70b.log 2>&1 || { tail -20 gpurun_out/prof_70b.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mix -o p -- python -u bench.py --model mixtral-8x7b --layers 2 --fp8 --steps 2 --warmup 1 > gpurun_out/prof_mix.log 2>&1 || { tail -20 gpurun_out/prof_mix.log; exit 1; }
echo done
