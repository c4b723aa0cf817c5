set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "fused or graph or skinny or head_dim or attention" > gpurun_out/r3_dec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_dec_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r3_dec_tests.log | head -30; exit $rc; }
python -u tools/gpu_ab.py --cmd "python -u tools/bench_generate.py --modes graph --new 128" --arm base:DLA_DECODE_FUSED_NORM=0 --arm fused:DLA_DECODE_FUSED_NORM=1 --rounds 2 --timeout 200 --key decode_ms_per_token --out gpurun_out/r3_decode_ab.jsonl || exit 1
python -u tools/gpu_ab.py --cmd "python -u tools/attn_bench.py --D 80 --Hq 32 --Hkv 32 --T 2048 --B 4 --iters 20" --arm native:DLA_ATTN_D80=1 --arm padded:DLA_ATTN_D80=0 --rounds 2 --timeout 120 --metric-re "fwd ([0-9.]+) us" --out gpurun_out/r3_d80_ab.jsonl || exit 1
for f in gpurun_out/ab_native_*.log gpurun_out/ab_padded_*.log; do echo "$f: $(tail -1 $f)"; done
DLA_DECODE_FUSED_NORM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dec1 -o d -- python -u tools/bench_generate.py --modes graph --new 128 > gpurun_out/prof_dec1.log 2>&1 || exit 1
f=$(find gpurun_out/prof_dec1 -name "*kernel_stats.csv" | head -1)
python scripts/prof_summary.py $f 14 > gpurun_out/prof_dec1_summary.md
cat gpurun_out/prof_dec1_summary.md
