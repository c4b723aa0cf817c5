# Round-4 GPU pass 15: B=64 decode attention split target A/B (DLA_DECODE_BLOCKS).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r4o
mkdir -p $O
for r in 1 2; do
  for tb in 256 1024 640; do
    DLA_DECODE_BLOCKS=$tb timeout -k 10 300 python -u tools/bench_generate.py --modes graph --new 128 --batch 64 --prompt 512 > $O/gen64_tb$tb.log 2>&1 || exit 1
    echo "blocks=$tb $(tail -1 $O/gen64_tb$tb.log | cut -c1-200)"
  done
done
echo ALL_DONE
