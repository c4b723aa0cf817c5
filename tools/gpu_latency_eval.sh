#!/bin/bash
# The reference's latency harness grid (eval_latency) on 1x MI355X, results -> gpurun_out/latency.json
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m distributed_llm_alignment_amd.eval.eval_latency --config config/eval_latency_mi355x.yaml \
  --override logging.output_path=gpurun_out/results.json > gpurun_out/latency.log 2>&1 || { tail -20 gpurun_out/latency.log; exit 1; }
python -c "
import json; r = json.load(open('gpurun_out/latency.json'))
for m, rows in r.items():
    for x in rows:
        print(m, x['batch_size'], x['seq_length'], round(x['tokens_per_second']), round(x['latency_ms'], 2), round(x.get('decode_ms_per_token', 0), 2))
"
