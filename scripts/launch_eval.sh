#!/usr/bin/env bash
# Alignment heuristics + prefill/decode latency for every model in the eval config (1 GPU).
source "$(dirname "${BASH_SOURCE[0]}")/_launch_common.sh"
CONFIG=${1:-config/eval_config.yaml}
python -m distributed_llm_alignment_amd.eval.eval_alignment --config "$CONFIG"
python -m distributed_llm_alignment_amd.eval.eval_latency --config "$CONFIG"
