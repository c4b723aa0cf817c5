#!/usr/bin/env bash
# rlhf stage on all GPUs of this node: scripts/launch_rlhf.sh [CONFIG] [--override k=v ...]
source "$(dirname "${BASH_SOURCE[0]}")/_launch_common.sh"
CONFIG=${1:-config/rlhf_config.yaml}; shift || true
dla_run distributed_llm_alignment_amd.training.train_rlhf --config "$CONFIG" "$@"
