#!/usr/bin/env bash
# dpo stage on all GPUs of this node: scripts/launch_dpo.sh [CONFIG] [--override k=v ...]
source "$(dirname "${BASH_SOURCE[0]}")/_launch_common.sh"
CONFIG=${1:-config/dpo_config.yaml}; shift || true
dla_run distributed_llm_alignment_amd.training.train_dpo --config "$CONFIG" "$@"
