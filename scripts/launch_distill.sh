#!/usr/bin/env bash
# distill stage on all GPUs of this node: scripts/launch_distill.sh [CONFIG] [--override k=v ...]
source "$(dirname "${BASH_SOURCE[0]}")/_launch_common.sh"
CONFIG=${1:-config/distill_config.yaml}; shift || true
dla_run distributed_llm_alignment_amd.training.train_distill --config "$CONFIG" "$@"
