#!/usr/bin/env bash
# Teacher-ensemble KL distillation: enables use_kl/on_policy; pass teachers via the config's
# distill.teacher_model_names_or_paths (or --override distill.teacher_model_names_or_paths=[a,b]).
source "$(dirname "${BASH_SOURCE[0]}")/_launch_common.sh"
CONFIG=${1:-config/distill_config.yaml}; shift || true
dla_run distributed_llm_alignment_amd.training.train_distill --config "$CONFIG" \
  --override distill.use_kl=true --override distill.on_policy=true "$@"
