#!/usr/bin/env bash
# Teacher rollouts, prompts sharded over all GPUs: scripts/launch_teacher_gen.sh --teacher T --prompts P --output O [...]
source "$(dirname "${BASH_SOURCE[0]}")/_launch_common.sh"
dla_run distributed_llm_alignment_amd.training.generate_teacher_data "$@"
