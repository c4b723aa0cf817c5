"""`src.models.reward_model` names (reference src/models/reward_model.py): native RewardModel,
builder, fused pairwise loss, and the (unused upstream) `RewardArtifacts` record."""
from dataclasses import dataclass
from typing import Any, Literal

from distributed_llm_alignment_amd.models.loader import build_reward_model  # noqa: F401
from distributed_llm_alignment_amd.models.reward import RewardModel  # noqa: F401
from distributed_llm_alignment_amd.ops.losses import pairwise_loss  # noqa: F401

Pooling = Literal["last_token", "mean"]


@dataclass
class RewardArtifacts:
    model: Any
    tokenizer: Any
