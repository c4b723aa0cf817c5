"""`src.models.reward_model` names: native RewardModel, builder and fused pairwise loss."""
from distributed_llm_alignment_amd.models.loader import build_reward_model  # noqa: F401
from distributed_llm_alignment_amd.models.reward import RewardModel  # noqa: F401
from distributed_llm_alignment_amd.ops.losses import pairwise_loss  # noqa: F401
