"""`src.models.base_model` names on the native model zoo (no HF modeling, one device per rank)."""
from distributed_llm_alignment_amd.models.loader import (  # noqa: F401
    ModelBundle, count_trainable_params, freeze_except_lora, load_causal_lm)
