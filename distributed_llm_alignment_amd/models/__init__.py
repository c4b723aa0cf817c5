"""Native model zoo: Llama-3 / Mistral / Mixtral / GPT-2 / phi-2 decoders + reward model."""
from .config import HUB_ALIASES, PRESETS, ModelConfig, get_config
from .generation import GenerationConfig, KVCache, generate, sample_next
from .loader import (ModelBundle, build_reward_model, build_value_model, count_trainable_params, default_device,
                     freeze_except_lora, load_causal_lm, load_reward_checkpoint, read_state_dict,
                     save_hf_pretrained)
from .reward import RewardModel, ValueModel
from .tokenizer import ByteTokenizer, load_tokenizer
from .transformer import CausalLM, attention_layout, build_model, default_dtype

__all__ = [
    "HUB_ALIASES", "PRESETS", "ModelConfig", "get_config", "GenerationConfig", "KVCache",
    "generate", "sample_next", "ModelBundle", "build_reward_model", "build_value_model",
    "count_trainable_params", "default_device", "freeze_except_lora", "load_causal_lm",
    "load_reward_checkpoint", "read_state_dict", "save_hf_pretrained", "RewardModel", "ValueModel",
    "ByteTokenizer", "load_tokenizer",
    "CausalLM", "attention_layout", "build_model", "default_dtype",
]
