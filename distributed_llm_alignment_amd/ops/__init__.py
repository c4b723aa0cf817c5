"""gfx950 compute ops. GPU tensors run the in-tree HIP kernels (`torch.ops.dla.*`); CPU tensors
run the pure-PyTorch references (test tier / numerics oracles)."""
from . import _ext, decode, moe
from .embedding import embedding
from .activations import gelu_new, swiglu, swiglu_mlp, swiglu_mlp_ok
from .attention import RotaryCache, attention_core, qkv_attention, ref_attention
from .linear import (accumulate_weight_grad, enable_fp8_inference, fp8_inference_scope, linear,
                     linear_add)
from .logprob import linear_logprob, seq_reduce, sequence_logprob, shifted_targets, token_nll
from .losses import (dpo_loss, ensemble_kl, gae, kl_penalty_pg, pairwise_loss, ppo_policy_loss,
                     ppo_value_loss)
from .norm import add_norm, layer_norm, rms_norm

__all__ = [
    "embedding",
    "_ext", "decode", "moe", "gelu_new", "swiglu", "swiglu_mlp", "swiglu_mlp_ok", "RotaryCache", "attention_core", "qkv_attention",
    "ref_attention", "linear_logprob", "seq_reduce", "sequence_logprob", "shifted_targets",
    "token_nll", "dpo_loss", "ensemble_kl", "kl_penalty_pg", "pairwise_loss", "gae",
    "ppo_policy_loss", "ppo_value_loss", "add_norm", "layer_norm", "rms_norm", "linear", "linear_add",
    "accumulate_weight_grad",
]
