"""Model configurations + named presets (SURVEY Appendix B shapes).

The reference loads HF checkpoints by name (src/models/base_model.py:17-42). With no network,
the framework resolves `model_name_or_path` as: a local directory with config.json (HF layout,
loaded from safetensors), else a preset name below (random init), else a known HF hub id mapped
to its preset (e.g. "mistralai/Mistral-7B-v0.1" -> "mistral-7b", random init, shapes identical).
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, Optional


@dataclass
class ModelConfig:
    arch: str = "llama"  # llama | mistral | mixtral | gpt2 | phi
    vocab_size: int = 32000
    hidden_size: int = 4096
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    intermediate_size: int = 14336
    norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    rope_scaling: Optional[Dict[str, Any]] = None
    rotary_pct: float = 1.0
    max_position_embeddings: int = 8192
    sliding_window: int = 0
    tie_word_embeddings: bool = False
    num_experts: int = 0
    num_experts_per_tok: int = 2
    router_aux_loss_coef: float = 0.0
    norm_type: str = "rms"  # rms | layer
    activation: str = "swiglu"  # swiglu | gelu_new
    parallel_block: bool = False  # phi: attn and mlp both read the same normed input
    attn_bias: bool = False
    mlp_bias: bool = False
    lm_head_bias: bool = False
    learned_pos_emb: bool = False  # gpt2 wpe
    bos_token_id: int = 1
    eos_token_id: int = 2
    pad_token_id: Optional[int] = None
    init_std: float = 0.02
    name: str = "custom"

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def rot_dim(self) -> int:
        if self.learned_pos_emb:
            return 0
        return int(self.head_dim * self.rotary_pct)

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    def num_params(self, include_embedding: bool = True) -> int:
        H, F, L = self.hidden_size, self.intermediate_size, self.num_layers
        attn = H * (self.q_size + 2 * self.kv_size) + self.q_size * H
        mlp_one = (3 if self.activation == "swiglu" else 2) * H * F
        mlp = mlp_one * max(1, self.num_experts) + (H * self.num_experts if self.is_moe else 0)
        norms = (2 if not self.parallel_block else 1) * H
        per_layer = attn + mlp + norms
        emb = self.vocab_size * H if include_embedding else 0
        head = 0 if self.tie_word_embeddings else self.vocab_size * H
        return L * per_layer + emb + head + H

    def flops_per_token(self, seq_len: int) -> float:
        """Forward FLOPs/token: 2*matmul params (active experts only) + causal attention."""
        H, F, L = self.hidden_size, self.intermediate_size, self.num_layers
        attn_proj = H * (self.q_size + 2 * self.kv_size) + self.q_size * H
        n_mlp = self.num_experts_per_tok if self.is_moe else 1
        mlp = (3 if self.activation == "swiglu" else 2) * H * F * n_mlp
        matmul = L * (attn_proj + mlp) + self.vocab_size * H
        attn_scores = L * 2 * 2 * self.q_size * seq_len / 2  # QK^T + PV, causal half
        return 2.0 * matmul + attn_scores

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "ModelConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})

    # ----------------------------------------------------------------- HF config.json interop
    @classmethod
    def from_hf(cls, hf: Dict[str, Any]) -> "ModelConfig":
        mt = hf.get("model_type", "llama")
        if mt in ("llama", "mistral", "mixtral", "qwen2"):
            H = hf["hidden_size"]
            nh = hf["num_attention_heads"]
            return cls(
                arch=mt if mt != "qwen2" else "llama", vocab_size=hf["vocab_size"], hidden_size=H,
                num_layers=hf["num_hidden_layers"], num_heads=nh,
                num_kv_heads=hf.get("num_key_value_heads", nh),
                head_dim=hf.get("head_dim") or H // nh,
                intermediate_size=hf["intermediate_size"], norm_eps=hf.get("rms_norm_eps", 1e-6),
                rope_theta=hf.get("rope_theta", 10000.0), rope_scaling=hf.get("rope_scaling"),
                max_position_embeddings=hf.get("max_position_embeddings", 4096),
                sliding_window=hf.get("sliding_window") or 0,
                tie_word_embeddings=hf.get("tie_word_embeddings", False),
                num_experts=hf.get("num_local_experts", 0) if mt == "mixtral" else 0,
                num_experts_per_tok=hf.get("num_experts_per_tok", 2),
                router_aux_loss_coef=hf.get("router_aux_loss_coef", 0.0),
                attn_bias=hf.get("attention_bias", mt == "qwen2"),
                bos_token_id=hf.get("bos_token_id", 1) or 1, eos_token_id=_first(hf.get("eos_token_id", 2)),
                pad_token_id=hf.get("pad_token_id"), name=hf.get("_name_or_path", mt),
            )
        if mt == "gpt2":
            H = hf["n_embd"]
            nh = hf["n_head"]
            return cls(
                arch="gpt2", vocab_size=hf["vocab_size"], hidden_size=H, num_layers=hf["n_layer"],
                num_heads=nh, num_kv_heads=nh, head_dim=H // nh,
                intermediate_size=hf.get("n_inner") or 4 * H, norm_eps=hf.get("layer_norm_epsilon", 1e-5),
                max_position_embeddings=hf.get("n_positions", 1024), tie_word_embeddings=True,
                norm_type="layer", activation="gelu_new", attn_bias=True, mlp_bias=True,
                learned_pos_emb=True, bos_token_id=hf.get("bos_token_id", 50256),
                eos_token_id=hf.get("eos_token_id", 50256), name="gpt2",
            )
        if mt == "phi":
            H = hf["hidden_size"]
            nh = hf["num_attention_heads"]
            return cls(
                arch="phi", vocab_size=hf["vocab_size"], hidden_size=H,
                num_layers=hf["num_hidden_layers"], num_heads=nh,
                num_kv_heads=hf.get("num_key_value_heads") or nh, head_dim=H // nh,
                intermediate_size=hf["intermediate_size"], norm_eps=hf.get("layer_norm_eps", 1e-5),
                rope_theta=hf.get("rope_theta", 10000.0), rotary_pct=hf.get("partial_rotary_factor", 0.5),
                max_position_embeddings=hf.get("max_position_embeddings", 2048),
                norm_type="layer", activation="gelu_new", parallel_block=True, attn_bias=True,
                mlp_bias=True, lm_head_bias=True, bos_token_id=hf.get("bos_token_id", 50256) or 50256,
                eos_token_id=hf.get("eos_token_id", 50256) or 50256, name="phi",
            )
        raise ValueError(f"unsupported model_type {mt!r}")

    def to_hf(self) -> Dict[str, Any]:
        if self.arch == "gpt2":
            return {"model_type": "gpt2", "architectures": ["GPT2LMHeadModel"], "vocab_size": self.vocab_size,
                    "n_embd": self.hidden_size, "n_layer": self.num_layers, "n_head": self.num_heads,
                    "n_inner": self.intermediate_size, "n_positions": self.max_position_embeddings,
                    "layer_norm_epsilon": self.norm_eps, "activation_function": "gelu_new",
                    "bos_token_id": self.bos_token_id, "eos_token_id": self.eos_token_id,
                    "tie_word_embeddings": True, "torch_dtype": "bfloat16"}
        if self.arch == "phi":
            return {"model_type": "phi", "architectures": ["PhiForCausalLM"], "vocab_size": self.vocab_size,
                    "hidden_size": self.hidden_size, "num_hidden_layers": self.num_layers,
                    "num_attention_heads": self.num_heads, "num_key_value_heads": self.num_kv_heads,
                    "intermediate_size": self.intermediate_size, "layer_norm_eps": self.norm_eps,
                    "rope_theta": self.rope_theta, "partial_rotary_factor": self.rotary_pct,
                    "max_position_embeddings": self.max_position_embeddings, "hidden_act": "gelu_new",
                    "bos_token_id": self.bos_token_id, "eos_token_id": self.eos_token_id,
                    "torch_dtype": "bfloat16"}
        mt = self.arch
        arch_name = {"llama": "LlamaForCausalLM", "mistral": "MistralForCausalLM",
                     "mixtral": "MixtralForCausalLM"}[mt]
        d = {"model_type": mt, "architectures": [arch_name], "vocab_size": self.vocab_size,
             "hidden_size": self.hidden_size, "num_hidden_layers": self.num_layers,
             "num_attention_heads": self.num_heads, "num_key_value_heads": self.num_kv_heads,
             "head_dim": self.head_dim, "intermediate_size": self.intermediate_size,
             "rms_norm_eps": self.norm_eps, "rope_theta": self.rope_theta,
             "rope_scaling": self.rope_scaling, "max_position_embeddings": self.max_position_embeddings,
             "tie_word_embeddings": self.tie_word_embeddings, "hidden_act": "silu",
             "bos_token_id": self.bos_token_id, "eos_token_id": self.eos_token_id,
             "attention_bias": self.attn_bias, "torch_dtype": "bfloat16"}
        if mt in ("mistral", "mixtral"):
            d["sliding_window"] = self.sliding_window or None
        if mt == "mixtral":
            d["num_local_experts"] = self.num_experts
            d["num_experts_per_tok"] = self.num_experts_per_tok
            d["router_aux_loss_coef"] = self.router_aux_loss_coef
        return d


def _first(x):
    return x[0] if isinstance(x, (list, tuple)) else x


PRESETS: Dict[str, Dict[str, Any]] = {
    # north-star models
    "llama3-8b": dict(arch="llama", vocab_size=128256, hidden_size=4096, num_layers=32, num_heads=32,
                      num_kv_heads=8, head_dim=128, intermediate_size=14336, norm_eps=1e-5,
                      rope_theta=500000.0, max_position_embeddings=8192, bos_token_id=128000,
                      eos_token_id=128001),
    "llama3-70b": dict(arch="llama", vocab_size=128256, hidden_size=8192, num_layers=80, num_heads=64,
                       num_kv_heads=8, head_dim=128, intermediate_size=28672, norm_eps=1e-5,
                       rope_theta=500000.0, max_position_embeddings=8192, bos_token_id=128000,
                       eos_token_id=128001),
    "mistral-7b": dict(arch="mistral", vocab_size=32000, hidden_size=4096, num_layers=32, num_heads=32,
                       num_kv_heads=8, head_dim=128, intermediate_size=14336, norm_eps=1e-5,
                       rope_theta=10000.0, max_position_embeddings=32768, sliding_window=4096),
    "mixtral-8x7b": dict(arch="mixtral", vocab_size=32000, hidden_size=4096, num_layers=32, num_heads=32,
                         num_kv_heads=8, head_dim=128, intermediate_size=14336, norm_eps=1e-5,
                         rope_theta=1e6, max_position_embeddings=32768, num_experts=8,
                         num_experts_per_tok=2, router_aux_loss_coef=0.02),
    "gpt2": dict(arch="gpt2", vocab_size=50257, hidden_size=768, num_layers=12, num_heads=12,
                 num_kv_heads=12, head_dim=64, intermediate_size=3072, norm_eps=1e-5,
                 max_position_embeddings=1024, tie_word_embeddings=True, norm_type="layer",
                 activation="gelu_new", attn_bias=True, mlp_bias=True, learned_pos_emb=True,
                 bos_token_id=50256, eos_token_id=50256),
    "phi-2": dict(arch="phi", vocab_size=51200, hidden_size=2560, num_layers=32, num_heads=32,
                  num_kv_heads=32, head_dim=80, intermediate_size=10240, norm_eps=1e-5,
                  rope_theta=10000.0, rotary_pct=0.4, max_position_embeddings=2048,
                  norm_type="layer", activation="gelu_new", parallel_block=True, attn_bias=True,
                  mlp_bias=True, lm_head_bias=True, bos_token_id=50256, eos_token_id=50256),
    # test-scale models (CPU tier / smoke)
    "tiny-llama": dict(arch="llama", vocab_size=512, hidden_size=128, num_layers=2, num_heads=4,
                       num_kv_heads=2, head_dim=32, intermediate_size=256, norm_eps=1e-5,
                       rope_theta=10000.0, max_position_embeddings=512, bos_token_id=1, eos_token_id=2),
    "tiny-llama-d128": dict(arch="llama", vocab_size=1024, hidden_size=512, num_layers=2, num_heads=4,
                            num_kv_heads=2, head_dim=128, intermediate_size=1024, norm_eps=1e-5,
                            rope_theta=500000.0, max_position_embeddings=2048, bos_token_id=1,
                            eos_token_id=2),
    "tiny-mistral": dict(arch="mistral", vocab_size=512, hidden_size=128, num_layers=2, num_heads=4,
                         num_kv_heads=2, head_dim=32, intermediate_size=256, norm_eps=1e-5,
                         max_position_embeddings=512, sliding_window=16),
    "tiny-mixtral": dict(arch="mixtral", vocab_size=512, hidden_size=128, num_layers=2, num_heads=4,
                         num_kv_heads=2, head_dim=32, intermediate_size=128, norm_eps=1e-5,
                         max_position_embeddings=512, num_experts=4, num_experts_per_tok=2),
    "tiny-gpt2": dict(arch="gpt2", vocab_size=512, hidden_size=128, num_layers=2, num_heads=4,
                      num_kv_heads=4, head_dim=32, intermediate_size=512, max_position_embeddings=512,
                      tie_word_embeddings=True, norm_type="layer", activation="gelu_new",
                      attn_bias=True, mlp_bias=True, learned_pos_emb=True, bos_token_id=1,
                      eos_token_id=2),
    "tiny-phi": dict(arch="phi", vocab_size=512, hidden_size=160, num_layers=2, num_heads=2,
                     num_kv_heads=2, head_dim=80, intermediate_size=320, rotary_pct=0.4,
                     max_position_embeddings=512, norm_type="layer", activation="gelu_new",
                     parallel_block=True, attn_bias=True, mlp_bias=True, lm_head_bias=True,
                     bos_token_id=1, eos_token_id=2),
}

# HF hub ids used by the reference configs -> presets (random init offline, identical shapes)
HUB_ALIASES = {
    "mistralai/Mistral-7B-v0.1": "mistral-7b",
    "meta-llama/Meta-Llama-3-8B": "llama3-8b",
    "meta-llama/Meta-Llama-3-8B-Instruct": "llama3-8b",
    "meta-llama/Meta-Llama-3-70B": "llama3-70b",
    "mistralai/Mixtral-8x7B-v0.1": "mixtral-8x7b",
    "microsoft/phi-2": "phi-2",
    "gpt2": "gpt2",
    "openai-community/gpt2": "gpt2",
}


def tp_shard_config(cfg: ModelConfig, tp: int) -> ModelConfig:
    """The per-rank shapes of `cfg` under tensor parallelism of degree `tp` as a standalone
    (world-1) model: heads, KV heads, FFN width and vocabulary divided by tp, hidden size and
    depth kept. Used by `bench.py --tp-shape` to time one TP rank's real GEMM / attention / norm
    shapes on one GPU (e.g. Llama-3-70B at tp 8: 8 q heads / 1 kv head, FFN 3584, vocab 16032)."""
    if cfg.num_heads % tp or cfg.num_kv_heads % tp or cfg.intermediate_size % tp or cfg.vocab_size % tp:
        raise ValueError(f"{cfg.name}: heads / kv heads / FFN / vocab must divide tp={tp}")
    d = cfg.to_dict()
    d.update(num_heads=cfg.num_heads // tp, num_kv_heads=cfg.num_kv_heads // tp,
             intermediate_size=cfg.intermediate_size // tp, vocab_size=cfg.vocab_size // tp,
             name=f"{cfg.name}@tp{tp}")
    return ModelConfig.from_dict(d)


def get_config(name_or_path: str, **overrides) -> ModelConfig:
    """Resolve a preset / HF directory / hub alias into a ModelConfig. `<preset>@tp<N>` gives the
    per-rank shard shapes of that preset under TP degree N (tp_shard_config)."""
    name = str(name_or_path)
    if "@tp" in name and not Path(name).is_dir():
        base, tp = name.rsplit("@tp", 1)
        cfg = tp_shard_config(get_config(base), int(tp))
        for k, v in overrides.items():
            setattr(cfg, k, v)
        return cfg
    p = Path(str(name_or_path))
    if p.is_dir():
        if (p / "dla_config.json").exists():
            cfg = ModelConfig.from_dict(json.loads((p / "dla_config.json").read_text()))
        elif (p / "config.json").exists():
            cfg = ModelConfig.from_hf(json.loads((p / "config.json").read_text()))
        else:
            raise FileNotFoundError(f"{p} has no config.json")
    else:
        key = HUB_ALIASES.get(str(name_or_path), str(name_or_path))
        if key not in PRESETS:
            raise KeyError(f"unknown model {name_or_path!r}; presets: {sorted(PRESETS)}")
        cfg = ModelConfig(**PRESETS[key], name=key)
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg
