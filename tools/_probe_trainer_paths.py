"""Debug probe: which main-grad autograd nodes the SFT trainer's steps run through on the GPU
(counts _SwiGLUMLPFn / _LinearMainGradFn calls and checks main_grad attachment)."""
import sys
import tempfile
from pathlib import Path

import yaml

from distributed_llm_alignment_amd.data import write_jsonl
from distributed_llm_alignment_amd.data.synthetic import synthetic_instruction_records
import importlib

activations = importlib.import_module("distributed_llm_alignment_amd.ops.activations")
linear = importlib.import_module("distributed_llm_alignment_amd.ops.linear")
from distributed_llm_alignment_amd.training import train_sft

calls = {"mlp": 0, "lin": 0, "mlp_ok_false": 0}
_f, _l, _ok = activations._SwiGLUMLPFn.forward, linear._LinearMainGradFn.forward, activations.swiglu_mlp_ok


def f(ctx, *a):
    calls["mlp"] += 1
    return _f(ctx, *a)


def l(ctx, *a):
    calls["lin"] += 1
    return _l(ctx, *a)


def ok(h, wu, wd):
    r = _ok(h, wu, wd)
    if not r:
        calls["mlp_ok_false"] += 1
        if calls["mlp_ok_false"] < 3:
            print("swiglu_mlp_ok False:", h.shape, h.dtype, wu.requires_grad, getattr(wu, "main_grad", None) is not None)
    return r


activations._SwiGLUMLPFn.forward = staticmethod(f)
linear._LinearMainGradFn.forward = staticmethod(l)
activations.swiglu_mlp_ok = ok
import distributed_llm_alignment_amd.models.transformer as tr  # noqa: E402
tr.ops.swiglu_mlp_ok = ok
d = Path(tempfile.mkdtemp())
write_jsonl(d / "sft.jsonl", synthetic_instruction_records(32, seed=1))
cfg = {"seed": 42, "model": {"model_name_or_path": "tiny-llama-d128", "max_seq_length": 128,
                             "gradient_checkpointing": sys.argv[1] if len(sys.argv) > 1 else True},
       "data": {"source": "local", "train_path": str(d / "sft.jsonl"), "num_workers": 0},
       "optimization": {"micro_batch_size": 8, "learning_rate": 3e-3, "max_train_steps": 2},
       "logging": {"output_dir": str(d / "ck"), "log_dir": str(d / "logs")}}
(d / "c.yaml").write_text(yaml.safe_dump(cfg))
train_sft.main(["--config", str(d / "c.yaml")])
print("calls", calls)
