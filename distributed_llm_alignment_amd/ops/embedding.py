"""Token embedding on the HIP gather / deterministic scatter-add kernels (csrc/embedding.hip,
SURVEY K1).

Forward gathers table rows with 16-byte loads. Backward sorts the token ids on the device
(`torch.sort`, stable: no host sync) and sums every token's dY rows in sorted order straight into
the engine's flat main-grad buffer (bf16 or fp32), instead of eager PyTorch's dense [V, H]
gradient (zero-fill + segment sum) plus autograd's add into `.grad` -- two passes over V x H per
micro-batch. Tied / shared tables (`_dla_shared`: the LM head also writes the gradient) get a
dense gradient tensor through autograd as usual. CPU tensors use `F.embedding`.

Out-of-range ids: `F.embedding` raises on them. Checking on the host would cost a sync per
forward, and a device assert aborts the whole process, so the kernel instead writes a zero row,
never touches memory outside the table (forward and backward) and sets a sticky per-device error
word. `check_ids()` raises on it; the trainer calls it at every logging step (where it syncs
anyway), and DLA_EMBED_CHECK=1 checks after every forward (debug).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _ext


_BAD = {}  # device -> int32 [1] sticky out-of-range-id word
_CHECK_EVERY = os.environ.get("DLA_EMBED_CHECK", "0") == "1"


def _bad_word(device: torch.device) -> torch.Tensor:
    w = _BAD.get(device)
    if w is None:
        w = _BAD[device] = torch.zeros(1, dtype=torch.int32, device=device)
    return w


def check_ids(reset: bool = True, group=None, collective: bool = False) -> None:
    """Raise if any native embedding forward since the last check saw an id outside [0, V)
    (one host sync per device that ran the kernel).

    `collective=True` (the trainers' logging step, reached by every rank together): the sticky
    words are max-reduced over `group` first, so every rank raises at the same step instead of the
    ranks that saw no bad id blocking in their next collective until the RCCL timeout."""
    import torch.distributed as dist

    words = list(_BAD.items())
    if collective and dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dev = words[0][0] if words else (torch.device("cuda", torch.cuda.current_device())
                                         if dist.get_backend(group) == "nccl" else torch.device("cpu"))
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        for _, w in words:
            flag = torch.maximum(flag, (w != 0).int().to(dev))
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if int(flag.item()) != 0:
            local = [str(d) for d, w in words if int(w.item()) != 0]
            if reset:
                for _, w in words:
                    w.zero_()
            raise IndexError("embedding: token id out of range [0, vocab) on "
                             f"{', '.join(local) if local else 'another rank'} (the rows were "
                             "zero-filled and got no gradient); check the tokenizer / vocab_size")
        return
    for dev, w in words:
        if int(w.item()) != 0:
            if reset:
                w.zero_()
            raise IndexError(f"embedding: token id out of range [0, vocab) on {dev} (the rows were "
                             "zero-filled and got no gradient); check the tokenizer / vocab_size")


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight):
        flat = ids.reshape(-1).to(torch.int64).contiguous()
        out = _ext.require().embed_fwd(weight, flat, _bad_word(weight.device))
        if _CHECK_EVERY:
            check_ids()
        ctx.save_for_backward(flat)
        ctx.wshape = weight.shape
        ctx.weight = weight
        return out.view(*ids.shape, weight.shape[1])

    @staticmethod
    def backward(ctx, dy):
        (flat,) = ctx.saved_tensors
        weight = ctx.weight
        sid, perm = torch.sort(flat, stable=True)
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        mg = getattr(weight, "main_grad", None)
        if mg is not None and not getattr(weight, "_dla_shared", False) and mg.is_contiguous():
            _ext.require().embed_bwd(sid, perm, dy2, mg)
            hook = getattr(weight, "_dla_grad_hook", None)
            if hook is not None:
                hook(weight)
            return None, None
        g = torch.zeros(ctx.wshape, dtype=torch.float32 if weight.dtype != torch.bfloat16 else weight.dtype,
                        device=dy.device)
        _ext.require().embed_bwd(sid, perm, dy2, g)
        return None, g.to(weight.dtype)


NATIVE_EMBEDDING = os.environ.get("DLA_EMBED_KERNEL", "1") != "0"


def embedding(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    if (NATIVE_EMBEDDING and _ext.use_native(weight) and weight.dtype == torch.bfloat16 and weight.dim() == 2
            and weight.shape[1] % 8 == 0 and weight.stride(1) == 1 and weight.stride(0) % 8 == 0):
        return _EmbeddingFn.apply(ids, weight)
    return F.embedding(ids, weight)
