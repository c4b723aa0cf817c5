"""Streamed safetensors I/O for large device tensors (optimizer shards).

`torch.save` of a rank's optimizer shard first copies every tensor to host memory: at 70B with
TP=8 that is ~106 GB of fp32 moments + master per rank, ~850 GB of host RAM for the node at the
same moment. Here the file is written in the plain safetensors layout (8-byte little-endian
header length, JSON header, raw row-major bytes) by copying each device tensor through ONE
reusable pinned host buffer of `chunk_mb`, so host RSS stays at that buffer whatever the shard
size. Reading back maps the file (`np.memmap`, page cache, no anonymous memory) and copies
chunk-wise into the destination device tensors. Files are readable by `safetensors.safe_open`.
Non-tensor values (step, lr, betas, ...) travel in the header's `__metadata__` as JSON.
"""
from __future__ import annotations

import json
import os
import struct
from pathlib import Path
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

_DT = {torch.float32: "F32", torch.bfloat16: "BF16", torch.float16: "F16", torch.int64: "I64",
       torch.int32: "I32", torch.uint8: "U8", torch.int8: "I8", torch.float64: "F64"}
_NP = {"F32": np.float32, "F16": np.float16, "I64": np.int64, "I32": np.int32, "U8": np.uint8,
       "I8": np.int8, "F64": np.float64, "BF16": np.int16}
_TORCH = {v: k for k, v in _DT.items()}


def save_streamed(path, tensors: Dict[str, Optional[torch.Tensor]], meta: Optional[Dict[str, Any]] = None,
                  chunk_mb: int = 64) -> Path:
    """Write `tensors` (any device; None entries skipped) + JSON-able `meta` to `path`."""
    path = Path(path)
    items = [(k, t) for k, t in tensors.items() if t is not None]
    header: Dict[str, Any] = {"__metadata__": {"format": "pt", "dla_meta": json.dumps(meta or {})}}
    off = 0
    for k, t in items:
        if t.dtype not in _DT:
            raise TypeError(f"{k}: dtype {t.dtype} not supported")
        n = t.numel() * t.element_size()
        header[k] = {"dtype": _DT[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + n]}
        off += n
    hb = json.dumps(header, separators=(",", ":")).encode()
    hb += b" " * ((8 - len(hb) % 8) % 8)  # 8-byte aligned data start (spec allows trailing spaces)
    tmp = path.with_suffix(path.suffix + ".tmp")
    chunk = max(1, int(chunk_mb)) << 20
    buf = None
    with open(tmp, "wb") as f:
        f.write(struct.pack("<Q", len(hb)))
        f.write(hb)
        for _k, t in items:
            flat = t.detach().reshape(-1).view(torch.uint8) if t.numel() else t.new_empty(0, dtype=torch.uint8)
            if not flat.is_cuda:
                f.write(flat.contiguous().numpy().tobytes())
                continue
            if buf is None:
                buf = torch.empty(chunk, dtype=torch.uint8, pin_memory=True)
            for s in range(0, flat.numel(), chunk):
                e = min(flat.numel(), s + chunk)
                buf[:e - s].copy_(flat[s:e], non_blocking=False)
                f.write(memoryview(buf[:e - s].numpy()))
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    return path


def read_header(path) -> Tuple[Dict[str, Any], int, Dict[str, Any]]:
    """(tensor header, data start byte, meta dict)."""
    with open(path, "rb") as f:
        (n,) = struct.unpack("<Q", f.read(8))
        h = json.loads(f.read(n))
    md = h.pop("__metadata__", {}) or {}
    meta = json.loads(md.get("dla_meta", "{}"))
    return h, 8 + n, meta


def mmap_tensor(path, name: str, header=None) -> torch.Tensor:
    """Zero-copy host view (read-only page-cache mapping) of tensor `name`."""
    h, start, _ = header if header is not None else read_header(path)
    info = h[name]
    b, e = info["data_offsets"]
    dt = info["dtype"]
    count = (e - b) // np.dtype(_NP[dt]).itemsize
    if count == 0:
        return torch.empty(info["shape"], dtype=_TORCH[dt])
    arr = np.memmap(path, dtype=_NP[dt], mode="r", offset=start + b, shape=(count,))
    import warnings

    with warnings.catch_warnings():  # read-only mapping: callers only read / copy out of it
        warnings.simplefilter("ignore", UserWarning)
        t = torch.from_numpy(arr)
    if dt == "BF16":
        t = t.view(torch.bfloat16)
    return t.view(info["shape"])


def load_streamed(path, device=None, chunk_mb: int = 256) -> Tuple[Dict[str, torch.Tensor], Dict[str, Any]]:
    """Read every tensor onto `device` (chunked host->device copies from the mapping) + meta."""
    hdr = read_header(path)
    out = {}
    for k in hdr[0]:
        src = mmap_tensor(path, k, hdr)
        dst = torch.empty(src.shape, dtype=src.dtype, device=device or "cpu")
        copy_into(dst, src, chunk_mb)
        out[k] = dst
    return out, hdr[2]


def copy_into(dst: torch.Tensor, src: torch.Tensor, chunk_mb: int = 256) -> None:
    d, s = dst.reshape(-1), src.reshape(-1)
    if d.numel() != s.numel():
        raise ValueError(f"size mismatch {tuple(dst.shape)} vs {tuple(src.shape)}")
    step = max(1, (int(chunk_mb) << 20) // max(1, src.element_size()))
    for a in range(0, s.numel(), step):
        d[a:a + step].copy_(s[a:a + step])
