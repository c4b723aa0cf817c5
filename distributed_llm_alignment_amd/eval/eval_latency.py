"""Latency / throughput evaluation (reference: src/eval/eval_latency.py:22-84).

    python -m distributed_llm_alignment_amd.eval.eval_latency --config config/eval_config.yaml

For every model and (batch_size, seq_length) of `latency.*`: `warmup_steps` forwards, synchronise,
`measure_steps` timed forwards, synchronise; records `tokens_per_second = B*T*steps/dt` and
`latency_ms` (prefill/forward, the reference's metric). Additionally measures autoregressive
decode (`decode_tokens_per_second`, `decode_ms_per_token`) with the KV-cache decoder, which the
reference's harness claims but does not measure (Appendix A #19). Writes `latency.json` next to
`logging.output_path`.
"""
from __future__ import annotations

import argparse
import json
import time
from pathlib import Path
from typing import Dict, List

import torch

from ..models import KVCache, load_causal_lm
from ..utils.config import load_config


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Measure forward / decode latency")
    p.add_argument("--config", required=True)
    p.add_argument("--decode_tokens", type=int, default=32)
    p.add_argument("--overlay", action="append", default=[], help="YAML fragment merged over the config")
    p.add_argument("--override", action="append", default=[], help="dotted key.path=value override")
    return p.parse_args(argv)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


@torch.no_grad()
def measure_model(model, batch_sizes: List[int], seq_lengths: List[int], warmup_steps: int,
                  measure_steps: int, decode_tokens: int = 32) -> List[Dict[str, float]]:
    dev = model.embed.device
    V = model.cfg.vocab_size
    rows = []
    for b in batch_sizes:
        for t in seq_lengths:
            ids = torch.randint(0, V - 1, (b, t), device=dev)
            att = torch.ones_like(ids)
            for _ in range(warmup_steps):
                model.logits(model(ids, att))
            _sync(dev)
            t0 = time.perf_counter()
            for _ in range(measure_steps):
                model.logits(model(ids, att))
            _sync(dev)
            dt = time.perf_counter() - t0
            rec = {"batch_size": b, "seq_length": t, "tokens_per_second": b * t * measure_steps / dt,
                   "latency_ms": dt / measure_steps * 1000.0}
            if decode_tokens > 0 and t + decode_tokens <= model.cfg.max_position_embeddings:
                cache = KVCache(model, b, t + decode_tokens + 1, None)
                model(ids, cache=cache)
                nxt = torch.randint(0, V - 1, (b, 1), device=dev)
                _sync(dev)
                t0 = time.perf_counter()
                for _ in range(decode_tokens):
                    model.logits(model(nxt, cache=cache)[:, -1])
                _sync(dev)
                dd = time.perf_counter() - t0
                rec["decode_tokens_per_second"] = b * decode_tokens / dd
                rec["decode_ms_per_token"] = dd / decode_tokens * 1000.0
            rows.append(rec)
    return rows


def main(argv=None) -> int:
    args = parse_args(argv)
    cfg = load_config(args.config, args.overlay, args.override)
    lat = cfg["latency"]
    results: Dict[str, List[Dict[str, float]]] = {}
    for name, path in cfg["models"].items():
        bundle = load_causal_lm(path, gradient_checkpointing=False, seed=cfg.get("seed", 0),
                                device_map=(cfg.get("hardware", {}) or {}).get("device_map"))
        bundle.model.eval()
        results[name] = measure_model(bundle.model, lat["batch_sizes"], lat["seq_lengths"],
                                      lat.get("warmup_steps", 3), lat.get("measure_steps", 10),
                                      args.decode_tokens)
        del bundle
    out = Path((cfg.get("logging", {}) or {}).get("output_path", "logs/eval/results.json")).with_name("latency.json")
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(results, indent=2))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
