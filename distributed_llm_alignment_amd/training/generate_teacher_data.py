"""Teacher rollout generation (reference: src/training/generate_teacher_data.py:17-107).

    python -m distributed_llm_alignment_amd.training.generate_teacher_data \\
        --teacher checkpoints/dpo/latest --prompts prompts.jsonl --output rollouts.jsonl \\
        [--reward_model checkpoints/reward/latest] [--batch_size 4] [--max_new_tokens 256] \\
        [--temperature 0.7] [--top_p 0.9]

Output JSONL `{"prompt", "teacher_response", "reward"?}` (reward only with --reward_model).
Generation is batched, left-padded, on one GPU per process; under torchrun each rank generates a
contiguous shard of the prompts and rank 0 concatenates the shards in order (the reference
instead spreads one model over all GPUs with device_map="auto"). Reward scoring is batched.
"""
from __future__ import annotations

import argparse
import json
from pathlib import Path
from typing import List

import torch

from ..data import read_jsonl
from ..models import build_reward_model, generate, load_causal_lm, load_reward_checkpoint
from ..parallel.dist import barrier, init_distributed, split_for_rank


def parse_args(argv=None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description="Sample teacher responses")
    p.add_argument("--teacher", required=True, help="Path or preset/hub id for teacher model")
    p.add_argument("--prompts", required=True, help="JSONL prompts file")
    p.add_argument("--output", required=True, help="Destination JSONL")
    p.add_argument("--reward_model", default=None, help="Optional reward model checkpoint")
    p.add_argument("--batch_size", type=int, default=4)
    p.add_argument("--max_new_tokens", type=int, default=256)
    p.add_argument("--temperature", type=float, default=0.7)
    p.add_argument("--top_p", type=float, default=0.9)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--device_map", default=None,
                   help="'auto': split the teacher's layers over all visible GPUs in this one process "
                        "(reference behavior; only for models larger than one GPU's HBM)")
    return p.parse_args(argv)


def chunk_list(items: List[str], chunk_size: int) -> List[List[str]]:
    return [items[i: i + chunk_size] for i in range(0, len(items), chunk_size)]


def main(argv=None) -> int:
    args = parse_args(argv)
    st = init_distributed()
    torch.manual_seed(args.seed)
    if args.device_map and st.world_size > 1:
        raise SystemExit("--device_map is a single-process mode; launch one process (or drop it)")
    bundle = load_causal_lm(args.teacher, gradient_checkpointing=False, device=st.device, seed=args.seed,
                            device_map=args.device_map)
    model, tok = bundle.model, bundle.tokenizer
    model.eval()
    rm = rtok = None
    if args.reward_model:
        base = args.reward_model
        rm, rtok = build_reward_model(base, device=st.device, seed=args.seed)
        if Path(args.reward_model).exists():
            load_reward_checkpoint(rm, args.reward_model)
        rm.eval()
    prompts = [item["prompt"] for item in read_jsonl(args.prompts)]
    mine = split_for_rank(prompts)
    out_path = Path(args.output)
    out_path.parent.mkdir(parents=True, exist_ok=True)
    shard_path = out_path if st.world_size == 1 else out_path.with_suffix(out_path.suffix + f".rank{st.rank}")
    g = torch.Generator(device=st.device)
    g.manual_seed(args.seed * 1000 + st.rank)
    max_len = getattr(tok, "model_max_length", 4096)
    max_len = min(max_len, model.cfg.max_position_embeddings - args.max_new_tokens)
    with shard_path.open("w", encoding="utf-8") as writer:
        for batch_prompts in chunk_list(mine, args.batch_size):
            side = getattr(tok, "padding_side", "right")
            tok.padding_side = "left"
            enc = tok(batch_prompts, return_tensors="pt", padding=True, truncation=True, max_length=max_len)
            tok.padding_side = side
            ids, am = enc["input_ids"].to(st.device), enc["attention_mask"].to(st.device)
            seqs = generate(model, ids, am, max_new_tokens=args.max_new_tokens, do_sample=True,
                            temperature=args.temperature, top_p=args.top_p,
                            pad_token_id=tok.pad_token_id, generator=g)
            responses = tok.batch_decode(seqs[:, ids.shape[1]:], skip_special_tokens=True)
            rewards = [None] * len(responses)
            if rm is not None:
                fused = [f"{p}\n\n{r}" for p, r in zip(batch_prompts, responses)]
                renc = rtok(fused, return_tensors="pt", padding=True, truncation=True,
                            max_length=getattr(rtok, "model_max_length", 4096))
                with torch.no_grad():
                    rewards = rm(renc["input_ids"].to(st.device), renc["attention_mask"].to(st.device)).tolist()
            for p, r, rw in zip(batch_prompts, responses, rewards):
                rec = {"prompt": p, "teacher_response": r}
                if rw is not None:
                    rec["reward"] = float(rw)
                writer.write(json.dumps(rec) + "\n")
    barrier()
    if st.world_size > 1 and st.is_main:
        with out_path.open("w", encoding="utf-8") as w:
            for r in range(st.world_size):
                sp = out_path.with_suffix(out_path.suffix + f".rank{r}")
                w.write(sp.read_text(encoding="utf-8"))
                sp.unlink()
    barrier()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
