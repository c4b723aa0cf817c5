"""`python -m src.training.train_rlhf --config ...` plus `load_prompts` / `sequence_logprob`."""
from distributed_llm_alignment_amd.training.train_rlhf import load_prompts, main, parse_args  # noqa: F401


def sequence_logprob(model, input_ids, attention_mask):
    return model.sequence_logprob(input_ids, attention_mask, "mean")


if __name__ == "__main__":
    raise SystemExit(main())
