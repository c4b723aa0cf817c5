"""`python -m src.training.train_dpo --config ...` plus the reference's helper functions."""
from distributed_llm_alignment_amd.ops.losses import dpo_loss as _dpo_loss
from distributed_llm_alignment_amd.training.train_dpo import main, parse_args  # noqa: F401


def compute_logprobs(model, input_ids, attention_mask):
    """Length-normalised per-sequence log-prob (reference train_dpo.py:31-39)."""
    return model.sequence_logprob(input_ids, attention_mask, "mean")


def dpo_loss(policy_pos, policy_neg, ref_pos, ref_neg, beta: float):
    return _dpo_loss(policy_pos, policy_neg, ref_pos, ref_neg, beta)[0]


if __name__ == "__main__":
    raise SystemExit(main())
