"""`python -m src.training.train_sft --config ...` -> distributed_llm_alignment_amd.training.train_sft."""
from distributed_llm_alignment_amd.training.train_sft import *  # noqa: F401,F403
from distributed_llm_alignment_amd.training.train_sft import main, parse_args  # noqa: F401

if __name__ == "__main__":
    raise SystemExit(main())
