"""`python -m src.training.train_distill --config ...` -> distributed_llm_alignment_amd.training.train_distill."""
from distributed_llm_alignment_amd.training.train_distill import *  # noqa: F401,F403
from distributed_llm_alignment_amd.training.train_distill import main, parse_args  # noqa: F401

if __name__ == "__main__":
    raise SystemExit(main())
