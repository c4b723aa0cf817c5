"""`python -m src.training.train_reward --config ...` -> distributed_llm_alignment_amd.training.train_reward."""
from distributed_llm_alignment_amd.training.train_reward import *  # noqa: F401,F403
from distributed_llm_alignment_amd.training.train_reward import main, parse_args  # noqa: F401

if __name__ == "__main__":
    raise SystemExit(main())
