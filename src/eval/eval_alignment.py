"""`python -m src.eval.eval_alignment --config ... [--max_prompts N]`."""
from distributed_llm_alignment_amd.eval.eval_alignment import (  # noqa: F401
    generate_responses, load_prompts, main, parse_args, summarize_responses)

if __name__ == "__main__":
    raise SystemExit(main())
