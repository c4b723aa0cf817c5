"""`python -m src.training.generate_teacher_data --teacher ... --prompts ... --output ...`."""
from distributed_llm_alignment_amd.training.generate_teacher_data import chunk_list, main, parse_args  # noqa: F401

if __name__ == "__main__":
    raise SystemExit(main())
