"""`python -m src.eval.eval_latency --config ...`."""
from distributed_llm_alignment_amd.eval.eval_latency import main, measure_model, parse_args  # noqa: F401

if __name__ == "__main__":
    raise SystemExit(main())
