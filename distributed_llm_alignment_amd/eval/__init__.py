"""Evaluation CLIs: alignment keyword heuristics (eval_alignment) and prefill/decode latency
(eval_latency), reference layer L8."""
