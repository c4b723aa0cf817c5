"""Reference-compatible trainer entry points (see distributed_llm_alignment_amd.training)."""
