"""Reference-compatible data helpers (see distributed_llm_alignment_amd.data)."""
