"""Reference-compatible model helpers (see distributed_llm_alignment_amd.models)."""
