"""Reference-compatible eval CLIs (see distributed_llm_alignment_amd.eval)."""
