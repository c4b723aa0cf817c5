"""`src.data.datasets` names, implemented natively (distributed_llm_alignment_amd.data)."""
from distributed_llm_alignment_amd.data.datasets import (  # noqa: F401
    EvalPromptDataset, InstructionDataset, PreferenceDataset, Sample, TeacherRolloutDataset,
    build_instruction_dataset, build_preference_dataset, load_instruction_records,
    load_preference_records, pad_batch, read_jsonl)
