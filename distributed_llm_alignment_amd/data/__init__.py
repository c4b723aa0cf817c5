"""Data pipeline: reference-schema JSONL datasets, collation, HF/local/synthetic loaders."""
from .datasets import (EvalPromptDataset, InstructionDataset, PackedDataset, PreferenceDataset, Sample,
                       TeacherRolloutDataset, build_instruction_dataset, build_preference_dataset,
                       load_instruction_records, load_preference_records, pad_batch, read_jsonl,
                       write_jsonl)
from .loader import build_dataloader, get_distributed_sampler
from .synthetic import (synthetic_instruction_records, synthetic_lm_batch, synthetic_preference_batch,
                        synthetic_preference_records, synthetic_prompt_records)

__all__ = [
    "EvalPromptDataset", "InstructionDataset", "PackedDataset", "PreferenceDataset", "Sample", "TeacherRolloutDataset",
    "build_instruction_dataset", "build_preference_dataset", "load_instruction_records",
    "load_preference_records", "pad_batch", "read_jsonl", "write_jsonl", "build_dataloader",
    "get_distributed_sampler", "synthetic_instruction_records", "synthetic_lm_batch",
    "synthetic_preference_batch", "synthetic_preference_records", "synthetic_prompt_records",
]
