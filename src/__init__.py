"""Drop-in module paths of nikhil-lalgudi/distributed-llm-alignment (`src.*`), backed by the
MI355X-native `distributed_llm_alignment_amd` package. Existing scripts such as
`python -m src.training.train_dpo --config ...` keep working."""
