"""hipBLASLt solution selection for the plain GEMMs (PyTorch TunableOp, gfx950).

hipBLASLt's default heuristic picks a depth-32 Tensile tile for the NN-layout input-gradient
GEMMs of the transformer backward (~0.94 PF/s vs ~1.5 PF/s for the forward GEMMs on MI355X,
profiles/r1_*). TunableOp benchmarks every hipBLASLt/rocBLAS solution per (layout, M, N, K)
once and records the winner; the table tuned on MI355X ships in-tree
(`tuning/tunableop_gfx950.csv`) and is loaded read-only at startup, so production runs pay no
tuning cost. Re-tune by running any workload with DLA_GEMM_TUNE=1 (and DLA_GEMM_TABLE=<path>):
TunableOp writes the table at process exit. DLA_GEMM_TUNING=0 disables the table.
"""
from __future__ import annotations

import os
from pathlib import Path

TUNED_DIR = Path(__file__).resolve().parent.parent / "tuning"


def tuned_table(arch: str = "gfx950") -> Path:
    return TUNED_DIR / f"tunableop_{arch}.csv"


def enable_gemm_tuning(device_index: int = 0) -> str:
    """Enable TunableOp with the shipped table (read-only) or in tuning mode (DLA_GEMM_TUNE=1).
    Returns the mode used ("off" | "read" | "tune")."""
    if os.environ.get("DLA_GEMM_TUNING", "1") == "0":
        return "off"
    try:
        import torch

        if not torch.cuda.is_available():
            return "off"
        tun = torch.cuda.tunable
    except Exception:
        return "off"
    tune = os.environ.get("DLA_GEMM_TUNE", "0") == "1"
    table = Path(os.environ.get("DLA_GEMM_TABLE", str(tuned_table())))
    if not tune and not table.exists():
        return "off"
    # TunableOp appends the device ordinal to the file name; keep one table per device id.
    per_dev = table.with_name(table.stem + f"{device_index}" + table.suffix)
    if not tune and not per_dev.exists():
        try:
            per_dev.write_bytes(table.read_bytes())
        except OSError:
            return "off"
    tun.enable(True)
    tun.tuning_enable(tune)
    tun.record_untuned_enable(False)
    if tune:
        tun.set_max_tuning_duration(int(os.environ.get("DLA_GEMM_TUNE_MS", "40")))
        tun.set_max_tuning_iterations(int(os.environ.get("DLA_GEMM_TUNE_ITERS", "20")))
    tun.set_filename(str(table), insert_device_ordinal=True)
    if not tune:
        tun.read_file(str(per_dev))
    return "tune" if tune else "read"


_SOLUTIONS = {}


def hipblaslt_solution(m: int, n: int, k: int, lda: int, ldb: int, ldc: int) -> int:
    """The hipBLASLt solution index the shipped TunableOp table picked for the TN bf16 GEMM
    (m, n, k, lda, ldb, ldc) in BLAS column-major terms, or -1 (no row, or a rocBLAS pick). Offered
    as one more candidate to the C != D GEMM's own selection (csrc/gemm_lt.cpp)."""
    if not _SOLUTIONS:
        _SOLUTIONS[None] = None
        try:
            for line in tuned_table().read_text().splitlines():
                parts = line.split(",")
                if len(parts) >= 3 and parts[0] == "GemmTunableOp_BFloat16_TN" and parts[2].startswith("Gemm_Hipblaslt_"):
                    _SOLUTIONS[parts[1]] = int(parts[2].rsplit("_", 1)[1])
        except (OSError, ValueError):
            pass
    return _SOLUTIONS.get(f"tn_{m}_{n}_{k}_ld_{lda}_{ldb}_{ldc}", -1)
