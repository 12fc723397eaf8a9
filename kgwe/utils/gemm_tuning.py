"""Per-shape GEMM solution selection for MI355X (PyTorch TunableOp over
hipBLASLt / rocBLAS).

The projection and MLP GEMMs of a transformer step are a handful of fixed
shapes.  The library's default heuristic picks one kernel per shape; timing
the candidate solutions once on MI355X and pinning the fastest is pure gain.
``tools/tune_gemm.py`` runs real training steps with tuning on and writes
``kgwe/tuning/tunableop_mi355x.csv`` (committed: every MI355X with this ROCm
stack has the same solutions); ``enable()`` loads it read-only, so a timed run
never tunes.  Shapes missing from the file fall back to the default heuristic.
"""
from __future__ import annotations

import os
from pathlib import Path

RESULTS = Path(__file__).resolve().parents[1] / "tuning" / "tunableop_mi355x.csv"


def enable(path: str | os.PathLike | None = None, tune: bool = False) -> bool:
    """Turn TunableOp on with ``path`` (default: the committed results).
    tune=False: use recorded solutions only.  Returns True if active."""
    import torch

    if not torch.cuda.is_available() or os.environ.get("KGWE_GEMM_TUNING", "1") == "0":
        return False
    try:
        import torch.cuda.tunable as tunable
    except ImportError:
        return False
    p = Path(path or os.environ.get("KGWE_GEMM_TUNING_FILE") or RESULTS)
    if not tune and not p.exists():
        return False
    tunable.enable(True)
    tunable.tuning_enable(tune)
    if tune:
        tunable.set_max_tuning_duration(int(os.environ.get("KGWE_TUNE_MS_PER_SOLUTION", "30")))
        tunable.set_max_tuning_iterations(int(os.environ.get("KGWE_TUNE_ITERS", "20")))
    # Rank-qualified file names are TunableOp's convention for multi-GPU runs;
    # every rank reads the same committed file.
    tunable.set_filename(str(p), insert_device_ordinal=False)
    if p.exists():
        tunable.read_file(str(p))
    return True


def active() -> bool:
    try:
        import torch.cuda.tunable as tunable

        return tunable.is_enabled()
    except ImportError:
        return False
