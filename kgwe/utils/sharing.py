"""Apply a co-located share's limits inside the workload process.

The scheduler ledger gives every CoLocate client a disjoint CU range and an
HBM cap (``SharingManager`` / ``Scheduler`` shares, rendered by
``share_env``).  The CU range is enforced by ROCm itself through
``HSA_CU_MASK`` (set before the HIP runtime starts); the HBM cap has no ROCm
knob, so kgwe workloads call :func:`apply_from_env` at start, which caps
PyTorch's caching allocator with ``torch.cuda.set_per_process_memory_fraction``
(reference MPS memory limit: src/sharing/mig_controller.go:594-678, recorded
there and enforced nowhere).
"""
from __future__ import annotations

import os


def share_info() -> dict:
    return {"method": os.environ.get("KGWE_SHARING", ""),
            "cu_mask": os.environ.get("HSA_CU_MASK", ""),
            "cu_range": os.environ.get("KGWE_CU_RANGE", ""),
            "memory_fraction": float(os.environ.get("KGWE_GPU_MEMORY_FRACTION", "0") or 0.0)}


def apply_from_env(device=None) -> dict:
    """Cap this process's HBM use to the share's fraction (no-op without one)."""
    info = share_info()
    frac = info["memory_fraction"]
    if frac > 0:
        import torch

        if torch.cuda.is_available():
            torch.cuda.set_per_process_memory_fraction(min(1.0, frac),
                                                       device if device is not None else 0)
            info["applied"] = True
    return info
