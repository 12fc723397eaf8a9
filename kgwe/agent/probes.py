"""Python binding of the HIP bandwidth probes (``libkgwe_probes.so``).

HBM self-probe (1 GPU) and xGMI peer probes (pairwise and all-links) used by
the node agent to attach MEASURED bandwidth to the topology it reports
(replaces reference NVML-reported NVLink numbers:
src/discovery/discovery.go:341 GetNVLinkInfo, types.go:134-146).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from pathlib import Path

_PATH = Path(__file__).resolve().parent.parent / "_lib" / "libkgwe_probes.so"
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not _PATH.exists():
            raise RuntimeError(f"{_PATH} missing; run python -m kgwe._build")
        L = ctypes.CDLL(str(_PATH), mode=os.RTLD_NOW)
        L.kgwe_probe_device_count.restype = ctypes.c_int
        L.kgwe_probe_hbm.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_double)]
        L.kgwe_probe_hbm.restype = ctypes.c_int
        L.kgwe_probe_p2p.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_double)]
        L.kgwe_probe_p2p.restype = ctypes.c_int
        L.kgwe_probe_p2p_all.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_double)]
        L.kgwe_probe_p2p_all.restype = ctypes.c_int
        _lib = L
    return _lib


@dataclass
class HbmResult:
    device: int
    copy_gbps: float
    read_gbps: float
    write_gbps: float
    lds_copy_gbps: float


def device_count() -> int:
    return lib().kgwe_probe_device_count()


def probe_hbm(device: int = 0, nbytes: int = 1 << 30, iters: int = 10) -> HbmResult:
    out = (ctypes.c_double * 4)()
    rc = lib().kgwe_probe_hbm(device, nbytes, iters, out)
    if rc != 0:
        raise RuntimeError(f"kgwe_probe_hbm failed rc={rc}")
    return HbmResult(device, out[0], out[1], out[2], out[3])


def probe_p2p(src: int, dst: int, nbytes: int = 256 << 20, iters: int = 10) -> float | None:
    out = ctypes.c_double()
    rc = lib().kgwe_probe_p2p(src, dst, nbytes, iters, ctypes.byref(out))
    if rc == -1:
        return None
    if rc != 0:
        raise RuntimeError(f"kgwe_probe_p2p failed rc={rc}")
    return out.value


def probe_p2p_all(ndev: int, nbytes: int = 128 << 20, iters: int = 5) -> list[list[float]]:
    mat = (ctypes.c_double * (ndev * ndev))()
    rc = lib().kgwe_probe_p2p_all(ndev, nbytes, iters, mat)
    if rc < 0:
        raise RuntimeError(f"kgwe_probe_p2p_all failed rc={rc}")
    return [[mat[d * ndev + s] for s in range(ndev)] for d in range(ndev)]
