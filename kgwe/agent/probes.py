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
        L.kgwe_probe_gate_selftest.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.kgwe_probe_gate_selftest.restype = ctypes.c_int
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


def _stats(xs: list[float]) -> dict:
    xs = sorted(x for x in xs if x > 0)
    if not xs:
        return {"links": 0}
    return {"links": len(xs), "min_gbps": round(xs[0], 1), "median_gbps": round(xs[len(xs) // 2], 1),
            "max_gbps": round(xs[-1], 1)}


def xgmi_report(ndev: int, pair_bytes: int = 64 << 20, all_bytes: int = 64 << 20) -> dict:
    """Single links first (GPU 0 <-> GPU 1 and GPU 0 <-> GPU N-1, one at a
    time), then every ordered pair at once: the per-link numbers the agent
    attaches to the topology, measured on the node the job runs on.  Sized
    to finish in seconds at N = 8 (a link moves ~0.1 GB per ms)."""
    ndev = min(ndev, device_count())
    if ndev < 2:
        return {"devices": ndev, "error": "needs >= 2 visible GPUs"}
    single = {}
    for p in sorted({1, ndev - 1}):
        for src, dst in ((p, 0), (0, p)):
            try:
                g = probe_p2p(src, dst, pair_bytes, 4)
            except RuntimeError:  # peer access refused: reported as an unmeasured link
                g = None
            single[f"{src}->{dst}"] = round(g, 1) if g is not None else None
    mat = probe_p2p_all(ndev, all_bytes, 4)
    per_gpu_in = [round(sum(row), 1) for row in mat]
    return {"devices": ndev, "kernel": "lds_pull_kernel (global_load_lds, peer HBM -> LDS -> local HBM)",
            "single_link_gbps": single,
            "single_link": _stats([v for v in single.values() if v is not None]),
            "all_links": _stats([mat[d][s] for d in range(ndev) for s in range(ndev) if s != d]),
            "all_links_ingress_per_gpu_gbps": per_gpu_in,
            "matrix_gbps": [[round(x, 1) for x in row] for row in mat]}


def main(argv=None) -> int:
    import argparse
    import json

    ap = argparse.ArgumentParser(description="HIP HBM / xGMI bandwidth probes")
    ap.add_argument("--xgmi", type=int, default=0, metavar="N",
                    help="probe the xGMI links among the first N GPUs")
    ap.add_argument("--hbm", type=int, default=-1, metavar="DEV", help="HBM self-probe of one GPU")
    a = ap.parse_args(argv)
    out = {}
    if a.hbm >= 0:
        out["hbm"] = probe_hbm(a.hbm, 1 << 30, 10).__dict__
    if a.xgmi > 0:
        out["xgmi"] = xgmi_report(a.xgmi)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())


def gate_selftest(device: int = 0, raise_flag: bool = True, limit_us: int = 2000) -> int:
    """The all-links probe's start gate on one device: 1 = the kernel saw the
    host's flag, 0 = its bounded wait ran out (the flag was never raised)."""
    rc = lib().kgwe_probe_gate_selftest(device, 1 if raise_flag else 0, limit_us)
    if rc < 0:
        raise RuntimeError(f"kgwe_probe_gate_selftest failed rc={rc}")
    return rc
