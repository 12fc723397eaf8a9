"""amd-smi access (no NVML, no DCGM) + a GPU-utilisation sampler.

"GPU utilisation" on MI355X is amd-smi ``gfx_activity`` (GFX engine busy %),
the AMD counterpart of the SM-utilisation KPI the reference quotes
(reference: docs/PRD.md:439 "measured by DCGM"; README.md:157 87 %).

Everything degrades gracefully: on a host without the amdgpu driver (the CPU
build container) ``available()`` is False and samplers report ``None``.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field

_smi = None
_init_ok: bool | None = None
_lock = threading.Lock()


def _load():
    global _smi, _init_ok
    with _lock:
        if _init_ok is not None:
            return _smi if _init_ok else None
        try:
            import amdsmi  # noqa: PLC0415

            amdsmi.amdsmi_init()
            _smi = amdsmi
            _init_ok = True
        except Exception:  # noqa: BLE001 - no driver / no library
            _init_ok = False
        return _smi if _init_ok else None


def available() -> bool:
    return _load() is not None


def gpu_handles() -> list:
    smi = _load()
    if smi is None:
        return []
    try:
        return list(smi.amdsmi_get_processor_handles())
    except Exception:  # noqa: BLE001
        return []


def _norm_bdf(s: str) -> str:
    s = s.strip().lower()
    if s.count(":") == 1:  # "bb:dd.f" -> "0000:bb:dd.f"
        s = "0000:" + s
    return s


def handle_for_torch_device(index: int):
    """Map a torch/HIP device index to its amd-smi handle via PCI BDF (robust to
    HIP_VISIBLE_DEVICES renumbering)."""
    smi = _load()
    if smi is None:
        return None
    import torch  # noqa: PLC0415

    p = torch.cuda.get_device_properties(index)
    want = _norm_bdf(f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0")
    for h in gpu_handles():
        try:
            bdf = _norm_bdf(smi.amdsmi_get_gpu_device_bdf(h))
        except Exception:  # noqa: BLE001
            continue
        if bdf.rsplit(".", 1)[0] == want.rsplit(".", 1)[0]:
            return h
    hs = gpu_handles()
    return hs[index] if index < len(hs) else None


def gpu_processes_by_uuid(uuid: str) -> list:
    """Processes holding the GPU whose amd-smi uuid / kgwe id is ``uuid`` ([] when
    amd-smi is unavailable or the GPU is unknown)."""
    smi = _load()
    if smi is None:
        return []
    for h in gpu_handles():
        try:
            u = smi.amdsmi_get_gpu_device_uuid(h)
        except Exception:  # noqa: BLE001
            continue
        if uuid in (u, f"GPU-{u}") or uuid.endswith(str(u)):
            try:
                return list(smi.amdsmi_get_gpu_process_list(h) or [])
            except Exception:  # noqa: BLE001
                return []
    return []


def gfx_activity(handle) -> float | None:
    smi = _load()
    if smi is None or handle is None:
        return None
    try:
        a = smi.amdsmi_get_gpu_activity(handle)
        v = a.get("gfx_activity")
        return float(v) if isinstance(v, (int, float)) else None
    except Exception:  # noqa: BLE001
        return None


def snapshot(handle) -> dict:
    """Best-effort telemetry for the node agent / exporter."""
    smi = _load()
    out: dict = {}
    if smi is None or handle is None:
        return out

    def tryset(key, fn):
        try:
            out[key] = fn()
        except Exception:  # noqa: BLE001
            pass

    tryset("bdf", lambda: smi.amdsmi_get_gpu_device_bdf(handle))
    tryset("uuid", lambda: smi.amdsmi_get_gpu_device_uuid(handle))
    tryset("activity", lambda: smi.amdsmi_get_gpu_activity(handle))
    tryset("vram", lambda: smi.amdsmi_get_gpu_vram_usage(handle))
    tryset("compute_partition", lambda: smi.amdsmi_get_gpu_compute_partition(handle))
    tryset("memory_partition", lambda: smi.amdsmi_get_gpu_memory_partition(handle))
    tryset("numa", lambda: smi.amdsmi_get_gpu_topo_numa_affinity(handle))

    def metrics():
        m = smi.amdsmi_get_gpu_metrics_info(handle)
        keep = ("temperature_hotspot", "temperature_mem", "average_socket_power",
                "current_socket_power", "average_gfx_activity", "average_umc_activity",
                "current_gfxclk", "throttle_status", "xgmi_link_width", "xgmi_link_speed")
        return {k: m.get(k) for k in keep if k in m}

    tryset("metrics", metrics)
    return out


@dataclass
class UtilSampler:
    """Background sampler of gfx_activity for one GPU between start() and stop()."""

    device_index: int = 0
    interval_s: float = 0.05
    samples: list = field(default_factory=list)
    _thread: threading.Thread | None = None
    _stop: threading.Event = field(default_factory=threading.Event)

    def start(self) -> "UtilSampler":
        self.samples.clear()
        self._handle = handle_for_torch_device(self.device_index) if available() else None
        if self._handle is None:
            return self
        self._stop.clear()
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()
        return self

    def _run(self):
        while not self._stop.is_set():
            v = gfx_activity(self._handle)
            if v is not None:
                self.samples.append((time.perf_counter(), v))
            self._stop.wait(self.interval_s)

    def stop(self) -> "UtilSampler":
        if self._thread is not None:
            self._stop.set()
            self._thread.join(timeout=5)
            self._thread = None
        return self

    @property
    def mean(self) -> float | None:
        if not self.samples:
            return None
        return sum(v for _, v in self.samples) / len(self.samples)
