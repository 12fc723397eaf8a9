"""Per-phase timers for the scheduling path (+ optional span export).

The reference claims OpenTelemetry tracing (README.md:43, docs/PRD.md:290,440)
but imports nothing.  Here every extender verb and every controller
reconcile step is timed into a lock-free native histogram per phase; spans can
be exported as JSON lines (``KGWE_TRACE_FILE``) for offline analysis — the
OTLP SDK is not installed in this image, so no network exporter is wired.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time

_trace_file = os.environ.get("KGWE_TRACE_FILE")
_trace_lock = threading.Lock()


def _hist():
    from ..core import LatencyHistogram  # noqa: PLC0415 - native, loaded lazily

    return LatencyHistogram()


class PhaseTimer:
    def __init__(self):
        self._h: dict = {}
        self._lock = threading.Lock()

    @contextlib.contextmanager
    def phase(self, name: str, **attrs):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            dt = (time.perf_counter() - t0) * 1000.0
            h = self._h.get(name)
            if h is None:
                with self._lock:
                    h = self._h.setdefault(name, _hist())
            h.record_ms(dt)
            if _trace_file:
                rec = {"span": name, "ms": round(dt, 4), "ts": time.time(), **attrs}
                with _trace_lock, open(_trace_file, "a") as f:
                    f.write(json.dumps(rec) + "\n")

    def summary(self) -> dict:
        out = {}
        for k, h in list(self._h.items()):
            out[k] = {"count": h.count(), "mean_ms": round(h.mean_ms(), 4),
                      "p50_ms": h.quantile_ms(0.5), "p99_ms": h.quantile_ms(0.99),
                      "max_ms": h.max_ms()}
        return out
