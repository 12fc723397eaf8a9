"""Per-phase timers for the scheduling path, with span export.

The reference claims OpenTelemetry tracing (README.md:43, docs/PRD.md:290,440;
``opentelemetry-*`` in src/optimizer/requirements.txt:25-27) but imports
nothing.  Here every extender verb and controller reconcile step is timed into
a lock-free native histogram per phase, and spans can leave the process two
ways:

* ``KGWE_TRACE_FILE``: JSON lines, for offline analysis;
* ``OTEL_EXPORTER_OTLP_ENDPOINT`` (or ``..._TRACES_ENDPOINT``): OTLP/HTTP with
  the JSON encoding (``POST <endpoint>/v1/traces``), which an OpenTelemetry
  Collector accepts directly.  The SDK is not installed in this image, so the
  exporter is written against the wire format: spans are queued (bounded,
  dropped and counted on overflow — the scheduling path never blocks on
  telemetry) and shipped in batches by one background thread.

Spans of one pod's scheduling cycle (filter -> prioritize -> bind) share a
trace id derived from the pod uid, so a collector shows the whole cycle as one
trace without propagating context through kube-scheduler.
"""
from __future__ import annotations

import contextlib
import hashlib
import json
import os
import queue
import secrets
import threading
import time
import urllib.request

_trace_file = os.environ.get("KGWE_TRACE_FILE")
_trace_lock = threading.Lock()


def _hist():
    from ..core import LatencyHistogram  # noqa: PLC0415 - native, loaded lazily

    return LatencyHistogram()


def trace_id_for(key: str) -> str:
    """32-hex OTLP trace id, stable per key (pod uid)."""
    return hashlib.sha256(key.encode()).hexdigest()[:32]


def _attr(k: str, v) -> dict:
    if isinstance(v, bool):
        val = {"boolValue": v}
    elif isinstance(v, int):
        val = {"intValue": str(v)}
    elif isinstance(v, float):
        val = {"doubleValue": v}
    else:
        val = {"stringValue": str(v)}
    return {"key": k, "value": val}


class OtlpExporter:
    """Batching OTLP/HTTP JSON span exporter (no SDK dependency)."""

    def __init__(self, endpoint: str, service: str = "kgwe-controller", max_queue: int = 8192,
                 batch: int = 512, interval_s: float = 1.0, timeout_s: float = 5.0):
        ep = endpoint.rstrip("/")
        self.url = ep if ep.endswith("/v1/traces") else ep + "/v1/traces"
        self.service = service
        self.batch, self.interval_s, self.timeout_s = batch, interval_s, timeout_s
        self.q: queue.Queue = queue.Queue(max_queue)
        self.dropped = self.exported = self.failed_posts = 0
        self._stop = threading.Event()
        self._flushed = threading.Condition()
        self._t = threading.Thread(target=self._run, name="otlp-export", daemon=True)
        self._t.start()

    def add(self, name: str, start_ns: int, end_ns: int, attrs: dict, trace_key: str | None = None):
        span = {"traceId": trace_id_for(trace_key) if trace_key else secrets.token_hex(16),
                "spanId": secrets.token_hex(8), "name": name, "kind": 2,  # SPAN_KIND_SERVER
                "startTimeUnixNano": str(start_ns), "endTimeUnixNano": str(end_ns),
                "attributes": [_attr(k, v) for k, v in attrs.items()],
                "status": {"code": 2 if attrs.get("error") else 1}}
        try:
            self.q.put_nowait(span)
        except queue.Full:
            self.dropped += 1

    def _payload(self, spans: list) -> bytes:
        return json.dumps({"resourceSpans": [{
            "resource": {"attributes": [_attr("service.name", self.service),
                                        _attr("service.namespace", "kgwe"),
                                        _attr("host.name", os.uname().nodename)]},
            "scopeSpans": [{"scope": {"name": "kgwe.tracing", "version": "1"},
                            "spans": spans}]}]}).encode()

    def _post(self, spans: list) -> None:
        req = urllib.request.Request(self.url, data=self._payload(spans), method="POST",
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=self.timeout_s) as r:
                r.read()
            self.exported += len(spans)
        except Exception:  # noqa: BLE001 - telemetry must never take the scheduler down
            self.failed_posts += 1
            self.dropped += len(spans)

    def _drain(self) -> list:
        out = []
        while len(out) < self.batch:
            try:
                out.append(self.q.get_nowait())
            except queue.Empty:
                break
        return out

    def _run(self):
        while not self._stop.is_set():
            spans = self._drain()
            if spans:
                self._post(spans)
            else:
                with self._flushed:
                    self._flushed.notify_all()
                self._stop.wait(self.interval_s)
        while spans := self._drain():
            self._post(spans)

    def flush(self, timeout_s: float = 10.0) -> None:
        deadline = time.monotonic() + timeout_s
        while not self.q.empty() and time.monotonic() < deadline:
            with self._flushed:
                self._flushed.wait(0.05)
        time.sleep(0.05)  # the batch in flight

    def close(self) -> None:
        self._stop.set()
        self._t.join(timeout=self.timeout_s + 1)


_exporter: OtlpExporter | None = None
_exporter_lock = threading.Lock()


def otlp_exporter() -> OtlpExporter | None:
    """Process-wide exporter from the standard OTEL_* environment, or None."""
    global _exporter
    ep = (os.environ.get("OTEL_EXPORTER_OTLP_TRACES_ENDPOINT")
          or os.environ.get("OTEL_EXPORTER_OTLP_ENDPOINT"))
    if not ep:
        return None
    with _exporter_lock:
        if _exporter is None:
            _exporter = OtlpExporter(ep, os.environ.get("OTEL_SERVICE_NAME", "kgwe-controller"))
        return _exporter


class PhaseTimer:
    def __init__(self, exporter: OtlpExporter | None = None):
        self._h: dict = {}
        self._lock = threading.Lock()
        self.exporter = exporter if exporter is not None else otlp_exporter()

    @contextlib.contextmanager
    def phase(self, name: str, trace_key: str | None = None, **attrs):
        t0 = time.perf_counter()
        t0_ns = time.time_ns()
        try:
            yield attrs  # the body may add attributes (e.g. the bound node)
        except Exception as e:
            attrs["error"] = f"{type(e).__name__}: {e}"
            raise
        finally:
            dt = (time.perf_counter() - t0) * 1000.0
            h = self._h.get(name)
            if h is None:
                with self._lock:
                    h = self._h.setdefault(name, _hist())
            h.record_ms(dt)
            if self.exporter is not None:
                self.exporter.add("kgwe." + name, t0_ns, t0_ns + int(dt * 1e6), attrs, trace_key)
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
