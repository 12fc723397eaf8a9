"""OTLP/HTTP JSON span export of the extender's scheduling phases (reference
README.md:43 / docs/PRD.md:440: OpenTelemetry claimed, absent).
A stdlib HTTP server stands in for an OpenTelemetry Collector."""
from __future__ import annotations

import json
import threading
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from kgwe.core import Platform, make_fixture
from kgwe.extender.server import ExtenderServer
from kgwe.utils import tracing


@pytest.fixture
def collector():
    got = []

    class H(BaseHTTPRequestHandler):
        def do_POST(self):
            n = int(self.headers["Content-Length"])
            got.append((self.path, self.headers["Content-Type"], json.loads(self.rfile.read(n))))
            self.send_response(200)
            self.send_header("Content-Length", "2")
            self.end_headers()
            self.wfile.write(b"{}")

        def log_message(self, *a):
            pass

    srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    yield f"http://127.0.0.1:{srv.server_port}", got
    srv.shutdown()


def _post(url, body):
    req = urllib.request.Request(url, data=json.dumps(body).encode(), method="POST",
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=10) as r:
        return json.loads(r.read())


def test_extender_cycle_exports_one_trace_per_pod(collector):
    url, got = collector
    exp = tracing.OtlpExporter(url, service="kgwe-test", interval_s=0.05)
    plat = Platform({})
    plat.add_fake_node(make_fixture("n0", 8, 2))
    ext = ExtenderServer(plat, host="127.0.0.1", port=0)
    ext.tracer = tracing.PhaseTimer(exporter=exp)
    ext.start()
    try:
        pod = {"metadata": {"name": "p", "namespace": "ml", "uid": "uid-123"},
               "spec": {"containers": [{"name": "c", "resources": {"limits": {"amd.com/gpu": "2"}}}]}}
        f = _post(ext.url + "/filter", {"pod": pod, "nodenames": ["n0"]})
        assert f.get("nodenames") == ["n0"], f
        _post(ext.url + "/prioritize", {"pod": pod, "nodenames": ["n0"]})
        b = _post(ext.url + "/bind", {"podName": "p", "podNamespace": "ml", "podUID": "uid-123",
                                      "node": "n0"})
        assert not b.get("error"), b
        exp.flush()
    finally:
        ext.stop()
        exp.close()
    spans = [s for path, ctype, body in got for rs in body["resourceSpans"]
             for ss in rs["scopeSpans"] for s in ss["spans"]]
    assert all(path == "/v1/traces" and ctype == "application/json" for path, ctype, _ in got)
    names = [s["name"] for s in spans]
    assert names == ["kgwe.filter", "kgwe.prioritize", "kgwe.bind"], names
    assert len({s["traceId"] for s in spans}) == 1, "one trace per pod cycle"
    assert spans[0]["traceId"] == tracing.trace_id_for("uid-123")
    assert len({s["spanId"] for s in spans}) == 3
    for s in spans:
        assert len(s["traceId"]) == 32 and len(s["spanId"]) == 16
        assert int(s["endTimeUnixNano"]) >= int(s["startTimeUnixNano"]) > 0
    res = got[0][2]["resourceSpans"][0]["resource"]["attributes"]
    assert {"key": "service.name", "value": {"stringValue": "kgwe-test"}} in res
    assert exp.exported == 3 and exp.dropped == 0


def test_exporter_never_blocks_and_counts_drops():
    exp = tracing.OtlpExporter("http://127.0.0.1:9", max_queue=4, interval_s=10.0, timeout_s=0.2)
    for i in range(10):
        exp.add("x", 1, 2, {"i": i})
    assert exp.dropped >= 6  # full queue: dropped, not blocked
    exp.close()
    assert exp.failed_posts >= 1  # unreachable collector: counted, never raised


def test_env_configures_process_exporter(monkeypatch):
    monkeypatch.setattr(tracing, "_exporter", None)
    monkeypatch.delenv("OTEL_EXPORTER_OTLP_TRACES_ENDPOINT", raising=False)
    monkeypatch.delenv("OTEL_EXPORTER_OTLP_ENDPOINT", raising=False)
    assert tracing.otlp_exporter() is None
    assert tracing.PhaseTimer().exporter is None
    monkeypatch.setenv("OTEL_EXPORTER_OTLP_ENDPOINT", "http://127.0.0.1:4318")
    e = tracing.otlp_exporter()
    assert e is not None and e.url == "http://127.0.0.1:4318/v1/traces"
    e.close()
    monkeypatch.setattr(tracing, "_exporter", None)
