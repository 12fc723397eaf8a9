"""kube-scheduler extender HTTP server (filter / prioritize / bind).

Implements the contract declared by the reference's scheduler ConfigMap
(deploy/helm/kgwe/templates/scheduler-configmap.yaml:61-79: urlPrefix on the
controller service :8080, verbs filter / prioritize / bind, weight 100,
nodeCacheCapable false, ignorable false) — which the reference never served
(SURVEY.md D1/N7).  This module is only socket plumbing: request bodies go
straight into the C++ core (``kgwe.core.Platform``) and its JSON replies go
straight back; the GIL is released inside the core so concurrent extender
calls score in parallel.

On a successful bind the shell also:
  * POSTs the pods/binding subresource to the apiserver;
  * writes the placement to pod annotations (kgwe.amd.com/allocated-gpus,
    kgwe.amd.com/rccl-env, ...) — consumed at container start by
    ``kgwe.launch`` (downward API) to export HIP_VISIBLE_DEVICES and the RCCL
    rank environment;
  * (inside the C++ bind) records the pod-create -> bind latency into the
    p99 histogram, from the webhook's microsecond admission stamp or the
    pod's first filter call.
"""
from __future__ import annotations

import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from ..core import Platform
from ..utils import tracing

ANN_GPUS = "kgwe.amd.com/allocated-gpus"
ANN_PARTS = "kgwe.amd.com/allocated-partitions"
ANN_ENV = "kgwe.amd.com/rccl-env"
ANN_NODE = "kgwe.amd.com/node"
ANN_SCORE = "kgwe.amd.com/score"
ANN_BW = "kgwe.amd.com/estimated-bandwidth-gbps"
# The full ledger entry (scheduling semantics included: priority,
# preemptible, type, gang, share CU range) — what a new leader restores.
ANN_ALLOC = "kgwe.amd.com/allocation"


def allocation_record(pl: dict) -> dict:
    """Ledger entry of a bind placement, in the form
    ``Platform.restore_allocation`` takes back."""
    w = pl.get("workload") or {}
    rec = {"uid": pl.get("uid", ""), "node": pl.get("node", ""), "gpus": pl.get("gpus", []),
           "partitions": pl.get("partitions", []), "namespace": w.get("namespace", "default"),
           "team": w.get("team", ""), "type": w.get("type", "Training"),
           "priority": w.get("priority", 0), "preemptible": w.get("preemptible", True),
           "gang": w.get("gang", ""), "gang_size": w.get("gang_size", 0),
           "bandwidth_gbps": pl.get("bandwidth_gbps", 0.0)}
    if pl.get("sharing"):
        rec.update({k: pl[k] for k in ("sharing", "shared_gpu", "cu_begin", "cu_end", "share_memory_gb")
                    if k in pl})
    return rec


class ExtenderServer:
    def __init__(self, platform: Platform, kube=None, host: str = "0.0.0.0", port: int = 8080,
                 url_prefix: str = "", routes: dict | None = None):
        """routes: extra POST handlers {path_prefix: fn(path, body) -> (code, bytes)}
        (the controller mounts the admission webhook and the node-agent push
        endpoint here)."""
        self.platform = platform
        self.kube = kube
        self.prefix = url_prefix.rstrip("/")
        self.routes = dict(routes or {})
        self.ready = lambda: True
        self.tracer = tracing.PhaseTimer()
        outer = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"
            disable_nagle_algorithm = True

            def log_message(self, *a):
                pass

            def _send(self, code: int, data: bytes, ctype="application/json"):
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):
                p = self.path.split("?")[0]
                if p in ("/healthz", "/health"):
                    return self._send(200, b"ok", "text/plain")
                if p == "/readyz":
                    # Only the lease holder is Ready, so the Service routes
                    # extender verbs and agent pushes to the one replica whose
                    # ledger is authoritative.
                    if outer.ready():
                        return self._send(200, b"ok", "text/plain")
                    return self._send(503, b"standby", "text/plain")
                if p == "/metrics":
                    return self._send(200, outer.platform.expose_metrics().encode(),
                                      "text/plain; version=0.0.4")
                if p == "/debug/allocations":
                    return self._send(200, json.dumps(outer.platform.allocations()).encode())
                if p == "/debug/scheduler":
                    m = outer.platform.scheduler_metrics()
                    m["phases"] = outer.tracer.summary()
                    return self._send(200, json.dumps(m).encode())
                if p == "/debug/topology":
                    return self._send(200, json.dumps(outer.platform.snapshot()).encode())
                return self._send(404, b'{"error":"not found"}')

            def do_POST(self):
                n = int(self.headers.get("Content-Length") or 0)
                raw = self.rfile.read(n) if n else b"{}"
                path = self.path.split("?")[0]
                verb = path[len(outer.prefix):].strip("/")
                if verb in ("filter", "prioritize") and not outer.tracer.exporter:
                    # hot path: bytes straight into the C++ scanner and back
                    try:
                        with outer.tracer.phase(verb, None, verb=verb):
                            data = (outer.platform.filter_bytes(raw) if verb == "filter"
                                    else outer.platform.prioritize_bytes(raw))
                    except Exception as e:  # noqa: BLE001 - contract: errors go in the body
                        data = json.dumps({"error": f"{type(e).__name__}: {e}"}).encode()
                    return self._send(200, data)
                body = raw.decode()
                for pre, fn in outer.routes.items():
                    if path.startswith(pre):
                        try:
                            code, data = fn(path, body)
                        except Exception as e:  # noqa: BLE001
                            code, data = 500, json.dumps({"error": str(e)}).encode()
                        return self._send(code, data)
                verb = path[len(outer.prefix):].strip("/")
                key = outer.trace_key(verb, body) if outer.tracer.exporter else None
                try:
                    if verb == "filter":
                        with outer.tracer.phase("filter", key, verb="filter"):
                            out = outer.platform.filter(body)
                    elif verb == "prioritize":
                        with outer.tracer.phase("prioritize", key, verb="prioritize"):
                            out = outer.platform.prioritize(body)
                    elif verb == "bind":
                        with outer.tracer.phase("bind", key, verb="bind"):
                            out = json.dumps(outer.handle_bind(body))
                    elif verb == "preempt":
                        with outer.tracer.phase("preempt", key, verb="preempt"):
                            out = outer.platform.preempt(body)
                    else:
                        return self._send(404, b'{"error":"unknown verb"}')
                except Exception as e:  # noqa: BLE001 - contract: errors go in the body
                    out = json.dumps({"error": f"{type(e).__name__}: {e}"})
                return self._send(200, out.encode())

        self._handler = H
        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self._extra: list = []

    def add_tls_listener(self, host: str, port: int, certfile: str, keyfile: str):
        """Serve the same routes over HTTPS on a second port — the apiserver only
        calls admission webhooks over TLS, while kube-scheduler talks to the
        extender in-cluster over plain HTTP (reference webhook settings:
        deploy/helm/kgwe/values.yaml:375-392, service port 443)."""
        import ssl  # noqa: PLC0415

        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        ctx.load_cert_chain(certfile, keyfile)
        srv = ThreadingHTTPServer((host, port), self._handler)
        srv.daemon_threads = True
        srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
        t = threading.Thread(target=srv.serve_forever, daemon=True)
        self._extra.append((srv, t))
        return srv

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}{self.prefix}"

    @staticmethod
    def trace_key(verb: str, body: str) -> str | None:
        """Pod uid of an extender request: one trace per pod scheduling cycle."""
        try:
            j = json.loads(body)
        except ValueError:
            return None
        if verb == "bind":
            return j.get("podUID") or f'{j.get("podNamespace", "")}/{j.get("podName", "")}'
        meta = (j.get("pod") or j.get("Pod") or {}).get("metadata", {})
        return meta.get("uid") or f'{meta.get("namespace", "")}/{meta.get("name", "")}'

    def handle_bind(self, body: str) -> dict:
        args = json.loads(body)
        ns = args.get("podNamespace") or args.get("PodNamespace") or "default"
        name = args.get("podName") or args.get("PodName")
        uid = args.get("podUID") or args.get("PodUID") or ""
        node = args.get("node") or args.get("Node")
        pod = None
        res = self.platform.bind(body)
        result = res.get("result", {})
        if result.get("error") and "no filter call seen" in result["error"] and self.kube is not None:
            pod = self.kube.get_pod(ns, name)  # extender restarted between verbs
            res = self.platform.bind(body, pod)
            result = res.get("result", {})
        if result.get("error"):
            return result
        pl = res["placement"]
        if self.kube is not None:
            ann = {ANN_GPUS: ",".join(pl.get("gpus", []) or ([pl["shared_gpu"]] if pl.get("shared_gpu") else [])),
                   ANN_PARTS: ",".join(pl.get("partitions", [])),
                   ANN_ENV: json.dumps(pl.get("env", {}), sort_keys=True), ANN_NODE: node,
                   ANN_SCORE: str(pl.get("score", 0)), ANN_BW: f"{pl.get('bandwidth_gbps', 0.0):.1f}",
                   ANN_ALLOC: json.dumps(allocation_record(pl), sort_keys=True)}
            try:
                # one apiserver write: the Binding carries the placement annotations
                # (same latency as PATCH + Binding on the bench, measured; and the pod
                # is never seen bound without its placement, or the reverse)
                self.kube.bind_pod(ns, name, node, uid, annotations=ann)
            except Exception as e:  # noqa: BLE001
                self.platform.release(pl.get("uid") or uid)
                return {"error": f"binding failed: {e}"}
        return {}

    def start(self) -> "ExtenderServer":
        self.thread.start()
        for _, t in self._extra:
            t.start()
        return self

    def stop(self) -> None:
        for srv, _ in self._extra:
            srv.shutdown()
            srv.server_close()
        self.httpd.shutdown()
        self.httpd.server_close()
