"""kube-scheduler extender HTTP server (filter / prioritize / bind).

Implements the contract declared by the reference's scheduler ConfigMap
(deploy/helm/kgwe/templates/scheduler-configmap.yaml:61-79: urlPrefix on the
controller service :8080, verbs filter / prioritize / bind, weight 100,
nodeCacheCapable false, ignorable false), which the reference never served.
The socket, the HTTP parsing and the verbs are native
(``native/core/http_server.cpp`` on ``kgwe.core.Platform``); this module
configures that server and supplies the pieces that need the cluster
credentials or Python services.

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
    """The extender endpoint of the controller.

    The socket, HTTP parsing and the four verbs are served by the native
    server (``native/core/http_server.cpp``): filter / prioritize / preempt
    never enter Python, bind enters it once for the apiserver write
    (``_bind_sink``), and gang members' binds are held server-side until the
    gang is complete (Permit).  Python serves what is left through
    ``_fallback``: the admission webhook and agent-push ``routes``, the
    ``/debug/*`` pages, and — only while a span exporter is configured — the
    verbs themselves, each wrapped in a trace span.
    """

    def __init__(self, platform: Platform, kube=None, host: str = "0.0.0.0", port: int = 8080,
                 url_prefix: str = "", routes: dict | None = None, workers: int = 0,
                 gang_hold_s: float = 25.0, auth_routes=()):
        """routes: extra POST handlers {path_prefix: fn(path, body) -> (code, bytes)}
        (the controller mounts the admission webhook and the node-agent push
        endpoint here); a prefix also listed in auth_routes is called as
        fn(path, body, authorization_header).  gang_hold_s: how long a gang member's bind request is
        held for the rest of its gang before it is answered with a retryable
        error (keep it below the scheduler's extender httpTimeout, 30 s in the
        reference's profile); 0 answers at once, as an extender without Permit
        would."""
        from ..core import native  # noqa: PLC0415

        self.platform = platform
        self.kube = kube
        self.host = host
        self.prefix = url_prefix.rstrip("/")
        self.routes = dict(routes or {})
        self.auth_routes = set(auth_routes or ())
        self._ready = lambda: True
        self._tracer = tracing.PhaseTimer()
        self._srv = native.HttpServer(platform.raw, host, int(port), self.prefix, int(workers),
                                      int(gang_hold_s * 1000))
        if kube is not None:
            self._srv.set_bind_sink(self._bind_sink)
            self._srv.set_pod_lookup(self._pod_lookup)
        self._srv.set_fallback(self._fallback)
        self._stop = threading.Event()
        self._ready_thread: threading.Thread | None = None
        self._extra: list = []
        self._started = False

    # ---- configuration -----------------------------------------------------
    @property
    def tracer(self) -> tracing.PhaseTimer:
        return self._tracer

    @tracer.setter
    def tracer(self, t: tracing.PhaseTimer) -> None:
        self._tracer = t
        self._srv.set_verbs_via_fallback(t.exporter is not None)

    @property
    def ready(self):
        return self._ready

    @ready.setter
    def ready(self, fn) -> None:
        """fn() -> bool, polled into the native /readyz flag (only the lease
        holder is Ready, so the Service routes verbs to the authoritative ledger)."""
        self._ready = fn
        self._srv.set_ready(bool(fn()))

    @property
    def address(self) -> tuple:
        return self.host if self.host not in ("", "0.0.0.0", "::") else "127.0.0.1", self._srv.port

    @property
    def url(self) -> str:
        h, p = self.address
        return f"http://{h}:{p}{self.prefix}"

    def stats(self) -> dict:
        """Native server statistics: per-verb latency (request read -> reply
        written), connections, held gang binds."""
        return json.loads(self._srv.stats_json())

    def phase_summary(self) -> dict:
        """Verb latencies of the native server merged with the Python-side
        phase timers (traced verbs, fallback routes)."""
        out = {k: {kk: v[kk] for kk in ("count", "mean_ms", "p50_ms", "p99_ms", "max_ms")}
               for k, v in self.stats().get("verbs", {}).items()}
        for k, v in self._tracer.summary().items():
            out.setdefault(k, v)
        return out

    # ---- hooks the native server calls ----------------------------------------
    def _bind_sink(self, args: bytes, result: bytes) -> str:
        """Apiserver write of a successful bind; "" or the error (the native
        server then releases the reservation and fails the verb)."""
        a = json.loads(args)
        pl = json.loads(result).get("placement") or {}
        try:
            self._write_binding(a, pl)
        except Exception as e:  # noqa: BLE001
            return f"{type(e).__name__}: {e}"
        return ""

    def _pod_lookup(self, ns: str, name: str) -> str:
        pod = self.kube.get_pod(ns, name)
        return json.dumps(pod) if pod else ""

    def _write_binding(self, args: dict, pl: dict) -> None:
        ns = args.get("podNamespace") or args.get("PodNamespace") or "default"
        name = args.get("podName") or args.get("PodName")
        uid = args.get("podUID") or args.get("PodUID") or ""
        node = args.get("node") or args.get("Node")
        ann = {ANN_GPUS: ",".join(pl.get("gpus", []) or ([pl["shared_gpu"]] if pl.get("shared_gpu") else [])),
               ANN_PARTS: ",".join(pl.get("partitions", [])),
               ANN_ENV: json.dumps(pl.get("env", {}), sort_keys=True), ANN_NODE: node,
               ANN_SCORE: str(pl.get("score", 0)), ANN_BW: f"{pl.get('bandwidth_gbps', 0.0):.1f}",
               ANN_ALLOC: json.dumps(allocation_record(pl), sort_keys=True)}
        # one apiserver write: the Binding carries the placement annotations
        # (the pod is never seen bound without its placement, or the reverse)
        self.kube.bind_pod(ns, name, node, uid, annotations=ann)

    def _fallback(self, method: str, path: str, raw: bytes, authorization: str = ""):
        """(code, body, content type) for every request the native server does
        not answer itself.  Routes registered with ``auth_routes`` get the
        request's Authorization header as a third argument."""
        if method == "GET":
            if path == "/debug/allocations":
                return 200, json.dumps(self.platform.allocations()).encode(), "application/json"
            if path == "/debug/scheduler":
                m = self.platform.scheduler_metrics()
                m["phases"] = self.phase_summary()
                m["server"] = self.stats()
                return 200, json.dumps(m).encode(), "application/json"
            if path == "/debug/topology":
                return 200, json.dumps(self.platform.snapshot()).encode(), "application/json"
            if path in ("/healthz", "/health"):
                return 200, b"ok", "text/plain"
            if path == "/readyz":
                return (200, b"ok", "text/plain") if self._ready() else (503, b"standby", "text/plain")
            if path == "/metrics":
                return 200, self.platform.expose_metrics().encode(), "text/plain; version=0.0.4"
            return 404, b'{"error":"not found"}', "application/json"
        if method != "POST":
            return 404, b'{"error":"not found"}', "application/json"
        body = raw.decode()
        for pre, fn in self.routes.items():
            if path.startswith(pre):
                try:
                    code, data = (fn(path, body, authorization) if pre in self.auth_routes
                                  else fn(path, body))
                except Exception as e:  # noqa: BLE001
                    code, data = 500, json.dumps({"error": str(e)}).encode()
                return code, data, "application/json"
        verb = path[len(self.prefix):].strip("/")
        key = self.trace_key(verb, body) if self._tracer.exporter else None
        try:
            if verb == "filter":
                with self._tracer.phase("filter", key, verb="filter"):
                    out = self.platform.filter(body)
            elif verb == "prioritize":
                with self._tracer.phase("prioritize", key, verb="prioritize"):
                    out = self.platform.prioritize(body)
            elif verb == "bind":
                with self._tracer.phase("bind", key, verb="bind"):
                    out = json.dumps(self.handle_bind(body))
            elif verb == "preempt":
                with self._tracer.phase("preempt", key, verb="preempt"):
                    out = self.platform.preempt(body)
            else:
                return 404, b'{"error":"unknown verb"}', "application/json"
        except Exception as e:  # noqa: BLE001 - contract: errors go in the body
            out = json.dumps({"error": f"{type(e).__name__}: {e}"})
        return 200, out.encode(), "application/json"

    def add_tls_listener(self, host: str, port: int, certfile: str, keyfile: str):
        """Serve the fallback routes over HTTPS on a second port — the apiserver
        only calls admission webhooks over TLS, while kube-scheduler talks to the
        extender in-cluster over plain HTTP (reference webhook settings:
        deploy/helm/kgwe/values.yaml:375-392, service port 443)."""
        import ssl  # noqa: PLC0415

        outer = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"
            disable_nagle_algorithm = True

            def log_message(self, *a):
                pass

            def _serve(self, method: str):
                n = int(self.headers.get("Content-Length") or 0)
                raw = self.rfile.read(n) if n else b"{}"
                code, data, ctype = outer._fallback(method, self.path.split("?")[0], raw,
                                                    self.headers.get("Authorization") or "")
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):
                self._serve("GET")

            def do_POST(self):
                self._serve("POST")

        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        ctx.load_cert_chain(certfile, keyfile)
        srv = ThreadingHTTPServer((host, port), H)
        srv.daemon_threads = True
        srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
        t = threading.Thread(target=srv.serve_forever, daemon=True)
        self._extra.append((srv, t))
        if self._started:
            t.start()
        return srv

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
        """The bind verb on the Python path (traced verbs, direct callers):
        ExtenderBindingArgs -> ExtenderBindingResult.  A gang member whose gang
        is incomplete gets the retryable "waiting" error here; the native
        server holds such requests instead."""
        args = json.loads(body)
        ns = args.get("podNamespace") or args.get("PodNamespace") or "default"
        name = args.get("podName") or args.get("PodName")
        uid = args.get("podUID") or args.get("PodUID") or ""
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
            try:
                self._write_binding(args, pl)
            except Exception as e:  # noqa: BLE001
                self.platform.release(pl.get("uid") or uid)
                return {"error": f"binding failed: {e}"}
        return {}

    def _poll_ready(self):
        while not self._stop.wait(0.2):
            try:
                self._srv.set_ready(bool(self._ready()))
            except Exception:  # noqa: BLE001 - a broken probe reads as not ready
                self._srv.set_ready(False)

    def start(self) -> "ExtenderServer":
        self._srv.set_verbs_via_fallback(self._tracer.exporter is not None)
        self._srv.start()
        self._started = True
        self._ready_thread = threading.Thread(target=self._poll_ready, daemon=True)
        self._ready_thread.start()
        for _, t in self._extra:
            t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        for srv, _ in self._extra:
            srv.shutdown()
            srv.server_close()
        self._srv.stop()
