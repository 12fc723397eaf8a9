"""In-process fake kube-apiserver (nodes, pods + binding, events, kgwe CRDs).

Stands in for a cluster where kind / kubectl / Go are absent: it speaks enough of the Kubernetes REST surface — list / get /
create / merge-patch / delete, the pods/binding subresource, CR status
subresources and a long-poll watch — for the controller, the extender and the
kube-scheduler simulator to run unchanged against it, over real HTTP.
"""
from __future__ import annotations

import bisect
import copy
import json
import re
import threading
import time
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


def _merge(dst: dict, patch: dict) -> dict:
    """RFC 7386 JSON merge patch."""
    for k, v in patch.items():
        if v is None:
            dst.pop(k, None)
        elif isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


class Store:
    def __init__(self):
        self.lock = threading.Condition()
        self.rv = 0
        self.objs: dict[tuple, dict] = {}  # (collection, namespace, name) -> obj
        self.log: list[tuple[int, str, str, dict]] = []  # (rv, collection, type, obj)

    def _bump(self, coll, typ, obj):
        self.rv += 1
        obj["metadata"]["resourceVersion"] = str(self.rv)
        self.log.append((self.rv, coll, typ, copy.deepcopy(obj)))
        if len(self.log) > 50000:
            del self.log[:10000]
        self.lock.notify_all()

    def create(self, coll, ns, obj):
        with self.lock:
            md = obj.setdefault("metadata", {})
            name = md.get("name")
            if not name and md.get("generateName"):
                name = md["generateName"] + uuid.uuid4().hex[:5]
                md["name"] = name
            key = (coll, ns, name)
            if key in self.objs:
                return None
            md.setdefault("uid", str(uuid.uuid4()))
            md.setdefault("creationTimestamp", time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
            md["_created"] = time.perf_counter()
            if ns:
                md["namespace"] = ns
            self.objs[key] = obj
            self._bump(coll, "ADDED", obj)
            return obj

    def get(self, coll, ns, name):
        with self.lock:
            o = self.objs.get((coll, ns, name))
            return copy.deepcopy(o) if o else None

    def list(self, coll, ns=None):
        with self.lock:
            return [copy.deepcopy(o) for (c, n, _), o in self.objs.items()
                    if c == coll and (ns is None or n == ns)]

    def patch(self, coll, ns, name, patch):
        with self.lock:
            o = self.objs.get((coll, ns, name))
            if o is None:
                return None
            _merge(o, patch)
            self._bump(coll, "MODIFIED", o)
            return copy.deepcopy(o)

    def delete(self, coll, ns, name):
        with self.lock:
            o = self.objs.pop((coll, ns, name), None)
            if o is not None:
                self._bump(coll, "DELETED", o)
            return o

    def events_since(self, coll, ns, rv, timeout):
        deadline = time.time() + timeout
        with self.lock:
            while True:
                # The log is ordered by rv: binary-search the first newer entry.
                start = bisect.bisect_right(self.log, rv, key=lambda e: e[0])
                evs = [{"type": t, "object": o} for (r, c, t, o) in self.log[start:]
                       if c == coll and (ns is None or o["metadata"].get("namespace") == ns)]
                if evs or time.time() >= deadline:
                    return evs, self.rv
                self.lock.wait(timeout=max(0.0, deadline - time.time()))


_CORE = re.compile(r"^/api/v1(?:/namespaces/(?P<ns>[^/]+))?/(?P<coll>nodes|pods|events)"
                   r"(?:/(?P<name>[^/]+))?(?:/(?P<sub>binding|status))?$")
_CRD = re.compile(r"^/apis/kgwe\.amd\.com/v1(?:/namespaces/(?P<ns>[^/]+))?/(?P<coll>gpuworkloads|"
                  r"partitionstrategies|gpubudgets)(?:/(?P<name>[^/]+))?(?:/(?P<sub>status))?$")
_LEASE = re.compile(r"^/apis/coordination\.k8s\.io/v1/namespaces/(?P<ns>[^/]+)/(?P<coll>leases)"
                    r"(?:/(?P<name>[^/]+))?(?P<sub>)$")


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    disable_nagle_algorithm = True
    store: Store = None  # set by FakeApiServer

    def log_message(self, *a):  # silence
        pass

    def _send(self, code, obj):
        data = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def _body(self):
        n = int(self.headers.get("Content-Length") or 0)
        return json.loads(self.rfile.read(n) or b"{}") if n else {}

    def _route(self):
        path, _, q = self.path.partition("?")
        qs = dict(p.split("=", 1) for p in q.split("&") if "=" in p)
        m = _CORE.match(path) or _CRD.match(path) or _LEASE.match(path)
        if not m:
            return None, qs
        d = m.groupdict()
        d["sub"] = d.get("sub") or None
        if d["coll"] == "nodes" or d["coll"] == "partitionstrategies":
            d["ns"] = None
        return d, qs

    def do_GET(self):
        d, qs = self._route()
        if d is None:
            return self._send(404, {"kind": "Status", "message": "not found"})
        st = self.store
        if qs.get("watch") in ("1", "true"):
            evs, rv = st.events_since(d["coll"], d["ns"], int(qs.get("resourceVersion", "0")),
                                      float(qs.get("timeoutSeconds", "5")))
            return self._send(200, {"events": evs, "resourceVersion": rv})
        if d["name"]:
            o = st.get(d["coll"], d["ns"], d["name"])
            return self._send(200, o) if o else self._send(404, {"kind": "Status", "reason": "NotFound"})
        items = st.list(d["coll"], d["ns"])
        fs = qs.get("fieldSelector", "")
        if fs.startswith("spec.nodeName%3D") or fs.startswith("spec.nodeName="):
            want = fs.split("%3D")[-1].split("=")[-1]
            items = [i for i in items if i.get("spec", {}).get("nodeName") == want]
        return self._send(200, {"kind": "List", "items": items,
                                "metadata": {"resourceVersion": str(st.rv)}})

    def do_POST(self):
        d, _ = self._route()
        if d is None:
            return self._send(404, {"message": "not found"})
        body = self._body()
        st = self.store
        if d["sub"] == "binding":
            node = body.get("target", {}).get("name")
            pod = st.get("pods", d["ns"], d["name"])
            if pod is None:
                return self._send(404, {"reason": "NotFound"})
            if pod.get("spec", {}).get("nodeName"):
                return self._send(409, {"reason": "Conflict", "message": "pod already bound"})
            # kube-apiserver's binding REST copies the Binding's annotations
            # onto the pod together with spec.nodeName (one write).
            patch = {"spec": {"nodeName": node}, "status": {"phase": "Running"}}
            ann = (body.get("metadata") or {}).get("annotations")
            if ann:
                patch["metadata"] = {"annotations": ann}
            st.patch("pods", d["ns"], d["name"], patch)
            return self._send(201, {"kind": "Status", "status": "Success"})
        o = st.create(d["coll"], d["ns"], body)
        if o is None:
            return self._send(409, {"reason": "AlreadyExists"})
        return self._send(201, o)

    def do_PATCH(self):
        d, _ = self._route()
        if d is None or not d["name"]:
            return self._send(404, {"message": "not found"})
        o = self.store.patch(d["coll"], d["ns"], d["name"], self._body())
        return self._send(200, o) if o else self._send(404, {"reason": "NotFound"})

    def do_PUT(self):
        """Replace with optimistic concurrency: a stale metadata.resourceVersion
        gets 409 Conflict (what leader election relies on)."""
        d, _ = self._route()
        if d is None or not d["name"]:
            return self._send(404, {"message": "not found"})
        body = self._body()
        st = self.store
        with st.lock:
            cur = st.objs.get((d["coll"], d["ns"], d["name"]))
            if cur is None:
                return self._send(404, {"reason": "NotFound"})
            want = body.get("metadata", {}).get("resourceVersion")
            if want and want != cur["metadata"].get("resourceVersion"):
                return self._send(409, {"reason": "Conflict"})
            body.setdefault("metadata", {})
            for k in ("uid", "creationTimestamp", "namespace", "name"):
                if k in cur["metadata"]:
                    body["metadata"][k] = cur["metadata"][k]
            st.objs[(d["coll"], d["ns"], d["name"])] = body
            st._bump(d["coll"], "MODIFIED", body)
            return self._send(200, copy.deepcopy(body))

    def do_DELETE(self):
        d, _ = self._route()
        if d is None or not d["name"]:
            return self._send(404, {"message": "not found"})
        o = self.store.delete(d["coll"], d["ns"], d["name"])
        return self._send(200, o) if o else self._send(404, {"reason": "NotFound"})


class FakeApiServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.store = Store()
        handler = type("H", (_Handler,), {"store": self.store})
        ThreadingHTTPServer.request_queue_size = 256
        self.httpd = ThreadingHTTPServer((host, port), handler)
        self.httpd.daemon_threads = True
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}"

    def start(self) -> "FakeApiServer":
        self.thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()

    # convenience for fixtures
    def add_node(self, name: str, labels: dict | None = None, gpus: int = 8,
                 resource: str = "amd.com/gpu", taints: list | None = None) -> dict:
        node = {"apiVersion": "v1", "kind": "Node",
                "metadata": {"name": name, "labels": {"kubernetes.io/hostname": name, **(labels or {})}},
                "spec": {"taints": taints or []},
                "status": {"capacity": {resource: str(gpus)}, "allocatable": {resource: str(gpus)},
                           "conditions": [{"type": "Ready", "status": "True"}]}}
        return self.store.create("nodes", None, node)
