"""Minimal Kubernetes REST client (no `kubernetes` package in this image).

Speaks plain JSON over HTTP/1.1 keep-alive to either a real kube-apiserver
(in-cluster service-account token + CA) or the in-process FakeApiServer used
by the test-suite and the benchmark (reference: KubernetesClient interface,
src/discovery/discovery.go:74-89, which had no implementation at all).
"""
from __future__ import annotations

import http.client
import json
import os
import ssl
import threading
import urllib.parse

GROUP = "kgwe.amd.com"
VERSION = "v1"

_PLURALS = {
    "GPUWorkload": ("gpuworkloads", True),
    "PartitionStrategy": ("partitionstrategies", False),
    "GPUBudget": ("gpubudgets", True),
}


class ApiError(RuntimeError):
    def __init__(self, status: int, body: str):
        super().__init__(f"apiserver {status}: {body[:300]}")
        self.status = status
        self.body = body


class KubeClient:
    def __init__(self, base_url: str, token: str | None = None, ca_file: str | None = None,
                 insecure: bool = False, timeout: float = 30.0):
        u = urllib.parse.urlparse(base_url)
        self.scheme = u.scheme
        self.host = u.hostname
        self.port = u.port or (443 if u.scheme == "https" else 80)
        self.token = token
        self.timeout = timeout
        self._ctx = None
        if self.scheme == "https":
            self._ctx = ssl.create_default_context(cafile=ca_file)
            if insecure:
                self._ctx.check_hostname = False
                self._ctx.verify_mode = ssl.CERT_NONE
        self._local = threading.local()

    @classmethod
    def in_cluster(cls) -> "KubeClient":
        sa = "/var/run/secrets/kubernetes.io/serviceaccount"
        host = os.environ["KUBERNETES_SERVICE_HOST"]
        port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        with open(f"{sa}/token") as f:
            token = f.read().strip()
        return cls(f"https://{host}:{port}", token=token, ca_file=f"{sa}/ca.crt")

    # ---------------------------------------------------------------- transport
    def _conn(self):
        c = getattr(self._local, "conn", None)
        if c is None:
            if self.scheme == "https":
                c = http.client.HTTPSConnection(self.host, self.port, timeout=self.timeout,
                                                context=self._ctx)
            else:
                c = http.client.HTTPConnection(self.host, self.port, timeout=self.timeout)
            self._local.conn = c
        return c

    def request(self, method: str, path: str, body=None, content_type="application/json",
                ok=(200, 201, 202)):
        data = None if body is None else (body if isinstance(body, (bytes, str)) else json.dumps(body))
        if isinstance(data, str):
            data = data.encode()
        headers = {"Accept": "application/json"}
        if data is not None:
            headers["Content-Type"] = content_type
        if self.token:
            headers["Authorization"] = f"Bearer {self.token}"
        for attempt in range(2):
            c = self._conn()
            try:
                c.request(method, path, body=data, headers=headers)
                r = c.getresponse()
                raw = r.read().decode()
                break
            except (http.client.HTTPException, ConnectionError, OSError):
                self._local.conn = None
                if attempt:
                    raise
        if r.status not in ok:
            raise ApiError(r.status, raw)
        return json.loads(raw) if raw else {}

    # ---------------------------------------------------------------- core/v1
    def list_nodes(self) -> list:
        return self.request("GET", "/api/v1/nodes").get("items", [])

    def get_node(self, name: str) -> dict:
        return self.request("GET", f"/api/v1/nodes/{name}")

    def create_node(self, node: dict) -> dict:
        return self.request("POST", "/api/v1/nodes", node)

    def patch_node_labels(self, name: str, labels: dict) -> dict:
        return self.request("PATCH", f"/api/v1/nodes/{name}", {"metadata": {"labels": labels}},
                            content_type="application/merge-patch+json")

    def delete_node(self, name: str) -> dict:
        return self.request("DELETE", f"/api/v1/nodes/{name}", ok=(200, 202, 404))

    def patch_node_status(self, name: str, status: dict) -> dict:
        return self.request("PATCH", f"/api/v1/nodes/{name}/status", {"status": status},
                            content_type="application/merge-patch+json")

    def list_pods(self, namespace: str | None = None, field_selector: str = "") -> list:
        path = f"/api/v1/namespaces/{namespace}/pods" if namespace else "/api/v1/pods"
        if field_selector:
            path += "?fieldSelector=" + urllib.parse.quote(field_selector)
        return self.request("GET", path).get("items", [])

    def get_pod(self, namespace: str, name: str) -> dict:
        return self.request("GET", f"/api/v1/namespaces/{namespace}/pods/{name}")

    def create_pod(self, pod: dict) -> dict:
        ns = pod["metadata"].get("namespace", "default")
        return self.request("POST", f"/api/v1/namespaces/{ns}/pods", pod)

    def delete_pod(self, namespace: str, name: str) -> dict:
        return self.request("DELETE", f"/api/v1/namespaces/{namespace}/pods/{name}", ok=(200, 202, 404))

    def patch_pod(self, namespace: str, name: str, patch: dict) -> dict:
        return self.request("PATCH", f"/api/v1/namespaces/{namespace}/pods/{name}", patch,
                            content_type="application/merge-patch+json")

    def bind_pod(self, namespace: str, name: str, node: str, uid: str = "",
                 annotations: dict | None = None) -> dict:
        """pods/binding.  The apiserver copies the Binding's annotations onto
        the pod in the same write as spec.nodeName (BindingREST), so placement
        annotations need no separate PATCH round trip."""
        meta = {"name": name, "namespace": namespace, "uid": uid}
        if annotations:
            meta["annotations"] = annotations
        body = {"apiVersion": "v1", "kind": "Binding", "metadata": meta,
                "target": {"apiVersion": "v1", "kind": "Node", "name": node}}
        return self.request("POST", f"/api/v1/namespaces/{namespace}/pods/{name}/binding", body)

    def create_event(self, namespace: str, event: dict) -> dict:
        return self.request("POST", f"/api/v1/namespaces/{namespace}/events", event)

    # ---------------------------------------------------------------- CRDs
    def _cr_path(self, kind: str, namespace: str | None, name: str | None = None, sub: str = ""):
        plural, namespaced = _PLURALS[kind]
        p = f"/apis/{GROUP}/{VERSION}"
        if namespaced and namespace:
            p += f"/namespaces/{namespace}"
        p += f"/{plural}"
        if name:
            p += f"/{name}"
        if sub:
            p += f"/{sub}"
        return p

    def list_cr(self, kind: str, namespace: str | None = None) -> list:
        return self.request("GET", self._cr_path(kind, namespace)).get("items", [])

    def get_cr(self, kind: str, namespace: str | None, name: str) -> dict:
        return self.request("GET", self._cr_path(kind, namespace, name))

    def create_cr(self, obj: dict) -> dict:
        kind = obj["kind"]
        return self.request("POST", self._cr_path(kind, obj["metadata"].get("namespace")), obj)

    def delete_cr(self, kind: str, namespace: str | None, name: str) -> dict:
        return self.request("DELETE", self._cr_path(kind, namespace, name), ok=(200, 202, 404))

    def patch_cr_status(self, kind: str, namespace: str | None, name: str, status: dict) -> dict:
        return self.request("PATCH", self._cr_path(kind, namespace, name, "status"), {"status": status},
                            content_type="application/merge-patch+json")

    def watch(self, path: str, resource_version: str = "0", timeout_s: int = 10) -> tuple[list, str]:
        """Long-poll watch: returns (events, last resourceVersion)."""
        sep = "&" if "?" in path else "?"
        q = f"{path}{sep}watch=1&resourceVersion={resource_version}&timeoutSeconds={timeout_s}"
        res = self.request("GET", q)
        evs = res.get("events", [])
        return evs, str(res.get("resourceVersion", resource_version))
