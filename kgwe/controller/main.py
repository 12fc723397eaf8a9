"""kgwe-controller: one process serving the whole control plane.

* :8080  kube-scheduler extender (/filter /prioritize /bind), admission webhook
         (/validate /mutate), node-agent push (/v1/nodes/<name>/topology),
         /metrics, /healthz, /debug/*  (reference D1: Dockerfile.controller
         8080/8443, scheduler-configmap.yaml:62)
* reconcile loops for GPUWorkload / GPUBudget / PartitionStrategy
* optional optimizer gRPC client (:50051) for placement hints
"""
from __future__ import annotations

import argparse
import hmac
import json
import signal
import sys
import threading
import time

from ..api import webhook
from ..core import Platform, make_fixture
from ..extender.server import ExtenderServer
from ..utils.config import load_config
from .kube import KubeClient
from .labels import NodeLabeler
from .reconciler import Reconciler

DEFAULTS = {
    "listen": {"host": "0.0.0.0", "port": 8080, "urlPrefix": ""},
    "kube": {"url": "", "inCluster": False, "insecure": False},
    "scheduler": {"topologyWeight": 40, "resourceWeight": 35, "balanceWeight": 25,
                  "enablePreemption": True, "enableGangScheduling": True, "gangTimeoutMs": 30000,
                  "maxSchedulingAttempts": 3, "scoring": "xgmi", "placement": "pack",
                  "preemptionCandidateNodes": 8, "preemptionWaitWindowSeconds": 30.0,
                  "preemptionMaxWaitSeconds": 120.0, "preemptionUrgentPriority": 1000000,
                  "preemptionMaxRatePercent": 4.0, "preemptionWindowSeconds": 300, "preemptionBurst": 8},
    "webhook": {"port": 8443, "certFile": "", "keyFile": ""},
    "cost": {"journalPath": "", "enableSpotOptimization": True, "enableRightsizing": True},
    "shareSocketDir": "/run/kgwe/share",
    "partitionDryRun": False,
    "autoProvisionPartitions": True,
    "partitionReclaimIdleSeconds": 60.0,
    "enforceBudgets": True,
    "optimizer": {"target": "", "inProcess": True, "learn": True, "recommendEverySeconds": 30.0},
    "partitionConsolidation": True,
    "partitionConsolidateBelow": 0.75,
    "partitionConsolidateAfterSeconds": 120.0,
    "migrationCooldownSeconds": 3600.0,
    "agentActuation": {"enabled": True, "tokenFile": "/etc/kgwe/actuation/token", "timeoutSeconds": 30.0},
    # Node-agent pushes: with the actuation token configured they must carry it,
    # and an agent's advertised endpoint (which later receives that token) must
    # be an address of the Node object it claims to be.
    "agentPush": {"requireToken": True, "pinEndpointToNode": True},
    "fakeNodes": 0,
    "labelNodes": True,
    "tickSeconds": 5.0,
    "leaderElection": {"enabled": True, "namespace": "kube-system", "leaseName": "kgwe-controller",
                       "identity": "", "leaseSeconds": 15.0, "renewSeconds": 10.0, "retrySeconds": 2.0},
}


def build(cfg: dict):
    plat = Platform({k: cfg[k] for k in ("scheduler", "cost", "partitionDryRun", "shareSocketDir",
                                         "autoProvisionPartitions", "partitionReclaimIdleSeconds",
                                         "enforceBudgets", "partitionConsolidateBelow",
                                         "partitionConsolidateAfterSeconds", "migrationCooldownSeconds")})
    for i in range(int(cfg.get("fakeNodes", 0))):
        plat.add_fake_node(make_fixture(f"mi355x-sim-{i:03d}", 8, 2))
    kube = None
    if cfg["kube"]["inCluster"]:
        kube = KubeClient.in_cluster()
    elif cfg["kube"]["url"]:
        kube = KubeClient(cfg["kube"]["url"], insecure=cfg["kube"]["insecure"])

    labeler = NodeLabeler(kube) if kube is not None and cfg["labelNodes"] else None
    endpoints: dict[str, str] = {}  # node -> agent gRPC host:port (from its pushes)
    agents: dict[str, object] = {}

    def token() -> str:
        path = cfg["agentActuation"]["tokenFile"]
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            return ""

    def actuate(node: str, gpu: str, compute: str, memory: str) -> str:
        """Partition switch on an agent-pushed node: the agent's SetPartition,
        with the bearer token (the agent also refuses a GPU that runs anything)."""
        ep = endpoints.get(node)
        if not ep:
            return f"no agent endpoint known for node {node}"
        try:
            from ..agent.grpc_service import AgentClient  # noqa: PLC0415

            c = agents.get(ep)
            if c is None:
                c = agents[ep] = AgentClient(ep, timeout=float(cfg["agentActuation"]["timeoutSeconds"]))
            r = c.call("SetPartition", {"gpu": gpu, "compute": compute, "memory": memory}, token=token())
        except Exception as e:  # noqa: BLE001 - a failed op, not a crashed extender
            return f"agent {ep}: {e}"
        if r.get("error"):
            return f"agent {ep}: {r['error']}"
        return ""

    if cfg["agentActuation"]["enabled"]:
        plat.set_partition_actuator(actuate)

    node_addrs: dict[str, tuple[float, set]] = {}  # node -> (fetched at, addresses of its Node object)

    def addresses_of(name: str) -> set | None:
        """The Node object's own addresses (InternalIP, Hostname, ...), cached
        for a minute; None when there is no apiserver to ask."""
        if kube is None:
            return None
        hit = node_addrs.get(name)
        if hit and time.time() - hit[0] < 60.0:
            return hit[1]
        try:
            obj = kube.get_node(name)
            addrs = {a.get("address", "") for a in (obj.get("status") or {}).get("addresses") or []}
        except Exception:  # noqa: BLE001 - unknown node: nothing is pinned to it
            addrs = set()
        node_addrs[name] = (time.time(), addrs)
        return addrs

    def agent_push(path, body, authorization=""):
        """Topology push of a node agent.  With a token configured the push
        must carry it (401 otherwise), and only then may it name the endpoint
        the controller later sends that same token to; with an apiserver the
        endpoint's host must also be one of the Node object's addresses.  No
        token configured (development): topology is accepted, endpoints are
        not."""
        node = json.loads(body)
        name = path.rstrip("/").split("/")[-2]  # /v1/nodes/<name>/topology
        node["name"] = name
        want = token()
        got = authorization[7:] if authorization.startswith("Bearer ") else ""
        authed = bool(want) and hmac.compare_digest(got.encode(), want.encode())
        if want and not authed and cfg["agentPush"]["requireToken"]:
            return 401, b'{"error":"unauthorized: node agent pushes carry the actuation token"}'
        ep = node.pop("agent_endpoint", "")
        note = {}
        if ep:
            host = ep.rsplit(":", 1)[0].strip("[]")
            addrs = addresses_of(name)
            if not authed:
                note["endpointIgnored"] = "push not authenticated"
            elif addrs is not None and host not in addrs and cfg["agentPush"]["pinEndpointToNode"]:
                note["endpointIgnored"] = f"{host} is not an address of Node {name}"
            else:
                endpoints[name] = ep
        plat.upsert_node(node)
        if labeler is not None:
            try:
                labeler.update(name, node)
            except Exception as e:  # noqa: BLE001 - labels are advisory; keep the topology
                return 200, json.dumps({"ok": True, "labelError": str(e)}).encode()
        return 200, json.dumps(dict({"ok": True}, **note)).encode()

    def admission(path, body):
        return 200, json.dumps(webhook.review(json.loads(body), mutate=path.startswith("/mutate"))).encode()

    ext = ExtenderServer(plat, kube=kube, host=cfg["listen"]["host"], port=int(cfg["listen"]["port"]),
                         url_prefix=cfg["listen"]["urlPrefix"],
                         routes={"/v1/nodes/": agent_push, "/validate": admission, "/mutate": admission},
                         auth_routes={"/v1/nodes/"})
    optimizer = None
    if cfg["optimizer"]["target"]:  # the optimizer Deployment (gRPC :50051)
        from ..optimizer.server import OptimizerClient  # noqa: PLC0415

        optimizer = OptimizerClient(cfg["optimizer"]["target"])
    elif cfg["optimizer"]["inProcess"]:
        from ..optimizer.optimizer import OptimizerService  # noqa: PLC0415

        optimizer = OptimizerService(learn=bool(cfg["optimizer"]["learn"]))
    rec = (Reconciler(plat, kube, optimizer=optimizer, tick_s=float(cfg["tickSeconds"]),
                      consolidate=bool(cfg["partitionConsolidation"]),
                      recommend_every_s=float(cfg["optimizer"]["recommendEverySeconds"])) if kube else None)
    return plat, ext, rec


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kgwe controller")
    ap.add_argument("--config", help="YAML config file")
    ap.add_argument("--set", action="append", default=[], help="override key.path=value")
    a = ap.parse_args(argv)
    cfg = load_config(DEFAULTS, a.config, a.set, env_prefix="KGWE_CONTROLLER_")
    # The extender's verbs run in HTTP handler threads next to the reconciler:
    # every C++ call releases the GIL, so hand it back at 1 ms (not CPython's
    # 5 ms) and a verb waiting to re-enter Python is not parked behind a
    # reconcile pass (profiles/r02_sched).
    sys.setswitchinterval(0.001)
    plat, ext, rec = build(cfg)
    wh = cfg["webhook"]
    if wh["certFile"]:
        ext.add_tls_listener(cfg["listen"]["host"], int(wh["port"]), wh["certFile"], wh["keyFile"])
    ext.start()
    elector = None
    le = cfg["leaderElection"]
    if rec and le["enabled"]:
        import os  # noqa: PLC0415
        import socket  # noqa: PLC0415

        from .leader import LeaderElector  # noqa: PLC0415

        ident = le["identity"] or f"{socket.gethostname()}-{os.getpid()}"
        elector = LeaderElector(rec.kube, le["leaseName"], ident, le["namespace"], le["leaseSeconds"],
                                le["renewSeconds"], le["retrySeconds"], on_started=rec.start,
                                on_stopped=rec.stop).start()
        ext.ready = lambda: elector.is_leader
    elif rec:
        rec.start()
    print(f"kgwe-controller listening on {ext.url}", flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    try:
        while not stop.wait(1.0):
            if rec is None:
                plat.tick(time.time())
    except KeyboardInterrupt:
        pass
    if elector:
        elector.stop()
    if rec:
        rec.stop()
    ext.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
