"""kgwe node agent (DaemonSet): amd-smi discovery + HIP bandwidth probes ->
topology push to the controller; rocm-smi/amd-smi telemetry -> Prometheus
(:9400); partition actuation.

Reference: discovery DaemonSet + node agent (Makefile:52-54,68-70,
docker/Dockerfile.agent, values.yaml:130-168,324-373: gRPC :50052, 5 s
telemetry, MIG/MPS configuration) and the exporter (:9400, DCGM-fed) — none
implemented (D3/D4/D6/D10).  MI355X-native: no NVML, no DCGM, no NVIDIA
device plugin:
  * discovery through the C++ AmdSmiHal (libamd_smi: devices, xGMI link
    type/hops/rated bandwidth, NUMA, partitions, ECC, activity);
  * MEASURED bandwidth: the HIP HBM self-probe per GPU and, with >= 2 GPUs,
    the LDS-staged xGMI pull probe with every link busy at once; a GPU whose
    HBM copy rate is < 70 % of the node median is marked Degraded, a link
    under 70 % of rated stays up but is scored lower by the scheduler;
  * telemetry gauges (gfx_activity = the "GPU utilization" KPI, umc
    activity, VRAM, hotspot temperature, socket power, ECC, partition mode,
    xGMI link status/bandwidth) via the core's metric registry;
  * POST /v1/partition (and gRPC SetPartition) actuates compute/memory
    partition modes through amd-smi (needs privileges; dry-run by default);
  * gRPC :50052 (kgwe.agent.v1.NodeAgent: GetTopology / GetTelemetry /
    GetProbes / SetPartition, kgwe/agent/grpc_service.py).
"""
from __future__ import annotations

import argparse
import http.client
import json
import statistics
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from .. import core
from ..utils import amdsmi_util
from ..utils.config import load_config

DEFAULTS = {
    "nodeName": "",
    "controllerUrl": "",
    "advertise": "",  # host:port of this agent's gRPC, pushed with the topology
    "fixture": "",
    "listen": {"host": "0.0.0.0", "port": 9400},
    "grpc": {"enabled": True, "port": 50052},
    "intervalSeconds": 5.0,
    "probe": {"hbm": True, "xgmi": True, "bytesMB": 1024, "iters": 5, "degradedRatio": 0.7},
    # Actuation is privileged (amd-smi set_gpu_compute/memory_partition): a
    # request must carry the controller's bearer token (a Secret mounted into
    # both pods) and the GPU must be idle on THIS node (no process on it).
    "partition": {"dryRun": True, "authTokenFile": ""},
}


class NodeAgent:
    def __init__(self, cfg: dict):
        self.cfg = cfg
        self.name = cfg["nodeName"] or "local"
        self.local = core.Platform({"enforceBudgets": False})
        self.topology: dict | None = None
        self.probe_results: dict = {}
        self._stop = threading.Event()
        self.pushes = 0
        self.push_errors = 0

    # ------------------------------------------------------------- discovery
    def discover(self) -> dict:
        if self.cfg["fixture"]:
            with open(self.cfg["fixture"]) as f:
                node = json.load(f)
            node["name"] = self.name
        else:
            d = core.amdsmi_discover(self.name)
            if not d.get("ok"):
                raise RuntimeError(f"amd-smi discovery failed: {d.get('error')}")
            node = d["node"]
        if self.probe_results:
            self._apply_probes(node)
        # The core's canonical form (health policy applied to the raw amd-smi
        # / probe signals) is what the agent serves and pushes.
        self.local.upsert_node(node)
        self.topology = self.local.node(self.name) or node
        return self.topology

    def run_probes(self) -> dict:
        """HBM self-probe per GPU; xGMI all-links probe when >= 2 GPUs."""
        from . import probes  # noqa: PLC0415 - needs the HIP library / a GPU

        pc = self.cfg["probe"]
        n = probes.device_count()
        res: dict = {"devices": n, "hbm": {}, "xgmi": None}
        if pc["hbm"]:
            for d in range(n):
                r = probes.probe_hbm(d, int(pc["bytesMB"]) << 20, int(pc["iters"]))
                res["hbm"][d] = {"copy_gbps": r.copy_gbps, "read_gbps": r.read_gbps,
                                 "write_gbps": r.write_gbps, "lds_copy_gbps": r.lds_copy_gbps}
        if pc["xgmi"] and n >= 2:
            res["xgmi"] = probes.probe_p2p_all(n, 128 << 20, 3)
        self.probe_results = res
        return res

    def _apply_probes(self, node: dict) -> None:
        ratio = float(self.cfg["probe"]["degradedRatio"])
        hbm = self.probe_results.get("hbm", {})
        copies = [v["copy_gbps"] for v in hbm.values()]
        med = statistics.median(copies) if copies else 0.0
        by_index = {g["index"]: g for g in node["gpus"]}
        for idx, v in hbm.items():
            g = by_index.get(int(idx))
            if g is None:
                continue
            g["hbm_measured_gbps"] = v["copy_gbps"]
            if med and v["copy_gbps"] < ratio * med:
                why = f"HBM copy {v['copy_gbps']:.0f} GB/s < {ratio:.0%} of node median {med:.0f}"
                h = g.setdefault("health", {})
                h["perf_degraded"], h["perf_reason"] = True, why  # the core's health policy input
                if h.get("status", "Healthy") == "Healthy":
                    h["status"] = "Degraded"
                h.setdefault("reasons", []).append(why)
        mat = self.probe_results.get("xgmi")
        if mat:
            uuid_of = {g["index"]: g["uuid"] for g in node["gpus"]}
            for dst, row in enumerate(mat):
                g = by_index.get(dst)
                if g is None:
                    continue
                for link in g.get("links", []):
                    src = next((i for i, u in uuid_of.items() if u == link["peer"]), None)
                    if src is not None and row[src] > 0:
                        link["measured_gbps"] = row[src]

    # ------------------------------------------------------------- push loop
    def push(self) -> bool:
        url = self.cfg["controllerUrl"]
        if not url or self.topology is None:
            return False
        u = urllib.parse.urlparse(url)
        try:
            c = http.client.HTTPConnection(u.hostname, u.port or 80, timeout=5)
            body = dict(self.topology)
            if self.cfg.get("advertise"):  # where the controller reaches this agent's gRPC
                body["agent_endpoint"] = self.cfg["advertise"]
            headers = {"Content-Type": "application/json"}
            tok = self._token()
            if tok:  # the controller only accepts an advertised endpoint from an authenticated push
                headers["Authorization"] = "Bearer " + tok
            c.request("POST", f"/v1/nodes/{self.name}/topology", body=json.dumps(body), headers=headers)
            ok = c.getresponse().status == 200
        except OSError:
            ok = False
        self.pushes += ok
        self.push_errors += not ok
        return ok

    def loop(self):
        while not self._stop.is_set():
            try:
                self.discover()
                self.push()
            except Exception:  # noqa: BLE001 - keep telemetry flowing
                self.push_errors += 1
            self._stop.wait(float(self.cfg["intervalSeconds"]))

    # ------------------------------------------------------------- HTTP
    def serve(self) -> ThreadingHTTPServer:
        agent = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"
            disable_nagle_algorithm = True

            def log_message(self, *a):
                pass

            def _send(self, code, data: bytes, ctype="application/json"):
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):
                if self.path.startswith("/metrics"):
                    return self._send(200, agent.local.expose_metrics().encode(), "text/plain; version=0.0.4")
                if self.path.startswith("/healthz"):
                    return self._send(200, b"ok", "text/plain")
                if self.path.startswith("/v1/topology"):
                    return self._send(200, json.dumps(agent.topology).encode())
                if self.path.startswith("/v1/probes"):
                    return self._send(200, json.dumps(agent.probe_results).encode())
                return self._send(404, b"{}")

            def do_POST(self):
                n = int(self.headers.get("Content-Length") or 0)
                body = json.loads(self.rfile.read(n) or b"{}")
                if self.path.startswith("/v1/partition"):
                    auth = self.headers.get("Authorization", "")
                    res = agent.set_partition(body, auth[7:] if auth.startswith("Bearer ") else "")
                    code = 403 if res.get("denied") else 409 if res.get("error") else 200
                    return self._send(code, json.dumps(res).encode())
                return self._send(404, b"{}")

        srv = ThreadingHTTPServer((self.cfg["listen"]["host"], int(self.cfg["listen"]["port"])), H)
        srv.daemon_threads = True
        threading.Thread(target=srv.serve_forever, daemon=True).start()
        return srv

    def _token(self) -> str:
        path = self.cfg["partition"].get("authTokenFile") or ""
        if not path:
            return ""
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            return ""

    def set_partition(self, body: dict, token: str = "") -> dict:
        """Compute / memory partition actuation (dry-run unless configured).
        Refused without the controller's token, and on a GPU that runs any
        process (the scheduler's idle check + fence cover its own ledger; this
        guards against a caller that bypasses it)."""
        import hmac  # noqa: PLC0415

        if not body.get("gpu"):
            return {"error": "gpu required"}
        want = self._token()
        dry = body.get("dryRun", self.cfg["partition"]["dryRun"]) or self.cfg["partition"]["dryRun"]
        if not dry:
            if not want:
                return {"error": "actuation disabled: partition.authTokenFile is not configured",
                        "denied": True}
            if not token or not hmac.compare_digest(token, want):
                return {"error": "unauthorized", "denied": True}
        if dry:
            return {"dryRun": True, "planned": body}
        procs = amdsmi_util.gpu_processes_by_uuid(body["gpu"])
        if procs:
            return {"error": f"gpu {body['gpu']} busy: {len(procs)} process(es) running"}
        err = core.native.amdsmi_set_partition(body["gpu"], body.get("compute", ""), body.get("memory", ""))
        return {"error": err} if err else {"applied": body}

    def serve_grpc(self):
        from . import grpc_service

        server, port = grpc_service.serve(self, int(self.cfg["grpc"]["port"]),
                                          self.cfg["listen"]["host"])
        self.grpc_port = port
        return server

    def stop(self):
        self._stop.set()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kgwe agent")
    ap.add_argument("--config")
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--once", action="store_true", help="discover (+probe), print JSON, exit")
    a = ap.parse_args(argv)
    cfg = load_config(DEFAULTS, a.config, a.set, env_prefix="KGWE_AGENT_")
    agent = NodeAgent(cfg)
    if not cfg["fixture"] and (cfg["probe"]["hbm"] or cfg["probe"]["xgmi"]):
        try:
            agent.run_probes()
        except Exception as e:  # noqa: BLE001
            print(f"[agent] probes unavailable: {e}", flush=True)
    if a.once:
        print(json.dumps({"topology": agent.discover(), "probes": agent.probe_results}), flush=True)
        return 0
    agent.serve()
    if cfg["grpc"]["enabled"]:
        agent.serve_grpc()
    print(f"kgwe-agent {agent.name}: metrics on :{cfg['listen']['port']}"
          + (f", gRPC on :{agent.grpc_port}" if cfg["grpc"]["enabled"] else ""), flush=True)
    try:
        agent.loop()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
