"""gRPC surface of the node agent (reference: gRPC :50052 in values.yaml:324-373
and docker/Dockerfile.agent — declared, never implemented, D4).

Same transport convention as the optimizer (kgwe/optimizer/server.py): no
protoc in the image, so messages are JSON documents carried as gRPC bytes on
generic method handlers.  Service ``kgwe.agent.v1.NodeAgent``:

* ``GetTopology``   -> the node topology the agent last discovered (amd-smi +
                       measured probe bandwidth);
* ``GetTelemetry``  -> per-GPU gfx / umc activity, memory, power,
                       temperature, health (status + reasons);
* ``GetProbes``     -> last HBM / xGMI probe results;
* ``SetPartition``  -> {gpu, compute, memory, dryRun}: compute / memory
                       partition actuation through amd-smi (dry-run unless
                       the agent runs with partition.dryRun=false).
"""
from __future__ import annotations

import json
from concurrent import futures

import grpc

SERVICE = "kgwe.agent.v1.NodeAgent"
METHODS = ("GetTopology", "GetTelemetry", "GetProbes", "SetPartition")


def _ser(obj) -> bytes:
    return json.dumps(obj).encode()


def _de(b: bytes):
    return json.loads(b.decode() or "{}")


class AgentService:
    def __init__(self, agent):
        self.agent = agent

    def GetTopology(self, req: dict) -> dict:
        return {"node": self.agent.name, "topology": self.agent.topology}

    def GetTelemetry(self, req: dict) -> dict:
        topo = self.agent.topology or {"gpus": []}
        gpus = []
        for g in topo.get("gpus", []):
            u, h = g.get("util", {}), g.get("health", {})
            gpus.append({"uuid": g.get("uuid"), "index": g.get("index"),
                         "gfx_activity": u.get("gfx_activity"), "umc_activity": u.get("umc_activity"),
                         "memory_used_gb": g.get("memory_used_gb"),
                         "memory_total_gb": g.get("memory_total_gb"),
                         "power_w": u.get("power_w"), "temperature_c": u.get("temperature_c"),
                         "partition": g.get("partition", {}).get("compute"),
                         "health": h.get("status"), "reasons": h.get("reasons", [])})
        return {"node": self.agent.name, "gpus": gpus}

    def GetProbes(self, req: dict) -> dict:
        return {"node": self.agent.name, "probes": self.agent.probe_results}

    def SetPartition(self, req: dict, ctx=None) -> dict:
        token = ""
        if ctx is not None:
            md = dict(ctx.invocation_metadata() or ())
            auth = md.get("authorization", "")
            token = auth[7:] if auth.startswith("Bearer ") else ""
        return self.agent.set_partition(req, token)


def serve(agent, port: int = 50052, host: str = "0.0.0.0", workers: int = 4):
    svc = AgentService(agent)
    handlers = {m: grpc.unary_unary_rpc_method_handler(
        (lambda m: (lambda req, ctx: svc.SetPartition(req, ctx)) if m == "SetPartition"
         else (lambda req, ctx: getattr(svc, m)(req)))(m),
        request_deserializer=_de, response_serializer=_ser) for m in METHODS}
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers))
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))
    bound = server.add_insecure_port(f"{host}:{port}")
    server.start()
    return server, bound


class AgentClient:
    def __init__(self, target: str, timeout: float = 5.0):
        self.channel = grpc.insecure_channel(target)
        self.timeout = timeout
        self._stubs = {m: self.channel.unary_unary(f"/{SERVICE}/{m}", request_serializer=_ser,
                                                   response_deserializer=_de) for m in METHODS}

    def call(self, method: str, request: dict | None = None, token: str = "") -> dict:
        md = (("authorization", f"Bearer {token}"),) if token else None
        return self._stubs[method](request or {}, timeout=self.timeout, metadata=md)

    def close(self):
        self.channel.close()
