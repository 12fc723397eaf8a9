"""gRPC transport for the OptimizerService (reference port 50051:
docker/Dockerfile.optimizer:53, values.yaml:189-192 — the reference shipped the
port but no server).

No protoc in this image, so messages are JSON documents carried as gRPC bytes
(generic method handlers with JSON (de)serialisers).  The wire method names
are /kgwe.optimizer.v1.Optimizer/{PredictResources,GetPlacement,
IngestTelemetry,GetMetrics}; `OptimizerClient` is the matching stub used by
the controller (its hint becomes the scheduler's +10 preferred-node bonus).
"""
from __future__ import annotations

import json
from concurrent import futures

import grpc

from .optimizer import OptimizerService

SERVICE = "kgwe.optimizer.v1.Optimizer"
METHODS = ("PredictResources", "GetPlacement", "IngestTelemetry", "GetMetrics")


def _ser(obj) -> bytes:
    return json.dumps(obj).encode()


def _de(b: bytes):
    return json.loads(b.decode() or "{}")


def serve(port: int = 50051, host: str = "0.0.0.0", workers: int = 8,
          service: OptimizerService | None = None):
    svc = service or OptimizerService()
    handlers = {m: grpc.unary_unary_rpc_method_handler(
        (lambda m: lambda req, ctx: getattr(svc, m)(req))(m),
        request_deserializer=_de, response_serializer=_ser) for m in METHODS}
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers))
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))
    bound = server.add_insecure_port(f"{host}:{port}")
    server.start()
    return server, bound, svc


class OptimizerClient:
    def __init__(self, target: str, timeout: float = 2.0):
        self.channel = grpc.insecure_channel(target)
        self.timeout = timeout
        self._stubs = {m: self.channel.unary_unary(f"/{SERVICE}/{m}", request_serializer=_ser,
                                                   response_deserializer=_de) for m in METHODS}

    def call(self, method: str, request: dict | None = None) -> dict:
        return self._stubs[method](request or {}, timeout=self.timeout)

    # Same surface as OptimizerService, so the controller takes either.
    def PredictResources(self, request: dict) -> dict:  # noqa: N802
        return self.call("PredictResources", request)

    def GetPlacement(self, request: dict) -> dict:  # noqa: N802
        return self.call("GetPlacement", request)

    def IngestTelemetry(self, request: dict) -> dict:  # noqa: N802
        return self.call("IngestTelemetry", request)

    def GetMetrics(self, request: dict | None = None) -> dict:  # noqa: N802
        return self.call("GetMetrics", request)

    def close(self):
        self.channel.close()


def main(argv=None) -> int:
    import argparse
    import time

    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=50051)
    ap.add_argument("--sizing", default="mi355x", choices=["mi355x", "reference"])
    a = ap.parse_args(argv)
    server, port, _ = serve(a.port, service=OptimizerService(sizing=a.sizing))
    print(f"kgwe optimizer gRPC on :{port}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        server.stop(1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
