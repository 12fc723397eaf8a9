"""Workload optimizer: parity with the reference's documented behaviour, the
fixed defects, the MI355X memory model, online learning and the gRPC surface."""
import time

import pytest

from kgwe.core import Platform, make_fixture
from kgwe.optimizer.optimizer import (OptimizerService, TelemetryDataPoint, WorkloadOptimizer,
                                      WorkloadType)


def dp(t, util, mem_gb, total_gb=288):
    return TelemetryDataPoint(timestamp=t, gpu_uuid="g0", gpu_utilization=util,
                              memory_used_bytes=int(mem_gb * 2**30),
                              memory_total_bytes=int(total_gb * 2**30))


def test_reference_table_parity():
    opt = WorkloadOptimizer(sizing="reference", learn=False)
    # Outputs of the reference's predictor (workload_optimizer.py:275-285, run with numpy 2.2): 7B -> 2 GPUs, 13B -> 4, 70B -> 16.
    assert opt.predict_resources("a", {"model_params_billions": 7}).recommended_gpus == 2
    assert opt.predict_resources("a", {"model_params_billions": 13}).recommended_gpus == 4
    assert opt.predict_resources("a", {"model_params_billions": 70}).recommended_gpus == 16
    assert opt.predict_resources("a", {"model_params_billions": 0.05}).recommended_gpus == 1
    assert opt.predict_resources("a", {"model_params_billions": 600}).recommended_gpus == 64


def test_mi355x_memory_model():
    opt = WorkloadOptimizer(learn=False)
    p8 = opt.predict_resources("a", {"model_params_billions": 8, "strategy": "FSDP"})
    assert p8.recommended_gpus == 1  # 8B x 18 B/param x 1.25 = 180 GB < 230 GB usable
    p70 = opt.predict_resources("b", {"model_params_billions": 70, "strategy": "FSDP"})
    assert p70.recommended_gpus == 8 and p70.prefer_xgmi
    inf = opt.predict_resources("c", {"model_params_billions": 70, "workload_type": "Inference"})
    assert inf.recommended_gpus == 1


def test_string_enums_no_longer_crash():
    svc = OptimizerService(learn=False)
    r = svc.PredictResources({"workload_id": "w", "hints": {"strategy": "FSDP", "framework": "PyTorch",
                                                            "model_params_billions": 70}})
    assert "error" not in r and r["recommended_gpus"] >= 2
    assert any("FSDP" in s for s in r["reasoning"])
    assert "error" in svc.PredictResources({"hints": {"strategy": "NoSuchThing"}})


def test_samples_counted_once():
    opt = WorkloadOptimizer(learn=False)
    t = time.time()
    for i in range(20):
        opt.ingest_telemetry("w", dp(t + i, 70, 100))
    assert opt.get_profile("w").sample_count == 20


def test_constant_70pct_workload_is_training():
    opt = WorkloadOptimizer(learn=False)
    t = time.time()
    for i in range(30):
        opt.ingest_telemetry("w", dp(t + i, 70, 150))
    wt, conf = opt.predictor.classifier.classify("w")
    assert wt == WorkloadType.TRAINING and conf > 0.5


def test_low_util_inference_gets_cpx_partition():
    opt = WorkloadOptimizer(learn=False)
    t = time.time()
    for i in range(30):
        opt.ingest_telemetry("inf", dp(t + i, 15, 10))
    p = opt.predict_resources("inf", {"model_params_billions": 3, "workload_type": "Inference"})
    assert p.recommended_partition == "CPX"
    assert p.estimated_cost_per_hour == pytest.approx(2.95 / 8)


def test_online_model_learns_utilization():
    opt = WorkloadOptimizer(learn=True)
    t = time.time()
    for w in range(24):
        util = 20 + 3 * w
        for i in range(12):
            opt.ingest_telemetry(f"w{w}", dp(t + i, util, 50 + w))
        opt.complete(f"w{w}", 600 + 10 * w, train=False)
    loss0 = opt.predictor.model.train(epochs=5)
    loss1 = opt.predictor.model.train(epochs=300)
    assert loss1 < loss0
    p = opt.predict_resources("w10", {})
    assert any("Online model" in r for r in p.reasoning)
    assert abs(p.expected_utilization - 50) < 15


def test_placement_on_core_snapshot_uses_mutual_xgmi_cliques():
    plat = Platform({})
    plat.add_fake_node(make_fixture("n0", 8, 2))
    uu = [f"GPU-n0-{i:02d}" for i in range(8)]
    for j in range(2, 8):  # GPU 0 only linked to GPU 1: a star, not a clique
        plat.fake_set_link_up("n0", uu[0], uu[j], False)
    snap = plat.snapshot()
    opt = WorkloadOptimizer(learn=False)
    h = opt.get_optimal_placement("x", snap, {"gpu_count": 4, "prefer_xgmi": True})
    assert h.score == 90 and uu[0] not in h.preferred_gpus["n0"]


def test_grpc_roundtrip():
    from kgwe.optimizer.server import OptimizerClient, serve

    server, port, _ = serve(0, host="127.0.0.1", service=OptimizerService(learn=False))
    try:
        c = OptimizerClient(f"127.0.0.1:{port}")
        r = c.call("PredictResources", {"workload_id": "g", "hints": {"model_params_billions": 8}})
        assert r["recommended_gpus"] == 1
        ack = c.call("IngestTelemetry", {"workload_id": "g", "samples": [
            {"gpu_utilization": 80, "memory_used_bytes": 1, "memory_total_bytes": 2}] * 12})
        assert ack["accepted"] == 12
        assert c.call("GetMetrics")["total_samples"] == 12
        c.close()
    finally:
        server.stop(0)
