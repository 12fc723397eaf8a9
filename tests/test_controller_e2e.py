"""End-to-end on a fake cluster (BASELINE.json config 1): fake apiserver +
controller (reconciler + extender + webhook) + kube-scheduler stand-in, all
over real HTTP.  GPUWorkload -> Pod -> filter/prioritize/bind -> status with
allocated GPUs and RCCL env -> completion -> release + cost; budgets;
partition strategies; restart-safe ledger; admission webhook; config."""
import base64
import json
import time

import pytest

from kgwe.api import crds, webhook
from kgwe.controller.apiserver import FakeApiServer
from kgwe.controller.kube import KubeClient
from kgwe.controller.main import DEFAULTS, build
from kgwe.controller.schedsim import SchedulerSim
from kgwe.utils.config import ConfigError, load_config


def wait_for(fn, timeout=10.0, every=0.05):
    t0 = time.time()
    while time.time() - t0 < timeout:
        v = fn()
        if v:
            return v
        time.sleep(every)
    raise AssertionError("condition not met in time")


@pytest.fixture
def cluster():
    api = FakeApiServer().start()
    kube = KubeClient(api.url)
    for i in range(2):
        api.add_node(f"mi355x-{i}")
    cfg = load_config(DEFAULTS, sets=["listen.host=127.0.0.1", "listen.port=0", f"kube.url={api.url}",
                                      "tickSeconds=0.2"])
    plat, ext, rec = build(cfg)
    from kgwe.core import make_fixture
    for i in range(2):
        plat.add_fake_node(make_fixture(f"mi355x-{i}", 8, 2))
    ext.start()
    rec.start()
    sim = SchedulerSim(kube, ext.url).start()
    yield api, kube, plat, ext, rec
    sim.stop()
    rec.stop()
    ext.stop()
    api.stop()


def gw(name, count=8, **spec):
    s = {"gpuRequirements": {"count": count, "topology": {"preference": "NVLinkOptimal"}},
         "distributedConfig": {"strategy": "FSDP", "worldSize": count, "backend": "NCCL"},
         "podTemplate": {"spec": {"containers": [{"name": "train", "image": "rocm/pytorch",
                                                  "command": ["torchrun", "train.py"]}]}}}
    s.update(spec)
    return {"apiVersion": "kgwe.amd.com/v1", "kind": "GPUWorkload",
            "metadata": {"name": name, "namespace": "ml"}, "spec": s}


def test_gpuworkload_lifecycle(cluster):
    api, kube, plat, ext, rec = cluster
    kube.create_cr(gw("llama3-8b-fsdp"))
    st = wait_for(lambda: (kube.get_cr("GPUWorkload", "ml", "llama3-8b-fsdp").get("status") or {})
                  if (kube.get_cr("GPUWorkload", "ml", "llama3-8b-fsdp").get("status") or {}).get("phase")
                  in ("Scheduled", "Running") else None)
    assert len(st["allocatedGPUs"]) == 8 and st["scheduledNode"].startswith("mi355x-")
    env = st["rcclEnv"]
    assert env["WORLD_SIZE"] == "8" and env["HIP_VISIBLE_DEVICES"] == "0,1,2,3,4,5,6,7"
    assert env["TORCH_DISTRIBUTED_BACKEND"] == "nccl" and st["estimatedBandwidth"] > 100
    pod = kube.get_pod("ml", "llama3-8b-fsdp-gw")
    assert pod["spec"]["schedulerName"] == "kgwe-scheduler"
    assert pod["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"] == "8"
    assert plat.scheduler_metrics()["allocated_gpus"] == 8
    # completion -> release + cost + status
    kube.patch_pod("ml", "llama3-8b-fsdp-gw", {"status": {"phase": "Succeeded"}})
    wait_for(lambda: plat.scheduler_metrics()["allocated_gpus"] == 0)
    done = wait_for(lambda: kube.get_cr("GPUWorkload", "ml", "llama3-8b-fsdp")["status"]
                    if kube.get_cr("GPUWorkload", "ml", "llama3-8b-fsdp")["status"]["phase"] == "Succeeded"
                    else None)
    assert "completionTime" in done


def test_partition_workloads_bin_pack(cluster):
    api, kube, plat, ext, rec = cluster
    for i in range(8):
        kube.create_cr(gw(f"inf-{i}", count=0, workloadType="Inference",
                          gpuRequirements={"count": 0, "partition": {"mode": "CPX", "count": 1}},
                          distributedConfig={"backend": "RCCL"}))
    wait_for(lambda: plat.scheduler_metrics()["allocated_partitions"] == 8, timeout=15)
    slices = [a["partitions"][0] for a in plat.allocations()]
    assert len({s.rsplit("/p", 1)[0] for s in slices}) == 1


def test_invalid_workload_fails_with_condition(cluster):
    api, kube, plat, ext, rec = cluster
    bad = gw("bad", count=100)
    kube.create_cr(bad)
    st = wait_for(lambda: kube.get_cr("GPUWorkload", "ml", "bad").get("status"))
    assert st["phase"] == "Failed" and "maximum" in st["message"]


def test_budget_block_enforced_and_status(cluster):
    api, kube, plat, ext, rec = cluster
    kube.create_cr({"apiVersion": "kgwe.amd.com/v1", "kind": "GPUBudget",
                    "metadata": {"name": "tiny", "namespace": "ml"},
                    "spec": {"limit": "1", "enforcementPolicy": "Block"}})
    wait_for(lambda: plat.budgets())
    kube.create_cr(gw("blocked", count=8))
    time.sleep(0.6)
    assert plat.scheduler_metrics()["allocated_gpus"] == 0
    st = wait_for(lambda: kube.get_cr("GPUBudget", "ml", "tiny").get("status"))
    assert st["currentSpend"] == "0.00"


def test_partition_strategy_rebalanced(cluster):
    api, kube, plat, ext, rec = cluster
    kube.create_cr({"apiVersion": "kgwe.amd.com/v1", "kind": "PartitionStrategy",
                    "metadata": {"name": "mixed"},
                    "spec": {"profileDistribution": {"CPX": 0.25}, "rebalanceInterval": "5m"}})
    st = wait_for(lambda: kube.get_cr("PartitionStrategy", None, "mixed").get("status"), timeout=5)
    assert st["currentDistribution"].get("CPX") == 4


def test_restart_rebuilds_ledger(cluster):
    api, kube, plat, ext, rec = cluster
    kube.create_cr(gw("persist", count=4))
    wait_for(lambda: plat.scheduler_metrics()["allocated_gpus"] == 4)
    cfg = load_config(DEFAULTS, sets=["listen.host=127.0.0.1", "listen.port=0", f"kube.url={api.url}"])
    plat2, ext2, rec2 = build(cfg)
    from kgwe.core import make_fixture
    for i in range(2):
        plat2.add_fake_node(make_fixture(f"mi355x-{i}", 8, 2))
    assert rec2.rebuild_ledger() == 1
    assert plat2.scheduler_metrics()["allocated_gpus"] == 4
    ext2.httpd.server_close()


def test_agent_push_endpoint(cluster):
    import http.client
    api, kube, plat, ext, rec = cluster
    from kgwe.core import make_fixture
    node = make_fixture("pushed", 8, 2)
    h, p = ext.httpd.server_address[:2]
    c = http.client.HTTPConnection(h, p)
    c.request("POST", "/v1/nodes/pushed/topology", body=json.dumps(node))
    assert c.getresponse().status == 200
    assert plat.node("pushed")["name"] == "pushed"


def test_agent_push_labels_node(cluster):
    """D15: node labels follow the pushed topology (link down -> island not
    fully connected); an unchanged push does not re-patch."""
    import http.client
    api, kube, plat, ext, rec = cluster
    node = plat.node("mi355x-0")
    h, p = ext.httpd.server_address[:2]

    def push(n):
        c = http.client.HTTPConnection(h, p)
        c.request("POST", "/v1/nodes/mi355x-0/topology", body=json.dumps(n))
        r = c.getresponse()
        assert r.status == 200 and "labelError" not in json.loads(r.read())

    push(node)
    labels = kube.get_node("mi355x-0")["metadata"]["labels"]
    assert labels["kgwe.amd.com/gpu.count"] == "8"
    assert labels["kgwe.amd.com/xgmi.fully-connected"] == "true"
    assert labels["kgwe.amd.com/partition.compute"] == "SPX"
    rv = kube.get_node("mi355x-0")["metadata"]["resourceVersion"]
    push(node)
    assert kube.get_node("mi355x-0")["metadata"]["resourceVersion"] == rv
    g0 = node["gpus"][0]
    peer = g0["links"][0]["peer"]
    g0["links"][0]["up"] = False
    for g in node["gpus"]:
        if g["uuid"] == peer:
            for link in g["links"]:
                if link["peer"] == g0["uuid"]:
                    link["up"] = False
    push(node)
    labels = kube.get_node("mi355x-0")["metadata"]["labels"]
    assert labels["kgwe.amd.com/xgmi.fully-connected"] == "false"
    assert labels["kgwe.amd.com/xgmi.links-down"] == "1"


def test_webhook_mutates_and_validates():
    obj = gw("w", count=2, gpuRequirements={"count": 0, "mig": {"profile": "1g.10gb", "count": 2}})
    ar = {"request": {"uid": "u1", "operation": "CREATE", "object": obj}}
    out = webhook.review(ar, mutate=True)["response"]
    assert out["allowed"] and out["patchType"] == "JSONPatch"
    patch = json.loads(base64.b64decode(out["patch"]))
    spec = patch[0]["value"]
    assert spec["gpuRequirements"]["partition"] == {"mode": "CPX", "count": 2, "memoryMode": "NPS1"}
    assert spec["distributedConfig"]["backend"] == "RCCL"
    bad = webhook.review({"request": {"uid": "u2", "operation": "CREATE",
                                      "object": gw("x", count=65)}})["response"]
    assert not bad["allowed"] and "maximum" in bad["status"]["message"]
    both = gw("y", count=2, gpuRequirements={"count": 2, "partition": {"mode": "CPX"}})
    assert any("not both" in e for e in crds.validate(both))


def test_crd_render(tmp_path):
    import yaml
    paths = crds.render(tmp_path)
    assert len(paths) == 3
    doc = yaml.safe_load(paths[0].read_text())
    assert doc["spec"]["group"] == "kgwe.amd.com"


def test_config_rejects_unknown_keys(tmp_path):
    with pytest.raises(ConfigError):
        load_config(DEFAULTS, sets=["scheduler.noSuchKey=1"])
    f = tmp_path / "c.yaml"
    f.write_text("scheduler:\n  topologyWeight: 50\n")
    cfg = load_config(DEFAULTS, str(f), environ={"KGWE_CONTROLLER_SCHEDULER__BALANCEWEIGHT": "10"},
                      env_prefix="KGWE_CONTROLLER_")
    assert cfg["scheduler"]["topologyWeight"] == 50 and cfg["scheduler"]["balanceWeight"] == 10
    f.write_text("bogus: 1\n")
    with pytest.raises(ConfigError):
        load_config(DEFAULTS, str(f))


def test_leader_election_single_holder_and_failover():
    from kgwe.controller.leader import LeaderElector

    api = FakeApiServer().start()
    try:
        a = LeaderElector(KubeClient(api.url), "kgwe-controller", "a", lease_s=1.0)
        b = LeaderElector(KubeClient(api.url), "kgwe-controller", "b", lease_s=1.0)
        t0 = time.time()
        assert a.try_acquire_or_renew(t0)
        assert not b.try_acquire_or_renew(t0 + 0.1)
        assert a.try_acquire_or_renew(t0 + 0.5)      # renew
        assert b.try_acquire_or_renew(t0 + 3.0)      # a's lease expired -> failover
        assert not a.try_acquire_or_renew(t0 + 3.1)
    finally:
        api.stop()


def test_mixed_tenancy_training_and_partition_inference(cluster):
    """BASELINE.json config 5 (examples/mixed-tenancy.yaml): 4-GPU FSDP training
    + 4 single-slice inference services of another team, optimizer
    rightsizing and per-team cost attribution."""
    import yaml
    from pathlib import Path

    from kgwe.optimizer.optimizer import TelemetryDataPoint, WorkloadOptimizer

    api, kube, plat, ext, rec = cluster
    docs = [d for d in yaml.safe_load_all((Path(__file__).parents[1] / "examples" /
                                           "mixed-tenancy.yaml").read_text()) if d]
    for d in docs:
        kube.create_cr(d)
    wait_for(lambda: plat.scheduler_metrics()["allocated_gpus"] == 4
             and plat.scheduler_metrics()["allocated_partitions"] == 4, timeout=15)
    allocs = {a["uid"]: a for a in plat.allocations()}
    train = [a for a in allocs.values() if a["gpus"]]
    assert len(train) == 1 and len(train[0]["gpus"]) == 4
    node = plat.node(train[0]["node"])
    by_uuid = {g["uuid"]: g for g in node["gpus"]}
    assert len({by_uuid[u]["numa_node"] for u in train[0]["gpus"]}) == 1  # one NUMA domain
    st = kube.get_cr("GPUWorkload", "research", "llama3-8b-finetune")["status"]
    assert st["rcclEnv"]["WORLD_SIZE"] == "4" and st["estimatedBandwidth"] > 100
    # inference: 4 slices bin-packed onto ONE CPX GPU, disjoint from training's GPUs
    slices = [p for a in allocs.values() for p in a["partitions"]]
    gpus = {p.rsplit("/p", 1)[0] for p in slices}
    assert len(slices) == 4 and len(gpus) == 1 and not gpus & set(train[0]["gpus"])
    # rightsizing: low-utilisation inference telemetry -> CPX recommendation
    opt = WorkloadOptimizer(learn=False)
    t0 = time.time()
    for i in range(30):
        opt.ingest_telemetry("serve", TelemetryDataPoint(
            timestamp=t0 + i, gpu_uuid="g0", gpu_utilization=12.0,
            memory_used_bytes=20 * 2**30, memory_total_bytes=288 * 2**30))
    pred = opt.predict_resources("serve", {"model_params_billions": 1, "workload_type": "Inference"})
    assert pred.recommended_partition == "CPX"
    # completion -> cost records per team; slices metered at 1/8 of a GPU
    time.sleep(0.3)
    for name, ns in [("llama3-8b-finetune", "research")] + [(f"llama3-1b-serve-{i}", "serving")
                                                            for i in range(4)]:
        kube.patch_pod(ns, f"{name}-gw", {"status": {"phase": "Succeeded"}})
    wait_for(lambda: not plat.allocations(), timeout=10)
    cb = {ln["group"]: ln for ln in plat.chargeback("team")["lines"]}
    assert cb["research"]["workloads"] == 1 and cb["serving"]["workloads"] == 4
    rates = {}
    for uid, a in allocs.items():
        r = plat.cost_record(uid)
        rates[uid] = r["raw_cost"] / (r["duration_s"] / 3600.0) / r["gpu_count"]
    train_rate = rates[train[0]["uid"]]
    for uid, a in allocs.items():
        if a["partitions"]:
            assert rates[uid] == pytest.approx(train_rate / 8, rel=0.02)


def _status(kube, ns, name):
    return kube.get_cr("GPUWorkload", ns, name).get("status") or {}


def test_node_loss_reschedules_workload(cluster):
    """the reference evicts a deleted node from its cache and
    leaves the allocations on it stale.  Here the workload is evicted and,
    per spec.recovery, rescheduled onto the surviving node."""
    api, kube, plat, ext, rec = cluster
    kube.create_cr(gw("resilient", count=8))
    st = wait_for(lambda: _status(kube, "ml", "resilient") if _status(kube, "ml", "resilient")
                  .get("phase") in ("Scheduled", "Running") else None)
    first = st["scheduledNode"]
    kube.delete_node(first)
    st = wait_for(lambda: _status(kube, "ml", "resilient") if _status(kube, "ml", "resilient")
                  .get("restarts") == 1 and _status(kube, "ml", "resilient").get("phase") in
                  ("Scheduled", "Running") else None, timeout=15)
    assert st["scheduledNode"] != first and len(st["allocatedGPUs"]) == 8
    assert "node deleted" in st["lastFailure"]
    assert st["podName"] == "resilient-gw-r1"
    allocs = plat.allocations()
    assert len(allocs) == 1 and allocs[0]["node"] == st["scheduledNode"]
    assert first not in plat.snapshot()["nodes"]


def test_unhealthy_gpu_evicts_and_fail_policy(cluster):
    api, kube, plat, ext, rec = cluster
    kube.create_cr(gw("fragile", count=2, recovery={"policy": "Fail"}))
    st = wait_for(lambda: _status(kube, "ml", "fragile") if _status(kube, "ml", "fragile")
                  .get("phase") in ("Scheduled", "Running") else None)
    bad = st["allocatedGPUs"][0]
    plat.fake_set_health_signals(st["scheduledNode"], bad, {"ecc_uncorrectable": 3})
    st = wait_for(lambda: _status(kube, "ml", "fragile") if _status(kube, "ml", "fragile")
                  .get("phase") == "Failed" else None, timeout=10)
    assert bad in st["lastFailure"] and "uncorrectable ECC" in st["lastFailure"]
    assert not plat.allocations()


def test_unhealthy_gpu_reschedules_away_from_it(cluster):
    api, kube, plat, ext, rec = cluster
    kube.create_cr(gw("healer", count=4))
    st = wait_for(lambda: _status(kube, "ml", "healer") if _status(kube, "ml", "healer")
                  .get("phase") in ("Scheduled", "Running") else None)
    bad = st["allocatedGPUs"][1]
    plat.fake_set_health_signals(st["scheduledNode"], bad, {"retired_pages": 100})
    st = wait_for(lambda: _status(kube, "ml", "healer") if _status(kube, "ml", "healer")
                  .get("restarts") == 1 and _status(kube, "ml", "healer").get("phase") in
                  ("Scheduled", "Running") else None, timeout=15)
    assert bad not in st["allocatedGPUs"] and len(st["allocatedGPUs"]) == 4


def test_not_ready_node_evicts(cluster):
    api, kube, plat, ext, rec = cluster
    kube.create_cr(gw("nr", count=8))
    st = wait_for(lambda: _status(kube, "ml", "nr") if _status(kube, "ml", "nr")
                  .get("phase") in ("Scheduled", "Running") else None)
    first = st["scheduledNode"]
    kube.patch_node_status(first, {"conditions": [{"type": "Ready", "status": "False"}]})
    st = wait_for(lambda: _status(kube, "ml", "nr") if _status(kube, "ml", "nr")
                  .get("restarts") == 1 and _status(kube, "ml", "nr").get("phase") in
                  ("Scheduled", "Running") else None, timeout=15)
    assert st["scheduledNode"] != first and "NotReady" in st["lastFailure"]
