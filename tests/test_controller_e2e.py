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
                                      "tickSeconds=0.2", "optimizer.recommendEverySeconds=0.5"])
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
    ext2.stop()


def test_agent_push_endpoint(cluster):
    import http.client
    api, kube, plat, ext, rec = cluster
    from kgwe.core import make_fixture
    node = make_fixture("pushed", 8, 2)
    h, p = ext.address
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
    h, p = ext.address

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
    # rightsizing by the RUNNING controller: the serving GPU's amd-smi telemetry
    # (low gfx_activity) -> IngestTelemetry every tick -> status.recommendation
    plat.fake_set_util(node["name"], next(iter(gpus)), 12.0, 20.0)
    rec_ = wait_for(lambda: (_status(kube, "serving", "llama3-1b-serve-0").get("recommendation") or {})
                    if (_status(kube, "serving", "llama3-1b-serve-0").get("recommendation") or {})
                    .get("partition") == "CPX" else None, timeout=15)
    assert rec_["gpus"] == 1
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
    """The reference evicts a deleted node from its cache and
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


def _cluster(sets: list[str], nodes: int = 2):
    api = FakeApiServer().start()
    kube = KubeClient(api.url)
    for i in range(nodes):
        api.add_node(f"mi355x-{i}")
    cfg = load_config(DEFAULTS, sets=["listen.host=127.0.0.1", "listen.port=0", f"kube.url={api.url}",
                                      "tickSeconds=0.2"] + sets)
    plat, ext, rec = build(cfg)
    from kgwe.core import make_fixture
    for i in range(nodes):
        plat.add_fake_node(make_fixture(f"mi355x-{i}", 8, 2))
    ext.start()
    rec.start()
    sim = SchedulerSim(kube, ext.url).start()

    def stop():
        sim.stop()
        rec.stop()
        ext.stop()
        api.stop()
    return api, kube, plat, ext, rec, stop


def test_optimizer_loop_recommends_cpx_from_live_telemetry():
    """The running controller feeds per-allocation telemetry to the optimizer,
    writes status.recommendation (rightsizing) and trains the online model on
    completions — no hand-fed optimizer object."""
    api, kube, plat, ext, rec, stop = _cluster(["optimizer.recommendEverySeconds=0.5"])
    try:
        kube.create_cr(gw("serve", count=0, workloadType="Inference", framework="PyTorch",
                          gpuRequirements={"count": 0, "partition": {"mode": "CPX", "count": 1}},
                          distributedConfig={"backend": "RCCL"}))
        kube.create_cr(gw("train", count=2))
        st = wait_for(lambda: _status(kube, "ml", "serve") if _status(kube, "ml", "serve")
                      .get("phase") in ("Scheduled", "Running") else None, timeout=10)
        assert "recommendation" in st  # PredictResources at admission
        gpu = st["partitionSlices"][0].rsplit("/p", 1)[0]
        plat.fake_set_util(st["scheduledNode"], gpu, 12.0, 20.0)  # a lightly loaded server
        tr = wait_for(lambda: _status(kube, "ml", "train") if _status(kube, "ml", "train")
                      .get("phase") in ("Scheduled", "Running") else None, timeout=10)
        for g in tr["allocatedGPUs"]:
            plat.fake_set_util(tr["scheduledNode"], g, 97.0, 200.0)
        r = wait_for(lambda: (_status(kube, "ml", "serve").get("recommendation") or {})
                     if (_status(kube, "ml", "serve").get("recommendation") or {}).get("partition") == "CPX"
                     else None, timeout=15)
        assert r["gpus"] == 1 and r["expectedUtilization"] < 40
        rt = _status(kube, "ml", "train").get("recommendation") or {}
        assert rt.get("partition") is None  # a busy training job is not squeezed into a slice
        m = rec.optimizer.GetMetrics()
        assert m["total_samples"] >= 20 and {"ml/serve", "ml/train"} <= set(m["profiles"])
        # completion -> a training row of the online model
        kube.patch_pod("ml", "serve-gw", {"status": {"phase": "Succeeded"}})
        wait_for(lambda: (rec.optimizer.GetMetrics().get("model") or {}).get("training_rows", 0) > 0,
                 timeout=10)
        assert rec.errors == 0
    finally:
        stop()


def test_controller_consolidates_partitions_by_eviction():
    """Under-used CPX GPUs are emptied by evicting their preemptible inference
    pods (re-created and packed onto the fuller GPU), then go back to SPX."""
    api, kube, plat, ext, rec, stop = _cluster(["partitionConsolidateAfterSeconds=0",
                                                "partitionReclaimIdleSeconds=3600"], nodes=1)
    try:
        for i in range(12):
            kube.create_cr(gw(f"inf-{i}", count=0, workloadType="Inference",
                              gpuRequirements={"count": 0, "partition": {"mode": "CPX", "count": 1}},
                              distributedConfig={"backend": "RCCL"}))
        wait_for(lambda: plat.scheduler_metrics()["allocated_partitions"] == 12, timeout=20)
        assert plat.partition_metrics()["modes"]["CPX"]["gpus"] == 2
        # finish most pods on the first (full) GPU: it drops under the threshold
        by_gpu = {}
        for a in plat.allocations():
            by_gpu.setdefault(a["partitions"][0].rsplit("/p", 1)[0], []).append(a["uid"])
        full = max(by_gpu.values(), key=len)
        pods = {p["metadata"]["uid"]: p["metadata"]["name"] for p in kube.list_pods("ml")}
        for uid in full[:6]:
            kube.patch_pod("ml", pods[uid], {"status": {"phase": "Succeeded"}})
        wait_for(lambda: plat.partition_metrics()["modes"].get("CPX", {}).get("gpus") == 1
                 and plat.scheduler_metrics()["allocated_partitions"] == 6, timeout=20)
        m = plat.partition_metrics()
        assert m["slice_utilization"] == pytest.approx(6 / 8)
        moved = [n for n in (f"inf-{i}" for i in range(12)) if _status(kube, "ml", n).get("migrations")]
        assert moved and rec.migrations == len(moved)
        # the ledger holds the re-placed slice before the reconciler writes the
        # CR status, so wait for the status instead of sampling it once
        wait_for(lambda: all(_status(kube, "ml", n).get("phase") in ("Scheduled", "Running")
                             for n in moved), timeout=20)
        assert rec.errors == 0
    finally:
        stop()


def test_failover_keeps_scheduling_semantics_and_cost(tmp_path):
    """A new leader restores the FULL ledger entry (priority, preemptible, type,
    gang) and resumes the running cost record from the journal: a
    non-preemptible job survives a high-priority arrival after failover and
    is metered for its whole run."""
    journal = tmp_path / "cost.jsonl"
    sets = [f"cost.journalPath={journal}"]
    api, kube, plat, ext, rec, stop = _cluster(sets, nodes=1)
    try:
        kube.create_cr(gw("keep", count=8, priority=10, preemptible=False))
        wait_for(lambda: plat.scheduler_metrics()["allocated_gpus"] == 8)
        t_bind = time.time()
        time.sleep(1.2)
        plat.tick(time.time())  # a metering sample -> journal checkpoint path
        rec.stop()  # leader lost
        cfg = load_config(DEFAULTS, sets=["listen.host=127.0.0.1", "listen.port=0", f"kube.url={api.url}"]
                          + sets)
        plat2, ext2, rec2 = build(cfg)
        from kgwe.core import make_fixture
        plat2.add_fake_node(make_fixture("mi355x-0", 8, 2))
        assert rec2.rebuild_ledger() == 1
        assert plat2.cost_resumed() == 1
        a = plat2.allocations()[0]
        assert a["preemptible"] is False and a["priority"] == 10 and a["type"] == "Training"
        d = plat2.schedule({"uid": "vip", "priority": 1000, "gpuRequirements": {"count": 8}})
        assert not d["ok"] and "keep" not in str(d.get("preempted"))
        time.sleep(0.3)
        rel = plat2.release(a["uid"])
        dur = rel["cost"]["duration_s"]
        assert dur >= time.time() - t_bind - 0.5  # metered from the first leader's bind
        ext2.stop()
    finally:
        stop()
