"""Scheduler core (C++) — placement, filters, preemption, gangs, ledger safety.

Covers: scorers against the reference
formulas (compat mode), every filter constraint, ledger atomicity under
concurrency, bounded priority-aware preemption, gang all-or-nothing, and a p99
that comes from the histogram (not a running max).
"""
import json
import threading

import pytest

from kgwe.core import Platform, make_fixture


def wl(uid, count=1, topo="None", **spec):
    s = {"gpuRequirements": {"count": count, "topology": {"preference": topo}}}
    s["gpuRequirements"].update(spec.pop("req", {}))
    s.update(spec)
    return {"metadata": {"name": uid, "namespace": "ns", "uid": uid}, "spec": s}


@pytest.fixture
def plat():
    p = Platform({})
    for i in range(2):
        p.add_fake_node(make_fixture(f"n{i}", 8, 2))
    return p


def test_single_gpu_best_fit(plat):
    d = plat.schedule(wl("a", 1))
    assert d["ok"] and len(d["gpus"]) == 1 and d["score"] > 0
    # second single-GPU job packs into the same NUMA domain (best fit)
    d2 = plat.schedule(wl("b", 1))
    snap = plat.snapshot()
    numa = {g["uuid"]: g["numa_node"] for n in snap["nodes"].values() for g in n["gpus"]}
    if d2["node"] == d["node"]:
        assert numa[d2["gpus"][0]] == numa[d["gpus"][0]]


def test_xgmi_group_prefers_single_numa_domain(plat):
    d = plat.schedule(wl("j4", 4, "xGMIOptimal"))
    assert d["ok"]
    snap = plat.snapshot()
    numa = {g["uuid"]: g["numa_node"] for n in snap["nodes"].values() for g in n["gpus"]}
    assert len({numa[g] for g in d["gpus"]}) == 1
    assert d["score"] >= 80


def test_eight_gpu_fsdp_job_gets_whole_node_and_rccl_env(plat):
    d = plat.schedule(wl("fsdp", 8, "xGMIOptimal",
                         distributedConfig={"strategy": "FSDP", "worldSize": 8, "backend": "RCCL"}))
    assert d["ok"] and len(d["gpus"]) == 8
    env = d["env"]
    assert env["HIP_VISIBLE_DEVICES"] == "0,1,2,3,4,5,6,7"
    assert env["WORLD_SIZE"] == "8" and env["NPROC_PER_NODE"] == "8"
    assert env["TORCH_DISTRIBUTED_BACKEND"] == "nccl"  # RCCL on ROCm
    assert env["NCCL_IB_DISABLE"] == "1" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert float(env["KGWE_XGMI_BANDWIDTH_GBPS"]) > 100


def test_down_link_breaks_clique_for_xgmi_required(plat):
    uu = [f"GPU-n0-{i:02d}" for i in range(8)]
    for j in range(1, 8):
        plat.fake_set_link_up("n0", uu[0], uu[j], False)
    # n1 busy so only n0 is a candidate
    assert plat.schedule(wl("fill", 8, "None", constraints={"nodeSelector": {"kubernetes.io/hostname": "n1"}}))["ok"]
    d = plat.schedule(wl("req8", 8, "xGMIRequired"))
    assert not d["ok"]
    assert "xGMI" in d["failed_nodes"]["n0"]
    d7 = plat.schedule(wl("req7", 7, "xGMIRequired"))
    assert d7["ok"] and uu[0] not in d7["gpus"]


def test_degraded_measured_link_avoided(plat):
    a, b = "GPU-n0-00", "GPU-n0-01"
    plat.fake_set_measured_link("n0", a, b, 20.0)
    plat.fake_set_measured_link("n0", b, a, 20.0)
    plat.schedule(wl("x", 8, "None", constraints={"nodeSelector": {"kubernetes.io/hostname": "n1"}}))
    d = plat.schedule(wl("pair", 2, "xGMIOptimal"))
    assert d["ok"] and not ({a, b} <= set(d["gpus"]))


@pytest.mark.parametrize("field,value,expect", [
    ("nodeSelector", {"kubernetes.io/hostname": "n1"}, "n1"),
    ("excludeNodes", ["n0"], "n1"),
])
def test_constraints(plat, field, value, expect):
    d = plat.schedule(wl("c", 1, constraints={field: value}))
    assert d["ok"] and d["node"] == expect


def test_taints_and_tolerations():
    p = Platform({})
    fx = make_fixture("t0", 8, 2)
    fx["taints"] = [{"key": "dedicated", "value": "llm", "effect": "NoSchedule"}]
    p.add_fake_node(fx)
    assert not p.schedule(wl("no", 1))["ok"]
    ok = p.schedule(wl("yes", 1, constraints={"tolerations": [
        {"key": "dedicated", "operator": "Equal", "value": "llm", "effect": "NoSchedule"}]}))
    assert ok["ok"]


def test_min_memory_and_unhealthy(plat):
    plat.fake_set_health("n0", "GPU-n0-03", "Unhealthy", "uncorrectable ECC")
    plat.schedule(wl("big", 8, constraints={"nodeSelector": {"kubernetes.io/hostname": "n1"}}))
    d = plat.schedule(wl("seven", 8))
    assert not d["ok"]  # n0 has only 7 healthy GPUs
    assert not plat.schedule(wl("huge", 1, req={"minMemoryGB": 300}))["ok"]


def test_anti_affinity_and_colocation(plat):
    a = plat.schedule(wl("a", 1))
    b = plat.schedule(wl("b", 1, constraints={"antiAffinityWith": ["a"]}))
    assert b["ok"] and b["node"] != a["node"]
    c = plat.schedule(wl("c", 1, constraints={"colocateWith": ["a"]}))
    assert c["ok"] and c["node"] == a["node"]


def test_preemption_respects_priority_and_preemptible(plat):
    for i, n in enumerate(["n0", "n1"]):
        assert plat.schedule(wl(f"low{i}", 8, priority=10,
                                constraints={"nodeSelector": {"kubernetes.io/hostname": n}}))["ok"]
    # equal priority: no preemption
    assert not plat.schedule(wl("eq", 8, priority=10))["ok"]
    d = plat.schedule(wl("high", 8, priority=100))
    assert d["ok"] and len(d["preempted"]) == 1
    # non-preemptible victims are never chosen
    p = Platform({})
    p.add_fake_node(make_fixture("m0", 8, 2))
    assert p.schedule(wl("np", 8, priority=1, preemptible=False))["ok"]
    assert not p.schedule(wl("hi", 8, priority=1000))["ok"]


def test_gang_all_or_nothing(plat):
    members = [wl(f"g{i}", 8, "xGMIOptimal") for i in range(3)]
    res = plat.schedule_gang(members)
    assert not any(r["ok"] for r in res)  # 3 x 8 GPUs > 16 GPUs
    assert plat.scheduler_metrics()["allocated_gpus"] == 0
    res = plat.schedule_gang(members[:2])
    assert all(r["ok"] for r in res) and {r["node"] for r in res} == {"n0", "n1"}


def test_gang_member_waits_until_complete(plat):
    g = {"name": "ring", "size": 2}
    d1 = plat.schedule(wl("m1", 2, gang=g))
    assert d1["ok"] and d1["status"] == "Waiting"
    assert plat.permit("m1") == "Wait"
    d2 = plat.schedule(wl("m2", 2, gang=g))
    assert d2["status"] == "Scheduled"
    assert plat.permit("m1") == "Allow" and plat.permit("m2") == "Allow"


def test_gang_timeout_releases_reservations():
    p = Platform({"scheduler": {"gangTimeoutMs": 1}})
    p.add_fake_node(make_fixture("z", 8, 2))
    assert p.schedule(wl("only", 4, gang={"name": "gg", "size": 2}))["status"] == "Waiting"
    import time
    time.sleep(0.01)
    assert p.permit("only") == "Reject"
    assert p.scheduler_metrics()["allocated_gpus"] == 0


def test_concurrent_schedule_never_double_allocates():
    p = Platform({"scheduler": {"enablePreemption": False}})
    for i in range(4):
        p.add_fake_node(make_fixture(f"c{i}", 8, 2))
    results = []
    lock = threading.Lock()

    def worker(k):
        for j in range(20):
            d = p.schedule(wl(f"w{k}-{j}", 1 + (j % 3)))
            with lock:
                results.append(d)
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    owned = [g for d in results if d["ok"] for g in d["gpus"]]
    assert len(owned) == len(set(owned)), "a GPU was allocated twice"
    assert len(owned) <= 32
    assert p.scheduler_metrics()["allocated_gpus"] == len(owned)


def test_release_and_events(plat):
    d = plat.schedule(wl("r", 2))
    assert plat.release("r")["released"]
    assert not plat.release("r")["released"]
    evs = [e["type"] for e in plat.scheduler_events()]
    assert "Scheduled" in evs and "Released" in evs


def test_p99_is_a_quantile_not_max():
    p = Platform({})
    for _ in range(1000):
        p.observe_pod_latency_ms(1.0)
    p.observe_pod_latency_ms(5000.0)
    # the pod create -> bind histogram (kgwe_scheduling_latency_ms)
    assert p.pod_latency_quantile_ms(0.99) < 2.0 and p.pod_latency_quantile_ms(0.9999) >= 1000.0
    assert p.pod_latency_count() == 1001
    assert "kgwe_scheduling_latency_ms_count 1001" in p.expose_metrics()


def test_compat_mode_reproduces_reference_formulas():
    p = Platform({"scheduler": {"scoring": "compat"}})
    p.add_fake_node(make_fixture("k", 8, 2))
    s = p.score_node("k", wl("q", 2, "xGMIOptimal"))
    # reference: 50 + 50 * bw / (900 * C(k,2)) with 153.6 GB/s xGMI links
    assert s["topology"] == int(50 + 50 * 153.6 / 900)
    s = p.score_node("k", wl("q", 1))
    assert s["topology"] == 100
    assert s["resource"] == 100 and s["balance"] == 100
    assert s["total"] == (100 * 40 + 100 * 35 + 100 * 25) // 100


def test_optimizer_hint_bonus(plat):
    s0 = plat.score_node("n1", wl("h", 1))
    s1 = plat.score_node("n1", wl("h", 1, preferredNodes=["n1"]))
    assert s1["total"] == s0["total"] + 10


def test_topology_hints(plat):
    hs = plat.hints(4)
    assert hs and hs[0]["score"] >= 80 and len(hs[0]["gpus"]) == 4
    assert "fully connected xGMI group" in hs[0]["reasons"]


@pytest.mark.parametrize("signals,status,reason", [
    ({"ecc_uncorrectable": 2}, "Unhealthy", "uncorrectable ECC"),
    ({"retired_pages": 64}, "Unhealthy", "retired HBM pages"),
    ({"retired_pages": 3}, "Healthy", None),
    ({"pending_retired_pages": 1}, "Degraded", "pending retirement"),
    ({"ecc_correctable": 5000}, "Degraded", "ECC storm"),
    ({"ecc_correctable": 10}, "Healthy", None),
    ({"ecc_deferred": 1}, "Degraded", "deferred ECC"),
    ({"xgmi_errors": 1}, "Degraded", "xGMI errors"),
    ({"xgmi_links_down": 1}, "Healthy", "link(s) down"),
    ({"throttle": ["hbm_thermal"]}, "Healthy", "throttling: hbm_thermal"),
    ({"cper_fatal": 1}, "Unhealthy", "fatal CPER"),
    ({"cper_uncorrected": 2}, "Degraded", "uncorrected (non-fatal) CPER"),
    ({"cper_corrected": 150}, "Degraded", "corrected CPER storm"),
    ({"cper_corrected": 3}, "Healthy", None),
])
def test_health_policy_from_ras_signals(plat, signals, status, reason):
    """Fault injection through the fake amd-smi: raw RAS /
    xGMI / throttle signals -> the shared health policy -> schedulability."""
    gpu = "GPU-n0-02"
    plat.fake_set_health_signals("n0", gpu, signals)
    g = next(x for x in plat.node("n0")["gpus"] if x["uuid"] == gpu)
    assert g["health"]["status"] == status
    if reason:
        assert any(reason in r for r in g["health"]["reasons"]), g["health"]["reasons"]
    d = plat.schedule({"metadata": {"name": "all", "uid": "all"},
                       "spec": {"gpuRequirements": {"count": 8}}})
    assert d["ok"]
    # a whole-node job needs every GPU of the node healthy
    assert (d["node"] == "n0") == (status == "Healthy"), d["node"]


def test_health_signals_round_trip_and_recover(plat):
    gpu = "GPU-n0-05"
    plat.fake_set_health_signals("n0", gpu, {"ecc_uncorrectable": 1, "retired_pages": 7})
    snap = plat.node("n0")
    h = next(x for x in snap["gpus"] if x["uuid"] == gpu)["health"]
    assert h["retired_pages"] == 7 and h["status"] == "Unhealthy" and not h["pinned"]
    # agent push -> controller: the node JSON re-derives the same status
    from kgwe.core import Platform
    other = Platform({})
    other.upsert_node(snap)
    h2 = next(x for x in other.node("n0")["gpus"] if x["uuid"] == gpu)["health"]
    assert h2["status"] == "Unhealthy" and h2["retired_pages"] == 7
    plat.fake_set_health_signals("n0", gpu, {"ecc_uncorrectable": 0})  # after a reset
    h3 = next(x for x in plat.node("n0")["gpus"] if x["uuid"] == gpu)["health"]
    assert h3["status"] == "Healthy"


def test_group_stays_in_one_numa_domain_after_partial_use():
    """Regression: the domain count of a candidate group was inflated by
    map lookups of unused domains, so every 4-GPU group looked like it
    spanned both sockets and the first combination won (GPUs 1-4 across
    NUMA 0/1 instead of 4-7 on NUMA 1)."""
    from kgwe.core import Platform, make_fixture

    p = Platform({})
    p.add_fake_node(make_fixture("a", 8, 2))
    assert p.schedule({"metadata": {"name": "one", "uid": "one"},
                       "spec": {"gpuRequirements": {"count": 1}}})["ok"]
    d = p.schedule({"metadata": {"name": "t", "uid": "t"},
                    "spec": {"gpuRequirements": {"count": 4, "topology": {"preference": "xGMIOptimal"}}}})
    assert d["ok"]
    numa = {g["uuid"]: g["numa_node"] for g in p.node("a")["gpus"]}
    alloc = next(a for a in p.allocations() if a["uid"] == "t")
    assert len({numa[u] for u in alloc["gpus"]}) == 1, alloc["gpus"]
    assert d["score"] >= 90


def test_scale_bench_small_fleet():
    """The 10k-GPU scale bench (kgwe bench-scale) on a 128-node fleet: every
    op completes, and schedule / topology-query p99 stay far below the
    85 ms SLO (PRD target for topology queries: < 10 ms)."""
    from kgwe.bench import scale

    r = scale.run(nodes=128, ops=600, live_max=300)
    assert r["scheduled"] > 500
    assert r["schedule_ms"]["p99"] < 40.0 and r["topology_query_ms"]["p99"] < 40.0


# --- preemption policy: K best nodes, prefer waiting, rate window -----------------------------

def _alloc(p, uid):
    return next((a for a in p.allocations() if a["uid"] == uid), None)


def _full_fleet(p, nodes, priority=10, **spec):
    for i in range(nodes):
        p.add_fake_node(make_fixture(f"f{i:03d}", 8, 2))
    for i in range(nodes):
        assert p.schedule(wl(f"low{i:03d}", 8, priority=priority, **spec))["ok"]


def test_preemption_plans_exactly_on_the_cheapest_nodes_of_a_large_fleet():
    p = Platform({"scheduler": {"preemptionCandidateNodes": 4, "preemptionWaitWindowSeconds": 0}})
    for i in range(40):
        p.add_fake_node(make_fixture(f"f{i:03d}", 8, 2))
    # every node full; node f017 holds the only priority-1 job, f005 only non-preemptible work
    for i in range(40):
        sel = {"nodeSelector": {"kubernetes.io/hostname": f"f{i:03d}"}}
        pr, pre = (1, True) if i == 17 else (50, False) if i == 5 else (20, True)
        assert p.schedule(wl(f"j{i:03d}", 8, priority=pr, preemptible=pre, constraints=sel))["ok"]
    d = p.schedule(wl("vip", 8, priority=100))
    assert d["ok"] and d["preempted"] == ["j017"] and d["node"] == "f017"
    # the extender's dry run: at most K candidate plans, the non-preemptible node never among them
    plans = json.loads(p.preempt(json.dumps({
        "pod": {"metadata": {"name": "vip2", "uid": "vip2"},
                "spec": {"priority": 100, "containers": [{"resources": {"limits": {"amd.com/gpu": "8"}}}]}},
        "nodeNameToMetaVictims": {f"f{i:03d}": {"pods": []} for i in range(40)}})))["nodeNameToMetaVictims"]
    assert 1 <= len(plans) <= 4 and "f005" not in plans and "f017" not in plans
    assert all(len(v["pods"]) == 1 for v in plans.values())


def test_request_waits_for_a_job_that_is_about_to_finish_instead_of_preempting():
    p = Platform({"scheduler": {"preemptionWaitWindowSeconds": 30, "preemptionMaxWaitSeconds": 0.3,
                                "preemptionUrgentPriority": 1000}})
    p.add_fake_node(make_fixture("w0", 8, 2))
    assert p.schedule(wl("ending", 8, priority=1, expectedDurationSeconds=5))["ok"]
    d = p.schedule(wl("hi", 8, priority=100))
    assert not d["ok"]                                       # told to wait: nothing evicted
    m = p.scheduler_metrics()
    assert m["preemptions"] == 0 and m["preemptions_deferred_wait"] == 1
    assert _alloc(p, "ending") is not None
    # an urgent request does not wait
    u = p.schedule(wl("urgent", 8, priority=1000))
    assert u["ok"] and u["preempted"] == ["ending"]
    # and patience runs out: past preemptionMaxWaitSeconds the waiting request preempts too
    assert p.release("urgent")
    assert p.schedule(wl("ending2", 8, priority=1, expectedDurationSeconds=5))["ok"]
    assert not p.schedule(wl("hi2", 8, priority=100))["ok"]
    import time
    time.sleep(0.4)
    d = p.schedule(wl("hi2", 8, priority=100))
    assert d["ok"] and d["preempted"] == ["ending2"]


def test_long_running_victims_are_preempted_while_near_finishers_are_spared():
    p = Platform({"scheduler": {"preemptionWaitWindowSeconds": 30}})
    p.add_fake_node(make_fixture("w0", 8, 2))
    assert p.schedule(wl("long1", 3, priority=1, expectedDurationSeconds=86400))["ok"]
    assert p.schedule(wl("long2", 3, priority=1, expectedDurationSeconds=86400))["ok"]
    assert p.schedule(wl("short", 2, priority=1, expectedDurationSeconds=5))["ok"]   # youngest: first in line otherwise
    d = p.schedule(wl("hi", 4, priority=100))   # the near finisher's 2 GPUs are not enough to wait for
    assert d["ok"] and sorted(d["preempted"]) == ["long1", "long2"]
    assert _alloc(p, "short") is not None


def test_preemption_rate_window_caps_victims_and_counts_refusals():
    p = Platform({"scheduler": {"preemptionWaitWindowSeconds": 0, "preemptionMaxRatePercent": 5.0,
                                "preemptionBurst": 2, "preemptionWindowSeconds": 60}})
    _full_fleet(p, 6)
    got = [p.schedule(wl(f"hi{i}", 8, priority=100)) for i in range(4)]
    assert [d["ok"] for d in got] == [True, True, False, False]     # burst of 2, then 5 % of ~8 placements = 0
    m = p.scheduler_metrics()
    assert m["preemptions"] == 2 and m["preemptions_rate_limited"] == 2
    # no cap configured: everything preempts
    q = Platform({"scheduler": {"preemptionWaitWindowSeconds": 0, "preemptionMaxRatePercent": 0}})
    _full_fleet(q, 6)
    assert all(q.schedule(wl(f"hi{i}", 8, priority=100))["ok"] for i in range(4))


def test_lifetimes_are_learned_per_workload_type_when_not_declared():
    p = Platform({})
    p.add_fake_node(make_fixture("l0", 8, 2))
    for i in range(8):
        assert p.schedule(wl(f"s{i}", 1))["ok"]
        assert _alloc(p, f"s{i}")["expected_duration_s"] == 0     # nothing learned yet
        assert p.release(f"s{i}")
    assert p.schedule(wl("next", 1))["ok"]
    a = _alloc(p, "next")
    assert 0 < a["expected_duration_s"] < 5       # the observed (milliseconds-long) lifetimes
    import time
    assert abs(a["allocated_unix_s"] - time.time()) < 5
    assert p.schedule(wl("decl", 1, expectedDurationSeconds=3600))["ok"]
    a = _alloc(p, "decl")
    assert abs(a["expected_duration_s"] - 3600) < 1e-6
