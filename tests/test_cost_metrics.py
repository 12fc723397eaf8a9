"""Cost engine (pricing, adjusted cost, budgets/enforcement, alerts,
recommendations, chargeback, journal replay) and Prometheus exposition."""
import re

import pytest

from kgwe.core import Platform

T0 = 1_760_000_000.0  # fixed epoch for deterministic periods


@pytest.fixture
def plat(tmp_path):
    return Platform({"cost": {"journalPath": str(tmp_path / "cost.jsonl")}})


def run_usage(p, uid, hours, gfx, gpus=1, ns="ml", team="t1", tier="OnDemand", mode="", t=T0):
    assert p.cost_start({"uid": uid, "namespace": ns, "team": team, "gpu_count": gpus, "tier": tier,
                         "partition_mode": mode}, t) == ""
    steps = 10
    for i in range(1, steps + 1):
        p.cost_sample(uid, gfx, gfx, t + hours * 3600 * i / steps)
    return p.cost_finalize(uid, t + hours * 3600)


def test_raw_and_adjusted_cost_rules(plat):
    price = {x["gpu_type"]: x for x in plat.pricing()}["amd-mi355x-288gb"]
    r = run_usage(plat, "busy", 2.0, 90.0, gpus=8)
    assert r["raw_cost"] == pytest.approx(price["on_demand"] * 8 * 2)
    assert r["adjusted_cost"] == pytest.approx(round(r["raw_cost"] * 0.95, 2))  # >80 % util discount
    idle = run_usage(plat, "idle", 1.0, 1.0)
    assert idle["adjusted_cost"] == pytest.approx(round(idle["raw_cost"] * 1.1, 2), abs=0.011)
    short = plat.cost_start({"uid": "s", "namespace": "ml"}, T0)
    assert short == ""
    assert plat.cost_finalize("s", T0 + 30)["adjusted_cost"] == pytest.approx(
        price["on_demand"] * 30 / 3600)


def test_partition_pricing_is_fractional(plat):
    r = run_usage(plat, "cpx", 1.0, 50.0, gpus=1, mode="CPX")
    price = {x["gpu_type"]: x for x in plat.pricing()}["amd-mi355x-288gb"]
    assert r["raw_cost"] == pytest.approx(price["on_demand"] / 8)


def test_budget_alerts_and_block_enforcement(plat):
    assert plat.create_budget({"metadata": {"name": "b1", "namespace": "ml"},
                               "spec": {"limit": "100", "scope": "Namespace", "period": "Monthly",
                                        "enforcementPolicy": "Block"}}, T0) == ""
    run_usage(plat, "w1", 4.0, 50.0, gpus=8)  # ~ $94
    alerts = plat.alerts()
    assert {a["threshold"] for a in alerts} >= {0.5, 0.75, 0.9}
    assert any(a["severity"] == "Critical" for a in alerts)
    adm = plat.admit("ml", "", "", 50.0, T0 + 4 * 3600)
    assert not adm["allowed"] and "Block" in adm["reason"]
    assert plat.admit("other-ns", "", "", 50.0, T0)["allowed"]
    assert plat.acknowledge_alert(alerts[0]["id"])
    assert len(plat.alerts(unacknowledged_only=True)) == len(alerts) - 1


def test_team_project_cluster_scopes_match(plat):
    for scope, sid in (("Team", "t1"), ("Project", "p1"), ("Cluster", "default")):
        plat.create_budget({"name": f"b-{scope}", "limit": 1000, "scope": scope, "scopeId": sid}, T0)
    plat.cost_start({"uid": "x", "namespace": "ml", "team": "t1", "project": "p1", "gpu_count": 1}, T0)
    plat.cost_finalize("x", T0 + 3600)
    spends = {b["name"]: b["spend"] for b in plat.budgets(T0 + 3600)}
    assert all(v > 0 for v in spends.values()), spends


def test_budget_period_rolls_over(plat):
    plat.create_budget({"name": "daily", "limit": 10, "scope": "Namespace", "scopeId": "ml",
                        "period": "Daily"}, T0)
    run_usage(plat, "d1", 1.0, 50.0)
    assert plat.budgets(T0 + 3600)[0]["spend"] > 0
    assert plat.budgets(T0 + 2 * 86400)[0]["spend"] == 0


def test_recommendations_and_chargeback(plat):
    run_usage(plat, "lowutil", 10.0, 5.0, gpus=2)
    for i in range(6):
        run_usage(plat, "bursty", 0.5, 10.0, t=T0 + i * 7200)
    recs = plat.recommendations()
    types = {(r["uid"], r["type"]) for r in recs}
    assert ("lowutil", "Spot") in types and ("lowutil", "Rightsize") in types
    assert ("bursty", "Consolidate") in types
    assert recs == sorted(recs, key=lambda r: -r["projected_saving"])
    cb = plat.chargeback("team")
    assert cb["lines"][0]["group"] == "t1" and cb["total_cost"] > 0
    s = plat.cost_summary("Namespace", "ml")
    assert s["records"] == 7 and "amd-mi355x-288gb" in s["by_gpu_type"]


def test_journal_replay_restores_records(tmp_path):
    path = str(tmp_path / "j.jsonl")
    p1 = Platform({"cost": {"journalPath": path}})
    run_usage(p1, "persist", 1.0, 70.0)
    p2 = Platform({"cost": {"journalPath": path}})
    assert p2.cost_replayed() == 1
    assert p2.cost_summary("Namespace", "ml")["records"] == 1


def test_prometheus_exposition_has_label_sets(plat):
    from kgwe.core import make_fixture

    plat.add_fake_node(make_fixture("n0", 8, 2))
    plat.schedule({"metadata": {"name": "j", "uid": "j", "namespace": "ml"},
                   "spec": {"gpuRequirements": {"count": 2}}})
    plat.observe_pod_latency_ms(12.5)
    text = plat.expose_metrics()
    assert '# TYPE kgwe_scheduling_latency_ms histogram' in text
    assert 'kgwe_scheduling_latency_ms_bucket{le="25"} 1' in text
    assert 'kgwe_scheduling_latency_ms_bucket{le="+Inf"} 1' in text
    assert re.search(r'kgwe_gpu_utilization_percent\{gpu_uuid="GPU-n0-00",node="n0",model="[^"]+"\}', text)
    assert 'kgwe_xgmi_link_status{gpu_uuid_1="GPU-n0-00",gpu_uuid_2="GPU-n0-01",node="n0"} 1' in text
    assert 'kgwe_gpu_partition_mode{gpu_uuid="GPU-n0-00",node="n0",compute="SPX",memory="NPS1"} 1' in text
    assert 'kgwe_active_workloads{namespace="ml",workload_type="Training"} 1' in text
    fams = plat.raw.metric_families()
    assert len(fams) >= 27


def test_bench_cost_row_is_metered_by_engine():
    import bench

    c = bench.meter_cost(8, 160000.0, 99.0)
    assert c["gpus"] == 8 and c["run_tokens"] == 10**9
    assert c["run_hours"] == pytest.approx(1e9 / 160000.0 / 3600, rel=1e-3)
    # high utilisation earns the engine's efficiency discount, never a surcharge
    assert 0 < c["adjusted_cost_usd"] <= c["raw_cost_usd"]
    assert c["raw_cost_usd"] == pytest.approx(c["usd_per_gpu_hour"] * 8 * c["run_hours"], rel=1e-2)
