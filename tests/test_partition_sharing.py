"""MI355X partition controller (MIG replacement) and GPU sharing manager."""
import pytest

from kgwe.core import Platform, make_fixture


def part_wl(uid, mode="CPX", count=1):
    return {"metadata": {"name": uid, "namespace": "inf", "uid": uid},
            "spec": {"workloadType": "Inference",
                     "gpuRequirements": {"count": 0, "partition": {"mode": mode, "count": count}}}}


@pytest.fixture
def plat():
    p = Platform({})
    p.add_fake_node(make_fixture("n0", 8, 2))
    return p


def test_cpx_one_gpu_split_eight_ways_binpacks_eight_pods(plat):
    # BASELINE config 4: one GPU split 8-way, 8 inference pods bin-packed.
    decisions = [plat.schedule(part_wl(f"inf{i}")) for i in range(8)]
    assert all(d["ok"] for d in decisions)
    gpus = {d["partitions"][0].rsplit("/p", 1)[0] for d in decisions}
    assert len(gpus) == 1, "all 8 slices must come from ONE GPU (bin-packing)"
    assert len({d["partitions"][0] for d in decisions}) == 8
    assert plat.fake_partition_switches("n0") == 1
    m = plat.partition_metrics()
    assert m["modes"]["CPX"]["slices_in_use"] == 8 and m["slice_utilization"] == 1.0
    # CPX slice env: logical HIP device = GPU base + slice index
    envs = sorted(int(d["env"]["HIP_VISIBLE_DEVICES"]) for d in decisions)
    assert envs == list(range(min(envs), min(envs) + 8))


def test_ninth_pod_converts_a_second_gpu(plat):
    for i in range(9):
        assert plat.schedule(part_wl(f"p{i}"))["ok"]
    assert plat.fake_partition_switches("n0") == 2


def test_busy_gpu_never_repartitioned(plat):
    whole = plat.schedule({"metadata": {"name": "t", "uid": "t"},
                           "spec": {"gpuRequirements": {"count": 8}}})
    assert whole["ok"]
    d = plat.schedule(part_wl("x"))
    assert not d["ok"]
    assert plat.fake_partition_switches("n0") == 0


def test_strategy_validation_and_rebalance(plat):
    bad = {"metadata": {"name": "bad"}, "spec": {"profileDistribution": {"CPX": 0.8, "QPX": 0.5}}}
    assert "sums to more" in plat.register_strategy(bad)
    tpx = {"metadata": {"name": "tpx"}, "spec": {"profileDistribution": {"TPX": 0.5}}}
    assert "TPX" in plat.register_strategy(tpx)
    good = {"metadata": {"name": "mix"},
            "spec": {"profileDistribution": {"CPX": 0.25, "QPX": 0.25}, "rebalanceInterval": "5m"}}
    assert plat.register_strategy(good) == ""
    plan = plat.rebalance("mix", plan_only=True)
    assert len(plan) == 4 and plat.fake_partition_switches("n0") == 0
    ops = plat.rebalance("mix")
    assert all(o["state"] == "Completed" for o in ops)
    modes = [g["partition"]["compute"] for g in plat.node("n0")["gpus"]]
    assert modes.count("CPX") == 2 and modes.count("QPX") == 2 and modes.count("SPX") == 4


def test_reclaim_idle_partitioned_gpus(plat):
    plat.ensure_partitions("CPX", 8)
    assert plat.partition_metrics()["modes"]["CPX"]["gpus"] == 1
    ops = plat.reclaim_idle_partitions()
    assert len(ops) == 1
    assert "CPX" not in plat.partition_metrics()["modes"]


def test_tick_reclaims_only_after_idle_hysteresis():
    p = Platform({"partitionReclaimIdleSeconds": 30.0})
    p.add_fake_node(make_fixture("n0", 8, 2))
    d = p.schedule(part_wl("a"))
    assert d["ok"] and p.fake_partition_switches("n0") == 1
    p.tick(100.0)  # slice in use: not idle
    p.release("a", 101.0)
    p.tick(102.0)  # idle clock starts
    p.tick(120.0)
    assert p.partition_metrics()["modes"]["CPX"]["gpus"] == 1, "reclaimed before the hysteresis"
    assert p.schedule(part_wl("b"))["ok"]  # reuses the slice, no mode switch
    assert p.fake_partition_switches("n0") == 1
    p.tick(140.0)  # busy again: idle clock resets
    p.release("b", 141.0)
    p.tick(150.0)
    p.tick(175.0)
    assert "CPX" in p.partition_metrics()["modes"]
    p.tick(181.0)
    assert "CPX" not in p.partition_metrics()["modes"]
    assert p.fake_partition_switches("n0") == 2
    never = Platform({"partitionReclaimIdleSeconds": -1})
    never.add_fake_node(make_fixture("n0", 8, 2))
    never.ensure_partitions("CPX", 8)
    never.tick(0.0)
    never.tick(1e6)
    assert never.partition_metrics()["modes"]["CPX"]["gpus"] == 1


def test_dry_run_does_not_actuate():
    p = Platform({"partitionDryRun": True})
    p.add_fake_node(make_fixture("d0", 8, 2))
    ops = p.ensure_partitions("CPX", 8)
    assert ops and ops[0]["dry_run"] and p.fake_partition_switches("d0") == 0


def test_colocation_gets_disjoint_cu_masks(plat):
    g = "GPU-n0-00"
    a = plat.share_allocate({"uid": "a", "node": "n0", "gpu": g, "cuPercent": 25, "memoryGB": 40})
    b = plat.share_allocate({"uid": "b", "node": "n0", "gpu": g, "cuPercent": 50, "memoryGB": 40})
    assert a["error"] == "" and b["error"] == ""
    assert a["method"] == "CoLocate"
    assert a["env"]["HSA_CU_MASK"] == "0:0-63" and b["env"]["HSA_CU_MASK"] == "0:64-191"
    c = plat.share_allocate({"uid": "c", "node": "n0", "gpu": g, "cuPercent": 50})
    assert "no room" in c["error"]
    assert plat.share_release("a")
    c = plat.share_allocate({"uid": "c", "node": "n0", "gpu": g, "cuPercent": 25})
    assert c["error"] == "" and c["cu_begin"] == 0


def test_sharing_method_selection(plat):
    r = plat.share_allocate({"uid": "iso", "requireIsolation": True, "gpu": "GPU-n0-01"})
    assert r["method"] == "Partition"


def test_memory_mode_requests_cpx_nps2():
    """gpuRequirements.partition.memoryMode is honoured: a CPX/NPS2 slice
    converts an idle GPU to CPX + NPS2 (compute first, then memory, so every
    intermediate state is valid); a CPX/NPS1 request does not take NPS2
    slices; SPX+NPS2 is rejected; reclaim returns the GPU to SPX/NPS1."""
    p = Platform({})
    p.add_fake_node(make_fixture("n0", 8, 2))

    def wl(uid, mem=None):
        part = {"mode": "CPX", "count": 1}
        if mem:
            part["memoryMode"] = mem
        return {"metadata": {"name": uid, "namespace": "inf", "uid": uid},
                "spec": {"workloadType": "Inference", "gpuRequirements": {"count": 0, "partition": part}}}

    d = p.schedule(wl("a", "NPS2"))
    assert d["ok"]
    g_a = d["partitions"][0].rsplit("/p", 1)[0]
    gpu = {g["uuid"]: g for g in p.node("n0")["gpus"]}[g_a]
    assert gpu["partition"]["compute"] == "CPX" and gpu["partition"]["memory"] == "NPS2"
    d2 = p.schedule(wl("b", "NPS1"))
    assert d2["ok"] and d2["partitions"][0].rsplit("/p", 1)[0] != g_a
    d3 = p.schedule(wl("c"))  # no memory constraint: packs onto the fullest CPX GPU
    assert d3["ok"]
    assert p.ensure_partitions("SPX", 1, memory="NPS2") == []  # invalid combination: nothing planned
    for u in ("a", "b", "c"):
        p.release(u)
    ops = p.reclaim_idle_partitions()
    assert ops and all(o["to"] == "SPX" and o["memory_to"] == "NPS1" for o in ops)
    assert all(g["partition"]["memory"] == "NPS1" for g in p.node("n0")["gpus"])


def test_slice_pods_fill_the_fullest_partitioned_gpu_in_the_fleet():
    """Best fit across nodes is by the GPU that takes the slice: a slice pod
    scores the node whose CPX GPU is fuller higher, whatever the nodes' whole
    GPUs are doing, so the emptier partitioned GPU drains and can go back to
    SPX."""
    p = Platform({})
    for n in ("na", "nb"):
        p.add_fake_node(make_fixture(n, 8, 2))

    def on(node, uid, wl):
        wl = {**wl, "spec": {**wl["spec"], "nodeSelector": {"kubernetes.io/hostname": node}}}
        d = p.schedule(wl)
        assert d["ok"] and d["node"] == node, d
        return d

    p.ensure_partitions("CPX", 16)                  # one CPX GPU on each node (bin-packed per node)
    modes = {n: [g["partition"]["compute"] for g in p.node(n)["gpus"]].count("CPX") for n in ("na", "nb")}
    if modes != {"na": 1, "nb": 1}:
        pytest.skip(f"fixture partitions landed as {modes}")
    for i in range(6):
        on("na", f"a{i}", part_wl(f"a{i}"))         # na's CPX GPU: 6 of 8 in use
    for i in range(2):
        on("nb", f"b{i}", part_wl(f"b{i}"))         # nb's: 2 of 8
    # nb is the busier node by whole GPUs
    on("nb", "train", {"metadata": {"name": "train", "uid": "train"},
                       "spec": {"gpuRequirements": {"count": 6}}})
    sa, sb = p.score_node("na", part_wl("x")), p.score_node("nb", part_wl("x"))
    assert sa["total"] > sb["total"], (sa, sb)
    assert sa["resource"] == 100 * 7 // 8 and sb["resource"] == 100 * 3 // 8
    d = p.schedule(part_wl("x"))
    assert d["ok"] and d["node"] == "na"
