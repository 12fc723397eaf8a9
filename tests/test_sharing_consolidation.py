"""GPU sharing held in the scheduler ledger, partition consolidation, gangs
on one xGMI island, pod create -> bind latency recorded by bind itself,
queue depth, and failover restore of the full ledger entry."""
import json
import time

import pytest

from kgwe.core import Platform, make_fixture


def share_wl(uid, method="CoLocate", cu=12.5, mem=30.0, prio=0, preemptible=True):
    return {"metadata": {"name": uid, "namespace": "inf", "uid": uid},
            "spec": {"workloadType": "Inference", "priority": prio, "preemptible": preemptible,
                     "gpuRequirements": {"count": 1, "sharing": {"method": method, "cuPercent": cu,
                                                                  "memoryGB": mem}}}}


def whole_wl(uid, n, prio=0, preemptible=True, topo="xGMIOptimal", gang=None):
    w = {"metadata": {"name": uid, "namespace": "train", "uid": uid},
         "spec": {"workloadType": "Training", "priority": prio, "preemptible": preemptible,
                  "gpuRequirements": {"count": n, "topology": {"preference": topo}},
                  "distributedConfig": {"strategy": "DataParallel"}}}
    if gang:
        w["spec"]["gang"] = {"name": gang[0], "size": gang[1]}
    return w


def cpx_wl(uid):
    return {"metadata": {"name": uid, "namespace": "inf", "uid": uid},
            "spec": {"workloadType": "Inference",
                     "gpuRequirements": {"count": 0, "partition": {"mode": "CPX", "count": 1}}}}


@pytest.fixture
def plat():
    p = Platform({"enforceBudgets": False})
    p.add_fake_node(make_fixture("n0", 8, 2))
    return p


def test_eight_colocated_clients_pack_one_gpu_with_disjoint_xcd_masks(plat):
    ds = [plat.schedule(share_wl(f"c{i}")) for i in range(8)]
    assert all(d["ok"] for d in ds)
    gpus = {d["shared_gpu"] for d in ds}
    assert len(gpus) == 1  # best fit: one GPU, 8 x one XCD (32 CUs)
    ranges = sorted((d["cu_begin"], d["cu_end"]) for d in ds)
    assert ranges == [(32 * i, 32 * i + 32) for i in range(8)]
    masks = {d["env"]["HSA_CU_MASK"] for d in ds}
    assert len(masks) == 8 and all(m.startswith("0:") for m in masks)
    assert all(d["env"]["KGWE_SHARING"] == "CoLocate" for d in ds)
    assert all(float(d["env"]["KGWE_GPU_MEMORY_FRACTION"]) == pytest.approx(30 / 288, rel=1e-3)
               for d in ds)
    # a ninth client opens a second GPU
    d9 = plat.schedule(share_wl("c8"))
    assert d9["ok"] and d9["shared_gpu"] not in gpus
    m = plat.scheduler_metrics()
    assert m["shared_gpus"] == 2 and m["share_clients"] == 9


def test_shared_gpu_is_never_handed_out_whole_or_partitioned(plat):
    assert plat.schedule(share_wl("s0"))["ok"]
    shared = plat.allocations()[0]["shared_gpu"]
    d = plat.schedule(whole_wl("big", 8))  # needs all 8 GPUs: one is shared
    assert not d["ok"]
    d7 = plat.schedule(whole_wl("seven", 7))
    assert d7["ok"] and shared not in d7["gpus"]
    # the shared GPU is not idle: no partition switch may take it
    assert plat.ensure_partitions("CPX", 1) == [] or all(
        op["gpu"] != shared for op in plat.partition_ops())
    plat.release("seven")
    # and a whole-GPU holder never takes clients
    dw = plat.schedule(whole_wl("one", 1))
    for i in range(8):
        ds = plat.schedule(share_wl(f"x{i}"))
        assert ds["ok"] and ds["shared_gpu"] != dw["gpus"][0]


def test_timeslice_and_colocate_do_not_mix_on_one_gpu(plat):
    a = plat.schedule(share_wl("ts0", method="TimeSlice", mem=0))
    b = plat.schedule(share_wl("co0"))
    assert a["ok"] and b["ok"] and a["shared_gpu"] != b["shared_gpu"]
    assert "HSA_CU_MASK" not in a["env"] and a["env"]["KGWE_SHARING"] == "TimeSlice"


def test_memory_cap_limits_clients(plat):
    ds = [plat.schedule(share_wl(f"m{i}", cu=5, mem=100.0)) for i in range(3)]
    assert all(d["ok"] for d in ds)
    assert len({d["shared_gpu"] for d in ds}) == 2  # 2 x 100 GB fit 288 GB, the third does not


def test_share_release_frees_the_gpu_for_whole_allocation(plat):
    d = plat.schedule(share_wl("s0"))
    assert not plat.schedule(whole_wl("all8", 8))["ok"]
    plat.release("s0")
    assert plat.schedule(whole_wl("all8", 8))["ok"]


def test_share_clients_are_preemptible_victims(plat):
    for i in range(8):
        assert plat.schedule(whole_wl(f"w{i}", 1, prio=0))["ok"] or True
    plat.release("w7")
    assert plat.schedule(share_wl("s0", prio=1))["ok"]
    d = plat.schedule(whole_wl("urgent", 1, prio=100, preemptible=False))
    assert d["ok"] and d["preempted"]


def test_extender_pod_with_gpu_shared_resource_gets_cu_mask(plat):
    pod = {"metadata": {"name": "srv", "namespace": "inf", "uid": "u-srv",
                        "annotations": {"kgwe.amd.com/cu-percent": "25", "kgwe.amd.com/memory-gb": "36"}},
           "spec": {"containers": [{"name": "m", "resources": {"limits": {"amd.com/gpu-shared": "1"}}}]}}
    body = json.dumps({"pod": pod, "nodenames": ["n0"]})
    f = json.loads(plat.filter(body))
    assert f["nodenames"] == ["n0"]
    res = plat.bind(json.dumps({"podName": "srv", "podNamespace": "inf", "podUID": "u-srv", "node": "n0"}))
    assert res["result"] == {} or not res["result"].get("error")
    env = res["placement"]["env"]
    assert env["KGWE_SHARING"] == "CoLocate" and env["HSA_CU_MASK"] == "0:0-63"
    assert res["placement"]["workload"]["sharing"] == "CoLocate"


def test_gang_lands_on_one_xgmi_island():
    p = Platform({"enforceBudgets": False})
    for n in ("a", "b", "c"):
        p.add_fake_node(make_fixture(n, 8, 2))
    # fragment: 2 GPUs used on a and b each, c half used
    for i, node_fill in enumerate((2, 2, 4)):
        for k in range(node_fill):
            p.schedule(whole_wl(f"f{i}{k}", 1, topo="None"))
    members = [whole_wl(f"g{k}", 1, gang=("g", 4)) for k in range(4)]
    ds = p.schedule_gang(members)
    assert all(d["ok"] for d in ds)
    assert len({d["node"] for d in ds}) == 1
    assert len({g for d in ds for g in d["gpus"]}) == 4
    # xGMIRequired gang larger than any node's free GPUs: refused, nothing held
    big = [whole_wl(f"h{k}", 5, topo="xGMIRequired", gang=("h", 2)) for k in range(2)]
    before = len(p.allocations())
    assert not any(d["ok"] for d in p.schedule_gang(big))
    assert len(p.allocations()) == before


def test_preempting_a_gang_member_preempts_the_whole_gang():
    p = Platform({"enforceBudgets": False})
    p.add_fake_node(make_fixture("a", 8, 2))
    p.add_fake_node(make_fixture("b", 8, 2))
    # 2 x 5 GPUs cannot share a node: one member per node
    ds = p.schedule_gang([whole_wl(f"g{k}", 5, prio=1, topo="None", gang=("g", 2)) for k in range(2)])
    assert all(d["ok"] for d in ds) and len({d["node"] for d in ds}) == 2
    for n in ("a", "b"):
        assert p.schedule(whole_wl(f"fill-{n}", 3, prio=1000, preemptible=False, topo="None"))["ok"]
    d = p.schedule(whole_wl("urgent", 5, prio=500, preemptible=False, topo="None"))
    assert d["ok"]
    assert set(d["preempted"]) == {"g0", "g1"}  # both members, even the one on the other node
    assert not any(a["uid"] in ("g0", "g1") for a in p.allocations())


def test_consolidation_empties_underused_cpx_gpus_and_reclaims_them():
    p = Platform({"enforceBudgets": False, "partitionReclaimIdleSeconds": -1,
                  "partitionConsolidateAfterSeconds": 0, "migrationCooldownSeconds": 0})
    p.add_fake_node(make_fixture("n0", 8, 2))
    # 16 slices on 2 CPX GPUs, then free most of them: 3 left on each GPU
    uids = [f"i{k}" for k in range(16)]
    for u in uids:
        assert p.schedule(cpx_wl(u))["ok"]
    assert p.partition_metrics()["modes"]["CPX"]["gpus"] == 2
    by_gpu = {}
    for a in p.allocations():
        by_gpu.setdefault(a["partitions"][0].rsplit("/p", 1)[0], []).append(a["uid"])
    keep = []
    for g, us in by_gpu.items():
        for u in us[3:]:
            p.release(u)
        keep += us[:3]
    assert p.partition_metrics()["slice_utilization"] == pytest.approx(6 / 16)
    moves = p.consolidate_partitions(time.time(), plan_only=False)
    assert len(moves) == 3 and all(m["uid"] in keep for m in moves)
    m = p.partition_metrics()
    assert m["modes"]["CPX"]["gpus"] == 1 and m["slice_utilization"] == pytest.approx(6 / 8)
    assert m["migrations"] == 3
    # every workload still holds exactly one slice, all on one GPU
    held = [a["partitions"] for a in p.allocations()]
    assert len(held) == 6 and all(len(h) == 1 for h in held)
    assert len({h[0].rsplit("/p", 1)[0] for h in held}) == 1


def test_consolidation_never_moves_training_or_nonpreemptible():
    p = Platform({"enforceBudgets": False, "partitionReclaimIdleSeconds": -1,
                  "partitionConsolidateAfterSeconds": 0})
    p.add_fake_node(make_fixture("n0", 8, 2))
    w = cpx_wl("keep")
    w["spec"]["preemptible"] = False
    assert p.schedule(w)["ok"]
    for k in range(9):
        assert p.schedule(cpx_wl(f"x{k}"))["ok"]
    for k in range(1, 9):
        p.release(f"x{k}")
    # GPU A: keep + x0? (packing order) — whatever the layout, "keep" never moves
    moves = p.consolidate_partitions(time.time(), plan_only=False)
    assert all(m["uid"] != "keep" for m in moves)


def test_consolidation_hysteresis_waits():
    p = Platform({"enforceBudgets": False, "partitionReclaimIdleSeconds": -1,
                  "partitionConsolidateAfterSeconds": 100})
    p.add_fake_node(make_fixture("n0", 8, 2))
    for k in range(9):
        p.schedule(cpx_wl(f"x{k}"))
    for k in range(1, 8):
        p.release(f"x{k}")
    assert p.consolidate_partitions(1000.0, plan_only=True) == []
    assert p.consolidate_partitions(1050.0, plan_only=True) == []
    assert len(p.consolidate_partitions(1101.0, plan_only=True)) == 1


def test_plan_only_consolidation_bars_new_slices_on_the_donor_until_it_is_empty():
    """Controller path on two nodes: the plan names the moves, the caller
    evicts the donor's pods.  Until the donor is empty and back to SPX no new
    slice may land on it, so the evicted pods reschedule onto the receiver."""
    p = Platform({"enforceBudgets": False, "partitionReclaimIdleSeconds": -1,
                  "partitionConsolidateAfterSeconds": 0, "migrationCooldownSeconds": 0})
    for n in ("n0", "n1"):
        p.add_fake_node(make_fixture(n, 8, 2))
    for k in range(7):   # n0 keeps one GPU free: the first CPX GPU is there, the second on n1
        w = whole_wl(f"fill{k}", 1, topo="None")
        w["spec"]["constraints"] = {"nodeSelector": {"kubernetes.io/hostname": "n0"}}
        assert p.schedule(w)["ok"]
    for n in ("n0", "n1"):
        for k in range(8):
            d = p.schedule(cpx_wl(f"{n}-i{k}"))
            assert d["ok"] and d["node"] == n
    for k in range(2, 8):
        p.release(f"n0-i{k}")      # n0's GPU: 2 of 8 used
    for k in range(5, 8):
        p.release(f"n1-i{k}")      # n1's GPU: 5 of 8 used
    moves = p.consolidate_partitions(time.time(), plan_only=True)
    assert sorted(m["uid"] for m in moves) == ["n0-i0", "n0-i1"]
    assert all(m["node_from"] == "n0" and m["node_to"] == "n1" for m in moves)
    donor = moves[0]["from"].rsplit("/p", 1)[0]
    assert p.draining_gpus() == [donor]
    # the ledger is untouched by a plan, but the donor takes no new slice: a fresh
    # request that would otherwise pack onto n0's 6 free slices goes to n1
    assert len(p.allocations()) == 7 + 7
    d = p.schedule(cpx_wl("fresh"))
    assert d["ok"] and d["node"] == "n1"
    # the caller evicts the two pods; they come back and land on the receiver
    for m in moves:
        assert p.release(m["uid"])
        d = p.schedule(cpx_wl(m["uid"] + "-again"))
        assert d["ok"] and d["node"] == "n1" and not d["partitions"][0].startswith(donor)
    # donor empty: the next pass returns it to SPX and lifts the bar
    p.consolidate_partitions(time.time(), plan_only=True)
    assert p.draining_gpus() == []
    m = p.partition_metrics()
    assert m["modes"]["CPX"]["gpus"] == 1


def test_a_donor_that_never_empties_is_given_back():
    p = Platform({"enforceBudgets": False, "partitionReclaimIdleSeconds": -1,
                  "partitionConsolidateAfterSeconds": 0, "migrationCooldownSeconds": 0})
    p.add_fake_node(make_fixture("n0", 8, 2))
    for k in range(16):
        assert p.schedule(cpx_wl(f"i{k}"))["ok"]
    by_gpu = {}
    for a in p.allocations():
        by_gpu.setdefault(a["partitions"][0].rsplit("/p", 1)[0], []).append(a["uid"])
    (ga, ua), (gb, ub) = sorted(by_gpu.items())
    for u in ua[2:] + ub[5:]:
        p.release(u)
    t0 = 1000.0
    assert len(p.consolidate_partitions(t0, plan_only=True)) == 2
    assert p.draining_gpus() == [ga]
    assert p.consolidate_partitions(t0 + 200, plan_only=True) == [] and p.draining_gpus() == [ga]
    p.consolidate_partitions(t0 + 301, plan_only=True)   # nobody evicted the pods: bar lifted, planned again
    assert ga in p.draining_gpus() or p.draining_gpus() == []
    held_on_a = [a for a in p.allocations() if a["partitions"][0].startswith(ga)]
    assert len(held_on_a) == 2


def test_bind_records_pod_latency_and_queue_depth(plat):
    names = [f"p{i}" for i in range(5)]
    for n in names:
        pod = {"metadata": {"name": n, "namespace": "d", "uid": "u-" + n},
               "spec": {"containers": [{"name": "m", "resources": {"limits": {"amd.com/gpu": "1"}}}]}}
        plat.filter(json.dumps({"pod": pod, "nodenames": ["n0"]}))
    assert plat.queue_depth() == 5
    time.sleep(0.02)
    for n in names:
        r = plat.bind(json.dumps({"podName": n, "podNamespace": "d", "podUID": "u-" + n, "node": "n0"}))
        assert not r["result"].get("error")
    assert plat.queue_depth() == 0
    assert plat.pod_latency_count() == 5
    assert plat.pod_latency_quantile_ms(0.5) >= 20.0
    text = plat.expose_metrics()
    assert 'kgwe_scheduling_latency_ms_count 5' in text
    assert 'kgwe_workload_queue_depth 0' in text


def test_bind_uses_microsecond_creation_stamp(plat):
    pod = {"metadata": {"name": "s", "namespace": "d", "uid": "u-s",
                        "annotations": {"kgwe.amd.com/created-at": f"{time.time() - 0.25:.6f}"}},
           "spec": {"containers": [{"name": "m", "resources": {"limits": {"amd.com/gpu": "1"}}}]}}
    plat.filter(json.dumps({"pod": pod, "nodenames": ["n0"]}))
    plat.bind(json.dumps({"podName": "s", "podNamespace": "d", "podUID": "u-s", "node": "n0"}))
    assert 240.0 <= plat.pod_latency_quantile_ms(0.5) <= 400.0


def test_restore_keeps_preemptible_type_gang_and_share():
    p = Platform({"enforceBudgets": False})
    p.add_fake_node(make_fixture("n0", 8, 2))
    assert p.restore_allocation({"uid": "nonpre", "node": "n0", "gpus": ["GPU-n0-00"], "priority": 5,
                                 "preemptible": False, "type": "Training", "gang": "g", "gang_size": 2})
    assert p.restore_allocation({"uid": "share", "node": "n0", "sharing": "CoLocate",
                                 "shared_gpu": "GPU-n0-01", "cu_begin": 0, "cu_end": 32,
                                 "type": "Inference"})
    a = {x["uid"]: x for x in p.allocations()}
    assert a["nonpre"]["preemptible"] is False and a["nonpre"]["gang"] == "g"
    assert a["nonpre"]["gang_size"] == 2 and a["share"]["shared_gpu"] == "GPU-n0-01"
    assert p.permit("nonpre") == "Allow"
    # the non-preemptible entry survives a high-priority arrival
    for i in range(2, 8):
        p.schedule(whole_wl(f"f{i}", 1, prio=0, topo="None"))
    d = p.schedule(whole_wl("vip", 8, prio=10_000, topo="None"))
    assert not d["ok"] or "nonpre" not in d["preempted"]
    assert any(x["uid"] == "nonpre" for x in p.allocations())
    # and the restored share still blocks whole-GPU use of its GPU
    d1 = p.schedule(whole_wl("w1", 1, prio=0, topo="None"))
    assert not d1["ok"] or "GPU-n0-01" not in d1["gpus"]


def test_share_placement_counts_hbm_the_device_reports_in_use():
    """A co-located client's HBM cap must fit next to what the device itself
    reports as used, not only next to the caps the ledger promised."""
    node = make_fixture("m0", 2, 1)
    node["gpus"][0]["memory_used_gb"] = 270.0      # somebody outside the ledger holds 270 of 288 GB
    p = Platform({"enforceBudgets": False})
    p.upsert_node(node)
    busy, free = node["gpus"][0]["uuid"], node["gpus"][1]["uuid"]
    for k in range(8):      # eight 30 GB clients fill the other GPU's client slots
        d = p.schedule(share_wl(f"c{k}", mem=30.0))
        assert d["ok"] and d["shared_gpu"] == free
    # only the busy GPU is left: 270 + 30 > 288 is refused, 270 + 10 fits
    assert not p.schedule(share_wl("big", mem=30.0))["ok"]
    d = p.schedule(share_wl("small", mem=10.0))
    assert d["ok"] and d["shared_gpu"] == busy


# --- share groups: same-model clients behind one serving process ------------------------------

def group_wl(uid, group, cu=50.0, mem=40.0):
    w = share_wl(uid, cu=cu, mem=mem)
    w["spec"]["gpuRequirements"]["sharing"]["group"] = group
    return w


def test_share_group_members_ride_on_the_leaders_range_and_cap():
    p = Platform({"enforceBudgets": False, "shareSocketDir": "/run/kgwe/share"})
    for n in ("a", "b"):
        p.add_fake_node(make_fixture(n, 8, 2))
    lead = p.schedule(group_wl("m0", "llama-1b"))
    assert lead["ok"] and lead["share_leader"] and lead["share_leader_uid"] == "m0"
    assert (lead["cu_begin"], lead["cu_end"]) == (0, 128) and lead["share_memory_gb"] == 40.0
    env = lead["env"]
    assert env["KGWE_SHARE_ROLE"] == "leader" and env["KGWE_SHARE_GROUP"] == "llama-1b"
    sock = env["KGWE_BATCH_ENDPOINT"]
    assert sock == f"unix:/run/kgwe/share/{lead['shared_gpu']}-llama-1b.sock"
    members = [p.schedule(group_wl(f"m{k}", "llama-1b")) for k in range(1, 8)]
    for d in members:
        # same GPU, same CU range, no HBM of their own, and the leader's socket
        assert d["ok"] and d["shared_gpu"] == lead["shared_gpu"] and not d["share_leader"]
        assert (d["cu_begin"], d["cu_end"]) == (0, 128) and d["share_memory_gb"] == 0.0
        assert d["env"]["KGWE_SHARE_ROLE"] == "member" and d["env"]["KGWE_BATCH_ENDPOINT"] == sock
        assert d["env"]["KGWE_SHARE_LEADER"] == "m0" and "KGWE_GPU_MEMORY_FRACTION" not in d["env"]
    # the group is ONE client of the GPU: the other half of the CUs still takes an ordinary share
    other = p.schedule(share_wl("solo", cu=50.0, mem=100.0))
    assert other["ok"] and other["shared_gpu"] == lead["shared_gpu"]
    assert (other["cu_begin"], other["cu_end"]) == (128, 256)
    # another group gets a range (and a leader) of its own
    d = p.schedule(group_wl("x0", "mistral", cu=12.5, mem=20.0))
    assert d["ok"] and d["share_leader"] and d["shared_gpu"] != lead["shared_gpu"]
    m = p.scheduler_metrics()
    assert m["share_clients"] == 10


def test_share_group_size_is_bounded_and_a_full_group_starts_a_second_server():
    p = Platform({"enforceBudgets": False, "scheduler": {"maxGroupClients": 3}})
    p.add_fake_node(make_fixture("a", 2, 1))
    ds = [p.schedule(group_wl(f"c{k}", "g", cu=25.0, mem=10.0)) for k in range(5)]
    assert all(d["ok"] for d in ds)
    assert [d["share_leader"] for d in ds] == [True, False, False, True, False]
    assert ds[3]["share_leader_uid"] == "c3" and ds[4]["share_leader_uid"] == "c3"


def test_releasing_a_group_leader_names_its_orphans_and_blocks_new_joiners():
    p = Platform({"enforceBudgets": False})
    p.add_fake_node(make_fixture("a", 1, 1))
    for k in range(3):
        assert p.schedule(group_wl(f"c{k}", "g", cu=100.0, mem=10.0))["ok"]
    assert "orphaned_share_members" not in p.release("c2")          # a member leaves: nothing to do
    rel = p.release("c0")
    assert rel["orphaned_share_members"] == ["c1"]
    # nobody may join a group whose server is gone, and its CUs are still held by the orphan
    assert not p.schedule(group_wl("late", "g", cu=100.0, mem=10.0))["ok"]
    assert p.release("c1")["released"]
    d = p.schedule(group_wl("late", "g", cu=100.0, mem=10.0))
    assert d["ok"] and d["share_leader"]


def test_share_group_survives_a_ledger_rebuild():
    p = Platform({"enforceBudgets": False})
    p.add_fake_node(make_fixture("a", 1, 1))
    for k in range(2):
        assert p.schedule(group_wl(f"c{k}", "g", cu=50.0, mem=10.0))["ok"]
    saved = p.allocations()
    q = Platform({"enforceBudgets": False})
    q.add_fake_node(make_fixture("a", 1, 1))
    for a in saved:
        assert q.restore_allocation(a)
    d = q.schedule(group_wl("c2", "g", cu=50.0, mem=10.0))
    assert d["ok"] and not d["share_leader"] and d["share_leader_uid"] == "c0"
