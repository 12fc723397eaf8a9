"""The native extender HTTP server (native/core/http_server.cpp) and the
Permit semantics it gives gangs: wire behaviour (keep-alive, large and
chunked bodies, Expect: 100-continue, concurrent clients, fallback routes),
held gang binds completing with the last member, gang time-out releasing every
reservation, the preempt verb naming only victims on the node itself."""
import http.client
import json
import socket
import threading
import time

import pytest

from kgwe.controller.apiserver import FakeApiServer
from kgwe.controller.kube import KubeClient
from kgwe.controller.schedsim import SCHEDULER_NAME, SchedulerSim
from kgwe.core import Platform, make_fixture
from kgwe.extender.server import ExtenderServer


def _pod(name, gpus=1, uid=None, ann=None, priority=0):
    a = {"kgwe.amd.com/topology": "xGMIOptimal" if gpus > 1 else "None"}
    a.update(ann or {})
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": "t", "uid": uid or f"uid-{name}", "annotations": a},
            "spec": {"schedulerName": SCHEDULER_NAME, "priority": priority,
                     "containers": [{"name": "c", "image": "x",
                                     "resources": {"limits": {"amd.com/gpu": str(gpus)}}}]}}


def _post(conn, path, obj):
    data = obj if isinstance(obj, (bytes, bytearray)) else json.dumps(obj).encode()
    conn.request("POST", path, body=data, headers={"Content-Type": "application/json"})
    r = conn.getresponse()
    return r.status, json.loads(r.read() or b"null")


@pytest.fixture
def served():
    plat = Platform({})
    for i in range(4):
        plat.add_fake_node(make_fixture(f"n{i}", 8, 2))
    seen = []

    def route(path, body):
        seen.append((path, body))
        return 200, b'{"routed":true}'

    ext = ExtenderServer(plat, host="127.0.0.1", port=0, routes={"/v1/nodes/": route}).start()
    yield plat, ext, seen
    ext.stop()


def test_verbs_keepalive_and_native_routes(served):
    plat, ext, seen = served
    h, p = ext.address
    c = http.client.HTTPConnection(h, p)
    names = [f"n{i}" for i in range(4)] + ["stranger"]
    for k in range(3):  # one connection, several cycles
        pod = _pod(f"p{k}", 2)
        st, f = _post(c, "/filter", {"pod": pod, "nodenames": names})
        assert st == 200 and sorted(f["nodenames"]) == ["n0", "n1", "n2", "n3"]
        assert "stranger" in f["failedNodes"]
        st, pr = _post(c, "/prioritize", {"pod": pod, "nodenames": f["nodenames"]})
        assert [x["host"] for x in pr] == f["nodenames"] and all(0 <= x["score"] <= 10 for x in pr)
        st, b = _post(c, "/bind", {"podName": f"p{k}", "podNamespace": "t", "podUID": f"uid-p{k}",
                                   "node": "n1"})
        assert st == 200 and not b.get("error"), b
    assert plat.scheduler_metrics()["allocated_gpus"] == 6
    c.request("GET", "/healthz")
    r = c.getresponse()
    assert r.status == 200 and r.read() == b"ok"
    c.request("GET", "/metrics")
    r = c.getresponse()
    body = r.read().decode()
    assert r.status == 200 and "kgwe_scheduling_successes_total 3" in body
    assert r.getheader("Content-Type").startswith("text/plain")
    st, d = _post(c, "/v1/nodes/n9/topology", {"x": 1})  # Python route behind the native server
    assert st == 200 and d == {"routed": True} and seen[-1][0] == "/v1/nodes/n9/topology"
    c.request("GET", "/debug/scheduler")
    dbg = json.loads(c.getresponse().read())
    assert dbg["phases"]["filter"]["count"] == 3 and dbg["server"]["requests"] >= 9
    c.request("GET", "/nope")
    r = c.getresponse()
    r.read()
    assert r.status == 404
    st, d = _post(c, "/filter", b"{not json")
    assert st == 200 and "error" in d  # extender contract: errors travel in the body


def test_readyz_follows_the_ready_callable(served):
    plat, ext, _ = served
    h, p = ext.address
    state = {"leader": False}
    ext.ready = lambda: state["leader"]
    c = http.client.HTTPConnection(h, p)
    c.request("GET", "/readyz")
    r = c.getresponse()
    assert r.status == 503 and r.read() == b"standby"
    state["leader"] = True
    deadline = time.time() + 3
    while time.time() < deadline:
        c.request("GET", "/readyz")
        r = c.getresponse()
        r.read()
        if r.status == 200:
            break
        time.sleep(0.05)
    assert r.status == 200


def test_large_full_node_body_chunked_and_expect_continue(served):
    plat, ext, _ = served
    h, p = ext.address
    from kgwe.bench.sched_latency import full_node

    items = [full_node(f"n{i}", i) for i in range(4)] + [full_node(f"x{i}", 100 + i) for i in range(300)]
    pod = _pod("big", 4)
    body = json.dumps({"pod": pod, "nodes": {"items": items}}).encode()
    assert len(body) > 1_500_000
    c = http.client.HTTPConnection(h, p)
    st, f = _post(c, "/filter", body)  # Content-Length body, read in many recv()s
    got = [n["metadata"]["name"] for n in f["nodes"]["items"]]
    assert got == ["n0", "n1", "n2", "n3"] and len(f["failedNodes"]) == 300
    assert f["nodes"]["items"][0] == items[0]  # Node objects come back byte-for-byte

    def chunks():
        for i in range(0, len(body), 70_000):
            yield body[i:i + 70_000]

    c.request("POST", "/filter", body=chunks(), headers={"Transfer-Encoding": "chunked"},
              encode_chunked=True)
    f2 = json.loads(c.getresponse().read())
    assert [n["metadata"]["name"] for n in f2["nodes"]["items"]] == got

    s = socket.create_connection((h, p))
    small = json.dumps({"pod": pod, "nodenames": ["n0"]}).encode()
    s.sendall(b"POST /filter HTTP/1.1\r\nHost: x\r\nExpect: 100-continue\r\nContent-Length: "
              + str(len(small)).encode() + b"\r\n\r\n")
    assert s.recv(64).startswith(b"HTTP/1.1 100")
    s.sendall(small)
    data = b""
    while b"nodenames" not in data:
        data += s.recv(4096)
    assert b"200 OK" in data
    s.close()


def test_concurrent_clients_never_double_allocate(served):
    plat, ext, _ = served
    h, p = ext.address
    errs, oks = [], []

    def client(k):
        c = http.client.HTTPConnection(h, p)
        for j in range(8):
            name = f"c{k}-{j}"
            pod = _pod(name, 1)
            _, f = _post(c, "/filter", {"pod": pod, "nodenames": ["n0", "n1", "n2", "n3"]})
            if not f["nodenames"]:
                continue
            _, b = _post(c, "/bind", {"podName": name, "podNamespace": "t", "podUID": f"uid-{name}",
                                      "node": f["nodenames"][j % len(f["nodenames"])]})
            (errs if b.get("error") else oks).append(name)

    ts = [threading.Thread(target=client, args=(k,)) for k in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    allocs = plat.allocations()
    gpus = [g for a in allocs for g in a["gpus"]]
    assert len(gpus) == len(set(gpus)) == len(oks) <= 32
    assert len(oks) >= 30  # 64 one-GPU pods chase 32 GPUs


def _gang_pod(name, gang, size, gpus=1):
    return _pod(name, gpus, ann={"kgwe.amd.com/gang": gang, "kgwe.amd.com/gang-size": str(size)})


def test_gang_binds_are_held_until_the_last_member(served):
    plat, ext, _ = served
    h, p = ext.address
    size = 8
    results, t_done = {}, {}

    def member(i):
        c = http.client.HTTPConnection(h, p, timeout=30)
        name = f"g{i}"
        pod = _gang_pod(name, "ring", size)
        _, f = _post(c, "/filter", {"pod": pod, "nodenames": ["n0", "n1", "n2", "n3"]})
        _, b = _post(c, "/bind", {"podName": name, "podNamespace": "t", "podUID": f"uid-{name}",
                                  "node": f["nodenames"][0]})
        results[i], t_done[i] = b, time.perf_counter()

    ts = [threading.Thread(target=member, args=(i,)) for i in range(size - 1)]
    for t in ts:
        t.start()
    deadline = time.time() + 5
    while ext.stats()["parked"] < size - 1 and time.time() < deadline:
        time.sleep(0.01)
    assert ext.stats()["parked"] == size - 1 and not results  # held, not answered
    assert plat.scheduler_metrics()["allocated_gpus"] == size - 1  # reserved meanwhile (Reserve)
    t_last = time.perf_counter()
    member(size - 1)  # the last member completes the gang
    for t in ts:
        t.join(timeout=10)
    assert all(not results[i].get("error") for i in range(size)), results
    assert max(t_done.values()) - t_last < 0.085  # every held bind answered within the p99 bar
    st = ext.stats()
    assert st["parked"] == 0 and st["gang_binds_held"] == size - 1 and st["gang_binds_timed_out"] == 0
    assert plat.scheduler_metrics()["allocated_gpus"] == size
    assert plat.pod_latency_count() == size  # one latency sample per member, none doubled


def test_timed_out_gang_fails_held_binds_and_releases_everything():
    plat = Platform({"scheduler": {"gangTimeoutMs": 400}})
    plat.add_fake_node(make_fixture("n0", 8, 2))
    ext = ExtenderServer(plat, host="127.0.0.1", port=0).start()
    try:
        h, p = ext.address
        results = {}

        def member(i):
            c = http.client.HTTPConnection(h, p, timeout=30)
            name = f"g{i}"
            pod = _gang_pod(name, "never", 4, 2)
            _post(c, "/filter", {"pod": pod, "nodenames": ["n0"]})
            _, results[i] = _post(c, "/bind", {"podName": name, "podNamespace": "t",
                                               "podUID": f"uid-{name}", "node": "n0"})

        ts = [threading.Thread(target=member, args=(i,)) for i in range(2)]  # 2 of 4 ever arrive
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=10)
        dt = time.perf_counter() - t0
        assert 0.35 < dt < 3.0
        assert all("timed out" in r.get("error", "") for r in results.values()), results
        assert plat.scheduler_metrics()["allocated_gpus"] == 0 and not plat.allocations()
        assert ext.stats()["gang_binds_timed_out"] == 2
    finally:
        ext.stop()


def test_hold_limit_answers_retryable_error_and_keeps_the_reservation():
    plat = Platform({})
    plat.add_fake_node(make_fixture("n0", 8, 2))
    ext = ExtenderServer(plat, host="127.0.0.1", port=0, gang_hold_s=0.3).start()
    try:
        h, p = ext.address
        c = http.client.HTTPConnection(h, p, timeout=30)
        pod = _gang_pod("solo", "late", 2)
        _post(c, "/filter", {"pod": pod, "nodenames": ["n0"]})
        t0 = time.perf_counter()
        _, b = _post(c, "/bind", {"podName": "solo", "podNamespace": "t", "podUID": "uid-solo", "node": "n0"})
        assert 0.25 < time.perf_counter() - t0 < 2.0 and "waiting" in b["error"]
        assert plat.scheduler_metrics()["allocated_gpus"] == 1  # the gang timeout, not the hold, releases
        # the same connection still serves (the parked connection was re-armed)
        st, f = _post(c, "/filter", {"pod": pod, "nodenames": ["n0"]})
        assert st == 200 and f["nodenames"] == ["n0"]
    finally:
        ext.stop()


def test_gang_through_the_scheduler_stand_in_with_kube_backoff():
    """An 8-pod gang created over ~0.3 s: with kube-scheduler's 1 s -> 10 s pod
    backoff a "retry until complete" Permit would bind the gang seconds after
    its last member; held binds finish it within the p99 bar."""
    api = FakeApiServer().start()
    kube = KubeClient(api.url)
    plat = Platform({})
    for i in range(2):
        api.add_node(f"n{i}")
        plat.add_fake_node(make_fixture(f"n{i}", 8, 2))
    ext = ExtenderServer(plat, kube=kube, host="127.0.0.1", port=0).start()
    bound = {}
    sim = SchedulerSim(kube, ext.url, on_bound=lambda pod, node, t: bound.__setitem__(pod["metadata"]["name"], t),
                       node_cache_capable=True).start()
    try:
        assert sim.backoff0 == 1.0 and sim.backoff_max == 10.0  # kube-scheduler defaults
        time.sleep(0.3)
        created = {}
        for i in range(8):
            pod = _gang_pod(f"m{i}", "job", 8)
            del pod["metadata"]["uid"]
            created[f"m{i}"] = time.perf_counter()
            kube.create_pod(pod)
            time.sleep(0.04)
        deadline = time.time() + 10
        while len(bound) < 8 and time.time() < deadline:
            time.sleep(0.01)
        assert len(bound) == 8, (bound, sim.stats)
        last_created = max(created.values())
        assert max(bound.values()) - last_created < 0.085
        assert sim.stats["bind_errors"] == 0  # nobody was bounced into the backoff queue
        nodes = {kube.get_pod("t", f"m{i}")["spec"]["nodeName"] for i in range(8)}
        assert len(nodes) >= 1 and all(kube.get_pod("t", f"m{i}")["metadata"]["annotations"]
                                       ["kgwe.amd.com/allocated-gpus"] for i in range(8))
    finally:
        sim.stop()
        ext.stop()
        api.stop()


def test_preempt_verb_names_only_victims_on_the_node_and_hands_peers_to_release():
    plat = Platform({})
    for i in range(2):
        plat.add_fake_node(make_fixture(f"n{i}", 8, 2))
    members = [{"metadata": {"name": f"lo{i}", "uid": f"lo{i}"},
                "spec": {"gpuRequirements": {"count": 8}, "priority": 1, "preemptible": True,
                         "gang": {"name": "lowgang", "size": 2}}} for i in range(2)]
    ds = plat.schedule_gang(members)
    assert all(d["ok"] for d in ds) and {d["node"] for d in ds} == {"n0", "n1"}
    vip = _pod("vip", 8, priority=1000)
    res = json.loads(plat.preempt(json.dumps({"pod": vip, "nodeNameToMetaVictims": {
        "n0": {"pods": []}, "n1": {"pods": []}}})))
    on = {n: [p["uid"] for p in v["pods"]] for n, v in res["nodeNameToMetaVictims"].items()}
    by_node = {d["node"]: d["uid"] for d in ds}
    assert on == {"n0": [by_node["n0"]], "n1": [by_node["n1"]]}  # never a pod of another node
    # kube-scheduler evicts n0's victim; its release names the peer for the controller
    rel = plat.release(by_node["n0"])
    assert rel["evict_gang_peers"] == [by_node["n1"]]
    assert "evict_gang_peers" not in plat.release(by_node["n1"])


def test_standin_candidate_window_follows_the_profile_setting():
    """percentageOfNodesToScore: 100 hands every node to the extender; 0 is
    kube-scheduler's adaptive default (a rotating window of max(100, N * (50 -
    N / 125) %) nodes); an explicit value is taken as given."""
    from kgwe.controller.schedsim import SchedulerSim

    names = [f"n{i}" for i in range(1250)]
    every = SchedulerSim(None, "http://127.0.0.1:1", percentage_of_nodes_to_score=100)
    assert every._candidates(names) == names
    adaptive = SchedulerSim(None, "http://127.0.0.1:1")
    first, second = adaptive._candidates(names), adaptive._candidates(names)
    assert len(first) == 500 and first[0] == "n0" and second[0] == "n500"
    third = adaptive._candidates(names)  # wraps round the node list
    assert third[0] == "n1000" and third[-1] == "n249"
    ten = SchedulerSim(None, "http://127.0.0.1:1", percentage_of_nodes_to_score=10)
    assert len(ten._candidates(names)) == 125
    assert len(ten._candidates(names[:90])) == 90  # small fleets are never sampled
