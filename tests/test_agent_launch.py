"""Node agent (fixture backend, push to controller, exporter), the container
launcher, and the GPU-side probes / RCCL sweep (gpu-marked)."""
import http.client
import json
import os

import pytest

from kgwe.agent.agent import DEFAULTS, NodeAgent
from kgwe.core import Platform, make_fixture
from kgwe.extender.server import ExtenderServer
from kgwe.launch import parse_downward_api, placement_env
from kgwe.utils.config import load_config


def test_agent_fixture_push_and_metrics(tmp_path):
    fx = tmp_path / "node.json"
    fx.write_text(json.dumps(make_fixture("whatever", 8, 2)))
    plat = Platform({})

    def push(path, body):
        node = json.loads(body)
        node["name"] = path.rstrip("/").split("/")[-2]
        plat.upsert_node(node)
        return 200, b"{}"
    ext = ExtenderServer(plat, host="127.0.0.1", port=0, routes={"/v1/nodes/": push}).start()
    cfg = load_config(DEFAULTS, sets=["nodeName=gpu-node-7", f"fixture={fx}", f"controllerUrl={ext.url}",
                                      "listen.host=127.0.0.1", "listen.port=0"])
    agent = NodeAgent(cfg)
    # measured-probe merge: GPU 3 HBM at 50 % of the median -> Degraded
    agent.probe_results = {"hbm": {i: {"copy_gbps": 6000.0 if i != 3 else 3000.0} for i in range(8)},
                           "xgmi": [[0 if s == d else 150.0 for s in range(8)] for d in range(8)]}
    node = agent.discover()
    assert node["name"] == "gpu-node-7"
    assert node["gpus"][3]["health"]["status"] == "Degraded"
    assert node["gpus"][0]["links"][0]["measured_gbps"] == 150.0
    assert agent.push()
    assert plat.node("gpu-node-7")["gpus"][3]["health"]["status"] == "Degraded"
    srv = agent.serve()
    h, p = srv.server_address[:2]
    c = http.client.HTTPConnection(h, p)
    c.request("GET", "/metrics")
    text = c.getresponse().read().decode()
    assert 'kgwe_gpu_health_status{gpu_uuid="GPU-whatever-03",node="gpu-node-7"} 0.5' in text
    assert 'kgwe_gpu_hbm_bandwidth_gbps' in text
    c.request("POST", "/v1/partition", body=json.dumps({"gpu": "GPU-whatever-00", "compute": "CPX"}))
    r = json.loads(c.getresponse().read())
    assert r["dryRun"] is True
    srv.shutdown()
    ext.stop()


def test_launch_env_from_downward_api():
    env = {"HIP_VISIBLE_DEVICES": "0,1", "WORLD_SIZE": "2"}
    text = ('kgwe.amd.com/node="n1"\n'
            f'kgwe.amd.com/rccl-env={json.dumps(json.dumps(env))}\n')
    ann = parse_downward_api(text)
    assert ann["kgwe.amd.com/node"] == "n1"
    assert placement_env(ann) == env


@pytest.mark.gpu
def test_agent_probes_on_gpu():
    cfg = load_config(DEFAULTS, sets=["probe.bytesMB=512", "probe.iters=3"])
    agent = NodeAgent(cfg)
    res = agent.run_probes()
    assert res["devices"] >= 1
    assert res["hbm"][0]["copy_gbps"] > 2000


@pytest.mark.gpu
def test_rccl_native_sweep_single_gpu():
    from kgwe.parallel.busbw import native_sweep

    r = native_sweep(1, sizes=[1 << 20, 1 << 24], iters=5)
    assert r["ndev"] == 1 and len(r["rows"]) == 2
    assert all(row["us"] > 0 for row in r["rows"])


def test_probe_degradation_survives_push_to_controller():
    """A GPU the agent's HBM probe marks slow stays Degraded when the
    controller re-derives health from the pushed signals."""
    from kgwe.core import Platform, make_fixture

    src = Platform({})
    src.add_fake_node(make_fixture("a", 8, 2))
    node = src.node("a")
    node["gpus"][3]["health"].update(perf_degraded=True, perf_reason="HBM copy 3000 GB/s < 70% of median")
    ctl = Platform({})
    ctl.upsert_node(node)
    h = ctl.node("a")["gpus"][3]["health"]
    assert h["status"] == "Degraded" and any("HBM copy" in r for r in h["reasons"])


def test_agent_grpc_service(tmp_path):
    from kgwe.agent.grpc_service import AgentClient

    fx = tmp_path / "node.json"
    fx.write_text(json.dumps(make_fixture("n", 8, 2)))
    cfg = load_config(DEFAULTS, sets=["nodeName=grpc-node", f"fixture={fx}", "listen.host=127.0.0.1",
                                      "grpc.port=0"])
    agent = NodeAgent(cfg)
    agent.discover()
    server = agent.serve_grpc()
    c = AgentClient(f"127.0.0.1:{agent.grpc_port}")
    try:
        topo = c.call("GetTopology")
        assert topo["node"] == "grpc-node" and len(topo["topology"]["gpus"]) == 8
        tel = c.call("GetTelemetry")
        assert len(tel["gpus"]) == 8 and tel["gpus"][0]["health"] == "Healthy"
        assert c.call("SetPartition", {"gpu": tel["gpus"][0]["uuid"], "compute": "CPX"})["dryRun"] is True
        assert "error" in c.call("SetPartition", {})
        assert c.call("GetProbes")["probes"] == {}
        # real actuation: refused without a configured token, and with a wrong one
        g = tel["gpus"][0]["uuid"]
        agent.cfg["partition"]["dryRun"] = False
        r = c.call("SetPartition", {"gpu": g, "compute": "CPX"})
        assert r.get("denied") and "authTokenFile" in r["error"]
        tok = tmp_path / "token"
        tok.write_text("s3cret\n")
        agent.cfg["partition"]["authTokenFile"] = str(tok)
        assert c.call("SetPartition", {"gpu": g, "compute": "CPX"}, token="wrong")["error"] == "unauthorized"
        assert c.call("SetPartition", {"gpu": g, "compute": "CPX"})["error"] == "unauthorized"
        # the right token gets past auth (actuation itself fails here: no amd-smi on this host)
        r = c.call("SetPartition", {"gpu": g, "compute": "CPX"}, token="s3cret")
        assert not r.get("denied")
    finally:
        c.close()
        server.stop(0)


def test_agent_http_partition_requires_bearer_token(tmp_path):
    import urllib.error
    import urllib.request

    fx = tmp_path / "node.json"
    fx.write_text(json.dumps(make_fixture("n", 8, 2)))
    tok = tmp_path / "token"
    tok.write_text("abc")
    cfg = load_config(DEFAULTS, sets=["nodeName=h", f"fixture={fx}", "listen.host=127.0.0.1", "listen.port=0",
                                      "partition.dryRun=false", f"partition.authTokenFile={tok}"])
    agent = NodeAgent(cfg)
    srv = agent.serve()
    url = f"http://127.0.0.1:{srv.server_address[1]}/v1/partition"

    def post(headers):
        req = urllib.request.Request(url, data=json.dumps({"gpu": "GPU-n-00", "compute": "CPX"}).encode(),
                                     headers={"Content-Type": "application/json", **headers})
        try:
            with urllib.request.urlopen(req, timeout=5) as r:
                return r.status
        except urllib.error.HTTPError as e:
            return e.code

    try:
        assert post({}) == 403
        assert post({"Authorization": "Bearer nope"}) == 403
        assert post({"Authorization": "Bearer abc"}) in (200, 409)  # past auth
    finally:
        srv.shutdown()


def test_controller_actuates_pushed_node_partitions_through_the_agent(tmp_path):
    """A partition switch on an agent-pushed node goes through the agent's
    authenticated SetPartition (no HAL in the controller), and the pushed
    topology follows the switch."""
    import urllib.request

    from kgwe.controller.main import DEFAULTS as CDEF
    from kgwe.controller.main import build

    tok = tmp_path / "token"
    tok.write_text("tkn")
    fx = tmp_path / "node.json"
    fx.write_text(json.dumps(make_fixture("edge", 8, 2)))
    acfg = load_config(DEFAULTS, sets=["nodeName=edge", f"fixture={fx}", "listen.host=127.0.0.1",
                                       "grpc.port=0", "partition.dryRun=true",
                                       f"partition.authTokenFile={tok}"])
    agent = NodeAgent(acfg)
    agent.discover()
    gsrv = agent.serve_grpc()
    calls = []
    real = agent.set_partition

    def spy(body, token=""):
        calls.append((body, token))
        return real(body, token)
    agent.set_partition = spy
    ccfg = load_config(CDEF, sets=["listen.host=127.0.0.1", "listen.port=0",
                                   f"agentActuation.tokenFile={tok}", "autoProvisionPartitions=true"])
    plat, ext, _ = build(ccfg)
    ext.start()
    try:
        body = dict(agent.topology)
        body["agent_endpoint"] = f"127.0.0.1:{agent.grpc_port}"
        url = f"{ext.url}/v1/nodes/edge/topology"
        # a push without the token is refused outright: it could redirect the token-bearing
        # SetPartition call to an endpoint of its choosing
        rogue = dict(body, agent_endpoint="203.0.113.9:50052")
        with pytest.raises(urllib.error.HTTPError) as ei:
            urllib.request.urlopen(urllib.request.Request(
                url, data=json.dumps(rogue).encode(), headers={"Content-Type": "application/json"}), timeout=5)
        assert ei.value.code == 401
        with pytest.raises(urllib.error.HTTPError):
            urllib.request.urlopen(urllib.request.Request(
                url, data=json.dumps(rogue).encode(),
                headers={"Content-Type": "application/json", "Authorization": "Bearer wrong"}), timeout=5)
        assert plat.node("edge") is None
        req = urllib.request.Request(url, data=json.dumps(body).encode(),
                                     headers={"Content-Type": "application/json", "Authorization": "Bearer tkn"})
        assert urllib.request.urlopen(req, timeout=5).status == 200
        d = plat.schedule({"uid": "slice", "workloadType": "Inference",
                           "gpuRequirements": {"count": 0, "partition": {"mode": "CPX", "count": 1}}})
        assert d["ok"], d
        assert calls and calls[0][1] == "tkn" and calls[0][0]["compute"] == "CPX"
        g = d["partitions"][0].rsplit("/p", 1)[0]
        gpu = {x["uuid"]: x for x in plat.node("edge")["gpus"]}[g]
        assert gpu["partition"]["compute"] == "CPX" and len(gpu["partition"]["instances"]) == 8
    finally:
        ext.stop()
        gsrv.stop(0)


def test_advertised_endpoint_must_be_an_address_of_the_node_object(tmp_path):
    """With an apiserver the controller pins an agent's endpoint to the Node
    object's own addresses: an authenticated push naming another host keeps
    its topology but not its endpoint."""
    import urllib.request

    from kgwe.controller.apiserver import FakeApiServer
    from kgwe.controller.kube import KubeClient
    from kgwe.controller.main import DEFAULTS as CDEF
    from kgwe.controller.main import build

    tok = tmp_path / "token"
    tok.write_text("tkn")
    api = FakeApiServer().start()
    try:
        KubeClient(api.url).create_node({
            "apiVersion": "v1", "kind": "Node", "metadata": {"name": "edge"},
            "status": {"addresses": [{"type": "InternalIP", "address": "10.0.0.5"},
                                     {"type": "Hostname", "address": "edge"}]}})
        ccfg = load_config(CDEF, sets=["listen.host=127.0.0.1", "listen.port=0", f"kube.url={api.url}",
                                       f"agentActuation.tokenFile={tok}", "labelNodes=false"])
        plat, ext, _ = build(ccfg)
        ext.start()
        try:
            def push(endpoint):
                body = dict(make_fixture("edge", 8, 2), agent_endpoint=endpoint)
                req = urllib.request.Request(
                    f"{ext.url}/v1/nodes/edge/topology", data=json.dumps(body).encode(),
                    headers={"Content-Type": "application/json", "Authorization": "Bearer tkn"})
                return json.loads(urllib.request.urlopen(req, timeout=5).read())

            r = push("203.0.113.9:50052")
            assert r["ok"] and "not an address of Node edge" in r["endpointIgnored"]
            assert plat.node("edge") is not None
            assert push("10.0.0.5:50052") == {"ok": True}
            assert push("edge:50052") == {"ok": True}
        finally:
            ext.stop()
    finally:
        api.stop()


def test_launcher_installs_the_hbm_cap_hook_for_shares_only(tmp_path):
    """A placement with an HBM cap makes every Python process of the workload
    load kgwe/_sitehook first; the hook arms itself on `import torch` and does
    nothing before.  No cap in the placement: PYTHONPATH is left alone."""
    import subprocess
    import sys

    from kgwe import launch

    env = launch.enforce_share_limits({"KGWE_GPU_MEMORY_FRACTION": "0.25", "PYTHONPATH": "/x"})
    assert env["PYTHONPATH"].split(os.pathsep) == [launch.SITEHOOK, "/x"]
    assert "PYTHONPATH" not in launch.enforce_share_limits({"KGWE_GPU_MEMORY_FRACTION": "0"})
    assert "PYTHONPATH" not in launch.enforce_share_limits({})
    ann = tmp_path / "annotations"
    ann.write_text('kgwe.amd.com/rccl-env=' + json.dumps(json.dumps({"KGWE_GPU_MEMORY_FRACTION": "0.25"})) + "\n")
    code = ("import os, sys; print('pre', os.environ.get('KGWE_GPU_MEMORY_CAP_INSTALLED'), 'torch' in sys.modules); "
            "import torch; print('post', os.environ.get('KGWE_GPU_MEMORY_CAP_INSTALLED'))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "kgwe.launch", "--", sys.executable, "-c", code], cwd=root,
                       env=dict(os.environ, KGWE_ANNOTATIONS_FILE=str(ann)), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-800:]
    assert "pre None False" in r.stdout and "post 1" in r.stdout
