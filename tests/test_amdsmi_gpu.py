"""Real amd-smi through the C++ AmdSmiHal on an MI355X (real
discovery + telemetry sampler): device identity, HBM size, partition
modes, RAS / xGMI / throttle health signals and the health policy, the
scheduler running on the discovered node, and gfx_activity under load."""
from __future__ import annotations

import pytest
import torch


@pytest.mark.gpu
def test_amdsmi_discovery_and_health_signals():
    from kgwe.core import Platform, amdsmi_discover

    d = amdsmi_discover("box")
    assert d.get("ok"), d
    node = d["node"]
    assert node["name"] == "box" and len(node["gpus"]) >= 1
    for g in node["gpus"]:
        assert g["uuid"] and g["pcie"]["bdf"]
        assert 250 <= g["memory_total_gb"] <= 300, g["memory_total_gb"]  # 288 GB HBM3E
        assert g["partition"]["compute"] in ("SPX", "DPX", "QPX", "CPX")
        assert g["partition"]["memory"] in ("NPS1", "NPS2")
        h = g["health"]
        for k in ("ecc_correctable", "ecc_uncorrectable", "ecc_deferred", "retired_pages",
                  "pending_retired_pages", "xgmi_errors", "xgmi_links_down", "throttle",
                  "cper_fatal", "cper_uncorrected", "cper_corrected"):
            assert k in h, k
        assert h["status"] in ("Healthy", "Degraded", "Unhealthy")
        for k in ("ecc_correctable", "ecc_uncorrectable", "ecc_deferred", "retired_pages"):
            assert 0 <= h[k] < 2**40, (k, h[k])  # real counts, never uninitialised memory
        assert (h["status"] == "Unhealthy") == (h["ecc_uncorrectable"] > 0 or h["retired_pages"] >= 64
                                                or h["cper_fatal"] > 0)
    # the scheduler places onto the real node
    p = Platform({})
    p.upsert_node(node)
    healthy = [g for g in node["gpus"] if g["health"]["status"] == "Healthy"]
    dec = p.schedule({"metadata": {"name": "one", "uid": "one"}, "spec": {"gpuRequirements": {"count": 1}}})
    assert dec["ok"] == bool(healthy)


@pytest.mark.gpu
def test_gfx_activity_sampler_sees_load():
    """amd-smi gfx_activity is a smoothed busy %: it ramps over a few hundred
    ms (over a second on some hosts), so the check is on the loaded last
    third of a ~3 s GEMM loop."""
    import time

    from kgwe.utils.amdsmi_util import UtilSampler, available

    assert available()
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    (a @ a).sum().item()  # library init / first-kernel costs outside the window
    s = UtilSampler(0, interval_s=0.02).start()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 3.0:
        for _ in range(20):
            a = a @ a
            a = a / a.abs().amax().clamp_min(1e-3)
        torch.cuda.synchronize()
    s.stop()
    vals = [v for _, v in s.samples]
    assert len(vals) >= 20
    tail = vals[2 * len(vals) // 3:]
    assert max(vals) > 80.0 and sum(tail) / len(tail) > 60.0, vals
