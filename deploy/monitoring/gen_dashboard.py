"""Generate the KGWE MI355X Grafana dashboard.

Parity target: reference deploy/monitoring/grafana-dashboard.json (19 panels:
cluster overview stats, per-GPU utilisation/memory/temperature/power,
scheduling rate, topology score, NVLink bandwidth, cost by namespace, budget
gauge).  Here every query names a family declared by the native metric
registry (native/core/metrics.cpp, declare_kgwe_families); the NVLink panel
becomes xGMI per-link bandwidth, MIG becomes compute-partition instances, and
MI355X-specific panels are added (HBM/UMC activity, link status, partition
reconfigurations, preemptions).  tests/test_deploy.py checks every metric
referenced here is exported.

    python deploy/monitoring/gen_dashboard.py   # rewrites both JSON copies
"""
from __future__ import annotations

import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUTPUTS = [os.path.join(HERE, "grafana-dashboard.json"),
           os.path.join(HERE, "..", "helm", "kgwe-mi355x", "dashboards", "kgwe-mi355x.json")]

_id = [0]


def _next_id() -> int:
    _id[0] += 1
    return _id[0]


def row(title: str, y: int) -> dict:
    return {"type": "row", "title": title, "id": _next_id(), "collapsed": False,
            "gridPos": {"h": 1, "w": 24, "x": 0, "y": y}, "panels": []}


def panel(kind: str, title: str, exprs: list[tuple[str, str]], x: int, y: int, w: int, h: int,
          unit: str = "short", thresholds: list[tuple[str, float | None]] | None = None,
          max_: float | None = None) -> dict:
    steps = [{"color": c, "value": v} for c, v in (thresholds or [("green", None)])]
    defaults = {"unit": unit, "thresholds": {"mode": "absolute", "steps": steps}}
    if max_ is not None:
        defaults["max"] = max_
    return {
        "type": kind, "title": title, "id": _next_id(),
        "datasource": {"type": "prometheus", "uid": "${datasource}"},
        "gridPos": {"h": h, "w": w, "x": x, "y": y},
        "fieldConfig": {"defaults": defaults, "overrides": []},
        "options": {"legend": {"displayMode": "table", "placement": "bottom"}} if kind == "timeseries"
        else {"reduceOptions": {"calcs": ["lastNotNull"]}},
        "targets": [{"refId": chr(ord("A") + i), "expr": e, "legendFormat": lf}
                    for i, (e, lf) in enumerate(exprs)],
    }


def build() -> dict:
    _id[0] = 0
    P = []
    y = 0
    P.append(row("Cluster overview", y)); y += 1
    stats = [
        ("Total GPUs", "sum(kgwe_gpu_count)", "short", None),
        ("Avg GPU gfx activity", "avg(kgwe_gpu_gfx_activity_percent)", "percent",
         [("red", None), ("yellow", 50), ("green", 87)]),
        ("Active workloads", "sum(kgwe_active_workloads)", "short", None),
        ("Scheduling latency p99",
         "histogram_quantile(0.99, sum(rate(kgwe_scheduling_latency_ms_bucket[5m])) by (le))", "ms",
         [("green", None), ("yellow", 50), ("red", 85)]),
        ("Cost / hour", "sum(kgwe_gpu_cost_per_hour_dollars)", "currencyUSD", None),
        ("Partition instances", "sum(kgwe_partition_instance_count)", "short", None),
    ]
    for i, (t, e, u, th) in enumerate(stats):
        P.append(panel("stat", t, [(e, "")], 4 * i, y, 4, 4, u, th))
    y += 4
    P.append(row("MI355X devices", y)); y += 1
    P.append(panel("timeseries", "gfx activity by GPU",
                   [("kgwe_gpu_gfx_activity_percent", "{{node}}/{{gpu_uuid}}")], 0, y, 12, 8, "percent",
                   max_=100))
    P.append(panel("timeseries", "HBM (UMC) activity by GPU",
                   [("kgwe_gpu_umc_activity_percent", "{{node}}/{{gpu_uuid}}")], 12, y, 12, 8, "percent",
                   max_=100))
    y += 8
    P.append(panel("timeseries", "HBM3E used",
                   [("kgwe_gpu_memory_used_bytes", "{{node}}/{{gpu_uuid}}"),
                    ("kgwe_gpu_memory_total_bytes", "capacity {{node}}/{{gpu_uuid}}")], 0, y, 8, 8, "bytes"))
    P.append(panel("timeseries", "Junction temperature",
                   [("kgwe_gpu_temperature_celsius", "{{node}}/{{gpu_uuid}}")], 8, y, 8, 8, "celsius"))
    P.append(panel("timeseries", "Socket power",
                   [("kgwe_gpu_power_watts", "{{node}}/{{gpu_uuid}}")], 16, y, 8, 8, "watt"))
    y += 8
    P.append(row("Scheduling & xGMI topology", y)); y += 1
    P.append(panel("timeseries", "Scheduling rate",
                   [("sum(rate(kgwe_scheduling_successes_total[5m]))", "bound/s"),
                    ("sum(rate(kgwe_scheduling_failures_total[5m]))", "failed/s"),
                    ("sum(rate(kgwe_preemptions_total[5m]))", "preemptions/s")], 0, y, 8, 8, "ops"))
    P.append(panel("timeseries", "Scheduling latency quantiles",
                   [("histogram_quantile(0.5, sum(rate(kgwe_scheduling_latency_ms_bucket[5m])) by (le))", "p50"),
                    ("histogram_quantile(0.99, sum(rate(kgwe_scheduling_latency_ms_bucket[5m])) by (le))",
                     "p99")], 8, y, 8, 8, "ms"))
    P.append(panel("piechart", "Topology score by node",
                   [("avg(kgwe_topology_score) by (node)", "{{node}}")], 16, y, 8, 8))
    y += 8
    P.append(panel("timeseries", "xGMI link bandwidth (measured)",
                   [("kgwe_xgmi_bandwidth_gbps", "{{node}} {{gpu_uuid_1}}->{{gpu_uuid_2}}")], 0, y, 12, 8,
                   "GBs"))
    P.append(panel("stat", "xGMI links down",
                   [("count(kgwe_xgmi_link_status == 0) or vector(0)", "")], 12, y, 4, 8, "short",
                   [("green", None), ("red", 1)]))
    P.append(panel("timeseries", "Partition reconfigurations",
                   [("sum(increase(kgwe_partition_reconfigurations_total[1h])) by (result)", "{{result}}")],
                   16, y, 8, 8))
    y += 8
    P.append(row("Health & partitions", y)); y += 1
    P.append(panel("stat", "Unhealthy / degraded GPUs",
                   [("count(kgwe_gpu_health_status < 1) or vector(0)", "")], 0, y, 4, 8, "short",
                   [("green", None), ("red", 1)]))
    P.append(panel("timeseries", "ECC errors",
                   [("sum(kgwe_gpu_ecc_errors_total) by (node, type)", "{{node}} {{type}}")], 4, y, 7, 8))
    P.append(panel("timeseries", "Retired HBM pages",
                   [("sum(kgwe_gpu_retired_pages) by (node, state)", "{{node}} {{state}}")], 11, y, 7, 8))
    P.append(panel("timeseries", "Partition slice utilization",
                   [("kgwe_partition_instance_utilization_percent", "{{node}} {{mode}}")], 18, y, 6, 8,
                   "percent", max_=100))
    y += 8
    P.append(panel("timeseries", "Active throttling",
                   [("sum(kgwe_gpu_throttle_active) by (reason)", "{{reason}}")], 0, y, 12, 8))
    P.append(panel("stat", "GPUs with xGMI errors",
                   [("count(kgwe_gpu_xgmi_errors > 0) or vector(0)", "")], 12, y, 4, 8, "short",
                   [("green", None), ("red", 1)]))
    P.append(panel("stat", "Partition ops failed (1h)",
                   [("sum(increase(kgwe_partition_reconfigurations_total{result=\"failed\"}[1h])) or vector(0)",
                     "")], 16, y, 8, 8, "short", [("green", None), ("red", 1)]))
    y += 8
    P.append(row("Cost & budget", y)); y += 1
    P.append(panel("timeseries", "GPU cost by namespace (hourly)",
                   [("sum(kgwe_gpu_cost_per_hour_dollars) by (namespace)", "{{namespace}}")], 0, y, 12, 8,
                   "currencyUSD"))
    P.append(panel("gauge", "Budget utilization",
                   [("kgwe_budget_utilization_percent", "{{budget_id}}")], 12, y, 6, 8, "percent",
                   [("green", None), ("yellow", 75), ("red", 90)], max_=100))
    P.append(panel("stat", "Recommended savings",
                   [("sum(kgwe_cost_savings_recommended_dollars)", "")], 18, y, 6, 8, "currencyUSD"))
    return {
        "title": "KGWE - MI355X GPU Workload Enhancer",
        "uid": "kgwe-mi355x",
        "schemaVersion": 39,
        "version": 1,
        "tags": ["kgwe", "mi355x", "gpu"],
        "time": {"from": "now-6h", "to": "now"},
        "refresh": "30s",
        "templating": {"list": [{"name": "datasource", "type": "datasource", "query": "prometheus"}]},
        "panels": P,
    }


def main() -> None:
    text = json.dumps(build(), indent=2) + "\n"
    for out in OUTPUTS:
        os.makedirs(os.path.dirname(out), exist_ok=True)
        with open(out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
