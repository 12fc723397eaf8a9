"""Python face of the C++17 control-plane core (``_kgwe_core`` pybind11 module).

The native module MUST be built (``python -m kgwe._build``); there is no
pure-Python scheduler behind it.  JSON text crosses the boundary both ways;
this wrapper turns it into dicts.
"""
from __future__ import annotations

import importlib.util
import json
import sys
import time
from pathlib import Path
from typing import Any

_LIB = Path(__file__).resolve().parent.parent / "_lib"


def _load_native():
    for p in _LIB.glob("_kgwe_core*.so"):
        spec = importlib.util.spec_from_file_location("_kgwe_core", p)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        sys.modules["_kgwe_core"] = mod
        return mod
    raise ImportError(f"_kgwe_core not built in {_LIB}; run `python -m kgwe._build`")


native = _load_native()
LatencyHistogram = native.LatencyHistogram


def make_fixture(name: str, n_gpus: int = 8, numa_nodes: int = 2, prefix: str = "") -> dict:
    return json.loads(native.make_fixture(name, n_gpus, numa_nodes, prefix))


def amdsmi_discover(node: str = "local") -> dict:
    return json.loads(native.amdsmi_discover(node))


def workload_from_pod(pod: dict) -> dict:
    return json.loads(native.workload_from_pod(json.dumps(pod)))


def _j(s: str) -> Any:
    return json.loads(s)


class Platform:
    """Discovery + scheduler + partition controller + sharing + cost + metrics."""

    def __init__(self, config: dict | None = None):
        self._p = native.Platform(json.dumps(config or {}))

    @property
    def raw(self):
        return self._p

    # topology ---------------------------------------------------------------
    def add_fake_node(self, fixture: dict) -> str:
        return self._p.add_fake_node(json.dumps(fixture))

    def add_amdsmi_node(self, name: str) -> str:
        return self._p.add_amdsmi_node(name)

    def upsert_node(self, node: dict) -> None:
        self._p.upsert_node(json.dumps(node))

    def set_cordon(self, name: str, on: bool = True) -> None:
        self._p.set_cordon(name, on)

    def cordoned(self) -> list:
        return list(self._p.cordoned())

    def remove_node(self, name: str) -> None:
        self._p.remove_node(name)

    def refresh(self) -> None:
        self._p.refresh()

    def refresh_telemetry(self) -> None:
        self._p.refresh_telemetry()

    def snapshot(self) -> dict:
        return _j(self._p.snapshot_json())

    def node(self, name: str) -> dict | None:
        return _j(self._p.node_json(name))

    def topology_events(self) -> list:
        return _j(self._p.topology_events_json())

    def hints(self, count: int, min_memory_gb: float = 0.0, arch: str = "") -> list:
        return _j(self._p.hints_json(count, min_memory_gb, arch))

    # fault injection (fake nodes) --------------------------------------------
    def fake_set_link_up(self, node, a, b, up): self._p.fake_set_link_up(node, a, b, up)
    def fake_set_health(self, node, gpu, status, reason=""): self._p.fake_set_health(node, gpu, status, reason)
    def fake_set_health_signals(self, node, gpu, signals: dict):
        self._p.fake_set_health_signals(node, gpu, json.dumps(signals))

    def fake_set_util(self, node, gpu, gfx, mem_gb=0.0): self._p.fake_set_util(node, gpu, gfx, mem_gb)
    def fake_set_measured_link(self, node, a, b, gbps): self._p.fake_set_measured_link(node, a, b, gbps)
    def fake_partition_switches(self, node): return self._p.fake_partition_switches(node)

    # extender verbs (JSON text in/out: the HTTP shell passes bodies through) --
    def filter(self, body: str) -> str:
        return self._p.filter(body)

    def prioritize(self, body: str) -> str:
        return self._p.prioritize(body)

    def preempt(self, body: str) -> str:
        """ExtenderPreemptionArgs -> ExtenderPreemptionResult."""
        return self._p.preempt(body)

    def count_preemptions(self, n: int) -> None:
        """Victims actually evicted after a preempt verb (kgwe_preemptions_total)."""
        self._p.count_preemptions(n)

    def filter_bytes(self, body: bytes) -> bytes:
        """filter() without UTF-8 decode/encode of the (multi-MB) bodies."""
        return self._p.filter_bytes(body)

    def prioritize_bytes(self, body: bytes) -> bytes:
        return self._p.prioritize_bytes(body)

    def bind(self, body: str, pod: dict | None = None) -> dict:
        return _j(self._p.bind(body, json.dumps(pod) if pod else ""))

    def observe_pod_latency_ms(self, ms: float) -> None:
        self._p.observe_pod_latency_ms(ms)

    # scheduler -----------------------------------------------------------------
    def schedule(self, workload: dict) -> dict:
        return _j(self._p.schedule(json.dumps(workload)))

    def schedule_gang(self, workloads: list[dict]) -> list[dict]:
        return _j(self._p.schedule_gang(json.dumps(workloads)))

    def release(self, uid: str, now: float | None = None) -> dict:
        return _j(self._p.release(uid, time.time() if now is None else now))

    def permit(self, uid: str) -> str:
        return self._p.permit(uid)

    def restore_allocation(self, alloc: dict) -> bool:
        return self._p.restore_allocation(json.dumps(alloc))

    def allocations(self) -> list:
        return _j(self._p.allocations_json())

    def scheduler_metrics(self) -> dict:
        return _j(self._p.scheduler_metrics_json())

    def scheduler_events(self) -> list:
        return _j(self._p.scheduler_events_json())

    def score_node(self, node: str, workload: dict) -> dict:
        return _j(self._p.score_node_json(node, json.dumps(workload)))

    # partitions ---------------------------------------------------------------
    def register_strategy(self, strategy: dict) -> str:
        return self._p.register_strategy(json.dumps(strategy))

    def strategies(self) -> list:
        return _j(self._p.strategies_json())

    def ensure_partitions(self, mode: str, count: int, plan_only: bool = False, memory: str = "") -> list:
        return _j(self._p.ensure_partitions(mode, count, plan_only, memory))

    def rebalance(self, name: str, plan_only: bool = False) -> list:
        return _j(self._p.rebalance(name, plan_only))

    def reclaim_idle_partitions(self, plan_only: bool = False) -> list:
        return _j(self._p.reclaim_idle_partitions(plan_only))

    def reclaim_idle_after(self, now: float, min_idle_s: float) -> list:
        """Partitioned GPUs idle for >= min_idle_s go back to SPX (the tick's
        hysteresis reclaim, with an explicit clock — simulations)."""
        return _j(self._p.reclaim_idle_after(now, min_idle_s))

    def set_partition_actuator(self, fn) -> None:
        """fn(node, gpu, compute, memory) -> "" | error: how partition switches
        reach agent-pushed nodes (the controller's authenticated call to the
        node agent's SetPartition)."""
        self._p.set_partition_actuator(fn)

    def consolidate_partitions(self, now: float | None = None, plan_only: bool = True) -> list:
        """Consolidating rebalance of partitioned GPUs: list of slice moves
        {uid, from, to, node_from, node_to}.  plan_only=True (controller): the
        caller evicts the moved pods; False: the ledger moves them itself."""
        return _j(self._p.consolidate_partitions(time.time() if now is None else now, plan_only))

    def draining_gpus(self) -> list:
        """Consolidation donors that take no new slice work until they are
        empty and switched back to SPX."""
        return list(self._p.draining_gpus())

    def pod_latency_quantile_ms(self, q: float) -> float:
        """Pod create -> bind latency quantile recorded by bind() itself."""
        return self._p.pod_latency_quantile_ms(q)

    def pod_latency_count(self) -> int:
        return self._p.pod_latency_count()

    def queue_depth(self) -> int:
        return self._p.queue_depth()

    def count_error(self, step: str) -> None:
        """kgwe_controller_errors_total{step}."""
        self._p.count_error(step)

    def partition_ops(self) -> list:
        return _j(self._p.partition_ops_json())

    def partition_metrics(self) -> dict:
        return _j(self._p.partition_metrics_json())

    # sharing ---------------------------------------------------------------------
    def share_allocate(self, req: dict) -> dict:
        return _j(self._p.share_allocate(json.dumps(req)))

    def share_release(self, uid: str) -> bool:
        return self._p.share_release(uid)

    def share_allocations(self) -> list:
        return _j(self._p.share_allocations_json())

    # cost ------------------------------------------------------------------------
    def cost_start(self, record: dict, now: float | None = None) -> str:
        return self._p.cost_start(json.dumps(record), time.time() if now is None else now)

    def cost_sample(self, uid: str, gfx: float, mem: float, now: float | None = None) -> bool:
        return self._p.cost_sample(uid, gfx, mem, time.time() if now is None else now)

    def cost_finalize(self, uid: str, now: float | None = None) -> dict | None:
        return _j(self._p.cost_finalize(uid, time.time() if now is None else now))

    def cost_record(self, uid: str) -> dict | None:
        return _j(self._p.cost_record_json(uid))

    def create_budget(self, budget: dict, now: float | None = None) -> str:
        return self._p.create_budget(json.dumps(budget), time.time() if now is None else now)

    def budgets(self, now: float | None = None) -> list:
        return _j(self._p.budgets_json(time.time() if now is None else now))

    def alerts(self, unacknowledged_only: bool = False) -> list:
        return _j(self._p.alerts_json(unacknowledged_only))

    def acknowledge_alert(self, alert_id: str) -> bool:
        return self._p.acknowledge_alert(alert_id)

    def cost_summary(self, scope: str = "", scope_id: str = "", start: float = 0.0,
                     end: float = 0.0) -> dict:
        return _j(self._p.cost_summary_json(scope, scope_id, start, end))

    def recommendations(self, scope: str = "", scope_id: str = "") -> list:
        return _j(self._p.recommendations_json(scope, scope_id))

    def chargeback(self, group_by: str = "namespace", start: float = 0.0, end: float = 0.0) -> dict:
        return _j(self._p.chargeback_json(group_by, start, end))

    def admit(self, ns: str, team: str = "", project: str = "", estimated_cost: float = 0.0,
              now: float | None = None) -> dict:
        return _j(self._p.admit(ns, team, project, estimated_cost, time.time() if now is None else now))

    def pricing(self) -> list:
        return _j(self._p.pricing_json())

    def set_pricing(self, p: dict) -> None:
        self._p.set_pricing(json.dumps(p))

    def cost_resumed(self) -> int:
        """Running usage records restored from the journal (failover)."""
        return self._p.cost_resumed()

    def cost_replayed(self) -> int:
        return self._p.cost_replayed()

    # housekeeping ------------------------------------------------------------------
    def tick(self, now: float | None = None) -> None:
        self._p.tick(time.time() if now is None else now)

    def expose_metrics(self) -> str:
        return self._p.expose_metrics()

    def metric_value(self, name: str, labels: list[str] | tuple = ()) -> float:
        return self._p.metric_value(name, list(labels))
