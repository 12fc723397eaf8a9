"""Node labels derived from a pushed MI355X node topology.

Reference: the discovery service declares ``UpdateNodeLabels`` on its
Kubernetes client interface but never calls it (src/discovery/discovery.go:82).  Here the controller (lease holder) labels each node whenever the
agent's topology push changes a label, so ordinary nodeSelectors / affinities
(and the GPUWorkload ``constraints.nodeSelector``) can target hardware facts:
GPU model/arch/count/HBM size, whether the 8 GPUs form one fully connected xGMI
island, links down, homogeneous partition mode and healthy-GPU count.
"""
from __future__ import annotations

import threading

PREFIX = "kgwe.amd.com/"


def node_labels(node: dict) -> dict[str, str]:
    gpus = node.get("gpus") or []
    n = len(gpus)
    uuids = {g.get("uuid") for g in gpus}
    up_pairs = set()
    down = 0
    for g in gpus:
        for link in g.get("links") or []:
            if link.get("type", "XGMI") != "XGMI" or link.get("peer") not in uuids:
                continue
            if link.get("up", True):
                up_pairs.add(frozenset((g.get("uuid"), link["peer"])))
            else:
                down += 1
    full = n > 1 and len(up_pairs) == n * (n - 1) // 2
    computes = {(g.get("partition") or {}).get("compute", "SPX") for g in gpus}
    memories = {(g.get("partition") or {}).get("memory", "NPS1") for g in gpus}
    healthy = sum((g.get("health") or {}).get("status", "Healthy") == "Healthy" for g in gpus)
    models = {g.get("model") or "MI355X" for g in gpus}
    archs = {g.get("arch") or "gfx950" for g in gpus}
    mem = min((g.get("memory_total_gb") or 288.0) for g in gpus) if gpus else 0
    return {
        PREFIX + "gpu.present": "true" if n else "false",
        PREFIX + "gpu.count": str(n),
        PREFIX + "gpu.healthy": str(healthy),
        PREFIX + "gpu.model": models.pop() if len(models) == 1 else "mixed",
        PREFIX + "gpu.arch": archs.pop() if len(archs) == 1 else "mixed",
        PREFIX + "gpu.memory-gb": str(int(mem)),
        PREFIX + "xgmi.fully-connected": "true" if full else "false",
        PREFIX + "xgmi.links-down": str(down // 2 if down else 0),
        PREFIX + "partition.compute": computes.pop() if len(computes) == 1 else "mixed",
        PREFIX + "partition.memory": memories.pop() if len(memories) == 1 else "mixed",
    }


class NodeLabeler:
    """Patches only when a node's label set changed (pushes arrive every few
    seconds; label churn would wake every node watcher in the cluster)."""

    def __init__(self, kube):
        self.kube = kube
        self._last: dict[str, dict] = {}
        self._lock = threading.Lock()
        self.patches = 0

    def update(self, name: str, node: dict) -> bool:
        labels = node_labels(node)
        with self._lock:
            if self._last.get(name) == labels:
                return False
        self.kube.patch_node_labels(name, labels)
        with self._lock:
            self._last[name] = labels
            self.patches += 1
        return True
