"""CRD schemas (single source of truth), validation and defaulting.

Reference: deploy/helm/kgwe/crds/gpuworkload-crd.yaml — GPUWorkload (:1-246),
MIGStrategy (:248-366), GPUBudget (:368-513) in group kgwe.nvidia.io.  Here the
group is ``kgwe.amd.com/v1`` and the vocabulary is MI355X:
  * topology.preference: None | xGMIOptimal | xGMIRequired | SameNUMA |
    SamePCIeSwitch (the NVLink* values are accepted as deprecated aliases and
    rewritten by the mutating webhook);
  * ``partition`` {mode: CPX|QPX|DPX, memoryMode: NPS1|NPS2, count} replaces
    ``mig`` (the MIG field is still accepted and mapped);
  * distributedConfig.backend: RCCL (default) | Gloo | MPI, with NCCL mapped to
    RCCL (RCCL implements the NCCL API);
  * architecture: CDNA3 | CDNA4; gpuModel e.g. MI355X.
  * MIGStrategy -> PartitionStrategy (cluster-scoped), same fields with a mode
    distribution.
The YAML under deploy/ is rendered from these dicts (``python -m kgwe.api.crds``)
and the admission webhook validates against the same dicts.
"""
from __future__ import annotations

import copy
import json
import sys
from pathlib import Path

GROUP = "kgwe.amd.com"
VERSION = "v1"

_S = lambda **kw: kw  # noqa: E731 - schema literal helper

TOPOLOGY_PREFS = ["None", "xGMIOptimal", "xGMIRequired", "SameNUMA", "SamePCIeSwitch"]
TOPOLOGY_ALIASES = {"NVLinkOptimal": "xGMIOptimal", "NVLinkRequired": "xGMIRequired"}
PARTITION_MODES = ["SPX", "DPX", "QPX", "CPX"]
WORKLOAD_TYPES = ["Training", "Inference", "Batch", "Interactive", "Development",
                  "FineTuning", "DataPreprocessing"]
FRAMEWORKS = ["PyTorch", "TensorFlow", "JAX", "MXNet", "Triton", "vLLM", "SGLang"]
STRATEGIES = ["None", "DataParallel", "ModelParallel", "PipelineParallel", "Hybrid", "FSDP",
              "DeepSpeed", "ContextParallel", "ExpertParallel"]
BACKENDS = ["RCCL", "Gloo", "MPI", "NCCL"]
PHASES = ["Pending", "Scheduling", "Scheduled", "Running", "Succeeded", "Failed"]

_conditions = _S(type="array", items=_S(type="object", properties={
    "type": _S(type="string"), "status": _S(type="string"), "reason": _S(type="string"),
    "message": _S(type="string"), "lastTransitionTime": _S(type="string", format="date-time")}))

GPUWORKLOAD_SPEC = _S(
    type="object", required=["gpuRequirements"],
    properties={
        "gpuRequirements": _S(type="object", required=["count"], properties={
            "count": _S(type="integer", minimum=0, maximum=64,
                        description="Whole MI355X GPUs (0 when only partition slices are requested)"),
            "minMemoryGB": _S(type="integer", minimum=1, maximum=288),
            "minBandwidthGBps": _S(type="number", minimum=0),
            "topology": _S(type="object", properties={
                "preference": _S(type="string", enum=TOPOLOGY_PREFS + list(TOPOLOGY_ALIASES),
                                 default="None"),
                "minBandwidthGBps": _S(type="number", minimum=0)}),
            "partition": _S(type="object", required=["mode"], properties={
                "mode": _S(type="string", enum=PARTITION_MODES),
                "memoryMode": _S(type="string", enum=["NPS1", "NPS2"], default="NPS1"),
                "count": _S(type="integer", minimum=1, maximum=64, default=1)}),
            "sharing": _S(type="object", description=(
                "Share ONE whole SPX GPU with other workloads instead of owning it (reference MPS / "
                "time-slicing, src/sharing/mig_controller.go:545-857). CoLocate: a disjoint range of "
                "compute units (HSA_CU_MASK, rounded to whole XCDs) + an HBM cap; TimeSlice: the "
                "whole GPU, time-shared. The scheduler ledger never hands a shared GPU out whole "
                "or partitions it. Requires count 1."),
                properties={"method": _S(type="string", enum=["CoLocate", "TimeSlice", "MPS"],
                                         default="CoLocate"),
                            "cuPercent": _S(type="number", minimum=0, maximum=100,
                                            description="Share of the GPU's 256 CUs (12.5 = one XCD)"),
                            "memoryGB": _S(type="number", minimum=0, maximum=288),
                            "group": _S(type="string", maxLength=63, pattern="^[A-Za-z0-9._-]*$", description=(
                                "Share group: workloads of one group on a GPU (same model) hold ONE CU range "
                                "and ONE HBM cap, sized by the group's first workload (its leader, which runs "
                                "the serving process, python -m kgwe.serving.batch_server); the others connect "
                                "to it through KGWE_BATCH_ENDPOINT and add no weights of their own."))}),
            "mig": _S(type="object", description="Deprecated: mapped to partition",
                      properties={"profile": _S(type="string"), "count": _S(type="integer", minimum=1)}),
            "gpuModel": _S(type="string", description="e.g. MI355X"),
            "architecture": _S(type="string", enum=["CDNA3", "CDNA4"]),
        }),
        "workloadType": _S(type="string", enum=WORKLOAD_TYPES, default="Training"),
        "framework": _S(type="string", enum=FRAMEWORKS),
        "distributedConfig": _S(type="object", properties={
            "strategy": _S(type="string", enum=STRATEGIES),
            "worldSize": _S(type="integer", minimum=1),
            "backend": _S(type="string", enum=BACKENDS, default="RCCL")}),
        "modelParamsBillions": _S(type="number", minimum=0,
                                  description="Model size hint for the optimizer's rightsizing"),
        "priority": _S(type="integer", minimum=0, maximum=1000000, default=0),
        "preemptible": _S(type="boolean", default=True),
        "expectedDurationSeconds": _S(type="number", minimum=0, description=(
            "How long the workload expects to hold its GPUs; preemption spares a job within the wait window "
            "of its expected end and waits for it instead (reference WorkloadSpec.EstimatedDuration, "
            "src/scheduler/types.go:92-110, never read there).")),
        "team": _S(type="string"),
        "project": _S(type="string"),
        "gang": _S(type="object", properties={"name": _S(type="string"),
                                              "size": _S(type="integer", minimum=1)}),
        "constraints": _S(type="object", properties={
            "nodeSelector": _S(type="object", additionalProperties=_S(type="string")),
            "excludeNodes": _S(type="array", items=_S(type="string")),
            "colocateWith": _S(type="array", items=_S(type="string")),
            "antiAffinityWith": _S(type="array", items=_S(type="string")),
            "tolerations": _S(type="array", items=_S(type="object",
                                                     **{"x-kubernetes-preserve-unknown-fields": True})),
            "affinity": _S(type="object", **{"x-kubernetes-preserve-unknown-fields": True}),
            "maxLatencyMs": _S(type="number", minimum=0)}),
        "recovery": _S(type="object", description=(
            "What the controller does when the workload's node is lost or one of its GPUs turns "
            "Unhealthy (RAS / ECC / xGMI health from amd-smi): Reschedule re-creates the pod "
            "elsewhere (the job resumes from its own checkpoint), Fail ends the workload."),
            properties={"policy": _S(type="string", enum=["Reschedule", "Fail"], default="Reschedule"),
                        "maxRestarts": _S(type="integer", minimum=0, maximum=100, default=3)}),
        "podTemplate": _S(type="object", **{"x-kubernetes-preserve-unknown-fields": True}),
    })

GPUWORKLOAD_STATUS = _S(type="object", properties={
    "phase": _S(type="string", enum=PHASES),
    "scheduledNode": _S(type="string"),
    "allocatedGPUs": _S(type="array", items=_S(type="string")),
    "partitionSlices": _S(type="array", items=_S(type="string")),
    "schedulingScore": _S(type="integer"),
    "estimatedBandwidth": _S(type="number"),
    "rcclEnv": _S(type="object", additionalProperties=_S(type="string")),
    "podName": _S(type="string"),
    "message": _S(type="string"),
    "conditions": _conditions,
    "startTime": _S(type="string", format="date-time"),
    "completionTime": _S(type="string", format="date-time"),
    "restarts": _S(type="integer", minimum=0),
    "recoveryRestarts": _S(type="integer", minimum=0),
    "migrations": _S(type="integer", minimum=0),
    "lastFailure": _S(type="string"),
    "recommendation": _S(type="object", description="Workload optimizer rightsizing", properties={
        "gpus": _S(type="integer"), "memoryGB": _S(type="integer"), "partition": _S(type="string"),
        "expectedUtilization": _S(type="number"), "confidence": _S(type="number"),
        "costPerHour": _S(type="number"), "reasoning": _S(type="array", items=_S(type="string")),
        "updated": _S(type="string")}),
    "cost": _S(type="number")})

PARTITIONSTRATEGY_SPEC = _S(type="object", required=["profileDistribution"], properties={
    "nodeSelector": _S(type="object", additionalProperties=_S(type="string")),
    "gpuSelector": _S(type="object", properties={
        "model": _S(type="string"), "minMemoryGB": _S(type="integer", minimum=0),
        "architecture": _S(type="string"), "partitionCapable": _S(type="boolean")}),
    "profileDistribution": _S(type="object", additionalProperties=_S(type="number", minimum=0, maximum=1)),
    "memoryPartition": _S(type="string", enum=["NPS1", "NPS2"], default="NPS1"),
    "allowDynamicReconfig": _S(type="boolean", default=True),
    "rebalanceInterval": _S(type="string", default="5m", pattern=r"^[0-9]+(s|m|h)$"),
    "minUtilizationThreshold": _S(type="number", minimum=0, maximum=1, default=0.3),
    "priority": _S(type="integer", default=0)})

PARTITIONSTRATEGY_STATUS = _S(type="object", properties={
    "appliedNodes": _S(type="array", items=_S(type="string")),
    "currentDistribution": _S(type="object", additionalProperties=_S(type="number")),
    "lastRebalanceTime": _S(type="string", format="date-time"),
    "conditions": _conditions})

GPUBUDGET_SPEC = _S(type="object", required=["limit"], properties={
    "limit": _S(type="string", pattern=r"^[0-9]+(\.[0-9]+)?$"),
    "currency": _S(type="string", default="USD"),
    "period": _S(type="string", enum=["Daily", "Weekly", "Monthly"], default="Monthly"),
    "scope": _S(type="string", enum=["Namespace", "Team", "Project", "Cluster"], default="Namespace"),
    "teamId": _S(type="string"),
    "scopeId": _S(type="string"),
    "alertsEnabled": _S(type="boolean", default=True),
    "alertThresholds": _S(type="array", items=_S(type="integer", minimum=1, maximum=100)),
    "enforcementPolicy": _S(type="string", enum=["Alert", "Throttle", "Block"], default="Alert")})

GPUBUDGET_STATUS = _S(type="object", properties={
    "currentSpend": _S(type="string"), "utilizationPercent": _S(type="number"),
    "periodStart": _S(type="string", format="date-time"),
    "periodEnd": _S(type="string", format="date-time"),
    "alerts": _S(type="array", items=_S(type="object", **{"x-kubernetes-preserve-unknown-fields": True})),
    "conditions": _conditions})

KINDS = {
    "GPUWorkload": dict(plural="gpuworkloads", singular="gpuworkload", short=["gw", "gpuw"],
                        scope="Namespaced", spec=GPUWORKLOAD_SPEC, status=GPUWORKLOAD_STATUS,
                        columns=[("GPUs", "integer", ".spec.gpuRequirements.count"),
                                 ("Status", "string", ".status.phase"),
                                 ("Node", "string", ".status.scheduledNode"),
                                 ("Age", "date", ".metadata.creationTimestamp")]),
    "PartitionStrategy": dict(plural="partitionstrategies", singular="partitionstrategy",
                              short=["ps", "partstrat"], scope="Cluster", spec=PARTITIONSTRATEGY_SPEC,
                              status=PARTITIONSTRATEGY_STATUS,
                              columns=[("Age", "date", ".metadata.creationTimestamp")]),
    "GPUBudget": dict(plural="gpubudgets", singular="gpubudget", short=["gb", "gpub"],
                      scope="Namespaced", spec=GPUBUDGET_SPEC, status=GPUBUDGET_STATUS,
                      columns=[("Limit", "string", ".spec.limit"),
                               ("Spend", "string", ".status.currentSpend"),
                               ("Utilization", "number", ".status.utilizationPercent")]),
}


def crd(kind: str) -> dict:
    k = KINDS[kind]
    return {
        "apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{k['plural']}.{GROUP}",
                     "labels": {"app.kubernetes.io/name": "kgwe-mi355x", "app.kubernetes.io/part-of": "kgwe"}},
        "spec": {
            "group": GROUP,
            "names": {"kind": kind, "listKind": kind + "List", "plural": k["plural"],
                      "singular": k["singular"], "shortNames": k["short"]},
            "scope": k["scope"],
            "versions": [{
                "name": VERSION, "served": True, "storage": True, "subresources": {"status": {}},
                "additionalPrinterColumns": [{"name": n, "type": t, "jsonPath": p} for n, t, p in k["columns"]],
                "schema": {"openAPIV3Schema": {
                    "type": "object",
                    "properties": {"apiVersion": {"type": "string"}, "kind": {"type": "string"},
                                   "metadata": {"type": "object"},
                                   "spec": copy.deepcopy(k["spec"]),
                                   "status": copy.deepcopy(k["status"])}}},
            }],
        },
    }


# ---------------------------------------------------------------------------
# Validation + defaulting against the same schema dicts
# ---------------------------------------------------------------------------
_TYPES = {"object": dict, "array": list, "string": str, "boolean": bool}


def _validate(schema: dict, value, path: str, errors: list) -> None:
    t = schema.get("type")
    if t == "integer":
        if isinstance(value, bool) or not isinstance(value, int):
            errors.append(f"{path}: expected integer")
            return
    elif t == "number":
        if isinstance(value, bool) or not isinstance(value, (int, float)):
            errors.append(f"{path}: expected number")
            return
    elif t in _TYPES and not isinstance(value, _TYPES[t]):
        errors.append(f"{path}: expected {t}")
        return
    if "enum" in schema and value not in schema["enum"]:
        errors.append(f"{path}: {value!r} not in {schema['enum']}")
    if "minimum" in schema and isinstance(value, (int, float)) and value < schema["minimum"]:
        errors.append(f"{path}: {value} < minimum {schema['minimum']}")
    if "maximum" in schema and isinstance(value, (int, float)) and value > schema["maximum"]:
        errors.append(f"{path}: {value} > maximum {schema['maximum']}")
    if "pattern" in schema and isinstance(value, str):
        import re  # noqa: PLC0415

        if not re.match(schema["pattern"], value):
            errors.append(f"{path}: {value!r} does not match {schema['pattern']}")
    if t == "object" and isinstance(value, dict):
        if schema.get("x-kubernetes-preserve-unknown-fields"):
            return
        for r in schema.get("required", []):
            if r not in value:
                errors.append(f"{path}.{r}: required")
        props = schema.get("properties", {})
        addl = schema.get("additionalProperties")
        for k2, v2 in value.items():
            if k2 in props:
                _validate(props[k2], v2, f"{path}.{k2}", errors)
            elif isinstance(addl, dict):
                _validate(addl, v2, f"{path}.{k2}", errors)
            elif props:
                errors.append(f"{path}.{k2}: unknown field")
    if t == "array" and isinstance(value, list) and "items" in schema:
        for i, v2 in enumerate(value):
            _validate(schema["items"], v2, f"{path}[{i}]", errors)


def _defaults(schema: dict, value):
    if schema.get("type") != "object" or not isinstance(value, dict):
        return value
    for k2, sub in schema.get("properties", {}).items():
        if k2 not in value and "default" in sub:
            value[k2] = copy.deepcopy(sub["default"])
        if k2 in value:
            value[k2] = _defaults(sub, value[k2])
    return value


def validate(obj: dict) -> list[str]:
    """Schema + semantic validation of a kgwe custom resource. [] = valid."""
    kind = obj.get("kind")
    if kind not in KINDS:
        return [f"unknown kind {kind!r}"]
    errors: list[str] = []
    if not obj.get("metadata", {}).get("name"):
        errors.append("metadata.name: required")
    spec = obj.get("spec")
    if spec is None:
        return errors + ["spec: required"]
    _validate(KINDS[kind]["spec"], spec, "spec", errors)
    if kind == "GPUWorkload" and not errors:
        req = spec["gpuRequirements"]
        if req.get("count", 0) == 0 and not (req.get("partition") or req.get("mig")):
            errors.append("spec.gpuRequirements: count must be >= 1 unless partition slices are requested")
        if req.get("count", 0) > 0 and req.get("partition"):
            errors.append("spec.gpuRequirements: request whole GPUs or partition slices, not both")
        if req.get("sharing") and (req.get("count", 0) != 1 or req.get("partition")):
            errors.append("spec.gpuRequirements.sharing: requires count 1 and no partition")
        dc = spec.get("distributedConfig", {})
        ws = dc.get("worldSize")
        if ws and req.get("count", 0) and ws < req["count"]:
            errors.append("spec.distributedConfig.worldSize must be >= gpuRequirements.count")
        g = spec.get("gang")
        if g and not g.get("name"):
            errors.append("spec.gang.name: required when gang is set")
    if kind == "PartitionStrategy" and not errors:
        dist = spec["profileDistribution"]
        bad = [m for m in dist if m not in PARTITION_MODES]
        if bad:
            errors.append(f"spec.profileDistribution: unknown modes {bad} (MI355X: {PARTITION_MODES})")
        if sum(float(v) for v in dist.values()) > 1.01:
            errors.append("spec.profileDistribution: fractions sum to more than 1.0")
    return errors


def default(obj: dict) -> dict:
    """Apply schema defaults + MI355X vocabulary rewrites (mutating webhook)."""
    out = copy.deepcopy(obj)
    kind = out.get("kind")
    if kind not in KINDS:
        return out
    spec = out.setdefault("spec", {})
    if kind == "GPUWorkload":
        req = spec.setdefault("gpuRequirements", {})
        topo = req.get("topology")
        if isinstance(topo, dict) and topo.get("preference") in TOPOLOGY_ALIASES:
            topo["preference"] = TOPOLOGY_ALIASES[topo["preference"]]
        mig = req.pop("mig", None)
        if mig and "partition" not in req:
            prof = str(mig.get("profile", ""))
            mode = "CPX" if prof.startswith("1g") else "QPX" if prof.startswith("2g") else "DPX"
            req["partition"] = {"mode": mode, "count": int(mig.get("count", 1))}
            req.setdefault("count", 0)
        dc = spec.get("distributedConfig")
        if isinstance(dc, dict) and dc.get("backend") == "NCCL":
            dc["backend"] = "RCCL"
    _defaults(KINDS[kind]["spec"], spec)
    return out


def render(out_dir: str | Path) -> list[Path]:
    import yaml  # noqa: PLC0415

    out_dir = Path(out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    paths = []
    for kind, k in KINDS.items():
        p = out_dir / f"{k['plural']}.{GROUP}.yaml"
        p.write_text("# Generated by `python -m kgwe.api.crds` -- do not edit.\n" +
                     yaml.safe_dump(crd(kind), sort_keys=False))
        paths.append(p)
    return paths


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    target = argv[0] if argv else "deploy/helm/kgwe-mi355x/crds"
    for p in render(target):
        print(p)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
