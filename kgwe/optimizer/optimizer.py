"""Workload optimizer on PyTorch-ROCm: classification, resource prediction,
placement hints (reference: src/optimizer/workload_optimizer.py, C24a-e).

Kept (API + parity tables): WorkloadType / MLFramework / DistributionStrategy
enums, WorkloadProfile with the 9-feature vector (:346-370), the classifier
signatures (:153-178) and trend rule (:220-233), the reference MODEL_RESOURCE_MAP
(:275-285, half-open intervals), framework overheads (:288-293), strategy
efficiencies (:296-302), utilisation / duration / confidence estimators
(:477-518), placement with up to 2 alternatives (:533-612) and the
OptimizerService RPC surface (:798-875).

Fixed: enums are parsed from strings (the reference crashed on
``{"strategy": "FSDP"}``, :420-424); every sample is counted once (the
reference re-added the whole buffer on every ingest: 20 samples -> 165);
the xGMI group search checks MUTUAL connectivity (the reference grew a star
around one GPU, :656-694).

MI355X-native: resource sizing from a memory model of 288 GB HBM3E per GPU
(training: bf16 weights + fp32 master + fp32 grads + Adam moments, sharded by
FSDP; inference: bf16 weights + KV cache) instead of the H100-80GB table,
compute-partition recommendations (CPX = 1/8 GPU, 36 GB) instead of MIG
profiles, MI355X prices, and a small torch MLP trained online on completed
workloads (utilisation + duration regression, workload-type classification)
that takes over from the heuristics once it has seen enough data.
"""
from __future__ import annotations

import math
import threading
import time
from collections import defaultdict
from dataclasses import asdict, dataclass, field
from enum import Enum

import numpy as np


class WorkloadType(Enum):
    TRAINING = "Training"
    INFERENCE = "Inference"
    FINE_TUNING = "FineTuning"
    DATA_PREPROCESSING = "DataPreprocessing"
    REINFORCEMENT = "Reinforcement"
    VISUALIZATION = "Visualization"
    # GPUWorkload CRD types the reference's optimizer enum lacks
    BATCH = "Batch"
    INTERACTIVE = "Interactive"
    DEVELOPMENT = "Development"


class MLFramework(Enum):
    PYTORCH = "PyTorch"
    TENSORFLOW = "TensorFlow"
    JAX = "JAX"
    MXNET = "MXNet"
    TRITON = "Triton"
    VLLM = "vLLM"
    SGLANG = "SGLang"


class DistributionStrategy(Enum):
    DATA_PARALLEL = "DataParallel"
    MODEL_PARALLEL = "ModelParallel"
    PIPELINE_PARALLEL = "PipelineParallel"
    HYBRID = "Hybrid"
    FSDP = "FSDP"
    DEEPSPEED = "DeepSpeed"
    CONTEXT_PARALLEL = "ContextParallel"
    EXPERT_PARALLEL = "ExpertParallel"


def parse_enum(cls, v):
    """Accept enum members, values ("FSDP") or names ("FSDP"/"fsdp"); None passes."""
    if v is None or isinstance(v, cls):
        return v
    s = str(v)
    for m in cls:
        if s == m.value or s.upper() == m.name or s.lower() == m.value.lower():
            return m
    raise ValueError(f"unknown {cls.__name__}: {v!r}")


@dataclass
class TelemetryDataPoint:
    """One amd-smi sample of a workload's GPU."""
    timestamp: float
    gpu_uuid: str
    gpu_utilization: float          # gfx_activity %
    memory_used_bytes: int
    memory_total_bytes: int
    xgmi_bandwidth_gbps: float = 0.0
    power_watts: float = 0.0
    temperature_celsius: float = 0.0
    workload_id: str = ""


@dataclass
class WorkloadProfile:
    workload_id: str
    workload_type: WorkloadType
    framework: MLFramework | None = None
    avg_gpu_utilization: float = 0.0
    peak_gpu_utilization: float = 0.0
    avg_memory_utilization: float = 0.0
    peak_memory_utilization: float = 0.0
    utilization_variance: float = 0.0
    memory_growth_rate: float = 0.0  # MB/s
    avg_xgmi_bandwidth_usage: float = 0.0
    communication_compute_ratio: float = 0.0
    avg_duration_seconds: float = 0.0
    duration_variance: float = 0.0
    feature_vector: list = field(default_factory=list)
    created_at: float = field(default_factory=time.time)
    updated_at: float = field(default_factory=time.time)
    sample_count: int = 0


@dataclass
class ResourcePrediction:
    recommended_gpus: int
    recommended_memory_gb: int
    expected_utilization: float
    expected_duration_seconds: float
    confidence: float
    prefer_xgmi: bool = False
    prefer_same_numa: bool = False
    recommended_partition: str | None = None  # "CPX" / "QPX" / "DPX" or None (whole GPU)
    estimated_cost_per_hour: float = 0.0
    reasoning: list = field(default_factory=list)


@dataclass
class PlacementHint:
    preferred_nodes: list
    preferred_gpus: dict
    score: int
    reasoning: str
    alternatives: list = field(default_factory=list)


# ---------------------------------------------------------------------------
class WorkloadClassifier:
    """Signature matching (reference :144-262) + an online torch classifier."""

    WORKLOAD_SIGNATURES = {
        WorkloadType.TRAINING: {"min_gpu_util": 60, "memory_pattern": "growing",
                                "duration_pattern": "long", "communication_heavy": True},
        WorkloadType.INFERENCE: {"min_gpu_util": 20, "memory_pattern": "stable",
                                 "duration_pattern": "short", "communication_heavy": False},
        WorkloadType.FINE_TUNING: {"min_gpu_util": 50, "memory_pattern": "growing",
                                   "duration_pattern": "medium", "communication_heavy": True},
        WorkloadType.DATA_PREPROCESSING: {"min_gpu_util": 30, "memory_pattern": "variable",
                                          "duration_pattern": "variable",
                                          "communication_heavy": False},
    }

    def __init__(self):
        self.history: dict = defaultdict(list)

    def add_sample(self, workload_id: str, dp: TelemetryDataPoint):
        dp.workload_id = workload_id
        h = self.history[workload_id]
        h.append(dp)
        if len(h) > 1000:
            del h[: len(h) - 1000]

    @staticmethod
    def _calculate_trend(values) -> str:
        if len(values) < 3:
            return "stable"
        if float(np.mean(np.diff(values))) > 1.0:
            return "growing"
        if float(np.var(values)) > 100:
            return "variable"
        return "stable"

    @staticmethod
    def _match_signature(avg_util, trend, n, sig) -> float:
        score = 0.0
        if avg_util >= sig["min_gpu_util"]:
            score += 0.3
        elif avg_util >= sig["min_gpu_util"] * 0.8:
            score += 0.15
        if trend == sig["memory_pattern"]:
            score += 0.3
        expected = {"short": 10, "medium": 50, "long": 100}.get(sig["duration_pattern"], 50)
        if abs(n - expected) < expected * 0.3:
            score += 0.2
        return score + min(n / 100, 0.2)

    def classify(self, workload_id: str):
        samples = self.history.get(workload_id, [])
        if len(samples) < 5:
            return WorkloadType.TRAINING, 0.3
        utils = [s.gpu_utilization for s in samples]
        mems = [100.0 * s.memory_used_bytes / max(1, s.memory_total_bytes) for s in samples]
        avg = float(np.mean(utils))
        trend = self._calculate_trend(mems)
        best, best_score = WorkloadType.TRAINING, 0.0
        for wt, sig in self.WORKLOAD_SIGNATURES.items():
            s = self._match_signature(avg, trend, len(samples), sig)
            # Sustained high utilisation with flat memory is steady-state
            # training (weights + optimizer resident), not inference: the
            # reference mislabelled a constant 70 % workload as INFERENCE.
            if wt == WorkloadType.TRAINING and avg >= 60 and trend == "stable":
                s += 0.3
            if s > best_score:
                best, best_score = wt, s
        return best, min(best_score, 0.95)


# ---------------------------------------------------------------------------
class OnlineMLP:
    """Tiny torch MLP trained online on (9-feature profile -> [util, log duration])
    of completed workloads.  Runs on the ROCm GPU when present, else CPU."""

    def __init__(self, n_in: int = 9, hidden: int = 32, lr: float = 1e-2, min_samples: int = 16):
        import torch  # noqa: PLC0415

        self.torch = torch
        self.dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        g = torch.Generator().manual_seed(0)
        self.net = torch.nn.Sequential(torch.nn.Linear(n_in, hidden), torch.nn.GELU(),
                                       torch.nn.Linear(hidden, hidden), torch.nn.GELU(),
                                       torch.nn.Linear(hidden, 2))
        with torch.no_grad():
            for p in self.net.parameters():
                p.copy_(torch.randn(p.shape, generator=g) * 0.1)
        self.net.to(self.dev)
        self.opt = torch.optim.Adam(self.net.parameters(), lr=lr)
        self.min_samples = min_samples
        self.X: list = []
        self.Y: list = []
        self.lock = threading.Lock()
        self.steps = 0
        self.last_loss = float("nan")

    def add(self, features, util: float, duration_s: float):
        with self.lock:
            self.X.append(list(features))
            self.Y.append([util / 100.0, math.log1p(max(0.0, duration_s)) / 12.0])
            if len(self.X) > 5000:
                del self.X[:1000], self.Y[:1000]

    @property
    def ready(self) -> bool:
        return len(self.X) >= self.min_samples and self.steps > 0

    def train(self, epochs: int = 50):
        torch = self.torch
        with self.lock:
            if len(self.X) < self.min_samples:
                return None
            X = torch.tensor(self.X, dtype=torch.float32, device=self.dev)
            Y = torch.tensor(self.Y, dtype=torch.float32, device=self.dev)
        for _ in range(epochs):
            self.opt.zero_grad()
            loss = torch.nn.functional.mse_loss(self.net(X), Y)
            loss.backward()
            self.opt.step()
            self.steps += 1
        self.last_loss = float(loss.item())
        return self.last_loss

    def predict(self, features):
        torch = self.torch
        with torch.no_grad():
            y = self.net(torch.tensor([features], dtype=torch.float32, device=self.dev))[0].cpu()
        return float(y[0].clamp(0, 1)) * 100.0, float(math.expm1(float(y[1]) * 12.0))


# ---------------------------------------------------------------------------
MI355X_HBM_GB = 288.0
MI355X_PRICE = 2.95  # $/GPU-hour on demand (kept in sync with the C++ cost engine)
PARTITION_MEM = {"CPX": 36.0, "QPX": 72.0, "DPX": 144.0}


class ResourcePredictor:
    # Reference table (H100-80GB sizing), kept for parity / compat mode.
    MODEL_RESOURCE_MAP = {
        (0, 0.1): (1, 10, False), (0.1, 1): (1, 20, False), (1, 7): (1, 40, False),
        (7, 13): (2, 40, True), (13, 30): (4, 40, True), (30, 70): (8, 80, True),
        (70, 180): (16, 80, True), (180, 500): (32, 80, True),
    }
    FRAMEWORK_OVERHEAD = {MLFramework.PYTORCH: 1.0, MLFramework.TENSORFLOW: 1.1,
                          MLFramework.JAX: 0.95, MLFramework.TRITON: 0.8,
                          # serving engines size their KV-cache pool to what they are given
                          MLFramework.VLLM: 1.0, MLFramework.SGLANG: 1.0}
    STRATEGY_EFFICIENCY = {DistributionStrategy.DATA_PARALLEL: 0.85,
                           DistributionStrategy.MODEL_PARALLEL: 0.75,
                           DistributionStrategy.PIPELINE_PARALLEL: 0.80,
                           DistributionStrategy.FSDP: 0.90,
                           DistributionStrategy.DEEPSPEED: 0.92}

    def __init__(self, sizing: str = "mi355x", learn: bool = True):
        self.sizing = sizing
        self.profiles: dict = {}
        self.classifier = WorkloadClassifier()
        self.model = None
        if learn:
            try:
                self.model = OnlineMLP()
            except Exception:  # noqa: BLE001 - torch unavailable: heuristics only
                self.model = None

    # --------------------------------------------------------------- profiles
    def update_profile(self, workload_id: str, telemetry: list, new_samples: int | None = None):
        p = self.profiles.get(workload_id)
        if p is None:
            wt, _ = self.classifier.classify(workload_id)
            p = WorkloadProfile(workload_id=workload_id, workload_type=wt)
            self.profiles[workload_id] = p
        utils = [t.gpu_utilization for t in telemetry]
        mems = [100.0 * t.memory_used_bytes / max(1, t.memory_total_bytes) for t in telemetry]
        p.avg_gpu_utilization = float(np.mean(utils))
        p.peak_gpu_utilization = float(np.max(utils))
        p.avg_memory_utilization = float(np.mean(mems))
        p.peak_memory_utilization = float(np.max(mems))
        p.utilization_variance = float(np.var(utils))
        p.avg_xgmi_bandwidth_usage = float(np.mean([t.xgmi_bandwidth_gbps for t in telemetry]))
        if len(telemetry) >= 2:
            span = telemetry[-1].timestamp - telemetry[0].timestamp
            if span > 0:
                p.memory_growth_rate = (telemetry[-1].memory_used_bytes -
                                        telemetry[0].memory_used_bytes) / span / 2**20
        p.workload_type, _ = self.classifier.classify(workload_id)
        p.feature_vector = self._extract_features(p, telemetry)
        p.updated_at = time.time()
        p.sample_count += len(telemetry) if new_samples is None else new_samples
        return p

    @staticmethod
    def _extract_features(p: WorkloadProfile, telemetry: list) -> list:
        f = [p.avg_gpu_utilization / 100.0, p.peak_gpu_utilization / 100.0,
             p.avg_memory_utilization / 100.0, p.peak_memory_utilization / 100.0,
             min(p.utilization_variance / 1000.0, 1.0), min(abs(p.memory_growth_rate) / 1000.0, 1.0),
             1.0 if p.workload_type == WorkloadType.TRAINING else 0.0,
             1.0 if p.workload_type == WorkloadType.INFERENCE else 0.0]
        if len(telemetry) >= 2:
            f.append(min((telemetry[-1].timestamp - telemetry[0].timestamp) / 3600.0, 1.0))
        else:
            f.append(0.0)
        return f

    def record_completion(self, workload_id: str, duration_s: float):
        """Feed a finished workload to the online model (label = observed)."""
        p = self.profiles.get(workload_id)
        if p is None:
            return
        p.avg_duration_seconds = duration_s
        if self.model is not None and p.feature_vector:
            self.model.add(p.feature_vector, p.avg_gpu_utilization, duration_s)

    # --------------------------------------------------------------- sizing
    def _from_reference_table(self, params_b):
        if params_b is None:
            return 1, 20, False
        for (lo, hi), v in self.MODEL_RESOURCE_MAP.items():
            if lo <= params_b < hi:
                return v
        return 64, 80, True

    @staticmethod
    def _from_memory_model(params_b, wtype, strategy):
        """GPUs of 288 GB needed for the model (80 % usable for states)."""
        if params_b is None:
            return 1, 40, False
        usable = 0.8 * MI355X_HBM_GB
        if wtype in (WorkloadType.INFERENCE, WorkloadType.VISUALIZATION):
            need = params_b * 2.0 * 1.3  # bf16 weights + KV cache / activations
        else:
            # bf16 weights (2) + fp32 master (4) + fp32 grads (4) + Adam (8) = 18 B/param,
            # + activations (~25 % at micro-batch 1-2 with 288 GB of room).
            need = params_b * 18.0 * 1.25
        gpus = max(1, math.ceil(need / usable))
        if gpus > 1:
            gpus = 1 << (gpus - 1).bit_length()  # power of two: xGMI groups of 2/4/8
        per_gpu = min(MI355X_HBM_GB, need / gpus * 1.1)
        return gpus, int(math.ceil(per_gpu)), gpus > 1

    def predict_resources(self, workload_id: str, model_params_billions=None, framework=None,
                          strategy=None, batch_size=None, workload_type=None):
        framework = parse_enum(MLFramework, framework)
        strategy = parse_enum(DistributionStrategy, strategy)
        wtype = parse_enum(WorkloadType, workload_type)
        p = self.profiles.get(workload_id)
        if wtype is None:
            wtype = p.workload_type if p else WorkloadType.TRAINING
        reasoning = []
        if self.sizing == "reference":
            gpus, mem, xgmi = self._from_reference_table(model_params_billions)
            reasoning.append(f"Reference table ({model_params_billions}B params): {gpus} GPUs, {mem}GB")
        else:
            gpus, mem, xgmi = self._from_memory_model(model_params_billions, wtype, strategy)
            reasoning.append(f"MI355X memory model ({model_params_billions}B params, {wtype.value}): "
                             f"{gpus} x 288GB GPUs, {mem}GB/GPU")
        if p and p.sample_count >= 10:
            if p.peak_memory_utilization > 90:
                mem = int(mem * 1.25)
                reasoning.append("Increased memory due to high historical usage")
            elif p.peak_memory_utilization < 50:
                mem = max(10, int(mem * 0.75))
                reasoning.append("Reduced memory due to low historical usage")
        if framework in self.FRAMEWORK_OVERHEAD:
            mem = int(mem * self.FRAMEWORK_OVERHEAD[framework])
            reasoning.append(f"Applied {framework.value} overhead factor: "
                             f"{self.FRAMEWORK_OVERHEAD[framework]}")
        if strategy and gpus > 1:
            eff = self.STRATEGY_EFFICIENCY.get(strategy, 0.85)
            reasoning.append(f"Distribution strategy {strategy.value} efficiency: {eff:.0%}")
            if strategy in (DistributionStrategy.MODEL_PARALLEL, DistributionStrategy.CONTEXT_PARALLEL,
                            DistributionStrategy.EXPERT_PARALLEL):
                xgmi = True
                reasoning.append("Communication-heavy strategy: single xGMI island required")
        util, dur = self._estimate_utilization(p, gpus), self._estimate_duration(p, gpus)
        if self.model is not None and self.model.ready and p is not None and p.feature_vector:
            mu, md = self.model.predict(p.feature_vector)
            util = min(95.0, mu * (0.85 ** math.log2(gpus)) if gpus > 1 else mu)
            dur = md / (gpus ** 0.7)
            reasoning.append(f"Online model (n={len(self.model.X)}): util {mu:.0f}%, {md:.0f}s")
        part = None
        if p and p.avg_gpu_utilization < 40 and gpus == 1:
            for mode in ("CPX", "QPX", "DPX"):
                if mem <= PARTITION_MEM[mode]:
                    part = mode
                    break
            if part:
                reasoning.append(f"Low utilization: {part} compute partition "
                                 f"({PARTITION_MEM[part]:.0f} GB) recommended")
        cost = (MI355X_PRICE / {"CPX": 8, "QPX": 4, "DPX": 2}[part]) if part else gpus * MI355X_PRICE
        return ResourcePrediction(recommended_gpus=gpus, recommended_memory_gb=mem,
                                  expected_utilization=util, expected_duration_seconds=dur,
                                  confidence=self._calculate_confidence(p), prefer_xgmi=xgmi,
                                  prefer_same_numa=gpus <= 4, recommended_partition=part,
                                  estimated_cost_per_hour=cost, reasoning=reasoning)

    @staticmethod
    def _estimate_utilization(p, gpus):
        if p and p.sample_count >= 5:
            base = p.avg_gpu_utilization * (0.85 ** math.log2(gpus) if gpus > 1 else 1.0)
            return min(base, 95.0)
        return 70.0

    @staticmethod
    def _estimate_duration(p, gpus):
        if p and p.avg_duration_seconds > 0:
            return p.avg_duration_seconds / (gpus ** 0.7)
        return 3600.0

    @staticmethod
    def _calculate_confidence(p):
        if p is None:
            return 0.3
        s = min(p.sample_count / 100, 0.4)
        v = max(0.0, 0.3 - p.utilization_variance / 1000)
        age_h = (time.time() - p.updated_at) / 3600
        r = max(0.0, 0.3 - age_h / 24)
        return min(0.95, 0.3 + s + v + r)


# ---------------------------------------------------------------------------
class PlacementOptimizer:
    """Placement hints over a topology snapshot (kgwe.core Platform.snapshot())."""

    def __init__(self, predictor: ResourcePredictor):
        self.predictor = predictor

    def get_optimal_placement(self, workload_id: str, cluster_topology: dict, requirements: dict):
        k = int(requirements.get("gpu_count", 1))
        prefer = bool(requirements.get("prefer_xgmi", requirements.get("prefer_nvlink", False)))
        nodes = cluster_topology.get("nodes", {})
        if not nodes:
            return PlacementHint([], {}, 0, "No nodes available")
        scored = []
        for name, info in nodes.items():
            s, sel = self._score_node(info, k, prefer, set(requirements.get("busy_gpus", [])))
            scored.append((name, s, sel))
        scored.sort(key=lambda x: (-x[1], x[0]))
        if not scored or scored[0][1] == 0:
            return PlacementHint([], {}, 0, "No suitable placement found")
        best, bs, bg = scored[0]
        why = ["Optimal xGMI topology" if bs >= 80 else
               "Good topology with partial xGMI" if bs >= 60 else "PCIe-based placement"]
        if k > 1:
            why.append(f"Allocated {k} GPUs on single node")
        alts = [PlacementHint([n], {n: g}, s, f"Alternative placement (score: {s})")
                for n, s, g in scored[1:3] if s > 0]
        return PlacementHint([best], {best: bg}, bs, ", ".join(why), alts)

    def _score_node(self, info: dict, k: int, prefer: bool, busy: set):
        gpus = [g for g in info.get("gpus", [])
                if g.get("health", {}).get("status", "Healthy") == "Healthy" and g.get("uuid") not in busy]
        if len(gpus) < k:
            return 0, []
        if k == 1:
            gpus.sort(key=lambda g: -(g.get("memory_total_gb", 0) - g.get("memory_used_gb", 0)))
            return 80, [gpus[0]["uuid"]]
        if prefer or k >= 4:
            grp = self._find_xgmi_group(gpus, k)
            if len(grp) >= k:
                return 90, grp[:k]
        return 50, [g["uuid"] for g in gpus[:k]]

    @staticmethod
    def _find_xgmi_group(gpus: list, size: int) -> list:
        """Fully connected (every pair has an up xGMI link) group, greedy by
        connections into the group; checked for MUTUAL connectivity."""
        ids = [g["uuid"] for g in gpus]
        adj = {u: set() for u in ids}
        for g in gpus:
            for link in g.get("links", []):
                if link.get("up", True) and link.get("type", "XGMI") == "XGMI" and link.get("peer") in adj:
                    adj[g["uuid"]].add(link["peer"])
        for start in ids:
            group = [start]
            while len(group) < size:
                cands = [c for c in ids if c not in group and all(c in adj[m] and m in adj[c] for m in group)]
                if not cands:
                    break
                group.append(max(cands, key=lambda c: len(adj[c])))
            if len(group) >= size:
                return group
        return []


# ---------------------------------------------------------------------------
class WorkloadOptimizer:
    def __init__(self, sizing: str = "mi355x", learn: bool = True, profile_every: int = 10):
        self.predictor = ResourcePredictor(sizing=sizing, learn=learn)
        self.placement_optimizer = PlacementOptimizer(self.predictor)
        self.telemetry_buffer: dict = defaultdict(list)
        self._pending: dict = defaultdict(int)
        self.profile_every = profile_every
        self.total_samples = 0

    def ingest_telemetry(self, workload_id: str, dp: TelemetryDataPoint):
        self.telemetry_buffer[workload_id].append(dp)
        self.predictor.classifier.add_sample(workload_id, dp)
        self._pending[workload_id] += 1
        self.total_samples += 1
        buf = self.telemetry_buffer[workload_id]
        # Re-profile every `profile_every` NEW samples, counting each sample once.
        if len(buf) >= 10 and self._pending[workload_id] >= self.profile_every:
            self.predictor.update_profile(workload_id, buf, new_samples=self._pending[workload_id])
            self._pending[workload_id] = 0
            self.telemetry_buffer[workload_id] = buf[-100:]

    def complete(self, workload_id: str, duration_s: float, train: bool = True):
        buf = self.telemetry_buffer.get(workload_id)
        if buf and self._pending.get(workload_id):
            self.predictor.update_profile(workload_id, buf, new_samples=self._pending[workload_id])
            self._pending[workload_id] = 0
        self.predictor.record_completion(workload_id, duration_s)
        if train and self.predictor.model is not None:
            self.predictor.model.train(epochs=20)

    def predict_resources(self, workload_id: str, hints: dict | None = None):
        h = hints or {}
        return self.predictor.predict_resources(
            workload_id, model_params_billions=h.get("model_params_billions"),
            framework=h.get("framework"), strategy=h.get("strategy"),
            batch_size=h.get("batch_size"), workload_type=h.get("workload_type"))

    def get_optimal_placement(self, workload_id: str, cluster_topology: dict, requirements: dict):
        return self.placement_optimizer.get_optimal_placement(workload_id, cluster_topology, requirements)

    def get_profile(self, workload_id: str):
        return self.predictor.profiles.get(workload_id)

    def export_metrics(self) -> dict:
        m = self.predictor.model
        return {"total_profiles": len(self.predictor.profiles),
                "total_samples": self.total_samples,
                "model": None if m is None else {"device": str(m.dev), "training_rows": len(m.X),
                                                 "steps": m.steps, "last_loss": m.last_loss},
                "profiles": {wid: {"workload_type": p.workload_type.value,
                                   "avg_gpu_util": p.avg_gpu_utilization,
                                   "sample_count": p.sample_count,
                                   "updated_at": p.updated_at}
                             for wid, p in self.predictor.profiles.items()}}


def _enum_json(o):
    if isinstance(o, Enum):
        return o.value
    if isinstance(o, list):
        return [_enum_json(x) for x in o]
    if isinstance(o, dict):
        return {k: _enum_json(v) for k, v in o.items()}
    return o


class OptimizerService:
    """RPC surface (dict in, dict out); served over gRPC by kgwe.optimizer.server."""

    def __init__(self, **kw):
        self.optimizer = WorkloadOptimizer(**kw)

    def PredictResources(self, request: dict) -> dict:  # noqa: N802 - RPC name
        try:
            pr = self.optimizer.predict_resources(request.get("workload_id", "unknown"),
                                                  request.get("hints", {}))
        except ValueError as e:
            return {"error": str(e)}
        return _enum_json(asdict(pr))

    def GetPlacement(self, request: dict) -> dict:  # noqa: N802
        h = self.optimizer.get_optimal_placement(request.get("workload_id", "unknown"),
                                                 request.get("cluster_topology", {}),
                                                 request.get("requirements", {}))
        return _enum_json(asdict(h))

    def IngestTelemetry(self, request: dict) -> dict:  # noqa: N802
        wid = request.get("workload_id", "unknown")
        n = 0
        for s in request.get("samples", [request.get("sample")] if request.get("sample") else []):
            self.optimizer.ingest_telemetry(wid, TelemetryDataPoint(
                timestamp=float(s.get("timestamp", time.time())), gpu_uuid=s.get("gpu_uuid", ""),
                gpu_utilization=float(s.get("gpu_utilization", 0.0)),
                memory_used_bytes=int(s.get("memory_used_bytes", 0)),
                memory_total_bytes=int(s.get("memory_total_bytes", 1)),
                xgmi_bandwidth_gbps=float(s.get("xgmi_bandwidth_gbps", 0.0)),
                power_watts=float(s.get("power_watts", 0.0)),
                temperature_celsius=float(s.get("temperature_celsius", 0.0))))
            n += 1
        if request.get("completed"):
            self.optimizer.complete(wid, float(request.get("duration_seconds", 0.0)))
        return {"accepted": n}

    def GetMetrics(self, request: dict | None = None) -> dict:  # noqa: N802
        return self.optimizer.export_metrics()
