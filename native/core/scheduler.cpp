#include "scheduler.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <functional>
#include <numeric>

namespace kgwe {

constexpr size_t kSweepChunk = 32;  // nodes per shared-lock hold in filter / prioritize


// ---------------------------------------------------------------------------
// enums
// ---------------------------------------------------------------------------
const char* to_string(TopologyPreference p) {
  switch (p) {
    case TopologyPreference::None: return "None";
    case TopologyPreference::XgmiOptimal: return "xGMIOptimal";
    case TopologyPreference::XgmiRequired: return "xGMIRequired";
    case TopologyPreference::SameNUMA: return "SameNUMA";
    case TopologyPreference::SamePCIeSwitch: return "SamePCIeSwitch";
  }
  return "None";
}
TopologyPreference topology_preference_from(const std::string& s) {
  if (s == "xGMIOptimal" || s == "XGMIOptimal" || s == "NVLinkOptimal")
    return TopologyPreference::XgmiOptimal;
  if (s == "xGMIRequired" || s == "XGMIRequired" || s == "NVLinkRequired")
    return TopologyPreference::XgmiRequired;
  if (s == "SameNUMA") return TopologyPreference::SameNUMA;
  if (s == "SamePCIeSwitch") return TopologyPreference::SamePCIeSwitch;
  return TopologyPreference::None;
}
const char* to_string(WorkloadType t) {
  switch (t) {
    case WorkloadType::Training: return "Training";
    case WorkloadType::Inference: return "Inference";
    case WorkloadType::Batch: return "Batch";
    case WorkloadType::Interactive: return "Interactive";
    case WorkloadType::Development: return "Development";
    default: return "Unknown";
  }
}
WorkloadType workload_type_from(const std::string& s) {
  if (s == "Training") return WorkloadType::Training;
  if (s == "Inference") return WorkloadType::Inference;
  if (s == "Batch") return WorkloadType::Batch;
  if (s == "Interactive") return WorkloadType::Interactive;
  if (s == "Development") return WorkloadType::Development;
  return s.empty() ? WorkloadType::Training : WorkloadType::Unknown;
}
const char* to_string(DistributionStrategy s) {
  switch (s) {
    case DistributionStrategy::None: return "None";
    case DistributionStrategy::DataParallel: return "DataParallel";
    case DistributionStrategy::ModelParallel: return "ModelParallel";
    case DistributionStrategy::PipelineParallel: return "PipelineParallel";
    case DistributionStrategy::Hybrid: return "Hybrid";
    case DistributionStrategy::FSDP: return "FSDP";
    case DistributionStrategy::DeepSpeed: return "DeepSpeed";
    case DistributionStrategy::ContextParallel: return "ContextParallel";
    case DistributionStrategy::ExpertParallel: return "ExpertParallel";
  }
  return "None";
}
DistributionStrategy strategy_from(const std::string& s) {
  if (s == "DataParallel" || s == "DDP") return DistributionStrategy::DataParallel;
  if (s == "ModelParallel" || s == "TensorParallel") return DistributionStrategy::ModelParallel;
  if (s == "PipelineParallel") return DistributionStrategy::PipelineParallel;
  if (s == "Hybrid") return DistributionStrategy::Hybrid;
  if (s == "FSDP") return DistributionStrategy::FSDP;
  if (s == "DeepSpeed") return DistributionStrategy::DeepSpeed;
  if (s == "ContextParallel" || s == "SequenceParallel") return DistributionStrategy::ContextParallel;
  if (s == "ExpertParallel") return DistributionStrategy::ExpertParallel;
  return DistributionStrategy::None;
}
const char* to_string(CommBackend b) {
  switch (b) {
    case CommBackend::RCCL: return "RCCL";
    case CommBackend::Gloo: return "Gloo";
    case CommBackend::MPI: return "MPI";
  }
  return "RCCL";
}
CommBackend backend_from(const std::string& s) {
  if (s == "Gloo" || s == "gloo") return CommBackend::Gloo;
  if (s == "MPI" || s == "mpi") return CommBackend::MPI;
  return CommBackend::RCCL;  // "RCCL", "NCCL" (alias: RCCL implements the NCCL API)
}
const char* to_string(SchedEventType t) {
  switch (t) {
    case SchedEventType::Scheduled: return "Scheduled";
    case SchedEventType::Failed: return "Failed";
    case SchedEventType::Released: return "Released";
    case SchedEventType::Preempted: return "Preempted";
    case SchedEventType::GangReady: return "GangReady";
    case SchedEventType::GangTimeout: return "GangTimeout";
    case SchedEventType::Migrated: return "Migrated";
  }
  return "Unknown";
}
const char* to_string(SharingMethod m) {
  switch (m) {
    case SharingMethod::None: return "None";
    case SharingMethod::Partition: return "Partition";
    case SharingMethod::CoLocate: return "CoLocate";
    case SharingMethod::TimeSlice: return "TimeSlice";
  }
  return "None";
}
SharingMethod sharing_method_from(const std::string& s) {
  if (s == "Partition" || s == "MIG") return SharingMethod::Partition;
  if (s == "CoLocate" || s == "MPS") return SharingMethod::CoLocate;
  if (s == "TimeSlice") return SharingMethod::TimeSlice;
  return SharingMethod::None;
}

// ---------------------------------------------------------------------------
// JSON <-> WorkloadRequest (GPUWorkload custom resource or bare spec)
// ---------------------------------------------------------------------------
static std::vector<std::string> str_list(const Json& j) {
  std::vector<std::string> v;
  for (const auto& e : j.items()) v.push_back(e.str());
  return v;
}

static std::vector<AffinityTerm> terms_from(const Json& j) {
  std::vector<AffinityTerm> out;
  for (const auto& t : j.items()) {
    AffinityTerm a;
    a.key = t.get("key").str();
    a.op = t.get("operator").str("In");
    a.values = str_list(t.get("values"));
    a.weight = static_cast<int>(t.get("weight").as_int(0));
    out.push_back(a);
  }
  return out;
}

WorkloadRequest workload_from_json(const Json& in) {
  WorkloadRequest w;
  const Json& meta = in.get("metadata");
  const Json& spec = in.has("spec") ? in.get("spec") : in;
  w.uid = meta.get("uid").str(in.get("uid").str());
  w.name = meta.get("name").str(in.get("name").str());
  w.ns = meta.get("namespace").str(in.get("namespace").str("default"));
  if (w.uid.empty()) w.uid = w.ns + "/" + w.name;
  const Json& labels = meta.get("labels");
  w.team = spec.get("team").str(labels.get("kgwe.amd.com/team").str(labels.get("team").str()));
  w.project = spec.get("project").str(labels.get("kgwe.amd.com/project").str());
  const Json& req = spec.has("gpuRequirements") ? spec.get("gpuRequirements") : spec;
  w.gpu_count = static_cast<int>(req.get("count").as_int(req.get("gpuCount").as_int(1)));
  w.min_memory_gb = req.get("minMemoryGB").as_number(0.0);
  w.min_bandwidth_gbps = req.get("minBandwidthGBps").as_number(0.0);
  const Json& topo = req.get("topology");
  if (topo.is_object()) {
    w.topology = topology_preference_from(topo.get("preference").str("None"));
    if (topo.has("minBandwidthGBps"))
      w.min_bandwidth_gbps = std::max(w.min_bandwidth_gbps, topo.get("minBandwidthGBps").as_number());
  } else if (topo.is_string()) {
    w.topology = topology_preference_from(topo.str());
  }
  w.arch = req.get("architecture").str();
  w.model = req.get("gpuModel").str();
  const Json& part = req.get("partition");
  if (part.is_object()) {
    w.partition = true;
    w.partition_mode = compute_partition_from(part.get("mode").str("CPX"));
    w.partition_count = static_cast<int>(part.get("count").as_int(1));
    if (part.get("memoryMode").is_string()) {
      w.partition_memory_set = true;
      w.partition_memory = memory_partition_from(part.get("memoryMode").str());
    }
  }
  const Json& share = req.get("sharing");
  if (share.is_object()) {
    w.sharing = sharing_method_from(share.get("method").str("CoLocate"));
    if (w.sharing == SharingMethod::Partition) w.sharing = SharingMethod::None;  // use `partition`
    w.share_cu_percent = share.get("cuPercent").as_number(0.0);
    w.share_memory_gb = share.get("memoryGB").as_number(0.0);
    w.share_group = share.get("group").str();
    if (w.sharing != SharingMethod::None) w.gpu_count = 1;
  }
  const Json& mig = req.get("mig");  // legacy MIG field: map profile size to a mode
  if (!w.partition && mig.is_object()) {
    const std::string prof = mig.get("profile").str();
    w.partition = true;
    w.partition_count = static_cast<int>(mig.get("count").as_int(1));
    if (prof.rfind("1g", 0) == 0) w.partition_mode = ComputePartition::CPX;
    else if (prof.rfind("2g", 0) == 0) w.partition_mode = ComputePartition::QPX;
    else if (prof.rfind("3g", 0) == 0 || prof.rfind("4g", 0) == 0) w.partition_mode = ComputePartition::DPX;
    else w.partition_mode = ComputePartition::SPX;
  }
  w.type = workload_type_from(spec.get("workloadType").str("Training"));
  w.framework = spec.get("framework").str("PyTorch");
  const Json& dc = spec.get("distributedConfig");
  w.strategy = strategy_from(dc.get("strategy").str("None"));
  w.world_size = static_cast<int>(dc.get("worldSize").as_int(0));
  w.backend = backend_from(dc.get("backend").str("RCCL"));
  w.priority = spec.get("priority").as_int(0);
  w.preemptible = spec.get("preemptible").as_bool(true);
  w.expected_duration_s = spec.get("expectedDurationSeconds").as_number(0.0);
  const Json& c = spec.has("constraints") ? spec.get("constraints") : spec;
  for (const auto& kv : c.get("nodeSelector").fields()) w.node_selector[kv.first] = kv.second.str();
  const Json& aff = c.get("affinity");
  w.required_affinity = terms_from(aff.get("required"));
  w.preferred_affinity = terms_from(aff.get("preferred"));
  for (const auto& t : c.get("tolerations").items()) {
    Toleration tl;
    tl.key = t.get("key").str();
    tl.op = t.get("operator").str("Equal");
    tl.value = t.get("value").str();
    tl.effect = t.get("effect").str();
    w.tolerations.push_back(tl);
  }
  w.exclude_nodes = str_list(c.get("excludeNodes"));
  w.colocate_with = str_list(c.get("colocateWith"));
  w.anti_affinity_with = str_list(c.get("antiAffinityWith"));
  w.max_latency_ms = c.get("maxLatencyMs").as_number(0.0);
  const Json& gang = spec.get("gang");
  if (gang.is_object()) {
    w.gang = gang.get("name").str();
    w.gang_size = static_cast<int>(gang.get("size").as_int(0));
  }
  w.preferred_nodes = str_list(spec.get("preferredNodes"));
  return w;
}

Json to_json(const WorkloadRequest& w) {
  Json j = Json::object();
  j["uid"] = w.uid;
  j["name"] = w.name;
  j["namespace"] = w.ns;
  j["team"] = w.team;
  j["gpu_count"] = w.gpu_count;
  j["min_memory_gb"] = w.min_memory_gb;
  j["min_bandwidth_gbps"] = w.min_bandwidth_gbps;
  j["topology"] = to_string(w.topology);
  j["partition"] = w.partition;
  if (w.partition) {
    j["partition_mode"] = to_string(w.partition_mode);
    if (w.partition_memory_set) j["partition_memory"] = to_string(w.partition_memory);
    j["partition_count"] = w.partition_count;
  }
  j["type"] = to_string(w.type);
  j["strategy"] = to_string(w.strategy);
  j["backend"] = to_string(w.backend);
  j["world_size"] = w.world_size;
  j["priority"] = w.priority;
  j["preemptible"] = w.preemptible;
  if (w.expected_duration_s > 0) j["expectedDurationSeconds"] = w.expected_duration_s;
  j["gang"] = w.gang;
  j["gang_size"] = w.gang_size;
  if (w.sharing != SharingMethod::None) {
    j["sharing"] = to_string(w.sharing);
    j["share_cu_percent"] = w.share_cu_percent;
    j["share_memory_gb"] = w.share_memory_gb;
    if (!w.share_group.empty()) j["share_group"] = w.share_group;
  }
  return j;
}

Json to_json(const Decision& d) {
  Json j = Json::object();
  j["ok"] = d.ok;
  j["status"] = d.status;
  j["uid"] = d.uid;
  j["node"] = d.node;
  Json g = Json::array();
  for (const auto& x : d.gpus) g.push_back(x);
  j["gpus"] = g;
  Json p = Json::array();
  for (const auto& x : d.partitions) p.push_back(x);
  j["partitions"] = p;
  if (d.sharing != SharingMethod::None) {
    j["sharing"] = to_string(d.sharing);
    j["shared_gpu"] = d.shared_gpu;
    j["cu_begin"] = d.cu_begin;
    j["cu_end"] = d.cu_end;
    j["share_memory_gb"] = d.share_memory_gb;
    if (!d.share_group.empty()) {
      j["share_group"] = d.share_group;
      j["share_leader"] = d.share_leader;
      j["share_leader_uid"] = d.share_leader_uid;
    }
  }
  j["score"] = d.score;
  j["bandwidth_gbps"] = d.bandwidth_gbps;
  j["latency_ms"] = d.latency_ms;
  Json r = Json::array();
  for (const auto& x : d.reasons) r.push_back(x);
  j["reasons"] = r;
  Json pr = Json::array();
  for (const auto& x : d.preempted) pr.push_back(x);
  j["preempted"] = pr;
  Json f = Json::object();
  for (const auto& kv : d.failed_nodes) f[kv.first] = kv.second;
  j["failed_nodes"] = f;
  return j;
}

static double wall_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

Json to_json(const Allocation& a) {
  Json j = Json::object();
  j["uid"] = a.uid;
  j["node"] = a.node;
  j["namespace"] = a.ns;
  j["team"] = a.team;
  j["gang"] = a.gang;
  j["gang_size"] = a.gang_size;
  Json g = Json::array();
  for (const auto& x : a.gpus) g.push_back(x);
  j["gpus"] = g;
  Json p = Json::array();
  for (const auto& x : a.partitions) p.push_back(x);
  j["partitions"] = p;
  if (a.sharing != SharingMethod::None) {
    j["sharing"] = to_string(a.sharing);
    j["shared_gpu"] = a.shared_gpu;
    j["cu_begin"] = a.cu_begin;
    j["cu_end"] = a.cu_end;
    j["share_memory_gb"] = a.share_memory_gb;
    if (!a.share_group.empty()) {
      j["share_group"] = a.share_group;
      j["share_leader"] = a.share_leader;
      j["share_leader_uid"] = a.share_leader_uid;
    }
  }
  j["type"] = to_string(a.type);
  j["priority"] = a.priority;
  j["preemptible"] = a.preemptible;
  // Ledger times are on the monotonic clock; what leaves the process is wall
  // time of the allocation and the expected run time (0 = unknown).
  j["allocated_unix_s"] = a.allocated_ns ? wall_s() - static_cast<double>(now_ns() - a.allocated_ns) * 1e-9 : 0.0;
  j["expected_duration_s"] =
      a.expected_end_ns ? static_cast<double>(a.expected_end_ns - a.allocated_ns) * 1e-9 : 0.0;
  j["gang_pending"] = a.gang_pending;
  j["bandwidth_gbps"] = a.bandwidth_gbps;
  return j;
}

// The inverse of to_json(Allocation): a ledger entry as the controller
// persists it (pod annotations) and restores it after a restart / failover.
Allocation allocation_from_json(const Json& j) {
  Allocation a;
  a.uid = j.get("uid").str();
  a.node = j.get("node").str();
  a.ns = j.get("namespace").str("default");
  a.team = j.get("team").str();
  a.gang = j.get("gang").str();
  a.gang_size = static_cast<int>(j.get("gang_size").as_int(0));
  for (const auto& g : j.get("gpus").items()) a.gpus.push_back(g.str());
  for (const auto& p : j.get("partitions").items()) a.partitions.push_back(p.str());
  a.sharing = sharing_method_from(j.get("sharing").str("None"));
  a.shared_gpu = j.get("shared_gpu").str();
  a.cu_begin = static_cast<int>(j.get("cu_begin").as_int(0));
  a.cu_end = static_cast<int>(j.get("cu_end").as_int(0));
  a.share_memory_gb = j.get("share_memory_gb").as_number(0.0);
  a.share_group = j.get("share_group").str();
  a.share_leader = j.get("share_leader").as_bool(false);
  a.share_leader_uid = j.get("share_leader_uid").str();
  a.type = workload_type_from(j.get("type").str("Training"));
  a.priority = j.get("priority").as_int(0);
  a.preemptible = j.get("preemptible").as_bool(true);
  const double at = j.get("allocated_unix_s").as_number(0.0);
  if (at > 0.0) {
    a.allocated_ns = now_ns() - static_cast<int64_t>(std::max(0.0, wall_s() - at) * 1e9);
    const double dur = j.get("expected_duration_s").as_number(0.0);
    if (dur > 0.0) a.expected_end_ns = a.allocated_ns + static_cast<int64_t>(dur * 1e9);
  }
  a.bandwidth_gbps = j.get("bandwidth_gbps").as_number(0.0);
  return a;
}

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
namespace {

bool term_matches(const AffinityTerm& t, const std::map<std::string, std::string>& labels) {
  auto it = labels.find(t.key);
  const bool has = it != labels.end();
  if (t.op == "Exists") return has;
  if (t.op == "DoesNotExist") return !has;
  if (t.op == "In") return has && std::find(t.values.begin(), t.values.end(), it->second) != t.values.end();
  if (t.op == "NotIn") return !has || std::find(t.values.begin(), t.values.end(), it->second) == t.values.end();
  if ((t.op == "Gt" || t.op == "Lt") && has && !t.values.empty()) {
    try {
      const double a = std::stod(it->second), b = std::stod(t.values[0]);
      return t.op == "Gt" ? a > b : a < b;
    } catch (...) {
      return false;
    }
  }
  return false;
}

bool tolerated(const std::string& kv, const std::string& effect, const std::vector<Toleration>& ts) {
  auto eq = kv.find('=');
  const std::string key = kv.substr(0, eq);
  const std::string val = eq == std::string::npos ? "" : kv.substr(eq + 1);
  for (const auto& t : ts) {
    if (!t.effect.empty() && t.effect != effect) continue;
    if (t.op == "Exists" && (t.key.empty() || t.key == key)) return true;
    if (t.key == key && t.value == val) return true;
  }
  return false;
}

double pair_bw(const GpuDevice& a, const GpuDevice& b, bool* xgmi_up) {
  const XgmiLink* l1 = a.link_to(b.uuid);
  const XgmiLink* l2 = b.link_to(a.uuid);
  const bool up1 = l1 && l1->up && l1->type == LinkType::XGMI;
  const bool up2 = l2 ? (l2->up && l2->type == LinkType::XGMI) : up1;
  if (up1 && up2) {
    *xgmi_up = true;
    double bw = l1->effective_gbps();
    if (l2) bw = std::min(bw, l2->effective_gbps());
    return bw;
  }
  *xgmi_up = false;
  return std::min(a.pcie.bandwidth_gbps, b.pcie.bandwidth_gbps);
}

// Visit every k-combination of [0, n) (lexicographic), stop when f returns false.
void for_each_combination(int n, int k, const std::function<bool(const std::vector<int>&)>& f) {
  if (k > n || k <= 0) return;
  std::vector<int> idx(k);
  std::iota(idx.begin(), idx.end(), 0);
  for (;;) {
    if (!f(idx)) return;
    int i = k - 1;
    while (i >= 0 && idx[i] == n - k + i) --i;
    if (i < 0) return;
    ++idx[i];
    for (int j = i + 1; j < k; ++j) idx[j] = idx[j - 1] + 1;
  }
}

double n_choose_k(int n, int k) {
  if (k < 0 || k > n) return 0;
  double r = 1;
  for (int i = 1; i <= k; ++i) r = r * (n - k + i) / i;
  return r;
}

bool comm_heavy(DistributionStrategy s) {
  return s == DistributionStrategy::ModelParallel || s == DistributionStrategy::ContextParallel ||
         s == DistributionStrategy::ExpertParallel;
}

}  // namespace

// ---------------------------------------------------------------------------
// Scheduler
// ---------------------------------------------------------------------------
Scheduler::Scheduler(std::shared_ptr<DiscoveryService> disc, SchedulerConfig cfg)
    : disc_(std::move(disc)), cfg_(cfg) {}

void Scheduler::set_config(const SchedulerConfig& c) {
  std::unique_lock<RwLock> lk(mu_);
  cfg_ = c;
  global_gen_.fetch_add(1);
}

// Caller holds mu_ (shared or unique).
std::vector<const GpuDevice*> Scheduler::free_gpus(const NodeTopology& n,
                                                   const WorkloadRequest& w) const {
  std::vector<const GpuDevice*> out;
  for (const auto& g : n.gpus) {
    if (!g.healthy()) continue;
    if (g.partition.compute != ComputePartition::SPX || g.partition.switching) continue;
    if (gpu_owner_.count(g.uuid) || fenced_.count(g.uuid) || shared_.count(g.uuid)) continue;
    if (g.memory_free_gb() + 1e-9 < w.min_memory_gb) continue;
    if (!w.arch.empty() && g.arch != w.arch) continue;
    if (!w.model.empty() && g.model.find(w.model) == std::string::npos) continue;
    out.push_back(&g);
  }
  return out;
}

std::vector<const PartitionInstance*> Scheduler::free_partitions(
    const NodeTopology& n, const WorkloadRequest& w, std::vector<std::string>* gpu_of) const {
  std::vector<const PartitionInstance*> out;
  for (const auto& g : n.gpus) {
    if (!g.healthy() || g.partition.switching) continue;
    if (g.partition.compute != w.partition_mode) continue;
    if (w.partition_memory_set && g.partition.memory != w.partition_memory) continue;
    if (!w.arch.empty() && g.arch != w.arch) continue;
    if (gpu_owner_.count(g.uuid) || fenced_.count(g.uuid) || shared_.count(g.uuid))
      continue;  // whole GPU taken / shared / switching
    if (!draining_gpus_.empty() && draining_gpus_.count(g.uuid)) continue;  // consolidation donor
    for (const auto& pi : g.partition.instances) {
      if (pi.in_use || part_owner_.count(pi.id)) continue;
      if (pi.memory_gb + 1e-9 < w.min_memory_gb) continue;
      out.push_back(&pi);
      if (gpu_of) gpu_of->push_back(g.uuid);
    }
  }
  return out;
}

void Scheduler::set_cordon(const std::string& node, bool on) {
  std::lock_guard<std::mutex> lk(cordon_mu_);
  if (on) cordoned_.insert(node);
  else cordoned_.erase(node);
  global_gen_.fetch_add(1);
}

std::vector<std::string> Scheduler::cordoned() const {
  std::lock_guard<std::mutex> lk(cordon_mu_);
  return {cordoned_.begin(), cordoned_.end()};
}

// The constraints that no release of capacity changes: cordon, selectors,
// affinity, taints, placement relative to other workloads.
std::string Scheduler::admissible(const NodeTopology& n, const WorkloadRequest& w) const {
  {
    std::lock_guard<std::mutex> lk(cordon_mu_);
    if (!cordoned_.empty() && cordoned_.count(n.name)) return "node cordoned (not ready)";
  }
  if (std::find(w.exclude_nodes.begin(), w.exclude_nodes.end(), n.name) != w.exclude_nodes.end())
    return "node excluded by workload";
  for (const auto& kv : w.node_selector) {
    auto it = n.labels.find(kv.first);
    if (it == n.labels.end() || it->second != kv.second)
      return "node selector mismatch: " + kv.first + "=" + kv.second;
  }
  for (const auto& t : w.required_affinity)
    if (!term_matches(t, n.labels)) return "required node affinity not satisfied: " + t.key;
  for (const auto& t : n.taints) {
    if (t.second != "NoSchedule" && t.second != "NoExecute") continue;
    if (!tolerated(t.first, t.second, w.tolerations))
      return "untolerated taint " + t.first + ":" + t.second;
  }
  for (const auto& other : w.anti_affinity_with) {
    auto it = allocs_.find(other);
    if (it != allocs_.end() && it->second.node == n.name) return "anti-affinity with " + other;
  }
  for (const auto& other : w.colocate_with) {
    auto it = allocs_.find(other);
    if (it != allocs_.end() && it->second.node != n.name)
      return "must co-locate with " + other + " on " + it->second.node;
  }
  return "";
}

std::string Scheduler::eligible(const NodeTopology& n, const WorkloadRequest& w) const {
  std::string why = admissible(n, w);
  if (!why.empty()) return why;
  if (w.sharing != SharingMethod::None) {
    NodeScore tmp;
    if (!pick_share(n, w, &tmp))
      return std::string("no GPU can take a ") + to_string(w.sharing) + " client (" +
             std::to_string(w.share_cu_percent > 0 ? w.share_cu_percent : cfg_.default_cu_percent) +
             "% CUs, " + std::to_string(w.share_memory_gb) + " GB)";
    return "";
  }
  if (w.partition) {
    auto parts = free_partitions(n, w, nullptr);
    if (static_cast<int>(parts.size()) < w.partition_count)
      return "insufficient free " + std::string(to_string(w.partition_mode)) + " partitions (" +
             std::to_string(parts.size()) + " < " + std::to_string(w.partition_count) + ")";
    return "";
  }
  auto avail = free_gpus(n, w);
  if (static_cast<int>(avail.size()) < w.gpu_count)
    return "insufficient free GPUs (" + std::to_string(avail.size()) + " < " +
           std::to_string(w.gpu_count) + ")";
  const bool need_clique = w.topology == TopologyPreference::XgmiRequired ||
                           (comm_heavy(w.strategy) && w.topology == TopologyPreference::None);
  if (w.gpu_count > 1 && (need_clique || w.min_bandwidth_gbps > 0)) {
    std::vector<std::string> sel;
    double bw = 0.0;
    bool clique = false;
    topology_score(n, avail, w, &sel, &bw, &clique);
    if (need_clique && !clique) return "no fully connected xGMI group of " + std::to_string(w.gpu_count);
    if (w.min_bandwidth_gbps > 0) {
      // min pairwise bandwidth of the chosen group
      double mn = 1e30;
      for (size_t i = 0; i < sel.size(); ++i)
        for (size_t j = i + 1; j < sel.size(); ++j) {
          bool up = false;
          mn = std::min(mn, pair_bw(*n.gpu(sel[i]), *n.gpu(sel[j]), &up));
        }
      if (mn < w.min_bandwidth_gbps)
        return "group bandwidth " + std::to_string(static_cast<int>(mn)) + " GB/s < required " +
               std::to_string(static_cast<int>(w.min_bandwidth_gbps));
    }
  }
  return "";
}

// Memo of group searches.  A search's result depends only on the node's
// topology (links, NUMA, switches, health: NodeTopology::topo_fp), WHICH GPUs
// are free, the request size / preference and the scorer config — on a fleet
// of identical 8xMI355X nodes a 1,250-node prioritize repeats the same few
// searches thousands of times.  Thread-local: no lock on the hot path.
namespace {
struct TopoMemo {
  int score = 0;
  std::vector<int> positions;  // selected GPUs by position in NodeTopology::gpus
  double bw = 0.0;
  bool clique = false;
};
thread_local std::unordered_map<uint64_t, TopoMemo> t_topo_memo;
}  // namespace

int Scheduler::topology_score(const NodeTopology& n, const std::vector<const GpuDevice*>& avail,
                              const WorkloadRequest& w, std::vector<std::string>* sel, double* bw_out,
                              bool* clique_out) const {
  const size_t G = n.gpus.size();
  const bool indexed = n.topo_fp != 0 && n.link_bw.size() == G * G && G <= 64;
  uint64_t key = 0;
  if (indexed) {
    uint64_t mask = 0;
    for (auto* g : avail) mask |= 1ull << n.position(g);
    key = n.topo_fp;
    auto mix = [&key](uint64_t v) {
      key ^= v + 0x9e3779b97f4a7c15ull + (key << 6) + (key >> 2);
    };
    mix(mask);
    mix(static_cast<uint64_t>(w.gpu_count));
    mix(static_cast<uint64_t>(w.topology));
    mix(static_cast<uint64_t>(cfg_.rated_link_gbps * 1000));
    mix(static_cast<uint64_t>(cfg_.degraded_link_ratio * 1000));
    mix(cfg_.exhaustive_limit);
    auto it = t_topo_memo.find(key);
    if (it != t_topo_memo.end()) {
      sel->clear();
      for (int p : it->second.positions) sel->push_back(n.gpus[p].uuid);
      *bw_out = it->second.bw;
      *clique_out = it->second.clique;
      return it->second.score;
    }
  }
  const int score = topology_search(n, avail, w, sel, bw_out, clique_out);
  if (indexed) {
    if (t_topo_memo.size() > 65536) t_topo_memo.clear();
    TopoMemo mm;
    mm.score = score;
    mm.bw = *bw_out;
    mm.clique = *clique_out;
    for (const auto& u : *sel)
      for (size_t p = 0; p < G; ++p)
        if (n.gpus[p].uuid == u) mm.positions.push_back(static_cast<int>(p));
    t_topo_memo.emplace(key, std::move(mm));
  }
  return score;
}

int Scheduler::topology_search(const NodeTopology& n, const std::vector<const GpuDevice*>& avail,
                               const WorkloadRequest& w, std::vector<std::string>* sel, double* bw_out,
                               bool* clique_out) const {
  const int k = w.gpu_count;
  sel->clear();
  *bw_out = 0.0;
  *clique_out = false;
  if (static_cast<int>(avail.size()) < k || k <= 0) return 0;
  // Free GPUs per NUMA domain / PCIe switch (fragmentation + locality terms).
  std::map<int, int> free_numa, total_numa;
  for (const auto& g : n.gpus) total_numa[g.numa_node]++;
  for (auto* g : avail) free_numa[g->numa_node]++;

  if (k == 1) {
    // Best fit: the GPU in the NUMA domain with the FEWEST free GPUs (keeps
    // whole domains / large cliques free), then the one with the most
    // degraded links (least useful for future multi-GPU jobs).
    const GpuDevice* best = nullptr;
    std::tuple<int, int, int> bkey{1 << 30, 0, 0};
    for (auto* g : avail) {
      int degraded = 0;
      for (const auto& l : g->links)
        if (!l.up || (l.measured_gbps > 0 && l.measured_gbps < cfg_.degraded_link_ratio * l.rated_gbps))
          ++degraded;
      std::tuple<int, int, int> key{free_numa[g->numa_node], -degraded, g->index};
      if (!best || key < bkey) {
        best = g;
        bkey = key;
      }
    }
    sel->push_back(best->uuid);
    *clique_out = true;
    return 100;
  }

  const int m = static_cast<int>(avail.size());
  // Minimal number of NUMA domains a k-group can span.
  std::vector<int> sizes;
  for (auto& kv : free_numa) sizes.push_back(kv.second);
  std::sort(sizes.rbegin(), sizes.rend());
  int need_domains = 0;
  for (int acc = 0; acc < k && need_domains < static_cast<int>(sizes.size()); ++need_domains)
    acc += sizes[need_domains];

  // Dense per-call tables, so the (up to exhaustive_limit) candidate groups
  // are scored with array lookups only: pairwise effective bandwidth / xGMI
  // up-ness (pair_bw resolves links by uuid), NUMA domain and PCIe switch of
  // every free GPU as small integers.
  std::vector<double> bwm(static_cast<size_t>(m) * m, 0.0);
  std::vector<char> upm(static_cast<size_t>(m) * m, 0);
  const size_t G = n.gpus.size();
  const bool indexed = n.link_bw.size() == G * G;
  for (int i = 0; i < m; ++i)
    for (int j = i + 1; j < m; ++j) {
      bool up = false;
      double bw;
      if (indexed) {  // dense table built with the snapshot (index_links)
        const size_t a = static_cast<size_t>(n.position(avail[i])), b = static_cast<size_t>(n.position(avail[j]));
        bw = n.link_bw[a * G + b];
        up = n.link_up[a * G + b] != 0;
      } else {
        bw = pair_bw(*avail[i], *avail[j], &up);
      }
      bwm[i * m + j] = bwm[j * m + i] = bw;
      upm[i * m + j] = upm[j * m + i] = up;
    }
  std::vector<int> dom_of(m), sw_of(m);
  std::vector<int> dom_ids;  // numa node -> dense index
  std::vector<std::string> sw_ids;
  for (int i = 0; i < m; ++i) {
    auto d = std::find(dom_ids.begin(), dom_ids.end(), avail[i]->numa_node);
    dom_of[i] = static_cast<int>(d - dom_ids.begin());
    if (d == dom_ids.end()) dom_ids.push_back(avail[i]->numa_node);
    auto sw = std::find(sw_ids.begin(), sw_ids.end(), avail[i]->pcie.switch_id);
    sw_of[i] = static_cast<int>(sw - sw_ids.begin());
    if (sw == sw_ids.end()) sw_ids.push_back(avail[i]->pcie.switch_id);
  }
  const int ndom = static_cast<int>(dom_ids.size());
  std::vector<int> dom_free(ndom), dom_total(ndom, 0);
  for (int d = 0; d < ndom; ++d) {
    dom_free[d] = free_numa[dom_ids[d]];
    dom_total[d] = total_numa[dom_ids[d]];
  }
  // Domains with no free GPU can never become "whole free" after placement.
  int whole_free_elsewhere = 0;
  for (auto& kv : total_numa)
    if (std::find(dom_ids.begin(), dom_ids.end(), kv.first) == dom_ids.end() && kv.second == 0)
      ++whole_free_elsewhere;

  struct Best {
    double obj = -1e30;
    std::vector<int> idx;
    double agg = 0, minbw = 0;
    bool clique = false;
    int domains = 0;
  } best;
  const double ideal = cfg_.rated_link_gbps * k * (k - 1) / 2.0;
  std::vector<int> used(ndom);
  auto evaluate = [&](const std::vector<int>& idx) {
    double agg = 0.0, minbw = 1e30;
    bool clique = true;
    std::fill(used.begin(), used.end(), 0);
    uint64_t swmask = 0;
    bool multi_sw = false;
    for (size_t i = 0; i < idx.size(); ++i) {
      const int a = idx[i];
      used[dom_of[a]]++;
      if (sw_of[a] < 64) swmask |= 1ull << sw_of[a];
      else multi_sw = true;
      const double* row = &bwm[static_cast<size_t>(a) * m];
      const char* urow = &upm[static_cast<size_t>(a) * m];
      for (size_t j = i + 1; j < idx.size(); ++j) {
        clique &= urow[idx[j]] != 0;
        agg += row[idx[j]];
        minbw = std::min(minbw, row[idx[j]]);
      }
    }
    int domains = 0, whole_free_after = whole_free_elsewhere;
    for (int d = 0; d < ndom; ++d) {
      domains += used[d] > 0;
      if (dom_free[d] - used[d] == dom_total[d]) ++whole_free_after;  // domain left completely free
    }
    double obj = (clique ? 1000.0 : 0.0) + 300.0 * std::min(1.0, agg / ideal) +
                 100.0 * (need_domains > 0 ? static_cast<double>(need_domains) / domains : 1.0) +
                 20.0 * whole_free_after + 5.0 * (minbw / cfg_.rated_link_gbps);
    if (w.topology == TopologyPreference::SamePCIeSwitch)
      obj += (!multi_sw && __builtin_popcountll(swmask) == 1) ? 500.0 : 0.0;
    if (w.topology == TopologyPreference::SameNUMA) obj += domains == 1 ? 500.0 : 0.0;
    if (obj > best.obj) {
      best.obj = obj;
      best.idx = idx;
      best.agg = agg;
      best.minbw = minbw;
      best.clique = clique;
      best.domains = domains;
    }
    return true;
  };
  if (n_choose_k(m, k) <= static_cast<double>(cfg_.exhaustive_limit)) {
    for_each_combination(m, k, evaluate);
  } else {
    // Greedy clique growth from every start GPU (reference-style search,
    // but on effective bandwidth and with the same objective to pick).
    for (int s0 = 0; s0 < m; ++s0) {
      std::vector<int> grp{s0};
      std::vector<bool> in(m, false);
      in[s0] = true;
      while (static_cast<int>(grp.size()) < k) {
        int pick = -1;
        double pick_bw = -1;
        for (int c = 0; c < m; ++c) {
          if (in[c]) continue;
          double aggc = 0;
          bool ok = true;
          for (int g : grp) {
            aggc += bwm[static_cast<size_t>(c) * m + g];
            ok &= upm[static_cast<size_t>(c) * m + g] != 0;
          }
          double keyv = (ok ? 1e6 : 0) + aggc + (dom_of[c] == dom_of[s0] ? 1 : 0);
          if (keyv > pick_bw) {
            pick = c;
            pick_bw = keyv;
          }
        }
        grp.push_back(pick);
        in[pick] = true;
      }
      std::sort(grp.begin(), grp.end());
      evaluate(grp);
    }
  }
  for (int i : best.idx) sel->push_back(avail[i]->uuid);
  const int pairs = k * (k - 1) / 2;
  *bw_out = pairs ? best.agg / pairs : 0.0;
  *clique_out = best.clique;
  const double bwn = std::min(1.0, best.agg / ideal);
  const double numa_term = need_domains > 0 ? static_cast<double>(need_domains) / best.domains : 1.0;
  switch (w.topology) {
    case TopologyPreference::None:
      return 50;
    case TopologyPreference::SameNUMA:
      return best.domains == 1 ? 90 : 50;
    case TopologyPreference::SamePCIeSwitch: {
      std::set<std::string> sw;
      for (int i : best.idx) sw.insert(avail[i]->pcie.switch_id);
      return sw.size() == 1 ? 80 : 40;
    }
    default:
      break;
  }
  if (!best.clique) return static_cast<int>(30.0 * bwn);
  return static_cast<int>(std::lround(60.0 + 25.0 * bwn + 15.0 * numa_term));
}

// The reference's scorer, kept verbatim in behaviour for A/B (ScoringMode::Compat):
// NVLink-style greedy clique normalised to 900 GB/s per pair, NUMA 90/50,
// PCIe switch 80/40, None 50 with the first k GPUs.
int Scheduler::topology_score_compat(const NodeTopology& n,
                                     const std::vector<const GpuDevice*>& avail,
                                     const WorkloadRequest& w, std::vector<std::string>* sel) const {
  const int k = w.gpu_count;
  sel->clear();
  if (k <= 1) {
    if (avail.empty()) return 0;
    sel->push_back(avail[0]->uuid);
    return 100;
  }
  if (static_cast<int>(avail.size()) < k) return 0;
  auto first_k = [&]() {
    for (int i = 0; i < k; ++i) sel->push_back(avail[i]->uuid);
  };
  switch (w.topology) {
    case TopologyPreference::XgmiOptimal:
    case TopologyPreference::XgmiRequired: {
      std::vector<std::string> best;
      double best_bw = 0.0;
      for (auto* start : avail) {
        std::vector<const GpuDevice*> grp{start};
        double tot = 0.0;
        while (static_cast<int>(grp.size()) < k) {
          const GpuDevice* cand = nullptr;
          double cand_bw = 0.0;
          for (auto* c : avail) {
            if (std::find(grp.begin(), grp.end(), c) != grp.end()) continue;
            double agg = 0.0;
            bool full = true;
            for (auto* m : grp) {
              const XgmiLink* l = c->link_to(m->uuid);
              if (l && l->up) agg += l->effective_gbps();
              else full = false;
            }
            if (full && agg > cand_bw) {
              cand = c;
              cand_bw = agg;
            }
          }
          if (!cand) break;
          grp.push_back(cand);
          tot += cand_bw;
        }
        if (static_cast<int>(grp.size()) >= k && tot > best_bw) {
          best.clear();
          for (auto* g : grp) best.push_back(g->uuid);
          best_bw = tot;
        }
      }
      if (static_cast<int>(best.size()) < k) {
        first_k();
        return 30;
      }
      *sel = best;
      return static_cast<int>(50 + 50 * best_bw / (900.0 * (k * (k - 1) / 2)));
    }
    case TopologyPreference::SameNUMA: {
      std::map<int, std::vector<const GpuDevice*>> groups;
      for (auto* g : avail) groups[g->numa_node].push_back(g);
      for (auto& kv : groups)
        if (static_cast<int>(kv.second.size()) >= k) {
          for (int i = 0; i < k; ++i) sel->push_back(kv.second[i]->uuid);
          return 90;
        }
      first_k();
      return 50;
    }
    case TopologyPreference::SamePCIeSwitch: {
      std::map<std::string, std::vector<const GpuDevice*>> groups;
      for (auto* g : avail) groups[g->pcie.switch_id.empty() ? "default" : g->pcie.switch_id].push_back(g);
      for (auto& kv : groups)
        if (static_cast<int>(kv.second.size()) >= k) {
          for (int i = 0; i < k; ++i) sel->push_back(kv.second[i]->uuid);
          return 80;
        }
      first_k();
      return 40;
    }
    default:
      first_k();
      return 50;
  }
}

int Scheduler::resource_score(const std::vector<const GpuDevice*>& avail,
                              const WorkloadRequest& w) const {
  if (avail.empty()) return 0;
  int score = 50;
  double free_gb = 0.0, util = 0.0;
  for (auto* g : avail) {
    free_gb += g->memory_free_gb();
    util += g->util.gfx_activity;
  }
  util /= static_cast<double>(avail.size());
  const double need = w.min_memory_gb * std::max(1, w.gpu_count);
  if (free_gb >= 2 * need) score += 25;
  else if (free_gb >= need) score += 10;
  if (util < 30) score += 25;
  else if (util < 60) score += 10;
  return std::min(100, score);
}

int Scheduler::balance_score(const NodeTopology& n, int requested) const {
  if (n.gpus.empty()) return 0;
  double used;
  if (cfg_.mode == ScoringMode::Compat) {
    int allocs = 0;  // reference counts WORKLOADS on the node
    for (const auto& kv : allocs_) allocs += kv.second.node == n.name;
    used = allocs;
  } else {
    auto it = node_gpus_used_.find(n.name);
    used = it == node_gpus_used_.end() ? 0 : it->second;
  }
  if (cfg_.mode != ScoringMode::Compat && cfg_.pack) {
    // Best fit across nodes: prefer the node that is fullest AFTER this
    // placement, so whole 8-GPU xGMI islands stay free for FSDP/TP jobs
    // (spreading small jobs fragments every node and makes 8-GPU jobs wait).
    return std::min(100, static_cast<int>(100.0 * (used + requested) / n.gpus.size()));
  }
  return std::max(0, static_cast<int>(100.0 * (1.0 - used / n.gpus.size())));
}

double Scheduler::bandwidth_of(const NodeTopology& n, const std::vector<std::string>& gpus) const {
  double sum = 0;
  int pairs = 0;
  for (size_t i = 0; i < gpus.size(); ++i)
    for (size_t j = i + 1; j < gpus.size(); ++j) {
      const GpuDevice* a = n.gpu(gpus[i]);
      const GpuDevice* b = n.gpu(gpus[j]);
      if (!a || !b) continue;
      bool up = false;
      sum += pair_bw(*a, *b, &up);
      ++pairs;
    }
  return pairs ? sum / pairs : 0.0;
}

// Caller holds mu_.  Can GPU g take the sharing client w?  CoLocate clients
// get a disjoint CU range rounded to whole XCDs (32 CUs share one L2) when
// the request is at least an XCD; TimeSlice clients share the whole GPU.
bool Scheduler::share_fits(const GpuDevice& g, const WorkloadRequest& w, int* cu_begin, int* cu_end) const {
  if (!g.healthy() || g.partition.compute != ComputePartition::SPX || g.partition.switching) return false;
  if (gpu_owner_.count(g.uuid) || fenced_.count(g.uuid) || gpu_has_slice_owner_locked(g.uuid)) return false;
  if (!w.arch.empty() && g.arch != w.arch) return false;
  std::vector<const Allocation*> clients;
  auto sh = shared_.find(g.uuid);
  if (sh != shared_.end()) {
    if (sh->second.method != w.sharing) return false;  // one method per GPU
    for (const auto& uid : sh->second.clients) {
      auto it = allocs_.find(uid);
      if (it != allocs_.end()) clients.push_back(&it->second);
    }
  }
  if (!w.share_group.empty()) {
    // Join the group's share on this GPU: its CU range and HBM cap, no new ones.
    int members = 0;
    const Allocation* lead = nullptr;
    for (auto* c : clients)
      if (c->share_group == w.share_group) {
        ++members;
        if (c->share_leader || !lead) lead = c;
      }
    if (lead) {
      if (!lead->share_leader) return false;  // the group's server is gone: its orphans are being evicted
      if (members >= cfg_.max_group_clients) return false;
      *cu_begin = lead->cu_begin;
      *cu_end = lead->cu_end;
      return true;
    }
  }
  // A group counts as one client of the GPU.
  {
    std::set<std::string> groups;
    std::vector<const Allocation*> distinct;
    for (auto* c : clients)
      if (c->share_group.empty() || groups.insert(c->share_group).second) distinct.push_back(c);
    clients.swap(distinct);  // (members carry no HBM cap of their own: the leader's covers the group)
  }
  double mem = 0.0;
  for (auto* c : clients) mem += c->share_memory_gb;
  const double cap = g.memory_total_gb > 0 ? g.memory_total_gb : 288.0;
  if (w.share_memory_gb > 0 && mem + w.share_memory_gb > cap + 1e-9) return false;
  // HBM the device reports in use beyond what the ledger's clients were
  // promised (another tenant, a leak) is not there for a new client either.
  if (w.share_memory_gb > 0 && g.memory_total_gb > 0) {
    const double unaccounted = std::max(0.0, g.memory_used_gb - mem);
    if (mem + unaccounted + w.share_memory_gb > cap + 1e-9) return false;
  }
  if (w.sharing == SharingMethod::TimeSlice) {
    if (static_cast<int>(clients.size()) >= cfg_.max_timeslice_replicas) return false;
    *cu_begin = 0;
    *cu_end = g.cu_count > 0 ? g.cu_count : 256;
    return true;
  }
  if (static_cast<int>(clients.size()) >= cfg_.max_share_clients) return false;
  const int cus = g.cu_count > 0 ? g.cu_count : 256;
  const int xcds = g.xcd_count > 0 ? g.xcd_count : 8;
  const int per_xcd = cus / xcds;
  const double pct = w.share_cu_percent > 0 ? w.share_cu_percent : cfg_.default_cu_percent;
  int want = std::max(1, static_cast<int>(std::lround(cus * pct / 100.0)));
  if (want >= per_xcd) want = (want + per_xcd - 1) / per_xcd * per_xcd;
  if (want > cus) return false;
  std::vector<std::pair<int, int>> used;
  for (auto* c : clients) used.emplace_back(c->cu_begin, c->cu_end);
  std::sort(used.begin(), used.end());
  // Best fit among the free gaps (smallest gap that holds `want`), aligned to
  // an XCD boundary when the request is XCD-sized.
  const int align = want % per_xcd == 0 ? per_xcd : 1;
  int best = -1, best_gap = 1 << 30, start = 0;
  auto consider = [&](int lo, int hi) {
    lo = (lo + align - 1) / align * align;
    if (hi - lo >= want && hi - lo < best_gap) {
      best = lo;
      best_gap = hi - lo;
    }
  };
  for (const auto& u : used) {
    consider(start, u.first);
    start = std::max(start, u.second);
  }
  consider(start, cus);
  if (best < 0) return false;
  *cu_begin = best;
  *cu_end = best + want;
  return true;
}

// Caller holds mu_.  Best fit: join the most loaded compatible shared GPU
// (fewest CUs left after placement); open a fresh whole GPU only when none
// has room — so whole GPUs stay free for training jobs.
bool Scheduler::pick_share(const NodeTopology& n, const WorkloadRequest& w, NodeScore* s) const {
  const GpuDevice* best = nullptr;
  std::tuple<int, int, int> bkey{1, 0, 0};  // (fresh GPU?, -clients, index)
  int bb = 0, be = 0;
  for (const auto& g : n.gpus) {
    int b = 0, e = 0;
    if (!share_fits(g, w, &b, &e)) continue;
    auto sh = shared_.find(g.uuid);
    const int clients = sh == shared_.end() ? 0 : static_cast<int>(sh->second.clients.size());
    std::tuple<int, int, int> key{clients == 0 ? 1 : 0, -clients, g.index};
    if (!w.share_group.empty() && sh != shared_.end())
      for (const auto& uid : sh->second.clients) {
        auto it = allocs_.find(uid);
        if (it != allocs_.end() && it->second.share_group == w.share_group) std::get<0>(key) = -1;  // its group is here
      }
    if (!best || key < bkey) {
      best = &g;
      bkey = key;
      bb = b;
      be = e;
    }
  }
  if (!best) return false;
  s->shared_gpu = best->uuid;
  s->cu_begin = bb;
  s->cu_end = be;
  return true;
}

NodeScore Scheduler::score_node(const NodeTopology& n, const WorkloadRequest& w) const {
  NodeScore s;
  s.node = n.name;
  int group_bonus = 0;
  if (w.sharing != SharingMethod::None) {
    if (!pick_share(n, w, &s)) return s;
    auto sh = shared_.find(s.shared_gpu);
    const int clients = sh == shared_.end() ? 0 : static_cast<int>(sh->second.clients.size());
    s.topology = 100;
    s.resource = clients > 0 ? 100 : 50;  // packing onto already-shared GPUs
    s.balance = balance_score(n, clients > 0 ? 0 : 1);
    if (!w.share_group.empty() && sh != shared_.end())
      for (const auto& uid : sh->second.clients) {
        auto it = allocs_.find(uid);
        if (it != allocs_.end() && it->second.share_group == w.share_group && group_bonus == 0) {
          group_bonus = 30;  // join the group's server rather than start a second one elsewhere
          s.reasons.push_back("share group " + w.share_group + " is served on this GPU");
        }
      }
  } else if (w.partition) {
    std::vector<std::string> gpu_of;
    auto parts = free_partitions(n, w, &gpu_of);
    if (static_cast<int>(parts.size()) < w.partition_count) return s;
    // Best fit: fill GPUs that already have the most slices in use.
    std::map<std::string, int> used_on;
    for (const auto& g : n.gpus)
      for (const auto& pi : g.partition.instances)
        used_on[g.uuid] += (pi.in_use || part_owner_.count(pi.id)) ? 1 : 0;
    std::vector<size_t> order(parts.size());
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
      return used_on[gpu_of[a]] > used_on[gpu_of[b]];
    });
    for (int i = 0; i < w.partition_count; ++i) s.partitions.push_back(parts[order[i]]->id);
    // Best fit across the fleet: the score is how full the GPU that takes the
    // (first) slice is afterwards, so slice pods fill the fullest partitioned
    // GPU anywhere and the emptiest ones drain and go back to SPX.  Slices on
    // an existing partition take no whole GPU from the node, so the node's
    // whole-GPU balance does not enter.
    const std::string& target = gpu_of[order[0]];
    int on_target = 0, target_slices = 0;
    for (int i = 0; i < w.partition_count; ++i) on_target += gpu_of[order[i]] == target;
    if (const GpuDevice* tg = n.gpu(target)) target_slices = static_cast<int>(tg->partition.instances.size());
    const int fullness = target_slices ? 100 * (used_on[target] + on_target) / target_slices : 0;
    s.topology = 100;
    s.resource = std::min(100, fullness);
    s.balance = s.resource;
  } else {
    auto avail = free_gpus(n, w);
    if (static_cast<int>(avail.size()) < w.gpu_count) return s;
    bool clique = false;
    if (cfg_.mode == ScoringMode::Compat) {
      s.topology = topology_score_compat(n, avail, w, &s.gpus);
      s.bandwidth_gbps = bandwidth_of(n, s.gpus);
    } else {
      s.topology = topology_score(n, avail, w, &s.gpus, &s.bandwidth_gbps, &clique);
    }
    s.resource = resource_score(avail, w);
    s.balance = balance_score(n, w.gpu_count);
  }
  s.total = (s.topology * cfg_.topology_weight + s.resource * cfg_.resource_weight +
             s.balance * cfg_.balance_weight) / 100;
  s.total += group_bonus;
  if (std::find(w.preferred_nodes.begin(), w.preferred_nodes.end(), n.name) != w.preferred_nodes.end()) {
    s.total += 10;
    s.reasons.push_back("workload optimizer prefers this node");
  }
  int wsum = 0, wmatch = 0;
  for (const auto& t : w.preferred_affinity) {
    wsum += std::max(1, t.weight);
    if (term_matches(t, n.labels)) wmatch += std::max(1, t.weight);
  }
  if (wsum) {
    s.affinity = 10 * wmatch / wsum;
    s.total += s.affinity;
  }
  if (s.topology >= 80) s.reasons.push_back(w.gpu_count > 1 ? "optimal xGMI connectivity" : "single GPU, best-fit placement");
  if (s.resource >= 80) s.reasons.push_back("sufficient resources with headroom");
  if (s.balance >= 80) s.reasons.push_back("good load distribution");
  return s;
}

// ---------------------------------------------------------------------------
// Per-node verdict / score memo (see NodeCache in scheduler.h).
// ---------------------------------------------------------------------------
Scheduler::NodeCache& Scheduler::cache_of(const std::string& node) const {
  {
    std::shared_lock<std::shared_mutex> lk(cache_map_mu_);
    auto it = node_cache_.find(node);
    if (it != node_cache_.end()) return *it->second;
  }
  std::unique_lock<std::shared_mutex> lk(cache_map_mu_);
  auto& p = node_cache_[node];
  if (!p) p = std::make_unique<NodeCache>();
  return *p;
}

void Scheduler::touch_node(const std::string& node) {
  cache_of(node).epoch.fetch_add(1, std::memory_order_release);
}

uint64_t Scheduler::request_signature(const WorkloadRequest& w) {
  if (!w.anti_affinity_with.empty() || !w.colocate_with.empty()) return 0;
  uint64_t h = 1469598103934665603ull;
  auto bytes = [&h](const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  };
  auto num = [&](double v) { bytes(&v, sizeof v); };
  auto str = [&](const std::string& s) {
    bytes(s.data(), s.size());
    const unsigned char sep = 0xff;
    bytes(&sep, 1);
  };
  num(w.gpu_count);
  num(w.min_memory_gb);
  num(w.min_bandwidth_gbps);
  num(static_cast<int>(w.topology));
  str(w.arch);
  str(w.model);
  num(w.partition);
  num(static_cast<int>(w.partition_mode));
  num(w.partition_count);
  num(w.partition_memory_set);
  num(static_cast<int>(w.partition_memory));
  num(static_cast<int>(w.strategy));
  num(static_cast<int>(w.sharing));
  num(w.share_cu_percent);
  num(w.share_memory_gb);
  str(w.share_group);
  for (const auto& kv : w.node_selector) {
    str(kv.first);
    str(kv.second);
  }
  for (const auto* terms : {&w.required_affinity, &w.preferred_affinity}) {
    num(static_cast<double>(terms->size()));
    for (const auto& t : *terms) {
      str(t.key);
      str(t.op);
      num(t.weight);
      for (const auto& v : t.values) str(v);
    }
  }
  for (const auto& t : w.tolerations) {
    str(t.key);
    str(t.op);
    str(t.value);
    str(t.effect);
  }
  num(static_cast<double>(w.exclude_nodes.size()));
  for (const auto& n : w.exclude_nodes) str(n);
  num(static_cast<double>(w.preferred_nodes.size()));
  for (const auto& n : w.preferred_nodes) str(n);
  return (h && h != ~0ull) ? h : 1;
}

// Caller holds mu_ (shared or unique).  Returns the verdict ("" = eligible);
// the reference stays valid until the next call with the same scratch.
const std::string& Scheduler::eligible_cached(const NodeTopology& n, const WorkloadRequest& w, uint64_t sig,
                                              std::string* scratch) const {
  if (sig == 0) {
    *scratch = eligible(n, w);
    return *scratch;
  }
  NodeCache& c = cache_of(n.name);
  const uint64_t epoch = c.epoch.load(std::memory_order_acquire);
  const uint64_t gen = global_gen_.load(std::memory_order_acquire);
  {
    std::lock_guard<std::mutex> lk(c.mu);
    for (auto& e : c.entries)
      if (e.sig == sig && e.epoch == epoch && e.gen == gen && e.topo == &n && e.topo_ns == n.updated_ns &&
          e.has_why) {
        e.used = ++c.clock;
        *scratch = e.why;
        return *scratch;
      }
  }
  *scratch = eligible(n, w);
  std::lock_guard<std::mutex> lk(c.mu);
  NodeCacheEntry* slot = nullptr;
  for (auto& e : c.entries)
    if (e.sig == sig) slot = &e;
  if (!slot) {
    if (c.entries.size() < 12) {
      c.entries.emplace_back();
      slot = &c.entries.back();
    } else {
      slot = &*std::min_element(c.entries.begin(), c.entries.end(),
                                [](const NodeCacheEntry& a, const NodeCacheEntry& b) { return a.used < b.used; });
    }
    *slot = NodeCacheEntry();
  }
  if (slot->epoch != epoch || slot->gen != gen || slot->topo != &n || slot->topo_ns != n.updated_ns)
    slot->has_total = false;
  slot->sig = sig;
  slot->epoch = epoch;
  slot->gen = gen;
  slot->topo = &n;
  slot->topo_ns = n.updated_ns;
  slot->has_why = true;
  slot->why = *scratch;
  slot->used = ++c.clock;
  return *scratch;
}

// Caller holds mu_.  Total score of an ELIGIBLE node (0 when nothing fits).
int Scheduler::total_cached(const NodeTopology& n, const WorkloadRequest& w, uint64_t sig) const {
  if (sig == 0) return score_node(n, w).total;
  NodeCache& c = cache_of(n.name);
  const uint64_t epoch = c.epoch.load(std::memory_order_acquire);
  const uint64_t gen = global_gen_.load(std::memory_order_acquire);
  {
    std::lock_guard<std::mutex> lk(c.mu);
    for (auto& e : c.entries)
      if (e.sig == sig && e.epoch == epoch && e.gen == gen && e.topo == &n && e.topo_ns == n.updated_ns &&
          e.has_total) {
        e.used = ++c.clock;
        return e.total;
      }
  }
  const int total = score_node(n, w).total;
  std::lock_guard<std::mutex> lk(c.mu);
  NodeCacheEntry* slot = nullptr;
  for (auto& e : c.entries)
    if (e.sig == sig) slot = &e;
  if (!slot) {
    if (c.entries.size() < 12) {
      c.entries.emplace_back();
      slot = &c.entries.back();
    } else {
      slot = &*std::min_element(c.entries.begin(), c.entries.end(),
                                [](const NodeCacheEntry& a, const NodeCacheEntry& b) { return a.used < b.used; });
    }
    *slot = NodeCacheEntry();
  }
  if (slot->epoch != epoch || slot->gen != gen || slot->topo != &n || slot->topo_ns != n.updated_ns)
    slot->has_why = false;
  slot->sig = sig;
  slot->epoch = epoch;
  slot->gen = gen;
  slot->topo = &n;
  slot->topo_ns = n.updated_ns;
  slot->has_total = true;
  slot->total = total;
  slot->used = ++c.clock;
  return total;
}

Scheduler::NodeSummary Scheduler::node_summary(const NodeTopology& n) const {
  constexpr uint64_t kSig = ~0ull;  // reserved signature of the summary entry
  NodeCache& c = cache_of(n.name);
  std::shared_lock<RwLock> lk(mu_);
  const uint64_t epoch = c.epoch.load(std::memory_order_acquire);
  const uint64_t gen = global_gen_.load(std::memory_order_acquire);
  {
    std::lock_guard<std::mutex> ck(c.mu);
    for (auto& e : c.entries)
      if (e.sig == kSig && e.epoch == epoch && e.gen == gen && e.topo == &n && e.topo_ns == n.updated_ns &&
          e.has_summary) {
        e.used = ++c.clock;
        return e.summary;
      }
  }
  NodeSummary out;
  out.free_slices.assign(n.gpus.size(), 0);
  for (size_t p = 0; p < n.gpus.size(); ++p) {
    const GpuDevice& g = n.gpus[p];
    if (!g.healthy() || g.partition.switching) continue;
    const bool whole = gpu_owner_.count(g.uuid) || shared_.count(g.uuid) || fenced_.count(g.uuid);
    bool any_busy = whole;
    int free_n = 0;
    for (const auto& pi : g.partition.instances) {
      const bool taken = pi.in_use || (!part_owner_.empty() && part_owner_.count(pi.id));
      any_busy |= taken;
      free_n += taken ? 0 : 1;
    }
    out.free_slices[p] = whole || draining_gpus_.count(g.uuid) ? 0 : static_cast<uint8_t>(std::min(free_n, 255));
    if (!any_busy && g.util.gfx_activity < 5.0 && p < 64) out.idle_mask |= 1ull << p;
  }
  std::lock_guard<std::mutex> ck(c.mu);
  NodeCacheEntry* slot = nullptr;
  for (auto& e : c.entries)
    if (e.sig == kSig) slot = &e;
  if (!slot) {
    if (c.entries.size() < 12) {
      c.entries.emplace_back();
      slot = &c.entries.back();
    } else {
      slot = &*std::min_element(c.entries.begin(), c.entries.end(),
                                [](const NodeCacheEntry& a, const NodeCacheEntry& b) { return a.used < b.used; });
    }
  }
  *slot = NodeCacheEntry();
  slot->sig = kSig;
  slot->epoch = epoch;
  slot->gen = gen;
  slot->topo = &n;
  slot->topo_ns = n.updated_ns;
  slot->has_summary = true;
  slot->summary = out;
  slot->used = ++c.clock;
  return out;
}

void Scheduler::filter_verdicts(const WorkloadRequest& w, const std::vector<std::string>& nodes,
                                std::vector<std::string>* why) {
  why->assign(nodes.size(), std::string());
  auto snap = disc_->snapshot();
  const uint64_t sig = request_signature(w);
  std::string scratch;
  // The ledger is read in chunks of kSweepChunk nodes: a sweep over 1,250
  // candidates must not hold binds / releases off the ledger for its whole
  // length (each node's verdict is advisory anyway: bind re-checks).
  std::shared_lock<RwLock> lk(mu_);
  auto mine = allocs_.find(w.uid);
  for (size_t i = 0; i < nodes.size(); ++i) {
    if ((i + 1) % kSweepChunk == 0) {
      lk.unlock();
      lk.lock();
      mine = allocs_.find(w.uid);
    }
    const std::string& name = nodes[i];
    auto it = snap->nodes.find(name);
    if (it == snap->nodes.end()) {
      (*why)[i] = "node not managed by kgwe (no MI355X topology)";
      continue;
    }
    if (mine != allocs_.end()) {  // already reserved (gang member / retry): only that node
      if (mine->second.node != name) (*why)[i] = "workload already reserved on " + mine->second.node;
      continue;
    }
    const std::string& v = eligible_cached(it->second, w, sig, &scratch);
    if (!v.empty()) (*why)[i] = v;
  }
}

void Scheduler::prioritize_totals(const WorkloadRequest& w, const std::vector<std::string>& nodes,
                                  std::vector<int>* totals) {
  totals->assign(nodes.size(), 0);
  auto snap = disc_->snapshot();
  const uint64_t sig = request_signature(w);
  std::string scratch;
  std::shared_lock<RwLock> lk(mu_);
  for (size_t i = 0; i < nodes.size(); ++i) {
    if ((i + 1) % kSweepChunk == 0) {  // see filter_verdicts()
      lk.unlock();
      lk.lock();
    }
    auto it = snap->nodes.find(nodes[i]);
    if (it == snap->nodes.end()) continue;
    if (!eligible_cached(it->second, w, sig, &scratch).empty()) continue;
    (*totals)[i] = total_cached(it->second, w, sig);
  }
}

bool Scheduler::gpu_has_slice_owner_locked(const std::string& gpu_uuid) const {
  if (part_owner_.empty()) return false;
  for (int i = 0; i < 8; ++i)  // slice ids are "<uuid>/p<i>", at most 8 (CPX)
    if (part_owner_.count(gpu_uuid + "/p" + std::to_string(i))) return true;
  return false;
}

bool Scheduler::fence_gpu(const std::string& gpu_uuid, const std::string& node) {
  std::unique_lock<RwLock> lk(mu_);
  if (gpu_owner_.count(gpu_uuid) || gpu_has_slice_owner_locked(gpu_uuid) || fenced_.count(gpu_uuid) ||
      shared_.count(gpu_uuid))
    return false;
  fenced_.insert(gpu_uuid);
  if (node.empty()) global_gen_.fetch_add(1);
  else touch_node(node);
  return true;
}

void Scheduler::set_draining(const std::string& gpu_uuid, const std::string& node, bool on) {
  std::unique_lock<RwLock> lk(mu_);
  const bool changed = on ? draining_gpus_.insert(gpu_uuid).second : draining_gpus_.erase(gpu_uuid) > 0;
  if (!changed) return;
  if (node.empty()) global_gen_.fetch_add(1);
  else touch_node(node);
}

std::vector<std::string> Scheduler::draining() const {
  std::shared_lock<RwLock> lk(mu_);
  return {draining_gpus_.begin(), draining_gpus_.end()};
}

void Scheduler::unfence_gpu(const std::string& gpu_uuid, const std::string& node) {
  std::unique_lock<RwLock> lk(mu_);
  fenced_.erase(gpu_uuid);
  if (node.empty()) global_gen_.fetch_add(1);
  else touch_node(node);
}

// Caller holds mu_ exclusively.  The score may come from an older topology
// snapshot than the ledger: a whole GPU is only reservable when none of its
// slices is held, a slice only when its GPU is not held whole, and neither
// while the GPU is fenced for a partition switch.
bool Scheduler::reserve_locked(const WorkloadRequest& w, const NodeScore& s, bool gang_pending) {
  for (const auto& g : s.gpus)
    if (gpu_owner_.count(g) || fenced_.count(g) || gpu_has_slice_owner_locked(g) || shared_.count(g))
      return false;
  for (const auto& p : s.partitions) {
    if (part_owner_.count(p)) return false;
    const std::string gpu = p.substr(0, p.rfind("/p"));
    if (gpu_owner_.count(gpu) || fenced_.count(gpu) || shared_.count(gpu) || draining_gpus_.count(gpu)) return false;
  }
  if (w.sharing != SharingMethod::None) {
    // Re-check the CU range against the ledger as it is now (the score may
    // come from a concurrent reader's view).
    if (s.shared_gpu.empty()) return false;
    auto snap = disc_->snapshot();
    auto nit = snap->nodes.find(s.node);
    const GpuDevice* g = nit == snap->nodes.end() ? nullptr : nit->second.gpu(s.shared_gpu);
    int b = 0, e = 0;
    if (!g || !share_fits(*g, w, &b, &e)) return false;
    // (b, e) may differ from the scored range when the gap moved: take the
    // range that fits now.
    Allocation a;
    a.uid = w.uid;
    a.node = s.node;
    a.ns = w.ns;
    a.team = w.team;
    a.sharing = w.sharing;
    a.shared_gpu = s.shared_gpu;
    a.cu_begin = b;
    a.cu_end = e;
    a.share_memory_gb = w.share_memory_gb;
    a.share_group = w.share_group;
    if (!w.share_group.empty()) {
      a.share_leader = true;
      a.share_leader_uid = w.uid;
      auto cur = shared_.find(s.shared_gpu);
      if (cur != shared_.end())
        for (const auto& uid : cur->second.clients) {
          auto it = allocs_.find(uid);
          if (it != allocs_.end() && it->second.share_group == w.share_group && it->second.share_leader) {
            a.share_leader = false;  // a member: the leader's range and cap cover it
            a.share_leader_uid = uid;
            a.share_memory_gb = 0.0;
          }
        }
    }
    a.type = w.type;
    a.priority = w.priority;
    a.preemptible = w.preemptible;
    a.allocated_ns = now_ns();
    a.expected_end_ns = expected_end_locked(w, a.allocated_ns);
    SharedGpu& sg = shared_[s.shared_gpu];
    sg.method = w.sharing;
    sg.clients.push_back(w.uid);
    index_alloc_locked(a);
    allocs_[w.uid] = std::move(a);
    touch_node(s.node);
    return true;
  }
  if (s.gpus.empty() && s.partitions.empty()) return false;
  Allocation a;
  a.uid = w.uid;
  a.node = s.node;
  a.ns = w.ns;
  a.team = w.team;
  a.gang = w.gang;
  a.gang_size = w.gang_size;
  a.gpus = s.gpus;
  a.partitions = s.partitions;
  a.type = w.type;
  a.priority = w.priority;
  a.preemptible = w.preemptible;
  a.gang_pending = gang_pending;
  a.allocated_ns = now_ns();
  a.expected_end_ns = expected_end_locked(w, a.allocated_ns);
  a.bandwidth_gbps = s.bandwidth_gbps;
  for (const auto& g : s.gpus) gpu_owner_[g] = w.uid;
  for (const auto& p : s.partitions) part_owner_[p] = w.uid;
  node_gpus_used_[s.node] += static_cast<int>(s.gpus.size());
  index_alloc_locked(a);
  allocs_[w.uid] = std::move(a);
  touch_node(s.node);
  return true;
}

// Caller holds mu_ exclusively: drop one ledger entry and everything it holds.
void Scheduler::erase_locked(std::unordered_map<std::string, Allocation>::iterator it) {
  const Allocation& a = it->second;
  touch_node(a.node);
  for (const auto& g : a.gpus) gpu_owner_.erase(g);
  for (const auto& p : a.partitions) part_owner_.erase(p);
  node_gpus_used_[a.node] -= static_cast<int>(a.gpus.size());
  if (!a.shared_gpu.empty()) {
    auto sh = shared_.find(a.shared_gpu);
    if (sh != shared_.end()) {
      auto& cl = sh->second.clients;
      cl.erase(std::remove(cl.begin(), cl.end(), a.uid), cl.end());
      if (cl.empty()) shared_.erase(sh);
    }
  }
  auto na = node_allocs_.find(a.node);
  if (na != node_allocs_.end()) {
    auto& v = na->second;
    auto pos = std::find(v.begin(), v.end(), a.uid);
    if (pos != v.end()) {
      *pos = std::move(v.back());
      v.pop_back();
    }
    if (v.empty()) node_allocs_.erase(na);
  }
  allocs_.erase(it);
}

void Scheduler::index_alloc_locked(const Allocation& a) { node_allocs_[a.node].push_back(a.uid); }

// Caller holds mu_.  When the workload says how long it runs, that; else the
// learned mean lifetime of its type once 8 allocations of it have completed.
int64_t Scheduler::expected_end_locked(const WorkloadRequest& w, int64_t start_ns) const {
  double s = w.expected_duration_s;
  if (s <= 0.0) {
    const Lifetime& l = lifetimes_[static_cast<int>(w.type) & 7];
    if (l.n >= 8) s = l.mean_s;
  }
  return s > 0.0 ? start_ns + static_cast<int64_t>(s * 1e9) : 0;
}

void Scheduler::emit(SchedEvent e) {
  std::lock_guard<std::mutex> lk(ev_mu_);
  if (events_.size() >= cfg_.event_capacity) events_.pop_front();
  events_.push_back(std::move(e));
}

std::vector<SchedEvent> Scheduler::drain_events(size_t max) {
  std::lock_guard<std::mutex> lk(ev_mu_);
  std::vector<SchedEvent> out;
  size_t n = max == 0 ? events_.size() : std::min(max, events_.size());
  for (size_t i = 0; i < n; ++i) {
    out.push_back(std::move(events_.front()));
    events_.pop_front();
  }
  return out;
}

static Decision decision_from(const Allocation& a, int score, const std::string& status) {
  Decision d;
  d.ok = true;
  d.status = status;
  d.uid = a.uid;
  d.node = a.node;
  d.gpus = a.gpus;
  d.partitions = a.partitions;
  d.sharing = a.sharing;
  d.shared_gpu = a.shared_gpu;
  d.cu_begin = a.cu_begin;
  d.cu_end = a.cu_end;
  d.share_memory_gb = a.share_memory_gb;
  d.share_group = a.share_group;
  d.share_leader = a.share_leader;
  d.share_leader_uid = a.share_leader_uid;
  d.score = score;
  d.bandwidth_gbps = a.bandwidth_gbps;
  return d;
}

Decision Scheduler::schedule(const WorkloadRequest& w) {
  const auto t0 = std::chrono::steady_clock::now();
  Decision d;
  d.uid = w.uid;
  auto snap = disc_->snapshot();
  auto finish = [&](Decision& dd) {
    dd.latency_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    latency_.record_ms(dd.latency_ms);
    std::lock_guard<std::mutex> lk(stat_mu_);
    stats_.attempts++;
    if (dd.ok) {
      stats_.scheduled++;
      note_placement();
      preempt_wait_.erase(dd.uid);
    } else {
      stats_.failed++;
    }
  };
  {
    std::shared_lock<RwLock> lk(mu_);
    auto it = allocs_.find(w.uid);
    if (it != allocs_.end()) {  // idempotent re-schedule
      d = decision_from(it->second, 0, it->second.gang_pending ? "Waiting" : "Scheduled");
      finish(d);
      return d;
    }
  }
  for (int attempt = 0; attempt < 2; ++attempt) {
    std::vector<NodeScore> scores;
    {
      std::shared_lock<RwLock> lk(mu_);
      for (const auto& kv : snap->nodes) {
        std::string why = eligible(kv.second, w);
        if (!why.empty()) {
          d.failed_nodes[kv.first] = why;
          continue;
        }
        NodeScore s = score_node(kv.second, w);
        if (s.total > 0 && (!s.gpus.empty() || !s.partitions.empty() || !s.shared_gpu.empty()))
          scores.push_back(std::move(s));
      }
    }
    std::sort(scores.begin(), scores.end(), [](const NodeScore& a, const NodeScore& b) {
      return a.total != b.total ? a.total > b.total : a.node < b.node;
    });
    const int tries = std::min<int>(static_cast<int>(scores.size()), std::max(1, cfg_.max_attempts));
    for (int i = 0; i < tries; ++i) {
      std::unique_lock<RwLock> lk(mu_);
      NodeScore s = scores[i];
      const NodeTopology& n = snap->nodes.at(s.node);
      bool stale = false;
      for (const auto& g : s.gpus) stale |= gpu_owner_.count(g) > 0 || shared_.count(g) > 0;
      for (const auto& p : s.partitions) stale |= part_owner_.count(p) > 0;
      if (!s.shared_gpu.empty()) {
        int b = 0, e = 0;
        const GpuDevice* g = n.gpu(s.shared_gpu);
        stale |= !g || !share_fits(*g, w, &b, &e);
      }
      if (stale) {  // lost a race: re-score this node under the write lock
        if (!eligible(n, w).empty()) continue;
        s = score_node(n, w);
        if (s.gpus.empty() && s.partitions.empty() && s.shared_gpu.empty()) continue;
      }
      const bool gang = cfg_.enable_gang && !w.gang.empty() && w.gang_size > 1;
      if (!reserve_locked(w, s, gang)) continue;
      std::vector<std::string> preempted = std::move(d.preempted);
      d = decision_from(allocs_.at(w.uid), s.total, "Scheduled");
      d.preempted = std::move(preempted);
      d.bandwidth_gbps = s.bandwidth_gbps;
      d.reasons = s.reasons;
      d.failed_nodes.clear();
      if (gang) {
        Gang& gg = gangs_[w.gang];
        gg.size = w.gang_size;
        if (gg.members.empty()) gg.first_ns = now_ns();
        gg.members.insert(w.uid);
        if (static_cast<int>(gg.members.size()) >= gg.size) {
          gg.ready = true;
          for (const auto& m : gg.members) allocs_[m].gang_pending = false;
          emit({SchedEventType::GangReady, w.gang, s.node, std::to_string(gg.size), now_ns()});
        } else {
          d.status = "Waiting";
        }
      }
      if (s.topology >= 80) {
        std::lock_guard<std::mutex> sl(stat_mu_);
        stats_.topology_optimal++;
      }
      lk.unlock();
      emit({SchedEventType::Scheduled, w.uid, s.node, "", now_ns()});
      finish(d);
      return d;
    }
    if (attempt == 0 && cfg_.enable_preemption && w.priority > 0 && try_preempt(w, snap, &d)) continue;
    break;
  }
  d.ok = false;
  d.status = "Unschedulable";
  emit({SchedEventType::Failed, w.uid, "", "", now_ns()});
  finish(d);
  return d;
}

// An allocation expected to finish before `soon_ns`, and not overdue by more
// than its own expected run time (an estimate that far off says nothing).
bool Scheduler::near_completion(const Allocation& a, int64_t now, int64_t soon_ns) const {
  if (!a.expected_end_ns || a.expected_end_ns > soon_ns) return false;
  return now - a.expected_end_ns <= a.expected_end_ns - a.allocated_ns;
}

// Caller holds mu_ (shared).  Walks only the allocations on `n`.  Room is
// counted in GPUs (a slice = 1/8, a share = 1/8: generous, so "false" is a
// true negative); the cost is that of the cheapest victims, in eviction
// order, whose room covers the shortfall.
bool Scheduler::estimate_node_preemption(const WorkloadRequest& w, const NodeTopology& n, int64_t now,
                                         int64_t soon_ns, PreemptCost* cost, bool* wait) const {
  *wait = false;
  auto na = node_allocs_.find(n.name);
  if (na == node_allocs_.end()) return false;
  const bool frac = w.partition || w.sharing != SharingMethod::None;
  const double need = frac ? std::max(1, w.partition ? w.partition_count : 1) / 8.0 : std::max(1, w.gpu_count);
  auto room_of = [&](const Allocation& a) {
    const double whole = static_cast<double>(a.gpus.size());
    const double part = (a.partitions.size() + (a.shared_gpu.empty() ? 0 : 1)) / 8.0;
    return frac ? whole + part : whole + part;  // slices free a whole GPU only together: still an upper bound
  };
  struct Cand {
    int64_t prio, age_ns;
    double room;
  };
  std::vector<Cand> cands;
  double held = 0.0, soon = 0.0;
  for (const auto& uid : na->second) {
    auto it = allocs_.find(uid);
    if (it == allocs_.end()) continue;
    const Allocation& a = it->second;
    const double r = room_of(a);
    held += r;
    if (near_completion(a, now, soon_ns)) {
      soon += r;
      continue;  // about to finish: not a victim
    }
    if (a.preemptible && a.priority < w.priority) cands.push_back({a.priority, a.allocated_ns, r});
  }
  const double free_now = std::max(0.0, static_cast<double>(n.gpus.size()) - held);
  if (soon > 0.0 && free_now + soon >= need) *wait = true;
  if (cands.empty()) return false;
  std::sort(cands.begin(), cands.end(), [](const Cand& a, const Cand& b) {
    return a.prio != b.prio ? a.prio < b.prio : a.age_ns > b.age_ns;
  });
  double room = free_now;
  int64_t prio = 0;
  size_t k = 0;
  for (const auto& c : cands) {
    room += c.room;
    prio += c.prio;
    ++k;
    if (room >= need) break;
  }
  if (room < need && !frac) return false;
  *cost = {prio, k, static_cast<size_t>(room * 8)};
  return true;
}

// Caller holds mu_ exclusively (the ledger is edited and restored).  The
// cheapest set of lower-priority preemptible allocations (whole gangs) on
// `n`, none expected to finish before `protect_until_ns`, whose removal makes
// the node eligible for `w`; false if there is none.
bool Scheduler::plan_node_preemption(const WorkloadRequest& w, const NodeTopology& n, int64_t protect_until_ns,
                                     std::vector<std::string>* victims_out, PreemptCost* cost_out) {
  auto na = node_allocs_.find(n.name);
  if (na == node_allocs_.end()) return false;
  const int64_t now = now_ns();
  auto victim_ok = [&](const Allocation& a) {
    return a.preemptible && a.priority < w.priority && !near_completion(a, now, protect_until_ns);
  };
  // A gang is preempted as a unit: its other members (on any node) would
  // otherwise keep their GPUs while the job cannot run.
  auto unit_of = [&](const Allocation& a, std::vector<const Allocation*>* out) {
    if (a.gang.empty()) {
      out->push_back(&a);
      return true;
    }
    auto g = gangs_.find(a.gang);
    if (g == gangs_.end()) {
      out->push_back(&a);
      return true;
    }
    for (const auto& m : g->second.members) {
      auto it = allocs_.find(m);
      if (it == allocs_.end()) continue;
      if (!victim_ok(it->second)) return false;
      out->push_back(&it->second);
    }
    return true;
  };
  std::vector<const Allocation*> cands;
  for (const auto& uid : na->second) {
    auto it = allocs_.find(uid);
    if (it != allocs_.end() && victim_ok(it->second)) cands.push_back(&it->second);
  }
  if (cands.empty()) return false;
  std::sort(cands.begin(), cands.end(), [](const Allocation* a, const Allocation* b) {
    if (a->priority != b->priority) return a->priority < b->priority;
    return a->allocated_ns > b->allocated_ns;  // youngest first: least work lost
  });
  // Temporarily hide victims (whole gangs) one unit at a time until the node
  // becomes eligible.
  std::vector<std::string> victims;
  std::set<std::string> hidden_uids;
  std::vector<std::pair<std::string, std::string>> hidden_g, hidden_p;
  std::vector<std::pair<std::string, SharedGpu>> hidden_s;
  int64_t prio = 0;
  size_t ngpu = 0;
  bool ok = false;
  for (const Allocation* c : cands) {
    if (hidden_uids.count(c->uid)) continue;
    std::vector<const Allocation*> unit;
    if (!unit_of(*c, &unit)) continue;
    for (const Allocation* a : unit) {
      if (!hidden_uids.insert(a->uid).second) continue;
      victims.push_back(a->uid);
      prio += a->priority;
      ngpu += a->gpus.size() + a->partitions.size() + (a->shared_gpu.empty() ? 0 : 1);
      for (const auto& g : a->gpus) {
        hidden_g.emplace_back(g, gpu_owner_[g]);
        gpu_owner_.erase(g);
      }
      for (const auto& p : a->partitions) {
        hidden_p.emplace_back(p, part_owner_[p]);
        part_owner_.erase(p);
      }
      if (!a->shared_gpu.empty()) {
        auto sh = shared_.find(a->shared_gpu);
        if (sh != shared_.end()) {
          hidden_s.emplace_back(sh->first, sh->second);
          auto& cl = sh->second.clients;
          cl.erase(std::remove(cl.begin(), cl.end(), a->uid), cl.end());
          if (cl.empty()) shared_.erase(sh);
        }
      }
    }
    if (eligible(n, w).empty()) {
      ok = true;
      break;
    }
  }
  for (auto& h : hidden_g) gpu_owner_[h.first] = h.second;
  for (auto& h : hidden_p) part_owner_[h.first] = h.second;
  // Restore shares in reverse so the earliest (fullest) snapshot wins.
  for (auto it = hidden_s.rbegin(); it != hidden_s.rend(); ++it) shared_[it->first] = it->second;
  if (!ok) return false;
  *victims_out = std::move(victims);
  *cost_out = {prio, victims_out->size(), ngpu};
  return true;
}

// Caller holds stat_mu_.  Victims the rate window still allows: a percentage
// of the placements inside the window, never less than the burst.
int Scheduler::preemption_budget_locked(int64_t now) {
  if (cfg_.preemption_max_rate_percent <= 0.0) return INT32_MAX;
  const int64_t sec = now / 1000000000;
  while (!rate_.empty() && rate_.front().sec <= sec - std::max(1, cfg_.preemption_window_s)) rate_.pop_front();
  uint64_t placed = 0, victims = 0;
  for (const auto& b : rate_) {
    placed += b.placed;
    victims += b.victims;
  }
  const double allowed =
      std::max<double>(cfg_.preemption_burst, cfg_.preemption_max_rate_percent * 0.01 * static_cast<double>(placed));
  return static_cast<int>(std::max(0.0, std::floor(allowed) - static_cast<double>(victims)));
}

void Scheduler::note_placement() {  // caller holds stat_mu_
  const int64_t sec = now_ns() / 1000000000;
  if (rate_.empty() || rate_.back().sec != sec) rate_.push_back({sec, 0, 0});
  rate_.back().placed++;
}

std::vector<Scheduler::PreemptPlan> Scheduler::select_preemption(const WorkloadRequest& w,
                                                                 const TopologySnapshot& snap,
                                                                 const std::vector<std::string>* nodes,
                                                                 bool commit) {
  std::vector<PreemptPlan> out;
  const int64_t now = now_ns();
  // ---- policy: window budget, and whether this request may still be told to wait
  int budget;
  bool may_wait = cfg_.preemption_wait_window_s > 0.0 && w.priority < cfg_.preemption_urgent_priority;
  {
    std::lock_guard<std::mutex> sl(stat_mu_);
    budget = preemption_budget_locked(now);
    if (budget <= 0) {
      stats_.preemptions_rate_limited++;
      return out;
    }
    if (may_wait) {
      auto it = preempt_wait_.find(w.uid);
      if (it != preempt_wait_.end() &&
          now - it->second > static_cast<int64_t>(cfg_.preemption_max_wait_s * 1e9))
        may_wait = false;  // waited long enough: completions did not make room
    }
  }
  const int64_t soon = now + static_cast<int64_t>(cfg_.preemption_wait_window_s * 1e9);
  const int64_t protect = may_wait ? soon : 0;  // past its patience a request may also evict near-finishers

  // ---- estimates over the candidates, under the shared lock
  struct Est {
    const NodeTopology* n;
    PreemptCost cost;
  };
  std::vector<Est> est;
  bool wait_node = false;
  {
    std::shared_lock<RwLock> lk(mu_);
    auto visit = [&](const NodeTopology& n) {
      PreemptCost c;
      bool wait = false;
      const bool ok = estimate_node_preemption(w, n, now, protect, &c, &wait);
      // waiting only helps on a node the request could run on at all
      if (wait && !wait_node) wait_node = admissible(n, w).empty();
      if (ok) est.push_back({&n, c});
    };
    if (nodes) {
      for (const auto& name : *nodes) {
        auto it = snap->nodes.find(name);
        if (it != snap->nodes.end()) visit(it->second);
      }
    } else {
      for (const auto& kv : snap->nodes) visit(kv.second);
    }
  }
  if (may_wait && wait_node) {
    std::lock_guard<std::mutex> sl(stat_mu_);
    stats_.preemptions_deferred_wait++;
    preempt_wait_.emplace(w.uid, now);
    if (preempt_wait_.size() > 65536) {  // requests that went away without ever being placed
      for (auto it = preempt_wait_.begin(); it != preempt_wait_.end();)
        it = now - it->second > 3600LL * 1000000000 ? preempt_wait_.erase(it) : std::next(it);
    }
    return out;
  }
  if (est.empty()) return out;
  auto cheaper = [](const Est& a, const Est& b) {
    return a.cost != b.cost ? a.cost < b.cost : a.n->name < b.n->name;
  };
  const size_t K = static_cast<size_t>(std::max(1, cfg_.preemption_candidate_nodes));

  // ---- exact plans on the K cheapest (then the next K, at most 4 rounds), under the exclusive lock
  size_t done = 0;
  for (int round = 0; round < 4 && done < est.size() && out.empty(); ++round) {
    const size_t end = std::min(est.size(), done + K);
    std::partial_sort(est.begin() + done, est.begin() + end, est.end(), cheaper);
    std::unique_lock<RwLock> lk(mu_);
    for (size_t i = done; i < end; ++i) {
      PreemptPlan p;
      p.node = est[i].n->name;
      if (!plan_node_preemption(w, *est[i].n, protect, &p.victims, &p.cost)) continue;
      // over the window's budget: only the window's first preemption may exceed it
      if (static_cast<int>(p.victims.size()) > budget && budget < cfg_.preemption_burst) continue;
      out.push_back(std::move(p));
    }
    done = end;
    if (out.empty()) continue;
    std::sort(out.begin(), out.end(), [](const PreemptPlan& a, const PreemptPlan& b) {
      return a.cost != b.cost ? a.cost < b.cost : a.node < b.node;
    });
    if (commit) {
      out.resize(1);
      for (const auto& uid : out[0].victims) {
        auto it = allocs_.find(uid);
        if (it == allocs_.end()) continue;
        const std::string gang = it->second.gang;
        const std::string node = it->second.node;
        erase_locked(it);
        if (!gang.empty()) {
          auto g = gangs_.find(gang);
          if (g != gangs_.end()) {
            g->second.members.erase(uid);
            if (g->second.members.empty()) gangs_.erase(g);
          }
        }
        emit({SchedEventType::Preempted, uid, node, "by " + w.uid, now_ns()});
      }
    }
  }
  if (!out.empty()) {  // book the cheapest plan's victims in the window
    std::lock_guard<std::mutex> sl(stat_mu_);
    const int64_t sec = now / 1000000000;
    if (rate_.empty() || rate_.back().sec != sec) rate_.push_back({sec, 0, 0});
    rate_.back().victims += static_cast<uint32_t>(out[0].victims.size());
    if (commit) stats_.preemptions += out[0].victims.size();
  }
  return out;
}

// Picks, over all nodes, the cheapest victim set and evicts it from the
// ledger; cost = (sum of victim priorities, #victims, victim GPUs).
bool Scheduler::try_preempt(const WorkloadRequest& w, const TopologySnapshot& snap, Decision* d) {
  auto plans = select_preemption(w, snap, nullptr, /*commit=*/true);
  if (plans.empty()) return false;
  for (const auto& uid : plans[0].victims) d->preempted.push_back(uid);
  return true;
}

std::map<std::string, std::vector<std::string>> Scheduler::preemption_plans(
    const WorkloadRequest& w, const std::vector<std::string>& nodes) {
  std::map<std::string, std::vector<std::string>> out;
  if (!cfg_.enable_preemption || w.priority <= 0) return out;
  auto snap = disc_->snapshot();
  {  // a candidate that fits as it is needs no victims
    std::shared_lock<RwLock> lk(mu_);
    const uint64_t sig = request_signature(w);
    std::string scratch;
    for (const auto& name : nodes) {
      auto it = snap->nodes.find(name);
      if (it != snap->nodes.end() && eligible_cached(it->second, w, sig, &scratch).empty()) out[name] = {};
    }
  }
  if (!out.empty()) return out;
  for (auto& p : select_preemption(w, snap, &nodes, /*commit=*/false)) out[p.node] = std::move(p.victims);
  return out;
}

void Scheduler::count_preemptions(size_t n) {
  std::lock_guard<std::mutex> sl(stat_mu_);
  stats_.preemptions += n;
}

std::vector<Decision> Scheduler::schedule_gang(const std::vector<WorkloadRequest>& members) {
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<Decision> out;
  auto snap = disc_->snapshot();
  std::unique_lock<RwLock> lk(mu_);
  std::vector<std::string> placed;
  bool ok = true;
  auto fill = [](Decision& d, const NodeScore& s) {
    d.ok = true;
    d.status = "Scheduled";
    d.node = s.node;
    d.gpus = s.gpus;
    d.partitions = s.partitions;
    d.score = s.total;
    d.bandwidth_gbps = s.bandwidth_gbps;
    d.reasons = s.reasons;
  };
  // One xGMI island first: a gang of whole-GPU members that together fit one
  // node and asked for xGMI connectivity (or runs a comm-heavy strategy) is
  // placed as ONE group on one node — its ranks' collectives then ride the
  // all-to-all xGMI mesh instead of the node NICs.  xGMIRequired gangs never
  // spill across nodes.
  int total = 0;
  bool whole = true, want_island = false, need_island = false;
  for (const auto& w : members) {
    total += w.gpu_count;
    whole &= !w.partition && w.sharing == SharingMethod::None && w.gpu_count > 0;
    want_island |= w.topology == TopologyPreference::XgmiOptimal ||
                   w.topology == TopologyPreference::XgmiRequired || comm_heavy(w.strategy) ||
                   w.strategy == DistributionStrategy::DataParallel || w.strategy == DistributionStrategy::FSDP;
    need_island |= w.topology == TopologyPreference::XgmiRequired;
  }
  if (whole && want_island && members.size() > 1) {
    WorkloadRequest merged = members.front();
    merged.gpu_count = total;
    merged.gang.clear();
    if (merged.topology == TopologyPreference::None) merged.topology = TopologyPreference::XgmiOptimal;
    NodeScore best;
    for (const auto& kv : snap->nodes) {
      bool all = true;
      for (const auto& w : members) all &= eligible(kv.second, w).empty();
      if (!all || !eligible(kv.second, merged).empty()) continue;
      NodeScore s = score_node(kv.second, merged);
      if (static_cast<int>(s.gpus.size()) != total || s.total <= 0) continue;
      if (s.total > best.total || (s.total == best.total && s.node < best.node)) best = s;
    }
    if (!best.node.empty()) {
      size_t off = 0;
      for (const auto& w : members) {
        NodeScore part = best;
        part.gpus.assign(best.gpus.begin() + off, best.gpus.begin() + off + w.gpu_count);
        off += w.gpu_count;
        WorkloadRequest wm = w;
        wm.gang.clear();
        Decision d;
        d.uid = w.uid;
        if (!reserve_locked(wm, part, false)) {
          ok = false;
          d.status = "Unschedulable";
          out.push_back(d);
          break;
        }
        allocs_[w.uid].gang = w.gang;
        allocs_[w.uid].gang_size = w.gang_size;
        placed.push_back(w.uid);
        fill(d, part);
        out.push_back(d);
      }
    } else if (need_island) {
      ok = false;
      for (const auto& w : members) {
        Decision d;
        d.uid = w.uid;
        d.status = "Unschedulable";
        d.reasons.push_back("no single node has " + std::to_string(total) + " free xGMI-connected GPUs");
        out.push_back(d);
      }
    }
  }
  if (ok && out.empty()) {
    for (const auto& w : members) {
      Decision d;
      d.uid = w.uid;
      NodeScore best;
      for (const auto& kv : snap->nodes) {
        std::string why = eligible(kv.second, w);
        if (!why.empty()) {
          d.failed_nodes[kv.first] = why;
          continue;
        }
        NodeScore s = score_node(kv.second, w);
        if ((s.gpus.empty() && s.partitions.empty() && s.shared_gpu.empty()) || s.total <= 0) continue;
        if (s.total > best.total || (s.total == best.total && s.node < best.node)) best = s;
      }
      WorkloadRequest wm = w;
      wm.gang.clear();  // the whole gang is placed atomically here
      if (best.node.empty() || !reserve_locked(wm, best, false)) {
        ok = false;
        d.status = "Unschedulable";
        out.push_back(d);
        break;
      }
      allocs_[w.uid].gang = w.gang;
      allocs_[w.uid].gang_size = w.gang_size;
      placed.push_back(w.uid);
      d = decision_from(allocs_.at(w.uid), best.total, "Scheduled");
      d.reasons = best.reasons;
      out.push_back(d);
    }
  }
  if (!ok) {  // roll back: all or nothing
    for (const auto& uid : placed) {
      auto it = allocs_.find(uid);
      if (it != allocs_.end()) erase_locked(it);
    }
    for (auto& d : out) {
      d.ok = false;
      d.status = "Unschedulable";
      d.gpus.clear();
      d.partitions.clear();
      d.shared_gpu.clear();
    }
  }
  if (ok) {  // the gang is complete from the start: its members are found (and preempted) as one unit
    for (const auto& w : members) {
      if (w.gang.empty()) continue;
      Gang& gg = gangs_[w.gang];
      gg.size = std::max<int>(gg.size, std::max<int>(w.gang_size, static_cast<int>(members.size())));
      if (gg.members.empty()) gg.first_ns = now_ns();
      gg.members.insert(w.uid);
      gg.ready = true;
    }
  }
  lk.unlock();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  latency_.record_ms(ms);
  std::lock_guard<std::mutex> sl(stat_mu_);
  stats_.attempts += members.size();
  if (ok) {
    stats_.scheduled += members.size();
    for (size_t i = 0; i < members.size(); ++i) note_placement();
  } else {
    stats_.failed += members.size();
  }
  return out;
}

std::map<std::string, std::string> Scheduler::filter(const WorkloadRequest& w,
                                                     const std::vector<std::string>& nodes,
                                                     std::vector<std::string>* passed) {
  std::map<std::string, std::string> failed;
  std::vector<std::string> why;
  filter_verdicts(w, nodes, &why);
  for (size_t i = 0; i < nodes.size(); ++i) {
    if (why[i].empty()) passed->push_back(nodes[i]);
    else failed[nodes[i]] = std::move(why[i]);
  }
  return failed;
}

std::vector<NodeScore> Scheduler::prioritize(const WorkloadRequest& w,
                                             const std::vector<std::string>& nodes) {
  std::vector<NodeScore> out;
  out.reserve(nodes.size());
  auto snap = disc_->snapshot();
  std::shared_lock<RwLock> lk(mu_);
  size_t k = 0;
  for (const auto& name : nodes) {
    if (++k % kSweepChunk == 0) {  // see filter()
      lk.unlock();
      lk.lock();
    }
    auto it = snap->nodes.find(name);
    NodeScore s;
    s.node = name;
    if (it != snap->nodes.end() && eligible(it->second, w).empty()) s = score_node(it->second, w);
    s.node = name;
    out.push_back(std::move(s));
  }
  return out;
}

Decision Scheduler::bind(const WorkloadRequest& w, const std::string& node) {
  const auto t0 = std::chrono::steady_clock::now();
  Decision d;
  d.uid = w.uid;
  auto snap = disc_->snapshot();
  auto it = snap->nodes.find(node);
  std::unique_lock<RwLock> lk(mu_);
  auto mine = allocs_.find(w.uid);
  if (mine != allocs_.end()) {
    if (mine->second.node != node) {
      d.status = "Unschedulable";
      d.failed_nodes[node] = "already reserved on " + mine->second.node;
      return d;
    }
    d = decision_from(mine->second, 0, mine->second.gang_pending ? "Waiting" : "Scheduled");
    return d;
  }
  if (it == snap->nodes.end()) {
    d.status = "Unschedulable";
    d.failed_nodes[node] = "unknown node";
    return d;
  }
  std::string why = eligible(it->second, w);
  NodeScore s;
  if (why.empty()) s = score_node(it->second, w);
  const bool gang = cfg_.enable_gang && !w.gang.empty() && w.gang_size > 1;
  if (!why.empty() || !reserve_locked(w, s, gang)) {
    d.status = "Unschedulable";
    d.failed_nodes[node] = why.empty() ? "reservation conflict" : why;
    lk.unlock();
    std::lock_guard<std::mutex> sl(stat_mu_);
    stats_.attempts++;
    stats_.failed++;
    return d;
  }
  d = decision_from(allocs_.at(w.uid), s.total, "Scheduled");
  d.bandwidth_gbps = s.bandwidth_gbps;
  d.reasons = s.reasons;
  if (gang) {
    Gang& gg = gangs_[w.gang];
    gg.size = w.gang_size;
    if (gg.members.empty()) gg.first_ns = now_ns();
    gg.members.insert(w.uid);
    if (static_cast<int>(gg.members.size()) >= gg.size) {
      gg.ready = true;
      for (const auto& m : gg.members) allocs_[m].gang_pending = false;
      emit({SchedEventType::GangReady, w.gang, node, std::to_string(gg.size), now_ns()});
    } else {
      d.status = "Waiting";
    }
  }
  const bool optimal = s.topology >= 80;
  lk.unlock();
  emit({SchedEventType::Scheduled, w.uid, node, "", now_ns()});
  d.latency_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  latency_.record_ms(d.latency_ms);  // core bind latency (pod create -> bind is the Platform's)
  std::lock_guard<std::mutex> sl(stat_mu_);
  stats_.attempts++;
  stats_.scheduled++;
  note_placement();
  preempt_wait_.erase(w.uid);
  if (optimal) stats_.topology_optimal++;
  return d;
}

std::string Scheduler::permit(const std::string& uid) {
  expire_gangs();
  std::shared_lock<RwLock> lk(mu_);
  auto it = allocs_.find(uid);
  if (it == allocs_.end()) return "Reject";
  if (it->second.gang.empty() || !it->second.gang_pending) return "Allow";
  auto g = gangs_.find(it->second.gang);
  if (g != gangs_.end() && g->second.ready) return "Allow";
  return "Wait";
}

void Scheduler::expire_gangs() {
  std::vector<std::string> expired;
  {
    std::unique_lock<RwLock> lk(mu_);
    const int64_t now = now_ns();
    for (auto it = gangs_.begin(); it != gangs_.end();) {
      Gang& g = it->second;
      if (!g.ready && !g.members.empty() &&
          now - g.first_ns > static_cast<int64_t>(cfg_.gang_timeout_ms) * 1000000) {
        for (const auto& uid : g.members) {
          auto a = allocs_.find(uid);
          if (a != allocs_.end()) erase_locked(a);
        }
        expired.push_back(it->first);
        it = gangs_.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (const auto& g : expired) emit({SchedEventType::GangTimeout, g, "", "", now_ns()});
  if (!expired.empty()) {
    std::lock_guard<std::mutex> sl(stat_mu_);
    stats_.gang_timeouts += expired.size();
  }
}

bool Scheduler::release(const std::string& uid) {
  std::string node;
  {
    std::unique_lock<RwLock> lk(mu_);
    auto it = allocs_.find(uid);
    if (it == allocs_.end()) return false;
    node = it->second.node;
    if (!it->second.gang.empty()) {
      auto g = gangs_.find(it->second.gang);
      if (g != gangs_.end()) {
        g->second.members.erase(uid);
        if (g->second.members.empty()) gangs_.erase(g);
      }
    }
    if (!it->second.gang_pending && it->second.allocated_ns) {  // a completed run: learn its lifetime
      Lifetime& l = lifetimes_[static_cast<int>(it->second.type) & 7];
      const double s = static_cast<double>(now_ns() - it->second.allocated_ns) * 1e-9;
      l.n++;
      l.mean_s += (s - l.mean_s) / static_cast<double>(std::min<uint64_t>(l.n, 64));
    }
    erase_locked(it);
  }
  emit({SchedEventType::Released, uid, node, "", now_ns()});
  std::lock_guard<std::mutex> sl(stat_mu_);
  stats_.releases++;
  return true;
}

bool Scheduler::restore(const Allocation& a) {
  std::unique_lock<RwLock> lk(mu_);
  if (allocs_.count(a.uid)) return false;
  for (const auto& g : a.gpus)
    if (gpu_owner_.count(g) || shared_.count(g)) return false;
  for (const auto& p : a.partitions)
    if (part_owner_.count(p)) return false;
  if (!a.shared_gpu.empty()) {
    if (gpu_owner_.count(a.shared_gpu)) return false;
    auto sh = shared_.find(a.shared_gpu);
    if (sh != shared_.end() && sh->second.method != a.sharing) return false;
  }
  for (const auto& g : a.gpus) gpu_owner_[g] = a.uid;
  for (const auto& p : a.partitions) part_owner_[p] = a.uid;
  node_gpus_used_[a.node] += static_cast<int>(a.gpus.size());
  if (!a.shared_gpu.empty()) {
    SharedGpu& sg = shared_[a.shared_gpu];
    sg.method = a.sharing;
    sg.clients.push_back(a.uid);
  }
  Allocation c = a;
  if (!c.allocated_ns) c.allocated_ns = now_ns();
  if (!c.gang.empty()) {  // a restored gang was complete when it was bound
    Gang& gg = gangs_[c.gang];
    gg.size = std::max(gg.size, c.gang_size);
    gg.members.insert(c.uid);
    gg.ready = true;
    if (!gg.first_ns) gg.first_ns = c.allocated_ns;
    c.gang_pending = false;
  }
  index_alloc_locked(c);
  allocs_[a.uid] = c;
  touch_node(a.node);
  return true;
}

bool Scheduler::migrate_partition(const std::string& uid, const std::string& from, const std::string& to) {
  std::string node;
  {
    std::unique_lock<RwLock> lk(mu_);
    auto it = allocs_.find(uid);
    if (it == allocs_.end()) return false;
    auto& parts = it->second.partitions;
    auto pos = std::find(parts.begin(), parts.end(), from);
    if (pos == parts.end() || part_owner_.count(to)) return false;
    const std::string gpu = to.substr(0, to.rfind("/p"));
    if (gpu_owner_.count(gpu) || fenced_.count(gpu) || shared_.count(gpu) || draining_gpus_.count(gpu)) return false;
    auto snap = disc_->snapshot();
    std::string to_node;
    for (const auto& kv : snap->nodes)
      if (kv.second.gpu(gpu)) to_node = kv.first;
    if (to_node.empty()) return false;
    // A multi-slice allocation stays on one node.
    if (parts.size() > 1 && to_node != it->second.node) return false;
    part_owner_.erase(from);
    part_owner_[to] = uid;
    *pos = to;
    touch_node(it->second.node);
    touch_node(to_node);
    it->second.node = to_node;
    node = to_node;
  }
  emit({SchedEventType::Migrated, uid, node, from + " -> " + to, now_ns()});
  return true;
}

Decision Scheduler::reserve_share(const WorkloadRequest& w, const std::string& node, const std::string& gpu) {
  Decision d;
  d.uid = w.uid;
  d.status = "Unschedulable";
  auto snap = disc_->snapshot();
  auto nit = snap->nodes.find(node);
  const GpuDevice* g = nit == snap->nodes.end() ? nullptr : nit->second.gpu(gpu);
  if (!g || w.sharing == SharingMethod::None || w.sharing == SharingMethod::Partition) {
    d.failed_nodes[node] = g ? "not a CoLocate / TimeSlice request" : "unknown gpu " + gpu;
    return d;
  }
  std::unique_lock<RwLock> lk(mu_);
  if (allocs_.count(w.uid)) {
    d.failed_nodes[node] = "already allocated: " + w.uid;
    return d;
  }
  NodeScore s;
  s.node = node;
  if (!share_fits(*g, w, &s.cu_begin, &s.cu_end)) {
    d.failed_nodes[node] = "no room for a " + std::string(to_string(w.sharing)) + " client on " + gpu;
    return d;
  }
  s.shared_gpu = gpu;
  if (!reserve_locked(w, s, false)) {
    d.failed_nodes[node] = "reservation conflict";
    return d;
  }
  d = decision_from(allocs_.at(w.uid), 100, "Scheduled");
  lk.unlock();
  emit({SchedEventType::Scheduled, w.uid, node, "share", now_ns()});
  return d;
}

std::vector<std::string> Scheduler::share_group_peers(const std::string& uid, bool* leader) const {
  std::vector<std::string> out;
  *leader = false;
  std::shared_lock<RwLock> lk(mu_);
  auto it = allocs_.find(uid);
  if (it == allocs_.end() || it->second.share_group.empty()) return out;
  *leader = it->second.share_leader;
  auto sh = shared_.find(it->second.shared_gpu);
  if (sh == shared_.end()) return out;
  for (const auto& c : sh->second.clients) {
    auto a = allocs_.find(c);
    if (c != uid && a != allocs_.end() && a->second.share_group == it->second.share_group) out.push_back(c);
  }
  return out;
}

int Scheduler::share_clients(const std::string& gpu_uuid) const {
  std::shared_lock<RwLock> lk(mu_);
  auto it = shared_.find(gpu_uuid);
  return it == shared_.end() ? 0 : static_cast<int>(it->second.clients.size());
}

bool Scheduler::gpu_busy(const GpuDevice& g) const {
  std::shared_lock<RwLock> lk(mu_);
  if (gpu_owner_.count(g.uuid) || shared_.count(g.uuid)) return true;
  for (const auto& pi : g.partition.instances)
    if (part_owner_.count(pi.id)) return true;
  return false;
}

std::vector<Allocation> Scheduler::allocations() const {
  std::shared_lock<RwLock> lk(mu_);
  std::vector<Allocation> out;
  out.reserve(allocs_.size());
  for (const auto& kv : allocs_) out.push_back(kv.second);
  std::sort(out.begin(), out.end(), [](const Allocation& a, const Allocation& b) { return a.uid < b.uid; });
  return out;
}

bool Scheduler::allocation(const std::string& uid, Allocation* out) const {
  std::shared_lock<RwLock> lk(mu_);
  auto it = allocs_.find(uid);
  if (it == allocs_.end()) return false;
  if (out) *out = it->second;
  return true;
}

SchedulerMetrics Scheduler::metrics() const {
  SchedulerMetrics m;
  {
    std::lock_guard<std::mutex> lk(stat_mu_);
    m = stats_;
  }
  m.avg_latency_ms = latency_.mean_ms();
  m.p50_ms = latency_.quantile_ms(0.50);
  m.p90_ms = latency_.quantile_ms(0.90);
  m.p99_ms = latency_.quantile_ms(0.99);
  m.max_ms = latency_.max_ms();
  std::shared_lock<RwLock> lk(mu_);
  m.active_allocations = allocs_.size();
  m.allocated_gpus = gpu_owner_.size();
  m.allocated_partitions = part_owner_.size();
  m.shared_gpus = shared_.size();
  for (const auto& kv : shared_) m.share_clients += kv.second.clients.size();
  return m;
}

}  // namespace kgwe
