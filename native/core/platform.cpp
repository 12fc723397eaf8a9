#include "platform.h"

#include "extender_scan.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <set>

namespace kgwe {

namespace {

const Json& field(const Json& j, const char* a, const char* b) {
  return j.has(a) ? j.get(a) : j.get(b);
}

double wall_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

int64_t quantity(const Json& q) {
  if (q.is_number()) return q.as_int();
  return std::atoll(q.str("0").c_str());
}

}  // namespace

WorkloadRequest workload_from_pod(const Json& pod, const std::string& gpu_resource) {
  const Json& meta = pod.get("metadata");
  const Json& ann = meta.get("annotations");
  const Json& spec = pod.get("spec");
  WorkloadRequest w;
  const std::string wl = ann.get("kgwe.amd.com/workload").str();
  if (!wl.empty()) {
    try {
      w = workload_from_json(Json::parse(wl));
    } catch (...) {
    }
  }
  w.name = meta.get("name").str();
  w.ns = meta.get("namespace").str("default");
  w.uid = meta.get("uid").str(w.ns + "/" + w.name);
  const Json& labels = meta.get("labels");
  if (w.team.empty()) w.team = labels.get("kgwe.amd.com/team").str(labels.get("team").str());
  if (w.project.empty()) w.project = labels.get("kgwe.amd.com/project").str();
  if (wl.empty()) {
    int64_t gpus = 0;
    for (const auto& c : spec.get("containers").items()) {
      const Json& lim = c.get("resources").get("limits");
      const Json& req = c.get("resources").get("requests");
      const Json& q = lim.has(gpu_resource) ? lim.get(gpu_resource) : req.get(gpu_resource);
      gpus += quantity(q);
      for (const char* mode : {"cpx", "qpx", "dpx"}) {
        const std::string r = gpu_resource + "-" + mode;
        const Json& pq = lim.has(r) ? lim.get(r) : req.get(r);
        const int64_t n = quantity(pq);
        if (n > 0) {
          w.partition = true;
          std::string up = mode;
          std::transform(up.begin(), up.end(), up.begin(), ::toupper);
          w.partition_mode = compute_partition_from(up);
          w.partition_count += static_cast<int>(n);
        }
      }
    }
    w.gpu_count = static_cast<int>(gpus > 0 ? gpus : (w.partition ? 0 : 1));
    w.topology = topology_preference_from(ann.get("kgwe.amd.com/topology").str("None"));
    w.min_memory_gb = std::atof(ann.get("kgwe.amd.com/min-memory-gb").str("0").c_str());
    w.min_bandwidth_gbps = std::atof(ann.get("kgwe.amd.com/min-bandwidth-gbps").str("0").c_str());
    w.type = workload_type_from(ann.get("kgwe.amd.com/workload-type").str("Training"));
    w.strategy = strategy_from(ann.get("kgwe.amd.com/strategy").str("None"));
    w.gang = ann.get("kgwe.amd.com/gang").str();
    w.gang_size = std::atoi(ann.get("kgwe.amd.com/gang-size").str("0").c_str());
    w.preemptible = ann.get("kgwe.amd.com/preemptible").str("true") != "false";
    // Co-located / time-sliced share of a whole GPU: amd.com/gpu-shared (or
    // the kgwe.amd.com/sharing annotation) + CU percentage and HBM cap.
    int64_t shared = 0;
    for (const auto& c : spec.get("containers").items()) {
      const Json& lim = c.get("resources").get("limits");
      const std::string r = gpu_resource + "-shared";
      shared += quantity(lim.has(r) ? lim.get(r) : c.get("resources").get("requests").get(r));
    }
    const std::string sm = ann.get("kgwe.amd.com/sharing").str(shared > 0 ? "CoLocate" : "");
    if (!sm.empty() && sharing_method_from(sm) != SharingMethod::None &&
        sharing_method_from(sm) != SharingMethod::Partition) {
      w.sharing = sharing_method_from(sm);
      w.gpu_count = 1;
      w.share_cu_percent = std::atof(ann.get("kgwe.amd.com/cu-percent").str("0").c_str());
      w.share_memory_gb = std::atof(ann.get("kgwe.amd.com/memory-gb").str("0").c_str());
      w.share_group = ann.get("kgwe.amd.com/share-group").str();
      if (!ann.has("kgwe.amd.com/workload-type")) w.type = WorkloadType::Inference;
    }
  }
  if (spec.has("priority")) w.priority = spec.get("priority").as_int(w.priority);
  if (w.expected_duration_s <= 0.0) {
    w.expected_duration_s = std::atof(ann.get("kgwe.amd.com/expected-duration-seconds").str("0").c_str());
    if (w.expected_duration_s <= 0.0) w.expected_duration_s = spec.get("activeDeadlineSeconds").as_number(0.0);
  }
  for (const auto& kv : spec.get("nodeSelector").fields()) w.node_selector[kv.first] = kv.second.str();
  for (const auto& t : spec.get("tolerations").items()) {
    Toleration tl;
    tl.key = t.get("key").str();
    tl.op = t.get("operator").str("Equal");
    tl.value = t.get("value").str();
    tl.effect = t.get("effect").str();
    w.tolerations.push_back(tl);
  }
  const Json& na = spec.get("affinity").get("nodeAffinity");
  for (const auto& term : na.get("requiredDuringSchedulingIgnoredDuringExecution").get("nodeSelectorTerms").items())
    for (const auto& e : term.get("matchExpressions").items()) {
      AffinityTerm a;
      a.key = e.get("key").str();
      a.op = e.get("operator").str("In");
      for (const auto& v : e.get("values").items()) a.values.push_back(v.str());
      w.required_affinity.push_back(a);
    }
  for (const auto& pt : na.get("preferredDuringSchedulingIgnoredDuringExecution").items())
    for (const auto& e : pt.get("preference").get("matchExpressions").items()) {
      AffinityTerm a;
      a.key = e.get("key").str();
      a.op = e.get("operator").str("In");
      a.weight = static_cast<int>(pt.get("weight").as_int(1));
      for (const auto& v : e.get("values").items()) a.values.push_back(v.str());
      w.preferred_affinity.push_back(a);
    }
  return w;
}

std::map<std::string, std::string> rccl_env(const WorkloadRequest& w, const Decision& d,
                                            const NodeTopology& node, int master_port,
                                            const std::string& master_addr) {
  std::map<std::string, std::string> env;
  // Logical HIP device indices: whole GPUs by index; partition slices are
  // enumerated GPU-major (every slice is its own HIP device).
  std::vector<int> idx;
  std::vector<int> base(node.gpus.size() + 1, 0);
  std::vector<const GpuDevice*> by_index(node.gpus.size(), nullptr);
  for (const auto& g : node.gpus)
    if (g.index >= 0 && g.index < static_cast<int>(by_index.size())) by_index[g.index] = &g;
  for (size_t i = 0; i < by_index.size(); ++i)
    base[i + 1] = base[i] + (by_index[i] ? partition_count(by_index[i]->partition.compute) : 1);
  for (const auto& u : d.gpus)
    if (const GpuDevice* g = node.gpu(u)) idx.push_back(base[g->index]);
  for (const auto& p : d.partitions) {
    auto slash = p.rfind("/p");
    if (slash == std::string::npos) continue;
    if (const GpuDevice* g = node.gpu(p.substr(0, slash)))
      idx.push_back(base[g->index] + std::atoi(p.c_str() + slash + 2));
  }
  std::sort(idx.begin(), idx.end());
  std::string vis;
  for (size_t i = 0; i < idx.size(); ++i) vis += (i ? "," : "") + std::to_string(idx[i]);
  const int nproc = static_cast<int>(idx.size());
  env["HIP_VISIBLE_DEVICES"] = vis;
  env["ROCR_VISIBLE_DEVICES"] = vis;
  env["KGWE_ALLOCATED_GPUS"] = [&] {
    std::string s;
    for (size_t i = 0; i < d.gpus.size(); ++i) s += (i ? "," : "") + d.gpus[i];
    for (size_t i = 0; i < d.partitions.size(); ++i) s += (s.empty() ? "" : ",") + d.partitions[i];
    return s;
  }();
  env["KGWE_NODE"] = d.node;
  char bw[32];
  std::snprintf(bw, sizeof bw, "%.1f", d.bandwidth_gbps);
  env["KGWE_XGMI_BANDWIDTH_GBPS"] = bw;
  if (w.backend == CommBackend::RCCL || w.backend == CommBackend::Gloo) {
    // torchrun-style rendezvous: one pod = one node's worth of ranks; a
    // multi-pod gang uses the gang leader's address (set by the controller).
    const int world = w.world_size > 0 ? w.world_size : std::max(1, nproc);
    env["NPROC_PER_NODE"] = std::to_string(std::max(1, nproc));
    env["LOCAL_WORLD_SIZE"] = std::to_string(std::max(1, nproc));
    env["WORLD_SIZE"] = std::to_string(world);
    env["NNODES"] = std::to_string(std::max(1, world / std::max(1, nproc)));
    env["MASTER_ADDR"] = master_addr.empty() ? "127.0.0.1" : master_addr;
    env["MASTER_PORT"] = std::to_string(master_port);
    env["TORCH_DISTRIBUTED_BACKEND"] = w.backend == CommBackend::RCCL ? "nccl" : "gloo";
  }
  if (w.backend == CommBackend::RCCL) {
    // RCCL reads the NCCL_* variables.  Single-node xGMI: no IB / sockets on
    // the data path; dmabuf IPC (legacy IPC mode off) for peer buffers.
    const bool single_node = w.world_size <= 0 || w.world_size <= nproc;
    env["NCCL_IB_DISABLE"] = single_node ? "1" : "0";
    env["NCCL_DEBUG"] = "WARN";
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0";
    env["NCCL_P2P_LEVEL"] = node.xgmi_fully_connected ? "SYS" : "PHB";
    env["TORCH_NCCL_ASYNC_ERROR_HANDLING"] = "1";
    if (nproc == 8 && node.xgmi_fully_connected) env["NCCL_MIN_NCHANNELS"] = "32";  // 7 links x rings
  }
  return env;
}

// ---------------------------------------------------------------------------
Platform::Platform(PlatformConfig cfg) : cfg_(std::move(cfg)) {
  disc_ = std::make_shared<DiscoveryService>();
  sched_ = std::make_shared<Scheduler>(disc_, cfg_.sched);
  part_ = std::make_shared<PartitionController>(disc_, sched_, cfg_.partition_dry_run);
  SharingPolicy sp;
  share_ = std::make_shared<SharingManager>(disc_, sched_, sp);
  cost_ = std::make_shared<CostEngine>(cfg_.cost);
  reg_ = std::make_shared<MetricRegistry>();
  reg_->declare_kgwe_families();
  auto reg = reg_;
  cost_->set_cost_hook([reg](const UsageRecord& r) {
    reg->add("kgwe_gpu_cost_total_dollars", {r.ns, r.team}, r.adjusted_cost);
  });
}

void Platform::remember_pod(const std::string& uid, const WorkloadRequest& w, double created_s) {
  std::lock_guard<std::mutex> lk(pods_mu_);
  pods_[uid] = w;
  name_to_uid_[w.ns + "/" + w.name] = uid;
  if (pods_.size() > 100000) {  // bounded: drop arbitrary old entries
    pods_.erase(pods_.begin());
  }
  // First sighting starts the pod's latency clock (a retried filter keeps it).
  if (!pending_.count(uid)) pending_[uid] = {now_ns(), created_s};
}

size_t Platform::queue_depth() const {
  std::lock_guard<std::mutex> lk(pods_mu_);
  return pending_.size();
}

namespace {
// Slow-verb log: with KGWE_SLOW_VERB_MS=<ms> set, a filter call that takes
// longer prints where its time went (stderr), for chasing latency tails.
struct PhaseLog {
  double limit_ms;
  int64_t t0, last;
  char buf[256];
  int n = 0;
  PhaseLog() : limit_ms([] {
      const char* e = std::getenv("KGWE_SLOW_VERB_MS");
      return e ? std::atof(e) : 0.0;
    }()), t0(limit_ms > 0 ? now_ns() : 0), last(t0) {}
  void mark(const char* what) {
    if (limit_ms <= 0) return;
    const int64_t t = now_ns();
    n += std::snprintf(buf + n, sizeof buf - static_cast<size_t>(n), " %s=%.2f", what, (t - last) / 1e6);
    if (n > 200) n = 200;
    last = t;
  }
  void done(const char* verb, size_t cands) {
    if (limit_ms <= 0) return;
    const double total = (now_ns() - t0) / 1e6;
    if (total >= limit_ms) std::fprintf(stderr, "kgwe slow %s %.2f ms (%zu candidates):%s\n", verb, total, cands, buf);
  }
};
}  // namespace

std::string Platform::filter(const std::string& body) {
  PhaseLog pl;
  // Fast path: zero-copy scan (names + byte spans of the Node items); the
  // reply splices the passing items' original bytes.  Fallback: full parse.
  ExtenderArgsScan scan;
  bool scanned = false;
  try {
    scanned = scan_extender_args(body, &scan);
  } catch (...) {
    scanned = false;
  }
  Json parsed;
  if (!scanned) {
    Json out = Json::object();
    try {
      parsed = Json::parse(body);
    } catch (const std::exception& e) {
      out["error"] = std::string("bad ExtenderArgs: ") + e.what();
      return out.dump();
    }
    scan = ExtenderArgsScan();
    scan.pod = field(parsed, "pod", "Pod");
    const Json& nodes = field(parsed, "nodes", "Nodes");
    scan.have_nodes = nodes.is_object();
    for (const auto& n : nodes.get("items").items()) {
      NodeSpan ns;
      ns.name = n.get("metadata").get("name").str();
      scan.nodes.push_back(ns);
    }
    for (const auto& n : field(parsed, "nodenames", "NodeNames").items()) scan.nodenames.push_back(n.str());
  }
  pl.mark("scan");
  const Json& pod = scan.pod;
  WorkloadRequest w = workload_from_pod(pod, cfg_.gpu_resource);
  // Microsecond creation stamp written by kgwe's mutating webhook (the
  // apiserver's creationTimestamp is whole seconds); else first filter call.
  remember_pod(w.uid, w,
               std::atof(pod.get("metadata").get("annotations").get("kgwe.amd.com/created-at").str("0").c_str()));
  pl.mark("pod");
  std::vector<std::string> names;
  names.reserve(scan.nodes.size() + scan.nodenames.size());
  for (const auto& n : scan.nodes) names.push_back(n.name);
  for (const auto& n : scan.nodenames) names.push_back(n);
  std::vector<std::string> why;  // per candidate: "" = passes, else the reason
  // The reply is written straight into its string: failedNodes, then the
  // passing candidates in request order (Node items are spliced from the
  // request's own bytes).
  auto reply = [&]() {
    std::string out;
    // Full Node objects come back byte for byte: the reply is about as long
    // as the request (growing a multi-megabyte string by doubling re-copies
    // and re-faults it several times).
    out.reserve(scan.have_nodes ? body.size() + 256 : 64 + names.size() * 48);
    out += "{\"failedNodes\":{";
    bool first = true;
    for (size_t i = 0; i < names.size(); ++i)
      if (!why[i].empty()) {
        if (!first) out += ',';
        first = false;
        out += '"';
        out += json_escape(names[i]);
        out += "\":\"";
        out += json_escape(why[i]);
        out += '"';
      }
    out += '}';
    if (scan.have_nodes) {
      out += ",\"nodes\":{\"items\":[";
      first = true;
      if (scanned) {
        for (size_t i = 0; i < scan.nodes.size(); ++i)
          if (why[i].empty()) {
            if (!first) out += ',';
            out.append(body, scan.nodes[i].begin, scan.nodes[i].end - scan.nodes[i].begin);
            first = false;
          }
      } else {
        size_t i = 0;
        for (const auto& n : field(parsed, "nodes", "Nodes").get("items").items()) {
          if (i < why.size() && why[i].empty()) {
            if (!first) out += ',';
            n.dump_to(out);
            first = false;
          }
          ++i;
        }
      }
      out += "]}";
    } else {
      out += ",\"nodenames\":[";
      first = true;
      for (size_t i = 0; i < names.size(); ++i)
        if (why[i].empty()) {
          if (!first) out += ',';
          first = false;
          out += '"';
          out += json_escape(names[i]);
          out += '"';
        }
      out += ']';
    }
    out += "}";
    return out;
  };
  if (cfg_.enforce_budgets) {
    // Estimate: one hour of this request at on-demand prices.
    const GpuPricing p = cost_->pricing("amd-mi355x-288gb");
    const double est = w.partition ? p.partition.at(to_string(w.partition_mode)) * w.partition_count
                                   : p.on_demand * w.gpu_count;
    Admission a = cost_->admit(w.ns, w.team, w.project, est, wall_s());
    if (!a.allowed) {
      why.assign(names.size(), a.reason);
      reg_->add("kgwe_scheduling_failures_total", {"budget"}, 1);
      return reply();
    }
  }
  pl.mark("admit");
  auto any_passed = [&why]() {
    for (const auto& v : why)
      if (v.empty()) return true;
    return false;
  };
  sched_->filter_verdicts(w, names, &why);
  pl.mark("verdicts");
  if (!any_passed() && w.partition && cfg_.auto_provision_partitions) {
    const std::unordered_set<std::string> cand(names.begin(), names.end());
    auto ops = part_->ensure_capacity(w.partition_mode, w.partition_count, false,
                                      w.partition_memory_set ? &w.partition_memory : nullptr, &cand);
    for (const auto& op : ops)
      reg_->add("kgwe_partition_reconfigurations_total",
                {op.node, op.state == OpState::Failed ? "failed" : "ok"}, 1);
    pl.mark("provision");
    if (!ops.empty()) sched_->filter_verdicts(w, names, &why);
    pl.mark("verdicts2");
  }
  if (!any_passed()) reg_->add("kgwe_scheduling_failures_total", {"filter"}, 1);
  std::string out = reply();
  pl.mark("reply");
  pl.done("filter", names.size());
  return out;
}

std::string Platform::prioritize(const std::string& body) {
  ExtenderArgsScan scan;
  bool scanned = false;
  try {
    scanned = scan_extender_args(body, &scan);
  } catch (...) {
    scanned = false;
  }
  if (!scanned) {
    Json args;
    try {
      args = Json::parse(body);
    } catch (...) {
      return "[]";
    }
    scan = ExtenderArgsScan();
    scan.pod = field(args, "pod", "Pod");
    for (const auto& n : field(args, "nodes", "Nodes").get("items").items()) {
      NodeSpan ns;
      ns.name = n.get("metadata").get("name").str();
      scan.nodes.push_back(ns);
    }
    for (const auto& n : field(args, "nodenames", "NodeNames").items()) scan.nodenames.push_back(n.str());
  }
  WorkloadRequest w = workload_from_pod(scan.pod, cfg_.gpu_resource);
  std::vector<std::string> names;
  for (const auto& n : scan.nodes) names.push_back(n.name);
  for (const auto& n : scan.nodenames) names.push_back(n);
  std::vector<int> totals;
  sched_->prioritize_totals(w, names, &totals);
  std::string out;
  out.reserve(8 + names.size() * 40);
  out += '[';
  for (size_t i = 0; i < names.size(); ++i) {
    if (i) out += ',';
    out += "{\"host\":\"";
    out += json_escape(names[i]);
    out += "\",\"score\":";
    // kube-scheduler MaxExtenderPriority = 10; our totals are 0..~120.
    out += std::to_string(static_cast<int>(std::min(10.0, std::round(totals[i] / 10.0))));
    out += '}';
  }
  out += ']';
  return out;
}

std::string Platform::preempt(const std::string& body) {
  Json args;
  Json out = Json::object();
  try {
    args = Json::parse(body);
  } catch (const std::exception& e) {
    out["error"] = std::string("bad ExtenderPreemptionArgs: ") + e.what();
    return out.dump();
  }
  WorkloadRequest w = workload_from_pod(field(args, "pod", "Pod"), cfg_.gpu_resource);
  std::vector<std::string> names;
  for (const auto& kv : field(args, "nodeNameToMetaVictims", "NodeNameToMetaVictims").fields())
    names.push_back(kv.first);
  for (const auto& kv : field(args, "nodeNameToVictims", "NodeNameToVictims").fields())
    if (std::find(names.begin(), names.end(), kv.first) == names.end()) names.push_back(kv.first);
  Json res = Json::object();
  const int64_t now = now_ns();
  for (const auto& kv : sched_->preemption_plans(w, names)) {
    // kube-scheduler resolves MetaVictims against the named node's own pods
    // and fails the whole preemption if one is not there, so only victims ON
    // the node are named.  A victim gang's members on other nodes are kept as
    // that victim's peers: when the victim is released (evicted), release()
    // hands them to the controller, which evicts the rest of the gang.
    Json mv = Json::object();
    Json pods = Json::array();
    std::vector<std::string> here, elsewhere;
    for (const auto& uid : kv.second) {
      Allocation a;
      if (sched_->allocation(uid, &a) && a.node != kv.first) elsewhere.push_back(uid);
      else here.push_back(uid);
    }
    if (here.empty() && !kv.second.empty()) continue;  // nothing evictable on this node itself
    for (const auto& uid : here) {
      Json p = Json::object();
      p["uid"] = uid;
      pods.push_back(p);
    }
    if (!elsewhere.empty()) {
      std::lock_guard<std::mutex> lk(pods_mu_);
      for (const auto& uid : here) gang_peers_[uid] = {elsewhere, now};
      for (auto it = gang_peers_.begin(); it != gang_peers_.end();)  // plans never acted on
        it = now - it->second.second > 300LL * 1000000000 ? gang_peers_.erase(it) : std::next(it);
    }
    mv["pods"] = pods;
    mv["numPDBViolations"] = static_cast<int64_t>(0);
    res[kv.first] = mv;
  }
  out["nodeNameToMetaVictims"] = res;
  return out.dump();
}

std::string Platform::placement_json(const WorkloadRequest& w, const Decision& d) {
  Json pl = to_json(d);
  NodeTopology n;
  Json env = Json::object();
  if (d.ok && disc_->node(d.node, &n)) {
    for (const auto& kv : rccl_env(w, d, n, cfg_.master_port)) env[kv.first] = kv.second;
  }
  if (d.ok && d.sharing != SharingMethod::None && !d.shared_gpu.empty()) {
    GpuDevice g;
    if (disc_->gpu(d.shared_gpu, &g))
      for (const auto& kv : share_env(d.sharing, g.index, d.cu_begin, d.cu_end, d.share_memory_gb,
                                      g.memory_total_gb))
        env[kv.first] = kv.second;
    if (!d.share_group.empty()) {
      // One serving process per (GPU, group): the leader listens on a socket
      // in the node's share directory, the members connect to it.
      env["KGWE_SHARE_GROUP"] = d.share_group;
      env["KGWE_SHARE_ROLE"] = d.share_leader ? "leader" : "member";
      env["KGWE_SHARE_LEADER"] = d.share_leader_uid;
      std::string file = d.shared_gpu + "-" + d.share_group;
      for (auto& c : file)
        if (!(std::isalnum(static_cast<unsigned char>(c)) || c == '-' || c == '_' || c == '.')) c = '_';
      env["KGWE_BATCH_ENDPOINT"] = "unix:" + cfg_.share_socket_dir + "/" + file + ".sock";
    }
  }
  pl["env"] = env;
  pl["workload"] = to_json(w);
  return pl.dump();
}

std::string Platform::bind(const std::string& body, const std::string& pod_json) {
  return bind_outcome(body, pod_json).json;
}

Platform::BindOutcome Platform::bind_outcome(const std::string& body, const std::string& pod_json) {
  BindOutcome bo;
  Json out = Json::object();
  Json res = Json::object();
  Json args;
  try {
    args = Json::parse(body);
  } catch (const std::exception& e) {
    bo.error = std::string("bad ExtenderBindingArgs: ") + e.what();
    res["error"] = bo.error;
    out["result"] = res;
    bo.json = out.dump();
    return bo;
  }
  const std::string name = field(args, "podName", "PodName").str();
  const std::string ns = field(args, "podNamespace", "PodNamespace").str("default");
  std::string uid = field(args, "podUID", "PodUID").str();
  const std::string node = field(args, "node", "Node").str();
  bo.ns = ns;
  bo.name = name;
  bo.node = node;
  WorkloadRequest w;
  bool have = false;
  if (!pod_json.empty()) {
    try {
      w = workload_from_pod(Json::parse(pod_json), cfg_.gpu_resource);
      have = true;
    } catch (...) {
    }
  }
  if (!have) {
    std::lock_guard<std::mutex> lk(pods_mu_);
    if (uid.empty()) {
      auto it = name_to_uid_.find(ns + "/" + name);
      if (it != name_to_uid_.end()) uid = it->second;
    }
    auto it = pods_.find(uid);
    if (it != pods_.end()) {
      w = it->second;
      have = true;
    }
  }
  bo.uid = uid;
  if (!have) {
    bo.unknown_pod = true;
    bo.error = "unknown pod " + ns + "/" + name + " (no filter call seen)";
    res["error"] = bo.error;
    out["result"] = res;
    bo.json = out.dump();
    return bo;
  }
  bo.uid = w.uid;
  bo.gang = w.gang;
  Decision d = sched_->bind(w, node);
  if (!d.ok) {
    auto it = d.failed_nodes.find(node);
    bo.error = it != d.failed_nodes.end() ? it->second : "bind failed";
    res["error"] = bo.error;
    reg_->add("kgwe_scheduling_failures_total", {"bind"}, 1);
  } else if (d.status == "Waiting") {
    // Gang member reserved (Permit "Wait"): a serving shell holds the request
    // until the gang is complete or the reservation times out; a caller that
    // cannot hold it sees this error and calls bind again.
    bo.waiting = true;
    bo.error = "gang " + w.gang + " waiting for members";
    res["error"] = bo.error;
  } else {
    bo.ok = true;
    reg_->add("kgwe_scheduling_successes_total", {}, 1);
    // Pod create -> bind latency, recorded by the extender itself at every
    // successful bind (the reference declares the histogram and never feeds
    // it: prometheus_exporter.go:643-648).
    std::pair<int64_t, double> seen{0, 0.0};
    bool first = false;
    {
      std::lock_guard<std::mutex> lk(pods_mu_);
      auto it = pending_.find(w.uid);
      if (it != pending_.end()) {
        seen = it->second;
        pending_.erase(it);
        first = true;
      }
    }
    double created = seen.second;
    if (!pod_json.empty()) first = true;  // bound from the pod object (no filter call seen)
    if (created <= 0 && !pod_json.empty()) {
      try {
        created = std::atof(Json::parse(pod_json).get("metadata").get("annotations")
                                .get("kgwe.amd.com/created-at").str("0").c_str());
      } catch (...) {
      }
    }
    if (first) {  // an idempotent re-bind of a bound pod is not a second sample
      if (created > 0) observe_pod_latency_ms(std::max(0.0, (wall_s() - created) * 1000.0));
      else if (seen.first > 0) observe_pod_latency_ms(static_cast<double>(now_ns() - seen.first) / 1e6);
      UsageRecord r;
      r.uid = w.uid;
      r.ns = w.ns;
      r.team = w.team;
      r.project = w.project;
      r.gpu_type = "amd-mi355x-288gb";
      r.gpu_count = w.partition ? w.partition_count : w.gpu_count;
      r.partition_mode = w.partition ? to_string(w.partition_mode) : "";
      cost_->start(r, wall_s());
      if (w.partition) reg_->add("kgwe_partition_allocations_total", {to_string(w.partition_mode)}, 1);
    }
  }
  reg_->add("kgwe_scheduling_attempts_total", {}, 1);
  out["result"] = res;
  out["placement"] = Json::parse(placement_json(w, d));
  bo.json = out.dump();
  return bo;
}

std::string Platform::schedule(const std::string& workload_json) {
  WorkloadRequest w = workload_from_json(Json::parse(workload_json));
  if (w.partition && cfg_.auto_provision_partitions) {
    Decision probe = sched_->schedule(w);
    if (probe.ok) return placement_json(w, probe);
    part_->ensure_capacity(w.partition_mode, w.partition_count, false,
                           w.partition_memory_set ? &w.partition_memory : nullptr);
  }
  Decision d = sched_->schedule(w);
  reg_->add("kgwe_scheduling_attempts_total", {}, 1);
  if (d.ok) reg_->add("kgwe_scheduling_successes_total", {}, 1);
  else reg_->add("kgwe_scheduling_failures_total", {"unschedulable"}, 1);
  reg_->add("kgwe_preemptions_total", {}, static_cast<double>(d.preempted.size()));
  // Victims lose their GPUs now: stop metering them (their pods must be
  // evicted by the caller — the controller's eviction path).
  for (const auto& v : d.preempted) {
    UsageRecord r;
    cost_->finalize(v, wall_s(), &r);
  }
  return placement_json(w, d);
}

std::string Platform::release(const std::string& uid, double now_s) {
  Allocation a;
  const bool had = sched_->allocation(uid, &a);
  bool was_leader = false;
  const std::vector<std::string> group_peers = sched_->share_group_peers(uid, &was_leader);
  bool ok = sched_->release(uid);
  {
    std::lock_guard<std::mutex> lk(pods_mu_);
    pending_.erase(uid);
  }
  UsageRecord r;
  Json out = Json::object();
  out["released"] = ok;
  if (ok && was_leader && !group_peers.empty()) {
    // The group's serving process went with its leader: the members have
    // nothing to connect to.  The controller evicts them; rescheduled, the
    // first becomes the new leader.
    Json oj = Json::array();
    for (const auto& p : group_peers) oj.push_back(p);
    out["orphaned_share_members"] = oj;
  }
  {
    // A preemption victim whose gang has members on other nodes: they are
    // the controller's to evict (see preempt()).
    std::vector<std::string> peers;
    {
      std::lock_guard<std::mutex> lk(pods_mu_);
      auto it = gang_peers_.find(uid);
      if (it != gang_peers_.end()) {
        if (now_ns() - it->second.second < 120LL * 1000000000) peers = it->second.first;
        gang_peers_.erase(it);
      }
    }
    Json pj = Json::array();
    for (const auto& p : peers)
      if (sched_->allocation(p, nullptr)) pj.push_back(p);
    if (pj.size()) out["evict_gang_peers"] = pj;
  }
  if (cost_->finalize(uid, now_s, &r)) {
    out["cost"] = to_json(r);
    reg_->observe("kgwe_workload_duration_seconds", {to_string(a.type)}, r.duration_s);
  }
  if (had && !a.partitions.empty()) {
    GpuDevice g;
    std::string mode = "CPX";
    if (disc_->gpu(a.partitions[0].substr(0, a.partitions[0].rfind("/p")), &g))
      mode = to_string(g.partition.compute);
    reg_->add("kgwe_partition_releases_total", {mode}, static_cast<double>(a.partitions.size()));
  }
  return out.dump();
}

void Platform::observe_pod_latency_ms(double ms) {
  reg_->observe("kgwe_scheduling_latency_ms", {}, ms);
  pod_latency_.record_ms(ms);
}

std::string Platform::consolidate_partitions(double now_s, bool move_in_ledger) {
  auto moves = part_->consolidate(now_s, cfg_.consolidate, move_in_ledger);
  Json out = Json::array();
  for (const auto& m : moves) {
    out.push_back(to_json(m));
    reg_->add("kgwe_partition_migrations_total", {}, 1);
  }
  return out.dump();
}

void Platform::tick(double now_s) {
  sched_->expire_gangs();
  // Feed cost metering with live utilisation of each allocation's GPUs.
  auto snap = disc_->snapshot();
  for (const auto& a : sched_->allocations()) {
    auto it = snap->nodes.find(a.node);
    if (it == snap->nodes.end()) continue;
    double gfx = 0, mem = 0;
    int n = 0;
    for (const auto& u : a.gpus)
      if (const GpuDevice* g = it->second.gpu(u)) {
        gfx += g->util.gfx_activity;
        mem += g->util.memory_used_pct;
        ++n;
      }
    for (const auto& p : a.partitions)
      if (const GpuDevice* g = it->second.gpu(p.substr(0, p.rfind("/p")))) {
        gfx += g->util.gfx_activity;
        mem += g->util.memory_used_pct;
        ++n;
      }
    if (n) cost_->sample(a.uid, gfx / n, mem / n, now_s);
  }
  if (cfg_.partition_reclaim_idle_s >= 0)
    part_->reclaim_idle_after(now_s, cfg_.partition_reclaim_idle_s);
  const int64_t t0 = now_ns();
  if (t0 >= gauges_next_ns_.load()) {
    refresh_gauges(now_s);
    const int64_t t1 = now_ns();
    gauges_next_ns_.store(t1 + 9 * (t1 - t0));
  }
}

void Platform::refresh_gauges(double now_s) {
  std::lock_guard<std::mutex> refresh_lk(gauges_mu_);  // tick and a scrape may both come here
  auto snap = disc_->snapshot();
  GaugeBatch batch;  // built off-lock, swapped in at the end
  for (const char* f : {"kgwe_gpu_count", "kgwe_gpu_utilization_percent", "kgwe_gpu_gfx_activity_percent",
                        "kgwe_gpu_umc_activity_percent", "kgwe_gpu_memory_used_bytes",
                        "kgwe_gpu_memory_total_bytes", "kgwe_gpu_temperature_celsius", "kgwe_gpu_power_watts",
                        "kgwe_gpu_health_status", "kgwe_gpu_hbm_bandwidth_gbps", "kgwe_gpu_ecc_errors_total",
                        "kgwe_gpu_retired_pages", "kgwe_gpu_xgmi_errors", "kgwe_gpu_cper_records",
                        "kgwe_gpu_throttle_active",
                        "kgwe_gpu_partition_mode", "kgwe_partition_instance_count",
                        "kgwe_partition_instance_utilization_percent", "kgwe_xgmi_bandwidth_gbps",
                        "kgwe_xgmi_link_status", "kgwe_pcie_bandwidth_gbps", "kgwe_topology_score",
                        "kgwe_active_workloads", "kgwe_budget_utilization_percent",
                        "kgwe_cost_savings_recommended_dollars", "kgwe_gpu_cost_per_hour_dollars",
                        "kgwe_gpu_share_clients"})
    batch.touch(f);
  const std::vector<Allocation> allocs = sched_->allocations();
  std::set<std::string> owned_parts;
  for (const auto& a : allocs)
    for (const auto& p : a.partitions) owned_parts.insert(p);
  // Everything that derives from a node's topology object alone goes into
  // per-node blocks, rebuilt only for nodes whose object changed since the
  // last refresh: at 10,000 GPUs a from-scratch refresh is ~250,000 series
  // (~0.5 s of CPU, and a million small allocations whose release stalled the
  // next allocation of the same thread for ~150 ms).
  for (auto it = node_gauges_.begin(); it != node_gauges_.end();)
    it = snap->nodes.count(it->first) ? std::next(it) : node_gauges_.erase(it);
  for (const auto& kv : snap->nodes) {
    const NodeTopology& n = kv.second;
    NodeGauges& ng = node_gauges_[n.name];
    if (ng.topo != &n || ng.updated_ns != n.updated_ns || ng.blocks.empty()) {
      std::map<std::string, MetricRegistry::Block> b;
      b["kgwe_gpu_count"].push_back({{n.name}, static_cast<double>(n.gpus.size())});
      int links_up = 0, links = 0;
      for (const auto& g : n.gpus) {
        b["kgwe_gpu_utilization_percent"].push_back({{g.uuid, n.name, g.model}, g.util.gfx_activity});
        b["kgwe_gpu_gfx_activity_percent"].push_back({{g.uuid, n.name}, g.util.gfx_activity});
        b["kgwe_gpu_umc_activity_percent"].push_back({{g.uuid, n.name}, g.util.umc_activity});
        b["kgwe_gpu_memory_used_bytes"].push_back({{g.uuid, n.name}, g.memory_used_gb * 1073741824.0});
        b["kgwe_gpu_memory_total_bytes"].push_back({{g.uuid, n.name}, g.memory_total_gb * 1073741824.0});
        b["kgwe_gpu_temperature_celsius"].push_back({{g.uuid, n.name}, g.util.temperature_c});
        b["kgwe_gpu_power_watts"].push_back({{g.uuid, n.name}, g.util.power_w});
        b["kgwe_gpu_health_status"].push_back(
            {{g.uuid, n.name}, g.health.status == HealthStatus::Healthy ? 1.0
                               : g.health.status == HealthStatus::Degraded ? 0.5 : 0.0});
        if (g.hbm_measured_gbps > 0)
          b["kgwe_gpu_hbm_bandwidth_gbps"].push_back({{g.uuid, n.name}, g.hbm_measured_gbps});
        auto& ecc = b["kgwe_gpu_ecc_errors_total"];
        ecc.push_back({{g.uuid, n.name, "correctable"}, static_cast<double>(g.health.ecc_correctable)});
        ecc.push_back({{g.uuid, n.name, "uncorrectable"}, static_cast<double>(g.health.ecc_uncorrectable)});
        ecc.push_back({{g.uuid, n.name, "deferred"}, static_cast<double>(g.health.ecc_deferred)});
        auto& rp = b["kgwe_gpu_retired_pages"];
        rp.push_back({{g.uuid, n.name, "retired"}, static_cast<double>(g.health.retired_pages)});
        rp.push_back({{g.uuid, n.name, "pending"}, static_cast<double>(g.health.pending_retired_pages)});
        b["kgwe_gpu_xgmi_errors"].push_back({{g.uuid, n.name}, static_cast<double>(g.health.xgmi_errors)});
        auto& cp = b["kgwe_gpu_cper_records"];
        cp.push_back({{g.uuid, n.name, "fatal"}, static_cast<double>(g.health.cper_fatal)});
        cp.push_back({{g.uuid, n.name, "uncorrected"}, static_cast<double>(g.health.cper_uncorrected)});
        cp.push_back({{g.uuid, n.name, "corrected"}, static_cast<double>(g.health.cper_corrected)});
        for (const auto& t : g.health.throttle_reasons)
          b["kgwe_gpu_throttle_active"].push_back({{g.uuid, n.name, t}, 1.0});
        b["kgwe_gpu_partition_mode"].push_back(
            {{g.uuid, n.name, to_string(g.partition.compute), to_string(g.partition.memory)}, 1.0});
        b["kgwe_partition_instance_count"].push_back(
            {{g.uuid, n.name, to_string(g.partition.compute)}, static_cast<double>(g.partition.instances.size())});
        b["kgwe_pcie_bandwidth_gbps"].push_back({{g.uuid, n.name}, g.pcie.bandwidth_gbps});
        for (const auto& l : g.links) {
          b["kgwe_xgmi_bandwidth_gbps"].push_back({{g.uuid, l.peer_uuid, n.name}, l.up ? l.effective_gbps() : 0.0});
          b["kgwe_xgmi_link_status"].push_back({{g.uuid, l.peer_uuid, n.name}, l.up ? 1.0 : 0.0});
          ++links;
          links_up += l.up && l.type == LinkType::XGMI;
        }
      }
      // Node topology score: 50 base, +30 full xGMI mesh, +20 proportional link health.
      const double ts = 50.0 + (n.xgmi_fully_connected ? 30.0 : 0.0) + (links ? 20.0 * links_up / links : 0.0);
      b["kgwe_topology_score"].push_back({{n.name}, ts});
      ng.topo = &n;
      ng.updated_ns = n.updated_ns;
      ng.blocks.clear();
      for (auto& fb : b)
        ng.blocks[fb.first] = std::make_shared<const MetricRegistry::Block>(std::move(fb.second));
    }
    for (const auto& fb : ng.blocks) batch.block(fb.first, n.name, fb.second);
    // Slice occupancy depends on the ledger: computed every time, only for
    // nodes that have partitioned GPUs.
    std::map<std::string, std::pair<int, int>> slices;  // mode -> (used, total)
    for (const auto& g : n.gpus) {
      if (g.partition.compute == ComputePartition::SPX) continue;
      auto& sl = slices[to_string(g.partition.compute)];
      for (const auto& pi : g.partition.instances) {
        sl.second++;
        sl.first += (pi.in_use || owned_parts.count(pi.id)) ? 1 : 0;
      }
    }
    for (const auto& sl : slices)
      batch.set("kgwe_partition_instance_utilization_percent", {n.name, sl.first},
                sl.second.second ? 100.0 * sl.second.first / sl.second.second : 0.0);
  }
  for (const auto& a : allocs)
    if (!a.shared_gpu.empty())
      batch.add("kgwe_gpu_share_clients", {a.shared_gpu, a.node, to_string(a.sharing)}, 1.0);
  std::map<std::pair<std::string, std::string>, int> active;
  for (const auto& a : allocs) active[{a.ns, to_string(a.type)}]++;
  for (const auto& kv : active)
    batch.set("kgwe_active_workloads", {kv.first.first, kv.first.second}, kv.second);
  for (const auto& b : cost_->budgets(now_s))
    batch.set("kgwe_budget_utilization_percent", {b.id, to_string(b.scope)},
              b.limit > 0 ? 100.0 * b.spend / b.limit : 0.0);
  std::map<std::string, double> saving;
  for (const auto& r : cost_->recommendations("", "")) saving[r.type] += r.saving;
  for (const auto& kv : saving) batch.set("kgwe_cost_savings_recommended_dollars", {kv.first}, kv.second);
  batch.set("kgwe_gpu_cost_per_hour_dollars", {"all"}, cost_->running_cost_per_hour());
  {
    // Pods filtered but never bound nor released within an hour were deleted
    // behind our back (no release call): age them out of the queue.
    std::lock_guard<std::mutex> lk(pods_mu_);
    const int64_t horizon = now_ns() - static_cast<int64_t>(3600) * 1000000000;
    for (auto it = pending_.begin(); it != pending_.end();)
      it = it->second.first < horizon ? pending_.erase(it) : std::next(it);
  }
  reg_->commit(std::move(batch));
  reg_->set("kgwe_workload_queue_depth", {}, static_cast<double>(queue_depth()));
  const SchedulerMetrics sm = sched_->metrics();
  reg_->set("kgwe_preemptions_deferred_total", {"wait"}, static_cast<double>(sm.preemptions_deferred_wait));
  reg_->set("kgwe_preemptions_deferred_total", {"rate"}, static_cast<double>(sm.preemptions_rate_limited));
}

std::string Platform::expose_metrics() {
  refresh_gauges(wall_s());
  return reg_->expose();
}

}  // namespace kgwe
