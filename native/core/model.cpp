#include "model.h"

#include <cstring>
#include <functional>

#include <chrono>

namespace kgwe {

void index_links(NodeTopology& n) {
  const size_t G = n.gpus.size();
  n.link_bw.assign(G * G, 0.0f);
  n.link_up.assign(G * G, 0);
  uint64_t h = 1469598103934665603ull;  // FNV-1a over everything placement reads
  auto mix = [&h](uint64_t v) {
    h ^= v;
    h *= 1099511628211ull;
  };
  mix(G);
  for (size_t i = 0; i < G; ++i) {
    const GpuDevice& a = n.gpus[i];
    mix(static_cast<uint64_t>(a.numa_node + 7));
    mix(std::hash<std::string>{}(a.pcie.switch_id));
    mix(a.healthy() ? 1 : 2);
    for (size_t j = 0; j < G; ++j) {
      if (i == j) continue;
      const GpuDevice& b = n.gpus[j];
      const XgmiLink* l1 = a.link_to(b.uuid);
      const XgmiLink* l2 = b.link_to(a.uuid);
      const bool up1 = l1 && l1->up && l1->type == LinkType::XGMI;
      const bool up2 = l2 ? (l2->up && l2->type == LinkType::XGMI) : up1;
      double bw;
      if (up1 && up2) {
        bw = l1->effective_gbps();
        if (l2) bw = std::min(bw, l2->effective_gbps());
      } else {
        bw = std::min(a.pcie.bandwidth_gbps, b.pcie.bandwidth_gbps);
      }
      n.link_bw[i * G + j] = static_cast<float>(bw);
      n.link_up[i * G + j] = up1 && up2;
      uint32_t bits;
      const float fb = static_cast<float>(bw);
      std::memcpy(&bits, &fb, sizeof bits);
      mix(bits ^ (static_cast<uint64_t>(up1 && up2) << 32));
      // degraded-link count input of the 1-GPU best fit
      if (l1) mix((l1->up ? 3 : 5) ^ static_cast<uint64_t>(l1->measured_gbps * 16));
    }
  }
  n.topo_fp = h ? h : 1;
}

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

const char* to_string(HealthStatus s) {
  switch (s) {
    case HealthStatus::Healthy: return "Healthy";
    case HealthStatus::Degraded: return "Degraded";
    case HealthStatus::Unhealthy: return "Unhealthy";
    default: return "Unknown";
  }
}
const char* to_string(LinkType t) {
  switch (t) {
    case LinkType::XGMI: return "XGMI";
    case LinkType::PCIE: return "PCIE";
    default: return "Unknown";
  }
}
const char* to_string(ComputePartition p) {
  switch (p) {
    case ComputePartition::SPX: return "SPX";
    case ComputePartition::DPX: return "DPX";
    case ComputePartition::TPX: return "TPX";
    case ComputePartition::QPX: return "QPX";
    case ComputePartition::CPX: return "CPX";
  }
  return "SPX";
}
const char* to_string(MemoryPartition p) {
  switch (p) {
    case MemoryPartition::NPS1: return "NPS1";
    case MemoryPartition::NPS2: return "NPS2";
    case MemoryPartition::NPS4: return "NPS4";
    case MemoryPartition::NPS8: return "NPS8";
  }
  return "NPS1";
}
HealthStatus health_from(const std::string& s) {
  if (s == "Healthy") return HealthStatus::Healthy;
  if (s == "Degraded") return HealthStatus::Degraded;
  if (s == "Unhealthy") return HealthStatus::Unhealthy;
  return HealthStatus::Unknown;
}
LinkType link_from(const std::string& s) {
  if (s == "XGMI" || s == "xgmi") return LinkType::XGMI;
  if (s == "PCIE" || s == "pcie" || s == "PCIe") return LinkType::PCIE;
  return LinkType::Unknown;
}
ComputePartition compute_partition_from(const std::string& s) {
  if (s == "DPX") return ComputePartition::DPX;
  if (s == "TPX") return ComputePartition::TPX;
  if (s == "QPX") return ComputePartition::QPX;
  if (s == "CPX") return ComputePartition::CPX;
  return ComputePartition::SPX;
}
MemoryPartition memory_partition_from(const std::string& s) {
  if (s == "NPS2") return MemoryPartition::NPS2;
  if (s == "NPS4") return MemoryPartition::NPS4;
  if (s == "NPS8") return MemoryPartition::NPS8;
  return MemoryPartition::NPS1;
}
int partition_count(ComputePartition p) {
  switch (p) {
    case ComputePartition::SPX: return 1;
    case ComputePartition::DPX: return 2;
    case ComputePartition::TPX: return 3;
    case ComputePartition::QPX: return 4;
    case ComputePartition::CPX: return 8;
  }
  return 1;
}

const XgmiLink* GpuDevice::link_to(const std::string& peer) const {
  for (const auto& l : links)
    if (l.peer_uuid == peer) return &l;
  return nullptr;
}

const GpuDevice* NodeTopology::gpu(const std::string& uuid) const {
  for (const auto& g : gpus)
    if (g.uuid == uuid) return &g;
  return nullptr;
}
GpuDevice* NodeTopology::gpu(const std::string& uuid) {
  for (auto& g : gpus)
    if (g.uuid == uuid) return &g;
  return nullptr;
}

int ClusterTopology::total_gpus() const {
  int n = 0;
  for (const auto& kv : nodes) n += static_cast<int>(kv.second.gpus.size());
  return n;
}

GpuDevice gpu_from_json(const Json& j, const std::string& node) {
  GpuDevice g;
  g.uuid = j.get("uuid").str();
  g.index = static_cast<int>(j.get("index").as_int(0));
  g.node = node;
  g.model = j.get("model").str(g.model);
  g.arch = j.get("arch").str(g.arch);
  g.cu_count = static_cast<int>(j.get("cu_count").as_int(g.cu_count));
  g.xcd_count = static_cast<int>(j.get("xcd_count").as_int(g.xcd_count));
  g.memory_total_gb = j.get("memory_total_gb").as_number(g.memory_total_gb);
  g.memory_used_gb = j.get("memory_used_gb").as_number(0.0);
  g.hbm_rated_gbps = j.get("hbm_rated_gbps").as_number(g.hbm_rated_gbps);
  g.hbm_measured_gbps = j.get("hbm_measured_gbps").as_number(0.0);
  g.peak_bf16_tflops = j.get("peak_bf16_tflops").as_number(g.peak_bf16_tflops);
  g.numa_node = static_cast<int>(j.get("numa_node").as_int(0));
  g.socket = static_cast<int>(j.get("socket").as_int(g.numa_node));
  const Json& pc = j.get("pcie");
  g.pcie.bdf = pc.get("bdf").str();
  g.pcie.switch_id = pc.get("switch_id").str();
  g.pcie.generation = static_cast<int>(pc.get("generation").as_int(5));
  g.pcie.width = static_cast<int>(pc.get("width").as_int(16));
  g.pcie.bandwidth_gbps = pc.get("bandwidth_gbps").as_number(63.0);
  for (const auto& lj : j.get("links").items()) {
    XgmiLink l;
    l.peer_uuid = lj.get("peer").str();
    l.type = link_from(lj.get("type").str("XGMI"));
    l.hops = static_cast<int>(lj.get("hops").as_int(1));
    l.rated_gbps = lj.get("rated_gbps").as_number(l.type == LinkType::XGMI ? 153.6 : 63.0);
    l.measured_gbps = lj.get("measured_gbps").as_number(0.0);
    l.up = lj.get("up").as_bool(true);
    g.links.push_back(l);
  }
  const Json& pj = j.get("partition");
  g.partition.compute = compute_partition_from(pj.get("compute").str("SPX"));
  g.partition.memory = memory_partition_from(pj.get("memory").str("NPS1"));
  g.partition.switching = pj.get("switching").as_bool(false);
  const int np = partition_count(g.partition.compute);
  const auto& inst = pj.get("instances").items();
  for (int i = 0; i < np; ++i) {
    PartitionInstance pi;
    pi.index = i;
    pi.id = g.uuid + "/p" + std::to_string(i);
    pi.cu_count = g.cu_count / np;
    pi.memory_gb = g.memory_total_gb / np;
    if (i < static_cast<int>(inst.size())) {
      pi.in_use = inst[i].get("in_use").as_bool(false);
      pi.owner = inst[i].get("owner").str();
    }
    g.partition.instances.push_back(pi);
  }
  const Json& u = j.get("util");
  g.util.gfx_activity = u.get("gfx_activity").as_number(0.0);
  g.util.umc_activity = u.get("umc_activity").as_number(0.0);
  g.util.memory_used_pct = g.memory_total_gb > 0 ? 100.0 * g.memory_used_gb / g.memory_total_gb : 0.0;
  g.util.power_w = u.get("power_w").as_number(0.0);
  g.util.temperature_c = u.get("temperature_c").as_number(0.0);
  g.util.gfx_clock_mhz = u.get("gfx_clock_mhz").as_number(0.0);
  const Json& h = j.get("health");
  g.health.status = health_from(h.get("status").str("Healthy"));
  for (const auto& r : h.get("reasons").items()) g.health.reasons.push_back(r.str());
  g.health.ecc_correctable = h.get("ecc_correctable").as_int(0);
  g.health.ecc_uncorrectable = h.get("ecc_uncorrectable").as_int(0);
  g.health.ecc_deferred = h.get("ecc_deferred").as_int(0);
  g.health.xgmi_errors = static_cast<int>(h.get("xgmi_errors").as_int(0));
  g.health.xgmi_links_down = static_cast<int>(h.get("xgmi_links_down").as_int(0));
  g.health.retired_pages = h.get("retired_pages").as_int(0);
  g.health.pending_retired_pages = h.get("pending_retired_pages").as_int(0);
  g.health.cper_fatal = h.get("cper_fatal").as_int(0);
  g.health.cper_uncorrected = h.get("cper_uncorrected").as_int(0);
  g.health.cper_corrected = h.get("cper_corrected").as_int(0);
  for (const auto& r : h.get("throttle").items()) g.health.throttle_reasons.push_back(r.str());
  g.health.perf_degraded = h.get("perf_degraded").as_bool(false);
  g.health.perf_reason = h.get("perf_reason").str();
  g.health.pinned = h.get("pinned").as_bool(h.get("status").is_string());
  if (!g.health.pinned) {
    int down = 0;
    for (const auto& l : g.links) down += !l.up;
    apply_health_policy(g.health, down);
  }
  return g;
}

void apply_health_policy(Health& h, int links_down_in_topology) {
  h.status = HealthStatus::Healthy;
  h.reasons.clear();
  auto degrade = [&](const std::string& why) {
    if (h.status == HealthStatus::Healthy) h.status = HealthStatus::Degraded;
    h.reasons.push_back(why);
  };
  auto note = [&](const std::string& why) { h.reasons.push_back(why); };
  auto fail = [&](const std::string& why) {
    h.status = HealthStatus::Unhealthy;
    h.reasons.push_back(why);
  };
  if (h.ecc_uncorrectable > 0) fail(std::to_string(h.ecc_uncorrectable) + " uncorrectable ECC errors");
  if (h.retired_pages >= kRetiredPageLimit)
    fail(std::to_string(h.retired_pages) + " retired HBM pages (limit " + std::to_string(kRetiredPageLimit) + ")");
  if (h.ecc_deferred > 0) degrade(std::to_string(h.ecc_deferred) + " deferred ECC errors");
  if (h.ecc_correctable >= kCorrectableStorm)
    degrade("correctable ECC storm (" + std::to_string(h.ecc_correctable) + ")");
  if (h.pending_retired_pages > 0)
    degrade(std::to_string(h.pending_retired_pages) + " HBM pages pending retirement");
  if (h.cper_fatal > 0) fail(std::to_string(h.cper_fatal) + " fatal CPER error records");
  if (h.xgmi_errors > 0) degrade("xGMI errors reported");
  if (h.cper_uncorrected > 0) degrade(std::to_string(h.cper_uncorrected) + " uncorrected (non-fatal) CPER records");
  if (h.cper_corrected >= kCperCorrectedStorm)
    degrade("corrected CPER storm (" + std::to_string(h.cper_corrected) + ")");
  if (h.perf_degraded) degrade(h.perf_reason.empty() ? "probe: degraded performance" : h.perf_reason);
  const int down = h.xgmi_links_down > links_down_in_topology ? h.xgmi_links_down : links_down_in_topology;
  // A down link is excluded per link by the group search; the GPU itself
  // stays schedulable (single-GPU and partition work never crosses it).
  if (down > 0) note(std::to_string(down) + " xGMI link(s) down");
  for (const auto& t : h.throttle_reasons) note("throttling: " + t);
}

Json to_json(const GpuDevice& g) {
  Json j = Json::object();
  j["uuid"] = g.uuid;
  j["index"] = g.index;
  j["node"] = g.node;
  j["model"] = g.model;
  j["arch"] = g.arch;
  j["cu_count"] = g.cu_count;
  j["xcd_count"] = g.xcd_count;
  j["memory_total_gb"] = g.memory_total_gb;
  j["memory_used_gb"] = g.memory_used_gb;
  j["hbm_rated_gbps"] = g.hbm_rated_gbps;
  j["hbm_measured_gbps"] = g.hbm_measured_gbps;
  j["peak_bf16_tflops"] = g.peak_bf16_tflops;
  j["numa_node"] = g.numa_node;
  j["socket"] = g.socket;
  Json pc = Json::object();
  pc["bdf"] = g.pcie.bdf;
  pc["switch_id"] = g.pcie.switch_id;
  pc["generation"] = g.pcie.generation;
  pc["width"] = g.pcie.width;
  pc["bandwidth_gbps"] = g.pcie.bandwidth_gbps;
  j["pcie"] = pc;
  Json links = Json::array();
  for (const auto& l : g.links) {
    Json lj = Json::object();
    lj["peer"] = l.peer_uuid;
    lj["type"] = to_string(l.type);
    lj["hops"] = l.hops;
    lj["rated_gbps"] = l.rated_gbps;
    lj["measured_gbps"] = l.measured_gbps;
    lj["up"] = l.up;
    links.push_back(lj);
  }
  j["links"] = links;
  Json pj = Json::object();
  pj["compute"] = to_string(g.partition.compute);
  pj["memory"] = to_string(g.partition.memory);
  pj["switching"] = g.partition.switching;
  Json inst = Json::array();
  for (const auto& pi : g.partition.instances) {
    Json ij = Json::object();
    ij["id"] = pi.id;
    ij["index"] = pi.index;
    ij["cu_count"] = pi.cu_count;
    ij["memory_gb"] = pi.memory_gb;
    ij["in_use"] = pi.in_use;
    ij["owner"] = pi.owner;
    inst.push_back(ij);
  }
  pj["instances"] = inst;
  j["partition"] = pj;
  Json u = Json::object();
  u["gfx_activity"] = g.util.gfx_activity;
  u["umc_activity"] = g.util.umc_activity;
  u["memory_used_pct"] = g.util.memory_used_pct;
  u["power_w"] = g.util.power_w;
  u["temperature_c"] = g.util.temperature_c;
  u["gfx_clock_mhz"] = g.util.gfx_clock_mhz;
  j["util"] = u;
  Json h = Json::object();
  h["status"] = to_string(g.health.status);
  Json rs = Json::array();
  for (const auto& r : g.health.reasons) rs.push_back(r);
  h["reasons"] = rs;
  h["ecc_correctable"] = g.health.ecc_correctable;
  h["ecc_uncorrectable"] = g.health.ecc_uncorrectable;
  h["ecc_deferred"] = g.health.ecc_deferred;
  h["xgmi_errors"] = g.health.xgmi_errors;
  h["xgmi_links_down"] = g.health.xgmi_links_down;
  h["retired_pages"] = g.health.retired_pages;
  h["pending_retired_pages"] = g.health.pending_retired_pages;
  h["cper_fatal"] = g.health.cper_fatal;
  h["cper_uncorrected"] = g.health.cper_uncorrected;
  h["cper_corrected"] = g.health.cper_corrected;
  h["pinned"] = g.health.pinned;
  h["perf_degraded"] = g.health.perf_degraded;
  h["perf_reason"] = g.health.perf_reason;
  Json th = Json::array();
  for (const auto& r : g.health.throttle_reasons) th.push_back(r);
  h["throttle"] = th;
  j["health"] = h;
  return j;
}

NodeTopology node_from_json(const Json& j) {
  NodeTopology n;
  n.name = j.get("name").str();
  for (const auto& kv : j.get("labels").fields()) n.labels[kv.first] = kv.second.str();
  for (const auto& t : j.get("taints").items())
    n.taints.emplace_back(t.get("key").str() + "=" + t.get("value").str(), t.get("effect").str());
  n.numa_nodes = static_cast<int>(j.get("numa_nodes").as_int(2));
  n.cpu_sockets = static_cast<int>(j.get("cpu_sockets").as_int(2));
  for (const auto& gj : j.get("gpus").items()) n.gpus.push_back(gpu_from_json(gj, n.name));
  // Fully connected iff every GPU has an up xGMI link to every other.
  bool full = n.gpus.size() > 1;
  for (const auto& a : n.gpus)
    for (const auto& b : n.gpus) {
      if (a.uuid == b.uuid) continue;
      const XgmiLink* l = a.link_to(b.uuid);
      if (!l || l->type != LinkType::XGMI || !l->up) full = false;
    }
  n.xgmi_fully_connected = full;
  n.updated_ns = now_ns();
  return n;
}

Json to_json(const NodeTopology& n) {
  Json j = Json::object();
  j["name"] = n.name;
  Json labels = Json::object();
  for (const auto& kv : n.labels) labels[kv.first] = kv.second;
  j["labels"] = labels;
  Json taints = Json::array();
  for (const auto& t : n.taints) {
    Json tj = Json::object();
    auto eq = t.first.find('=');
    tj["key"] = t.first.substr(0, eq);
    tj["value"] = eq == std::string::npos ? "" : t.first.substr(eq + 1);
    tj["effect"] = t.second;
    taints.push_back(tj);
  }
  j["taints"] = taints;
  j["numa_nodes"] = n.numa_nodes;
  j["cpu_sockets"] = n.cpu_sockets;
  j["xgmi_fully_connected"] = n.xgmi_fully_connected;
  Json gpus = Json::array();
  for (const auto& g : n.gpus) gpus.push_back(to_json(g));
  j["gpus"] = gpus;
  return j;
}

Json to_json(const ClusterTopology& c) {
  Json j = Json::object();
  j["generation"] = static_cast<int64_t>(c.generation);
  j["total_gpus"] = c.total_gpus();
  Json nodes = Json::object();
  for (const auto& kv : c.nodes) nodes[kv.first] = to_json(kv.second);
  j["nodes"] = nodes;
  return j;
}

}  // namespace kgwe
