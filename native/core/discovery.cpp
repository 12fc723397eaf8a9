#include "discovery.h"

#include <algorithm>
#include <chrono>
#include <set>

namespace kgwe {

const char* to_string(TopologyEventType t) {
  switch (t) {
    case TopologyEventType::NodeAdded: return "NodeAdded";
    case TopologyEventType::NodeRemoved: return "NodeRemoved";
    case TopologyEventType::NodeUpdated: return "NodeUpdated";
    case TopologyEventType::HealthChanged: return "HealthChanged";
    case TopologyEventType::LinkDown: return "LinkDown";
    case TopologyEventType::LinkUp: return "LinkUp";
    case TopologyEventType::PartitionChanged: return "PartitionChanged";
  }
  return "Unknown";
}

DiscoveryService::DiscoveryService(int refresh_interval_ms, size_t event_capacity)
    : snap_(std::make_shared<ClusterTopology>()), ev_cap_(event_capacity),
      interval_ms_(refresh_interval_ms) {}

DiscoveryService::~DiscoveryService() { stop(); }

void DiscoveryService::add_node(const std::string& name, std::shared_ptr<Hal> hal) {
  {
    std::lock_guard<std::mutex> lk(hal_mu_);
    hals_[name] = std::move(hal);
  }
  // Discover just this node and publish.
  std::shared_ptr<Hal> h = this->hal(name);
  NodeTopology n = h->discover(name);
  std::lock_guard<std::mutex> lk(publish_mu_);
  auto prev = snapshot();
  auto next = std::make_shared<ClusterTopology>(*prev);
  next->nodes[name] = std::move(n);
  publish(next, prev);
}

void DiscoveryService::remove_node(const std::string& name) {
  {
    std::lock_guard<std::mutex> lk(hal_mu_);
    hals_.erase(name);
    pushed_.erase(name);
  }
  std::lock_guard<std::mutex> lk(publish_mu_);
  auto prev = snapshot();
  auto next = std::make_shared<ClusterTopology>(*prev);
  next->nodes.erase(name);
  publish(next, prev);
}

void DiscoveryService::upsert_node(const NodeTopology& node) {
  {
    std::lock_guard<std::mutex> lk(hal_mu_);
    pushed_[node.name] = node;
  }
  std::lock_guard<std::mutex> lk(publish_mu_);
  auto prev = snapshot();
  auto next = std::make_shared<ClusterTopology>(*prev);
  next->nodes[node.name] = node;
  publish(next, prev);
}

void DiscoveryService::refresh() {
  std::vector<std::pair<std::string, std::shared_ptr<Hal>>> hs;
  std::map<std::string, NodeTopology> pushed;
  {
    std::lock_guard<std::mutex> lk(hal_mu_);
    hs.assign(hals_.begin(), hals_.end());
    pushed = pushed_;
  }
  // Discovery runs without any lock readers could contend on.
  auto next = std::make_shared<ClusterTopology>();
  for (auto& kv : hs) next->nodes[kv.first] = kv.second->discover(kv.first);
  for (auto& kv : pushed) next->nodes[kv.first] = kv.second;
  std::lock_guard<std::mutex> lk(publish_mu_);
  publish(next, snapshot());
}

bool DiscoveryService::refresh_node(const std::string& name) {
  std::shared_ptr<Hal> h = hal(name);
  if (!h) return false;
  NodeTopology n = h->discover(name);
  std::lock_guard<std::mutex> lk(publish_mu_);
  auto prev = snapshot();
  auto next = std::make_shared<ClusterTopology>(*prev);
  next->nodes[name] = std::move(n);
  publish(next, prev);
  return true;
}

void DiscoveryService::refresh_telemetry() {
  std::vector<std::pair<std::string, std::shared_ptr<Hal>>> hs;
  {
    std::lock_guard<std::mutex> lk(hal_mu_);
    hs.assign(hals_.begin(), hals_.end());
  }
  std::lock_guard<std::mutex> lk(publish_mu_);
  auto prev = snapshot();
  auto next = std::make_shared<ClusterTopology>(*prev);
  for (auto& kv : hs) {
    auto it = next->nodes.find(kv.first);
    if (it != next->nodes.end()) kv.second->refresh_telemetry(it->second);
  }
  publish(next, prev);
}

void DiscoveryService::publish(std::shared_ptr<ClusterTopology> next, const TopologySnapshot& prev) {
  next->generation = prev->generation + 1;
  next->updated_ns = now_ns();
  // Diff -> events.
  for (const auto& kv : next->nodes) {
    auto pit = prev->nodes.find(kv.first);
    if (pit == prev->nodes.end()) {
      emit({TopologyEventType::NodeAdded, kv.first, "", "", now_ns()});
      continue;
    }
    const NodeTopology& old = pit->second;
    for (const auto& g : kv.second.gpus) {
      const GpuDevice* og = old.gpu(g.uuid);
      if (!og) continue;
      if (og->health.status != g.health.status)
        emit({TopologyEventType::HealthChanged, kv.first, g.uuid,
              std::string(to_string(og->health.status)) + "->" + to_string(g.health.status),
              now_ns()});
      if (og->partition.compute != g.partition.compute ||
          og->partition.memory != g.partition.memory)
        emit({TopologyEventType::PartitionChanged, kv.first, g.uuid,
              std::string(to_string(g.partition.compute)) + "/" + to_string(g.partition.memory),
              now_ns()});
      for (const auto& l : g.links) {
        const XgmiLink* ol = og->link_to(l.peer_uuid);
        if (ol && ol->up != l.up)
          emit({l.up ? TopologyEventType::LinkUp : TopologyEventType::LinkDown, kv.first, g.uuid,
                l.peer_uuid, now_ns()});
      }
    }
  }
  for (const auto& kv : prev->nodes)
    if (!next->nodes.count(kv.first))
      emit({TopologyEventType::NodeRemoved, kv.first, "", "", now_ns()});
  std::shared_ptr<const ClusterTopology> c = std::move(next);
  std::atomic_store(&snap_, c);
}

TopologySnapshot DiscoveryService::snapshot() const { return std::atomic_load(&snap_); }

uint64_t DiscoveryService::generation() const { return snapshot()->generation; }

bool DiscoveryService::node(const std::string& name, NodeTopology* out) const {
  auto s = snapshot();
  auto it = s->nodes.find(name);
  if (it == s->nodes.end()) return false;
  if (out) *out = it->second;
  return true;
}

bool DiscoveryService::gpu(const std::string& uuid, GpuDevice* out) const {
  auto s = snapshot();
  for (const auto& kv : s->nodes)
    if (const GpuDevice* g = kv.second.gpu(uuid)) {
      if (out) *out = *g;
      return true;
    }
  return false;
}

std::shared_ptr<Hal> DiscoveryService::hal(const std::string& node) const {
  std::lock_guard<std::mutex> lk(hal_mu_);
  auto it = hals_.find(node);
  return it == hals_.end() ? nullptr : it->second;
}

void DiscoveryService::emit(TopologyEvent e) {
  std::lock_guard<std::mutex> lk(ev_mu_);
  if (events_.size() >= ev_cap_) {
    events_.pop_front();
    dropped_.fetch_add(1);
  }
  events_.push_back(std::move(e));
}

std::vector<TopologyEvent> DiscoveryService::drain_events(size_t max) {
  std::lock_guard<std::mutex> lk(ev_mu_);
  std::vector<TopologyEvent> out;
  size_t n = max == 0 ? events_.size() : std::min(max, events_.size());
  for (size_t i = 0; i < n; ++i) {
    out.push_back(std::move(events_.front()));
    events_.pop_front();
  }
  return out;
}

void DiscoveryService::start() {
  std::lock_guard<std::mutex> lk(run_mu_);
  if (running_) return;
  running_ = true;
  thread_ = std::thread([this] { loop(); });
}

void DiscoveryService::stop() {
  {
    std::lock_guard<std::mutex> lk(run_mu_);
    if (!running_) return;
    running_ = false;
  }
  run_cv_.notify_all();
  if (thread_.joinable()) thread_.join();
}

void DiscoveryService::loop() {
  std::unique_lock<std::mutex> lk(run_mu_);
  while (running_) {
    run_cv_.wait_for(lk, std::chrono::milliseconds(interval_ms_), [this] { return !running_; });
    if (!running_) break;
    lk.unlock();
    refresh();
    lk.lock();
  }
}

// ---------------------------------------------------------------------------
// Topology hints (reference C5: discovery.go:222-559), MI355X semantics:
// candidate GPUs are healthy and (whole-GPU) not busy (gfx < 90 %) or have a
// free partition slice; a group "is xGMI" when all pairs have an up xGMI link.
// Score: 50 base, +30 fully connected xGMI group, +10 single NUMA domain,
// +5 per GPU of the requested arch.
// ---------------------------------------------------------------------------
std::vector<TopologyHint> DiscoveryService::hints(const HintRequest& req, size_t max_results) const {
  auto s = snapshot();
  std::vector<TopologyHint> out;
  for (const auto& kv : s->nodes) {
    const NodeTopology& n = kv.second;
    std::vector<const GpuDevice*> avail;
    for (const auto& g : n.gpus) {
      if (!g.healthy()) continue;
      if (g.partition.compute != ComputePartition::SPX) {
        bool free_slice = false;
        for (const auto& pi : g.partition.instances) free_slice |= !pi.in_use;
        if (!free_slice) continue;
      } else if (g.util.gfx_activity >= 90.0) {
        continue;
      }
      if (g.memory_free_gb() < req.min_memory_gb) continue;
      avail.push_back(&g);
    }
    if (static_cast<int>(avail.size()) < req.gpu_count) continue;
    TopologyHint h;
    h.node = n.name;
    h.score = 50;
    // Greedy fully-connected group, started from each GPU, best by aggregate bw.
    std::vector<const GpuDevice*> best;
    double best_bw = -1.0;
    for (const GpuDevice* start : avail) {
      std::vector<const GpuDevice*> grp{start};
      double bw = 0.0;
      while (static_cast<int>(grp.size()) < req.gpu_count) {
        const GpuDevice* pick = nullptr;
        double pick_bw = -1.0;
        for (const GpuDevice* c : avail) {
          if (std::find(grp.begin(), grp.end(), c) != grp.end()) continue;
          double agg = 0.0;
          bool ok = true;
          for (const GpuDevice* m : grp) {
            const XgmiLink* l = c->link_to(m->uuid);
            if (!l || !l->up || l->type != LinkType::XGMI) { ok = false; break; }
            agg += l->effective_gbps();
          }
          if (ok && agg > pick_bw) { pick = c; pick_bw = agg; }
        }
        if (!pick) break;
        grp.push_back(pick);
        bw += pick_bw;
      }
      if (static_cast<int>(grp.size()) == req.gpu_count && bw > best_bw) {
        best = grp;
        best_bw = bw;
      }
    }
    bool xgmi_group = !best.empty() && req.gpu_count > 1;
    if (best.empty()) best.assign(avail.begin(), avail.begin() + req.gpu_count);
    if (xgmi_group && req.prefer_xgmi) {
      h.score += 30;
      h.reasons.push_back("fully connected xGMI group");
    }
    std::set<int> numa;
    for (auto* g : best) numa.insert(g->numa_node);
    if (numa.size() == 1 && req.prefer_same_numa) {
      h.score += 10;
      h.reasons.push_back("single NUMA domain");
    }
    for (auto* g : best) {
      h.gpus.push_back(g->uuid);
      if (!req.arch.empty() && g->arch == req.arch) h.score += 5;
    }
    // Bandwidth estimate: mean pairwise effective xGMI bw, PCIe when no link.
    double sum = 0.0;
    int pairs = 0;
    for (size_t i = 0; i < best.size(); ++i)
      for (size_t j = i + 1; j < best.size(); ++j) {
        const XgmiLink* l = best[i]->link_to(best[j]->uuid);
        sum += (l && l->up) ? l->effective_gbps() : best[i]->pcie.bandwidth_gbps;
        ++pairs;
      }
    h.bandwidth_gbps = pairs ? sum / pairs : 0.0;
    if (h.score >= 80) h.reasons.push_back("optimal xGMI placement");
    else if (h.score >= 60) h.reasons.push_back("partial xGMI placement");
    else h.reasons.push_back("PCIe placement");
    out.push_back(std::move(h));
  }
  std::sort(out.begin(), out.end(), [](const TopologyHint& a, const TopologyHint& b) {
    return a.score != b.score ? a.score > b.score : a.node < b.node;
  });
  if (max_results && out.size() > max_results) out.resize(max_results);
  return out;
}

}  // namespace kgwe
