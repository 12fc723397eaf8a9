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
  next->nodes.set(name, std::move(n));
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
  next->nodes.set(node.name, node);
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
  for (auto& kv : hs) next->nodes.set(kv.first, kv.second->discover(kv.first));
  for (auto& kv : pushed) next->nodes.set(kv.first, kv.second);
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
  next->nodes.set(name, std::move(n));
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
    if (next->nodes.count(kv.first)) {
      NodeTopology& n = next->nodes.mut(kv.first);
      kv.second->refresh_telemetry(n);
      index_links(n);  // telemetry carries link up/down and measured bandwidth
    }
  }
  publish(next, prev);
}

void DiscoveryService::publish(std::shared_ptr<ClusterTopology> next, const TopologySnapshot& prev) {
  std::vector<std::string> unindexed;  // new / re-discovered nodes arrive without link tables
  for (const auto& kv : next->nodes)
    if (kv.second.link_bw.size() != kv.second.gpus.size() * kv.second.gpus.size()) unindexed.push_back(kv.first);
  for (const auto& name : unindexed) index_links(next->nodes.mut(name));
  next->generation = prev->generation + 1;
  next->updated_ns = now_ns();
  // Diff -> events.
  for (const auto& kv : next->nodes) {
    if (next->nodes.same(kv.first, prev->nodes)) continue;  // untouched node: nothing to diff
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

namespace {
// HAL of an agent-pushed node: discovery = the last push; actuation = the
// remote actuator (node agent gRPC SetPartition, authenticated).
class RemoteHal : public Hal {
 public:
  RemoteHal(DiscoveryService* d, std::string node) : d_(d), node_(std::move(node)) {}
  std::string backend() const override { return "agent"; }
  NodeTopology discover(const std::string& name) override {
    NodeTopology n;
    d_->pushed_node(name, &n);
    return n;
  }
  void refresh_telemetry(NodeTopology&) override {}  // the agent pushes telemetry
  std::string set_compute_partition(const std::string& gpu, ComputePartition mode) override {
    return d_->actuate_remote(node_, gpu, to_string(mode), "");
  }
  std::string set_memory_partition(const std::string& gpu, MemoryPartition mode) override {
    return d_->actuate_remote(node_, gpu, "", to_string(mode));
  }

 private:
  DiscoveryService* d_;
  std::string node_;
};
}  // namespace

std::shared_ptr<Hal> DiscoveryService::hal(const std::string& node) const {
  std::lock_guard<std::mutex> lk(hal_mu_);
  auto it = hals_.find(node);
  if (it != hals_.end()) return it->second;
  if (actuator_ && pushed_.count(node))
    return std::make_shared<RemoteHal>(const_cast<DiscoveryService*>(this), node);
  return nullptr;
}

void DiscoveryService::set_remote_actuator(RemoteActuator fn) {
  std::lock_guard<std::mutex> lk(hal_mu_);
  actuator_ = std::move(fn);
}

bool DiscoveryService::pushed_node(const std::string& name, NodeTopology* out) const {
  std::lock_guard<std::mutex> lk(hal_mu_);
  auto it = pushed_.find(name);
  if (it == pushed_.end()) return false;
  *out = it->second;
  return true;
}

std::string DiscoveryService::actuate_remote(const std::string& node, const std::string& gpu,
                                             const std::string& compute, const std::string& memory) {
  RemoteActuator fn;
  {
    std::lock_guard<std::mutex> lk(hal_mu_);
    fn = actuator_;
  }
  if (!fn) return "no remote actuator for node " + node;
  std::string err = fn(node, gpu, compute, memory);  // no lock held across the remote call
  if (!err.empty()) return err;
  std::lock_guard<std::mutex> lk(hal_mu_);
  auto it = pushed_.find(node);
  if (it != pushed_.end())
    if (GpuDevice* g = it->second.gpu(gpu)) {
      if (!compute.empty()) apply_compute_partition(*g, compute_partition_from(compute));
      if (!memory.empty()) g->partition.memory = memory_partition_from(memory);
    }
  return "";
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
  // Pass 1: per node, the best group (greedy on a dense link table) and its
  // score — no strings.  Pass 2 materialises only the hints returned.
  struct Cand {
    const NodeTopology* node;
    std::vector<const GpuDevice*> group;
    int score;
    bool xgmi, one_numa;
  };
  std::vector<Cand> cands;
  cands.reserve(s->nodes.size());
  std::vector<const GpuDevice*> avail;
  std::vector<double> bwm;
  std::vector<int> grp;
  std::vector<char> in;
  for (const auto& kv : s->nodes) {
    const NodeTopology& n = kv.second;
    avail.clear();
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
    const int m = static_cast<int>(avail.size());
    std::vector<const GpuDevice*> best;
    if (req.gpu_count > 1) {
      bwm.assign(static_cast<size_t>(m) * m, -1.0);  // -1: no up xGMI link
      double max_link = 0.0;
      for (int i = 0; i < m; ++i)
        for (const auto& l : avail[i]->links) {
          if (!l.up || l.type != LinkType::XGMI) continue;
          for (int j = 0; j < m; ++j)
            if (j != i && avail[j]->uuid == l.peer_uuid) {
              bwm[static_cast<size_t>(i) * m + j] = l.effective_gbps();
              max_link = std::max(max_link, l.effective_gbps());
              break;
            }
        }
      // Greedy fully-connected group from each start GPU, best by aggregate
      // bandwidth; a group with every pair at the node's best link speed
      // cannot be beaten, so the search stops there.
      const int k = req.gpu_count;
      const double bound = max_link * k * (k - 1) / 2.0;
      double best_bw = -1.0;
      in.assign(m, 0);
      for (int start = 0; start < m && best_bw < bound - 1e-9; ++start) {
        grp.assign(1, start);
        std::fill(in.begin(), in.end(), 0);
        in[start] = 1;
        double bw = 0.0;
        while (static_cast<int>(grp.size()) < k) {
          int pick = -1;
          double pick_bw = -1.0;
          for (int c = 0; c < m; ++c) {
            if (in[c]) continue;
            double agg = 0.0;
            bool ok = true;
            const double* row = &bwm[static_cast<size_t>(c) * m];
            for (int g : grp) {
              if (row[g] < 0) { ok = false; break; }
              agg += row[g];
            }
            if (ok && agg > pick_bw) { pick = c; pick_bw = agg; }
          }
          if (pick < 0) break;
          grp.push_back(pick);
          in[pick] = 1;
          bw += pick_bw;
        }
        if (static_cast<int>(grp.size()) == k && bw > best_bw) {
          best.clear();
          for (int g : grp) best.push_back(avail[g]);
          best_bw = bw;
        }
      }
    }
    Cand c{&n, {}, 50, false, false};
    c.xgmi = !best.empty() && req.gpu_count > 1;
    if (best.empty()) best.assign(avail.begin(), avail.begin() + req.gpu_count);
    if (c.xgmi && req.prefer_xgmi) c.score += 30;
    c.one_numa = true;
    for (auto* g : best) c.one_numa &= g->numa_node == best[0]->numa_node;
    if (c.one_numa && req.prefer_same_numa) c.score += 10;
    for (auto* g : best)
      if (!req.arch.empty() && g->arch == req.arch) c.score += 5;
    c.group = std::move(best);
    cands.push_back(std::move(c));
  }
  auto better = [](const Cand& a, const Cand& b) {
    return a.score != b.score ? a.score > b.score : a.node->name < b.node->name;
  };
  const size_t keep = max_results ? std::min(max_results, cands.size()) : cands.size();
  std::partial_sort(cands.begin(), cands.begin() + static_cast<long>(keep), cands.end(), better);
  std::vector<TopologyHint> out;
  out.reserve(keep);
  for (size_t ci = 0; ci < keep; ++ci) {
    const Cand& c = cands[ci];
    TopologyHint h;
    h.node = c.node->name;
    h.score = c.score;
    if (c.xgmi && req.prefer_xgmi) h.reasons.push_back("fully connected xGMI group");
    if (c.one_numa && req.prefer_same_numa) h.reasons.push_back("single NUMA domain");
    for (auto* g : c.group) h.gpus.push_back(g->uuid);
    // Bandwidth estimate: mean pairwise effective xGMI bw, PCIe when no link.
    double sum = 0.0;
    int pairs = 0;
    for (size_t i = 0; i < c.group.size(); ++i)
      for (size_t j = i + 1; j < c.group.size(); ++j) {
        const XgmiLink* l = c.group[i]->link_to(c.group[j]->uuid);
        sum += (l && l->up) ? l->effective_gbps() : c.group[i]->pcie.bandwidth_gbps;
        ++pairs;
      }
    h.bandwidth_gbps = pairs ? sum / pairs : 0.0;
    if (h.score >= 80) h.reasons.push_back("optimal xGMI placement");
    else if (h.score >= 60) h.reasons.push_back("partial xGMI placement");
    else h.reasons.push_back("PCIe placement");
    out.push_back(std::move(h));
  }
  return out;
}

}  // namespace kgwe
