#include "partition.h"

#include <algorithm>
#include <cmath>

namespace kgwe {

const char* to_string(OpState s) {
  switch (s) {
    case OpState::Pending: return "Pending";
    case OpState::Draining: return "Draining";
    case OpState::Switching: return "Switching";
    case OpState::Completed: return "Completed";
    case OpState::Failed: return "Failed";
  }
  return "Unknown";
}

// ---------------------------------------------------------------------------
// strategies
// ---------------------------------------------------------------------------
bool valid_mode_combo(ComputePartition c, MemoryPartition m) {
  if (c == ComputePartition::TPX) return false;
  if (m == MemoryPartition::NPS1) return true;
  if (m == MemoryPartition::NPS2) return partition_count(c) % 2 == 0;
  return false;  // NPS4 / NPS8: not MI355X modes
}

std::string validate_strategy(const PartitionStrategy& s) {
  if (s.name.empty()) return "strategy name is required";
  if (s.distribution.empty()) return "profileDistribution must not be empty";
  double sum = 0.0;
  for (const auto& kv : s.distribution) {
    if (kv.first == ComputePartition::TPX) return "TPX is not a valid MI355X mode (8 XCDs)";
    if (kv.second < 0.0 || kv.second > 1.0) return "distribution fractions must be in [0, 1]";
    sum += kv.second;
  }
  if (sum > 1.01) return "distribution sums to more than 1.0";
  if (s.memory == MemoryPartition::NPS4 || s.memory == MemoryPartition::NPS8)
    return "MI355X supports NPS1 and NPS2 memory modes";
  if (s.min_utilization < 0.0 || s.min_utilization > 1.0) return "minUtilizationThreshold must be in [0, 1]";
  if (s.rebalance_interval_s < 0) return "rebalanceInterval must be >= 0";
  return "";
}

static int parse_duration_s(const std::string& d, int dflt) {
  if (d.empty()) return dflt;
  try {
    size_t pos = 0;
    double v = std::stod(d, &pos);
    std::string unit = d.substr(pos);
    if (unit == "s" || unit.empty()) return static_cast<int>(v);
    if (unit == "m") return static_cast<int>(v * 60);
    if (unit == "h") return static_cast<int>(v * 3600);
  } catch (...) {
  }
  return dflt;
}

PartitionStrategy strategy_from_json(const Json& in) {
  PartitionStrategy s;
  const Json& meta = in.get("metadata");
  const Json& spec = in.has("spec") ? in.get("spec") : in;
  s.name = meta.get("name").str(in.get("name").str());
  for (const auto& kv : spec.get("nodeSelector").fields()) s.node_selector[kv.first] = kv.second.str();
  const Json& gs = spec.get("gpuSelector");
  s.gpu_model = gs.get("model").str();
  s.min_memory_gb = gs.get("minMemoryGB").as_number(0.0);
  for (const auto& kv : spec.get("profileDistribution").fields())
    s.distribution[compute_partition_from(kv.first)] += kv.second.as_number(0.0);
  s.memory = memory_partition_from(spec.get("memoryPartition").str("NPS1"));
  s.allow_dynamic = spec.get("allowDynamicReconfig").as_bool(true);
  s.rebalance_interval_s = parse_duration_s(spec.get("rebalanceInterval").str("5m"), 300);
  s.min_utilization = spec.get("minUtilizationThreshold").as_number(0.3);
  s.priority = static_cast<int>(spec.get("priority").as_int(0));
  return s;
}

Json to_json(const PartitionStrategy& s) {
  Json j = Json::object();
  j["name"] = s.name;
  Json d = Json::object();
  for (const auto& kv : s.distribution) d[to_string(kv.first)] = kv.second;
  j["profileDistribution"] = d;
  j["memoryPartition"] = to_string(s.memory);
  j["allowDynamicReconfig"] = s.allow_dynamic;
  j["rebalanceIntervalSeconds"] = s.rebalance_interval_s;
  j["minUtilizationThreshold"] = s.min_utilization;
  j["priority"] = s.priority;
  return j;
}

Json to_json(const PartitionOp& op) {
  Json j = Json::object();
  j["id"] = op.id;
  j["node"] = op.node;
  j["gpu"] = op.gpu;
  j["from"] = to_string(op.from);
  j["to"] = to_string(op.to);
  j["memory_to"] = to_string(op.mem_to);
  j["state"] = to_string(op.state);
  j["reason"] = op.reason;
  j["error"] = op.error;
  j["dry_run"] = op.dry_run;
  return j;
}

// ---------------------------------------------------------------------------
// controller
// ---------------------------------------------------------------------------
PartitionController::PartitionController(std::shared_ptr<DiscoveryService> disc,
                                         std::shared_ptr<Scheduler> sched, bool dry_run)
    : disc_(std::move(disc)), sched_(std::move(sched)), dry_run_(dry_run) {}

std::string PartitionController::register_strategy(const PartitionStrategy& s) {
  std::string err = validate_strategy(s);
  if (!err.empty()) return err;
  std::lock_guard<std::mutex> lk(mu_);
  strategies_[s.name] = s;
  return "";
}

bool PartitionController::remove_strategy(const std::string& name) {
  std::lock_guard<std::mutex> lk(mu_);
  return strategies_.erase(name) > 0;
}

std::vector<PartitionStrategy> PartitionController::strategies() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<PartitionStrategy> out;
  for (const auto& kv : strategies_) out.push_back(kv.second);
  return out;
}

bool PartitionController::gpu_idle(const GpuDevice& g) const {
  if (!g.healthy() || g.partition.switching) return false;
  if (sched_ && sched_->gpu_busy(g)) return false;
  for (const auto& pi : g.partition.instances)
    if (pi.in_use) return false;
  return g.util.gfx_activity < 5.0;
}

int PartitionController::free_slices(const ClusterTopology& c, ComputePartition mode,
                                     const MemoryPartition* memory,
                                     const std::unordered_set<std::string>* within) const {
  int n = 0;
  std::set<std::string> owned;  // slices held in the ledger (one pass, not per slice)
  if (sched_)
    for (const auto& a : sched_->allocations())
      for (const auto& p : a.partitions) owned.insert(p);
  for (const auto& kv : c.nodes) {
    if (within && !within->count(kv.first)) continue;
    for (const auto& g : kv.second.gpus) {
      if (g.partition.compute != mode || !g.healthy() || g.partition.switching) continue;
      if (memory && g.partition.memory != *memory) continue;
      if (sched_ && g.partition.compute == ComputePartition::SPX && sched_->gpu_busy(g)) continue;
      for (const auto& pi : g.partition.instances)
        n += (pi.in_use || owned.count(pi.id)) ? 0 : 1;
    }
  }
  return n;
}

PartitionOp PartitionController::execute(const std::string& node, const GpuDevice& g,
                                         ComputePartition to, const std::string& reason,
                                         bool plan_only, const MemoryPartition* mem_to) {
  PartitionOp op;
  {
    std::lock_guard<std::mutex> lk(mu_);
    op.id = "op-" + std::to_string(next_op_++);
  }
  op.node = node;
  op.gpu = g.uuid;
  op.from = g.partition.compute;
  op.to = to;
  // Back to SPX always means NPS1 (SPX cannot span two memory domains).
  op.mem_to = mem_to ? *mem_to : to == ComputePartition::SPX ? MemoryPartition::NPS1 : g.partition.memory;
  op.reason = reason;
  op.dry_run = dry_run_ || plan_only;
  op.created_ns = now_ns();
  if (!plan_only) {
    // Drain: the GPU was chosen idle; re-verify right before switching.
    op.state = OpState::Draining;
    const bool fenced = !dry_run_ && sched_;
    if (!valid_mode_combo(to, op.mem_to)) {
      op.state = OpState::Failed;
      op.error = std::string("invalid mode combination ") + to_string(to) + "/" + to_string(op.mem_to);
    } else if (!gpu_idle(g) || (fenced && !sched_->fence_gpu(g.uuid, node))) {
      op.state = OpState::Failed;
      op.error = "gpu no longer idle";
    } else if (dry_run_) {
      op.state = OpState::Completed;
    } else {
      op.state = OpState::Switching;
      auto hal = disc_->hal(node);
      // Every intermediate state must be a valid combination: towards NPS2
      // switch compute first (X/NPS1 is always valid), towards NPS1 switch
      // memory first.
      std::string err = hal ? "" : "no HAL for node " + node;
      const bool mem_change = op.mem_to != g.partition.memory;
      const bool to_nps1 = op.mem_to == MemoryPartition::NPS1;
      if (err.empty() && mem_change && to_nps1) err = hal->set_memory_partition(g.uuid, op.mem_to);
      if (err.empty() && to != g.partition.compute) err = hal->set_compute_partition(g.uuid, to);
      if (err.empty() && mem_change && !to_nps1) err = hal->set_memory_partition(g.uuid, op.mem_to);
      if (err.empty()) {
        disc_->refresh_node(node);  // re-advertise the new slices
        op.state = OpState::Completed;
      } else {
        op.state = OpState::Failed;
        op.error = err;
      }
      if (fenced) sched_->unfence_gpu(g.uuid, node);
    }
    op.finished_ns = now_ns();
  }
  std::lock_guard<std::mutex> lk(mu_);
  ops_.push_back(op);
  if (ops_.size() > 4096) ops_.erase(ops_.begin(), ops_.begin() + 1024);
  return op;
}

std::vector<PartitionOp> PartitionController::ensure_capacity(ComputePartition mode, int count,
                                                              bool plan_only, const MemoryPartition* memory,
                                                              const std::unordered_set<std::string>* within) {
  std::vector<PartitionOp> out;
  if (memory && !valid_mode_combo(mode, *memory)) return out;
  auto snap = disc_->snapshot();
  // One memoised ledger summary per node (idle GPUs, free slices) instead of
  // a ledger probe per GPU: this runs inside the extender's filter verb.
  struct Cand {
    const std::string* node;
    const GpuDevice* g;
    int node_has_mode, node_idle;
    size_t seq;  // discovery order: the tie-break that keeps the choice deterministic
  };
  std::vector<Cand> cands;
  int have = 0;
  for (const auto& kv : snap->nodes) {
    if (within && !within->count(kv.first)) continue;
    const NodeTopology& n = kv.second;
    Scheduler::NodeSummary sum;
    if (sched_) {
      sum = sched_->node_summary(n);
    } else {
      sum.free_slices.assign(n.gpus.size(), 0);
      for (size_t p = 0; p < n.gpus.size(); ++p) {
        if (gpu_idle(n.gpus[p]) && p < 64) sum.idle_mask |= 1ull << p;
        for (const auto& pi : n.gpus[p].partition.instances) sum.free_slices[p] += pi.in_use ? 0 : 1;
      }
    }
    int has_mode = 0;
    const int idle = __builtin_popcountll(sum.idle_mask);
    for (size_t p = 0; p < n.gpus.size(); ++p) {
      const GpuDevice& g = n.gpus[p];
      has_mode += g.partition.compute == mode;
      if (g.partition.compute == mode && g.healthy() && !g.partition.switching &&
          (!memory || g.partition.memory == *memory))
        have += sum.free_slices[p];
    }
    if (idle == 0) continue;
    for (size_t p = 0; p < n.gpus.size() && p < 64; ++p) {
      const GpuDevice& g = n.gpus[p];
      const bool wrong = g.partition.compute != mode || (memory && g.partition.memory != *memory);
      if (wrong && (sum.idle_mask >> p & 1)) cands.push_back({&kv.first, &g, has_mode, idle, cands.size()});
    }
  }
  if (have >= count) return out;
  const int per_gpu = partition_count(mode);
  // Candidate idle GPUs in a different mode; prefer nodes already running the
  // target mode (consolidation), then nodes with the fewest idle GPUs (keep
  // whole idle nodes intact for large training jobs), then SPX sources.
  auto better = [](const Cand& a, const Cand& b) {
    if (a.node_has_mode != b.node_has_mode) return a.node_has_mode > b.node_has_mode;
    if (a.node_idle != b.node_idle) return a.node_idle < b.node_idle;
    const bool as = a.g->partition.compute == ComputePartition::SPX;
    const bool bs = b.g->partition.compute == ComputePartition::SPX;
    if (as != bs) return as;
    if (a.g->index != b.g->index) return a.g->index < b.g->index;
    return a.seq < b.seq;
  };
  // Only the few best candidates are needed (usually one GPU): order those,
  // and the rest only if conversions keep failing.
  size_t sorted = 0, next = 0;
  while (have < count && next < cands.size()) {
    if (next >= sorted) {
      const size_t want = static_cast<size_t>((count - have + per_gpu - 1) / per_gpu) + 4;
      const size_t upto = std::min(cands.size(), sorted + want);
      std::partial_sort(cands.begin() + sorted, cands.begin() + upto, cands.end(), better);
      sorted = upto;
    }
    const Cand& c = cands[next++];
    PartitionOp op = execute(*c.node, *c.g, mode,
                             "capacity: need " + std::to_string(count) + " " + to_string(mode) +
                                 (memory ? std::string("/") + to_string(*memory) : std::string()) +
                                 " slices, have " + std::to_string(have),
                             plan_only, memory);
    out.push_back(op);
    if (op.state != OpState::Failed) have += per_gpu;
  }
  return out;
}

std::vector<PartitionOp> PartitionController::rebalance(const std::string& name, bool plan_only) {
  std::vector<PartitionOp> out;
  PartitionStrategy st;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = strategies_.find(name);
    if (it == strategies_.end()) return out;
    st = it->second;
  }
  if (!st.allow_dynamic) return out;
  auto snap = disc_->snapshot();
  // Matching GPUs.
  std::vector<std::pair<std::string, const GpuDevice*>> match;
  for (const auto& kv : snap->nodes) {
    bool ok = true;
    for (const auto& sel : st.node_selector) {
      auto l = kv.second.labels.find(sel.first);
      ok &= l != kv.second.labels.end() && l->second == sel.second;
    }
    if (!ok) continue;
    for (const auto& g : kv.second.gpus) {
      if (!st.gpu_model.empty() && g.model.find(st.gpu_model) == std::string::npos) continue;
      if (g.memory_total_gb < st.min_memory_gb) continue;
      match.emplace_back(kv.first, &g);
    }
  }
  if (match.empty()) return out;
  const int total = static_cast<int>(match.size());
  std::map<ComputePartition, int> want, have;
  int assigned = 0;
  for (const auto& kv : st.distribution) {
    want[kv.first] = static_cast<int>(std::floor(kv.second * total + 1e-9));
    assigned += want[kv.first];
  }
  // Remainder stays / goes to SPX.
  want[ComputePartition::SPX] += total - assigned;
  for (const auto& m : match) have[m.second->partition.compute]++;
  // Idle GPUs of over-represented modes are converted to under-represented ones.
  for (const auto& m : match) {
    const ComputePartition cur = m.second->partition.compute;
    if (have[cur] <= want[cur] || !gpu_idle(*m.second)) continue;
    ComputePartition target = cur;
    int deficit = 0;
    for (const auto& kv : want) {
      int d = kv.second - have[kv.first];
      if (d > deficit) {
        deficit = d;
        target = kv.first;
      }
    }
    if (target == cur) break;
    const MemoryPartition* mem = target == ComputePartition::SPX ? nullptr : &st.memory;
    PartitionOp op = execute(m.first, *m.second, target, "rebalance strategy " + st.name, plan_only, mem);
    out.push_back(op);
    if (op.state != OpState::Failed) {
      have[cur]--;
      have[target]++;
    }
  }
  return out;
}

std::vector<PartitionOp> PartitionController::reclaim_idle(bool plan_only) {
  std::vector<PartitionOp> out;
  auto snap = disc_->snapshot();
  for (const auto& kv : snap->nodes)
    for (const auto& g : kv.second.gpus)
      if (g.partition.compute != ComputePartition::SPX && gpu_idle(g))
        out.push_back(execute(kv.first, g, ComputePartition::SPX, "reclaim idle partitioned GPU", plan_only));
  return out;
}

std::vector<PartitionOp> PartitionController::reclaim_idle_after(double now_s, double min_idle_s) {
  std::vector<PartitionOp> out;
  auto snap = disc_->snapshot();
  std::vector<std::pair<std::string, const GpuDevice*>> due;
  {
    std::lock_guard<std::mutex> lk(mu_);
    std::map<std::string, double> seen;
    for (const auto& kv : snap->nodes)
      for (const auto& g : kv.second.gpus) {
        if (g.partition.compute == ComputePartition::SPX || !gpu_idle(g)) continue;
        auto it = idle_since_.find(g.uuid);
        const double t0 = it == idle_since_.end() ? now_s : it->second;
        seen[g.uuid] = t0;
        if (now_s - t0 >= min_idle_s) due.emplace_back(kv.first, &g);
      }
    idle_since_.swap(seen);  // busy / SPX GPUs drop out of the idle map
  }
  for (const auto& d : due) {
    out.push_back(execute(d.first, *d.second, ComputePartition::SPX,
                          "reclaim partitioned GPU idle for >= " + std::to_string(min_idle_s) + " s",
                          false));
    std::lock_guard<std::mutex> lk(mu_);
    idle_since_.erase(d.second->uuid);
  }
  return out;
}

Json to_json(const PartitionMove& m) {
  Json j = Json::object();
  j["uid"] = m.uid;
  j["from"] = m.from;
  j["to"] = m.to;
  j["node_from"] = m.node_from;
  j["node_to"] = m.node_to;
  return j;
}

int PartitionController::migrations() const {
  std::lock_guard<std::mutex> lk(mu_);
  return migrations_;
}

std::vector<PartitionMove> PartitionController::consolidate(double now_s, const ConsolidationPolicy& pol,
                                                            bool move_in_ledger) {
  std::vector<PartitionMove> moves;
  if (!sched_) return moves;
  auto snap = disc_->snapshot();
  // Donors emptied earlier (controller path: their pods were evicted) go
  // back to SPX as soon as they are idle — no idle hysteresis for them.
  std::set<std::string> draining;
  {
    std::lock_guard<std::mutex> lk(mu_);
    draining = draining_;
  }
  // Until then the scheduler places no new slice work on them (plan-only
  // callers evict the donor's pods; without the bar the same pods could be
  // scheduled straight back).  A donor that has not emptied within the drain
  // limit (its pods were never evicted) is given back.
  const double drain_limit_s = std::max(300.0, 2.0 * pol.after_s);
  auto undrain = [&](const std::string& uuid, const std::string& node) {
    sched_->set_draining(uuid, node, false);
    std::lock_guard<std::mutex> lk(mu_);
    draining_.erase(uuid);
    draining_since_.erase(uuid);
  };
  for (const auto& uuid : draining) {
    bool found = false;
    for (const auto& kv : snap->nodes)
      if (const GpuDevice* g = kv.second.gpu(uuid)) {
        found = true;
        double since = now_s;
        {
          std::lock_guard<std::mutex> lk(mu_);
          auto it = draining_since_.find(uuid);
          if (it != draining_since_.end()) since = it->second;
        }
        if (g->partition.compute == ComputePartition::SPX) {
          undrain(uuid, kv.first);
        } else if (gpu_idle(*g)) {
          PartitionOp op = execute(kv.first, *g, ComputePartition::SPX, "consolidation: donor emptied", false);
          if (op.state != OpState::Failed) undrain(uuid, kv.first);
        } else if (now_s - since > drain_limit_s) {
          undrain(uuid, kv.first);
        }
      }
    if (!found) undrain(uuid, "");  // the GPU left the fleet
  }
  snap = disc_->snapshot();
  const auto allocs = sched_->allocations();
  std::map<std::string, const Allocation*> owner;  // slice id -> allocation
  for (const auto& a : allocs)
    for (const auto& p : a.partitions) owner[p] = &a;
  struct G {
    std::string node;
    const GpuDevice* g;
    int used = 0, total = 0;
    bool movable = true;
    std::vector<std::string> free_slices, used_slices;
  };
  std::map<ComputePartition, std::vector<G>> by_mode;
  std::map<std::string, double> low;
  std::map<std::string, double> migrated;
  {
    std::lock_guard<std::mutex> lk(mu_);
    low = low_since_;
    migrated = migrated_at_;
    draining = draining_;
  }
  std::map<std::string, double> low_next;
  for (const auto& kv : snap->nodes)
    for (const auto& g : kv.second.gpus) {
      if (g.partition.compute == ComputePartition::SPX || !g.healthy() || g.partition.switching) continue;
      if (draining.count(g.uuid)) continue;
      G e{kv.first, &g};
      for (const auto& pi : g.partition.instances) {
        e.total++;
        auto o = owner.find(pi.id);
        if (pi.in_use || o != owner.end()) {
          e.used++;
          e.used_slices.push_back(pi.id);
          // Only preemptible inference / batch work that has not moved
          // recently, holding nothing but slices, may be migrated.
          const Allocation* a = o == owner.end() ? nullptr : o->second;
          const bool ok = a && a->preemptible && a->gpus.empty() && a->gang.empty() &&
                          (a->type == WorkloadType::Inference || a->type == WorkloadType::Batch) &&
                          (!migrated.count(a->uid) || now_s - migrated[a->uid] >= pol.cooldown_s);
          e.movable &= ok;
        } else {
          e.free_slices.push_back(pi.id);
        }
      }
      if (e.total == 0) continue;
      if (e.used > 0 && e.used < pol.below * e.total) {
        auto it = low.find(g.uuid);
        low_next[g.uuid] = it == low.end() ? now_s : it->second;
      }
      by_mode[g.partition.compute].push_back(std::move(e));
    }
  std::vector<std::string> emptied;
  for (auto& mk : by_mode) {
    auto& gs = mk.second;
    // Donors: emptiest first.  Receivers: fullest first.
    std::vector<G*> donors, recv;
    for (auto& e : gs) {
      auto l = low_next.find(e.g->uuid);
      if (e.movable && l != low_next.end() && now_s - l->second >= pol.after_s) donors.push_back(&e);
    }
    std::sort(donors.begin(), donors.end(), [](const G* a, const G* b) {
      return a->used != b->used ? a->used < b->used : a->g->uuid < b->g->uuid;
    });
    std::set<const G*> is_donor, gone;
    for (auto* d : donors) is_donor.insert(d);
    for (auto* d : donors) {
      if (!is_donor.count(d)) continue;  // received slices meanwhile: no longer a donor
      recv.clear();
      for (auto& e : gs)
        if (&e != d && !gone.count(&e) && !e.free_slices.empty()) recv.push_back(&e);
      std::sort(recv.begin(), recv.end(), [&](const G* a, const G* b) {
        const bool ad = is_donor.count(a) && !gone.count(a), bd = is_donor.count(b) && !gone.count(b);
        if (ad != bd) return !ad;  // prefer non-donors
        return a->used != b->used ? a->used > b->used : a->g->uuid < b->g->uuid;
      });
      // Later (fuller or equal) donors may receive: they stop being donors.
      int room = 0;
      for (auto* r : recv) room += static_cast<int>(r->free_slices.size());
      if (room < d->used) continue;  // cannot be emptied completely: leave it
      std::vector<PartitionMove> mine;
      bool ok = true;
      for (const auto& sl : d->used_slices) {
        G* tgt = nullptr;
        for (auto* r : recv)
          if (!r->free_slices.empty()) {
            tgt = r;
            break;
          }
        if (!tgt) {
          ok = false;
          break;
        }
        PartitionMove m;
        m.uid = owner.at(sl)->uid;
        m.from = sl;
        m.to = tgt->free_slices.back();
        m.node_from = d->node;
        m.node_to = tgt->node;
        if (move_in_ledger && !sched_->migrate_partition(m.uid, m.from, m.to)) {
          ok = false;
          break;
        }
        tgt->free_slices.pop_back();
        tgt->used++;
        is_donor.erase(tgt);
        mine.push_back(m);
      }
      if (!ok) continue;  // ledger moved underneath us: the rest waits for the next tick
      gone.insert(d);
      emptied.push_back(d->g->uuid);
      for (auto& m : mine) moves.push_back(m);
    }
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    low_since_.swap(low_next);
    for (const auto& m : moves) migrated_at_[m.uid] = now_s;
    migrations_ += static_cast<int>(moves.size());
    for (const auto& u : emptied) {
      draining_.insert(u);
      draining_since_[u] = now_s;
      low_since_.erase(u);
    }
    if (migrated_at_.size() > 100000) migrated_at_.clear();
  }
  {
    auto s2 = disc_->snapshot();
    for (const auto& u : emptied)
      for (const auto& kv : s2->nodes)
        if (const GpuDevice* g = kv.second.gpu(u)) {
          sched_->set_draining(u, kv.first, true);  // no new slice work on a donor
          if (!move_in_ledger) continue;            // its pods are still to be evicted by the caller
          // donors are empty right now: switch them back
          PartitionOp op = execute(kv.first, *g, ComputePartition::SPX, "consolidation: donor emptied", false);
          if (op.state != OpState::Failed) undrain(u, kv.first);
        }
  }
  return moves;
}

std::vector<PartitionOp> PartitionController::operations() const {
  std::lock_guard<std::mutex> lk(mu_);
  return ops_;
}

PartitionMetrics PartitionController::metrics() const {
  PartitionMetrics m;
  auto snap = disc_->snapshot();
  std::vector<Allocation> allocs;
  if (sched_) allocs = sched_->allocations();
  std::set<std::string> owned;
  for (const auto& a : allocs)
    for (const auto& p : a.partitions) owned.insert(p);
  int slices = 0, used = 0;
  for (const auto& kv : snap->nodes)
    for (const auto& g : kv.second.gpus) {
      auto& md = m.modes[to_string(g.partition.compute)];
      md.gpus++;
      md.slices += static_cast<int>(g.partition.instances.size());
      for (const auto& pi : g.partition.instances) {
        const bool u = pi.in_use || owned.count(pi.id);
        md.slices_in_use += u;
        if (g.partition.compute != ComputePartition::SPX) {
          slices++;
          used += u;
        }
      }
    }
  m.slice_utilization = slices ? static_cast<double>(used) / slices : 0.0;
  std::lock_guard<std::mutex> lk(mu_);
  m.ops_total = static_cast<int>(ops_.size());
  for (const auto& op : ops_) {
    m.ops_failed += op.state == OpState::Failed;
    m.ops_pending += op.state == OpState::Pending || op.state == OpState::Draining ||
                     op.state == OpState::Switching;
  }
  return m;
}

// ---------------------------------------------------------------------------
// sharing
// ---------------------------------------------------------------------------
Json to_json(const SharingAllocation& a) {
  Json j = Json::object();
  j["uid"] = a.uid;
  j["node"] = a.node;
  j["gpu"] = a.gpu;
  j["method"] = to_string(a.method);
  j["cu_begin"] = a.cu_begin;
  j["cu_end"] = a.cu_end;
  j["memory_gb"] = a.memory_gb;
  j["gpu_index"] = a.gpu_index;
  Json env = Json::object();
  for (const auto& kv : a.env) env[kv.first] = kv.second;
  j["env"] = env;
  return j;
}

std::map<std::string, std::string> share_env(SharingMethod m, int gpu_index, int cu_begin, int cu_end,
                                             double memory_gb, double gpu_memory_gb) {
  std::map<std::string, std::string> env;
  env["KGWE_SHARING"] = to_string(m);
  env["HIP_VISIBLE_DEVICES"] = std::to_string(gpu_index);
  env["ROCR_VISIBLE_DEVICES"] = std::to_string(gpu_index);
  if (m == SharingMethod::CoLocate) {
    // ROCm CU masking: <device index>:<CU list>; the device is 0 once
    // ROCR_VISIBLE_DEVICES leaves only this GPU visible.
    env["HSA_CU_MASK"] = "0:" + std::to_string(cu_begin) + "-" + std::to_string(cu_end - 1);
    env["KGWE_CU_RANGE"] = std::to_string(cu_begin) + "-" + std::to_string(cu_end);
  }
  // Measured on MI355X (profiles/r02_colocate): co-located processes run
  // concurrently only while each holds <= 2 hardware queues; at the HIP
  // default (4) the scheduler time-slices the clients' queues and 8 clients
  // together decode 3-5x slower than ONE client alone.
  if (m == SharingMethod::CoLocate || m == SharingMethod::TimeSlice) env["GPU_MAX_HW_QUEUES"] = "2";
  if (memory_gb > 0 && gpu_memory_gb > 0) {
    char buf[32];
    std::snprintf(buf, sizeof buf, "%.4f", std::min(1.0, memory_gb / gpu_memory_gb));
    env["KGWE_GPU_MEMORY_FRACTION"] = buf;
  }
  return env;
}

SharingManager::SharingManager(std::shared_ptr<DiscoveryService> disc, std::shared_ptr<Scheduler> sched,
                               SharingPolicy policy)
    : disc_(std::move(disc)), sched_(std::move(sched)), policy_(std::move(policy)) {}

SharingMethod SharingManager::decide(const SharingRequest& r) const {
  if (r.method != SharingMethod::None) return r.method;
  auto it = policy_.by_type.find(r.type);
  if (it != policy_.by_type.end()) return it->second;
  if (r.require_isolation) return SharingMethod::Partition;
  if (r.prefer_partition) return SharingMethod::Partition;
  return SharingMethod::CoLocate;
}

int SharingManager::clients_on(const std::string& gpu) const { return sched_->share_clients(gpu); }

SharingAllocation SharingManager::from_alloc(const Allocation& a) const {
  SharingAllocation s;
  s.uid = a.uid;
  s.node = a.node;
  s.gpu = a.shared_gpu;
  s.method = a.sharing;
  s.cu_begin = a.cu_begin;
  s.cu_end = a.cu_end;
  s.memory_gb = a.share_memory_gb;
  GpuDevice g;
  double mem = 0.0;
  if (disc_->gpu(a.shared_gpu, &g)) {
    s.gpu_index = g.index;
    mem = g.memory_total_gb;
  }
  s.env = share_env(a.sharing, s.gpu_index, a.cu_begin, a.cu_end, a.share_memory_gb, mem);
  return s;
}

SharingAllocation SharingManager::allocate(const SharingRequest& r, std::string* error) {
  SharingAllocation a;
  a.uid = r.uid;
  a.method = decide(r);
  a.node = r.node;
  a.gpu = r.gpu;
  if (a.method == SharingMethod::Partition) {
    a.env["KGWE_SHARING"] = "Partition";
    a.env["KGWE_PARTITION_MODE"] = to_string(r.partition_mode);
    return a;
  }
  WorkloadRequest w;
  w.uid = r.uid;
  w.ns = r.ns;
  w.team = r.team;
  w.type = r.type;
  w.sharing = a.method;
  w.share_cu_percent = r.cu_percent;
  w.share_memory_gb = r.memory_gb;
  w.gpu_count = 1;
  Decision d = sched_->reserve_share(w, r.node, r.gpu);
  if (!d.ok) {
    *error = d.failed_nodes.empty() ? "share rejected" : d.failed_nodes.begin()->second;
    return a;
  }
  Allocation al;
  if (!sched_->allocation(r.uid, &al)) {
    *error = "share vanished";
    return a;
  }
  return from_alloc(al);
}

bool SharingManager::release(const std::string& uid) {
  Allocation a;
  if (!sched_->allocation(uid, &a) || a.sharing == SharingMethod::None) return false;
  return sched_->release(uid);
}

std::vector<SharingAllocation> SharingManager::allocations() const {
  std::vector<SharingAllocation> out;
  for (const auto& a : sched_->allocations())
    if (a.sharing != SharingMethod::None) out.push_back(from_alloc(a));
  return out;
}

}  // namespace kgwe
