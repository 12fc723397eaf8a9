#include "cost.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <ctime>
#include <fstream>
#include <sstream>

namespace kgwe {

const char* to_string(PricingTier t) {
  switch (t) {
    case PricingTier::OnDemand: return "OnDemand";
    case PricingTier::Spot: return "Spot";
    case PricingTier::Reserved: return "Reserved";
  }
  return "OnDemand";
}
const char* to_string(BudgetScope s) {
  switch (s) {
    case BudgetScope::Namespace: return "Namespace";
    case BudgetScope::Team: return "Team";
    case BudgetScope::Project: return "Project";
    case BudgetScope::Cluster: return "Cluster";
  }
  return "Namespace";
}
const char* to_string(BudgetPeriod p) {
  switch (p) {
    case BudgetPeriod::Daily: return "Daily";
    case BudgetPeriod::Weekly: return "Weekly";
    case BudgetPeriod::Monthly: return "Monthly";
  }
  return "Monthly";
}
const char* to_string(Enforcement e) {
  switch (e) {
    case Enforcement::Alert: return "Alert";
    case Enforcement::Throttle: return "Throttle";
    case Enforcement::Block: return "Block";
  }
  return "Alert";
}
const char* to_string(AlertSeverity s) {
  switch (s) {
    case AlertSeverity::Info: return "Info";
    case AlertSeverity::Warning: return "Warning";
    case AlertSeverity::Critical: return "Critical";
  }
  return "Info";
}
PricingTier tier_from(const std::string& s) {
  if (s == "Spot" || s == "spot") return PricingTier::Spot;
  if (s == "Reserved" || s == "reserved") return PricingTier::Reserved;
  return PricingTier::OnDemand;
}
BudgetScope scope_from(const std::string& s) {
  if (s == "Team") return BudgetScope::Team;
  if (s == "Project") return BudgetScope::Project;
  if (s == "Cluster") return BudgetScope::Cluster;
  return BudgetScope::Namespace;
}
BudgetPeriod period_from(const std::string& s) {
  if (s == "Daily") return BudgetPeriod::Daily;
  if (s == "Weekly") return BudgetPeriod::Weekly;
  return BudgetPeriod::Monthly;
}
Enforcement enforcement_from(const std::string& s) {
  if (s == "Throttle") return Enforcement::Throttle;
  if (s == "Block") return Enforcement::Block;
  return Enforcement::Alert;
}

static double cents(double v) { return std::round(v * 100.0) / 100.0; }

Json to_json(const UsageRecord& r) {
  Json j = Json::object();
  j["uid"] = r.uid;
  j["namespace"] = r.ns;
  j["team"] = r.team;
  j["project"] = r.project;
  j["cluster"] = r.cluster;
  j["gpu_type"] = r.gpu_type;
  j["partition_mode"] = r.partition_mode;
  j["gpu_count"] = r.gpu_count;
  j["tier"] = to_string(r.tier);
  Json l = Json::object();
  for (const auto& kv : r.labels) l[kv.first] = kv.second;
  j["labels"] = l;
  j["start_s"] = r.start_s;
  j["end_s"] = r.end_s;
  j["duration_s"] = r.duration_s;
  j["avg_gfx"] = r.avg_gfx();
  j["avg_mem"] = r.avg_mem();
  j["peak_gfx"] = r.peak_gfx;
  j["idle_s"] = r.idle_s;
  j["sampled_s"] = r.sampled_s;
  j["last_sample_s"] = r.last_sample_s;
  j["peak_mem"] = r.peak_mem;
  j["raw_cost"] = r.raw_cost;
  j["adjusted_cost"] = r.adjusted_cost;
  j["finalized"] = r.finalized;
  return j;
}

UsageRecord usage_from_json(const Json& j) {
  UsageRecord r;
  r.uid = j.get("uid").str();
  r.ns = j.get("namespace").str("default");
  r.team = j.get("team").str();
  r.project = j.get("project").str();
  r.cluster = j.get("cluster").str("default");
  r.gpu_type = j.get("gpu_type").str("amd-mi355x-288gb");
  r.partition_mode = j.get("partition_mode").str();
  r.gpu_count = static_cast<int>(j.get("gpu_count").as_int(1));
  r.tier = tier_from(j.get("tier").str("OnDemand"));
  for (const auto& kv : j.get("labels").fields()) r.labels[kv.first] = kv.second.str();
  r.start_s = j.get("start_s").as_number(0);
  r.end_s = j.get("end_s").as_number(0);
  r.duration_s = j.get("duration_s").as_number(0);
  r.sampled_s = j.get("sampled_s").as_number(0);
  r.gfx_integral = j.get("avg_gfx").as_number(0) * r.sampled_s;
  r.mem_integral = j.get("avg_mem").as_number(0) * r.sampled_s;
  r.peak_gfx = j.get("peak_gfx").as_number(0);
  r.idle_s = j.get("idle_s").as_number(0);
  r.last_sample_s = j.get("last_sample_s").as_number(r.start_s + r.sampled_s);
  r.peak_mem = j.get("peak_mem").as_number(0);
  r.raw_cost = j.get("raw_cost").as_number(0);
  r.adjusted_cost = j.get("adjusted_cost").as_number(0);
  r.finalized = j.get("finalized").as_bool(false);
  return r;
}

Json to_json(const Budget& b) {
  Json j = Json::object();
  j["id"] = b.id;
  j["name"] = b.name;
  j["scope"] = to_string(b.scope);
  j["scope_id"] = b.scope_id;
  j["limit"] = b.limit;
  j["spend"] = cents(b.spend);
  j["currency"] = b.currency;
  j["period"] = to_string(b.period);
  j["period_start_s"] = b.period_start_s;
  j["period_end_s"] = b.period_end_s;
  j["alerts_enabled"] = b.alerts_enabled;
  j["enforcement"] = to_string(b.enforcement);
  j["utilization_percent"] = b.limit > 0 ? 100.0 * b.spend / b.limit : 0.0;
  return j;
}

Budget budget_from_json(const Json& in) {
  Budget b;
  const Json& meta = in.get("metadata");
  const Json& spec = in.has("spec") ? in.get("spec") : in;
  b.name = meta.get("name").str(in.get("name").str());
  const std::string ns = meta.get("namespace").str("");
  b.id = in.get("id").str(ns.empty() ? b.name : ns + "/" + b.name);
  b.scope = scope_from(spec.get("scope").str("Namespace"));
  b.scope_id = spec.get("scopeId").str(spec.get("teamId").str(ns));
  const Json& lim = spec.get("limit");
  b.limit = lim.is_string() ? std::atof(lim.str().c_str()) : lim.as_number(0);
  b.currency = spec.get("currency").str("USD");
  b.period = period_from(spec.get("period").str("Monthly"));
  b.alerts_enabled = spec.get("alertsEnabled").as_bool(true);
  if (spec.get("alertThresholds").is_array()) {
    b.thresholds.clear();
    for (const auto& t : spec.get("alertThresholds").items()) {
      double v = t.is_string() ? std::atof(t.str().c_str()) : t.as_number();
      b.thresholds.push_back(v > 1.0 ? v / 100.0 : v);
    }
  }
  b.enforcement = enforcement_from(spec.get("enforcementPolicy").str("Alert"));
  return b;
}

Json to_json(const BudgetAlert& a) {
  Json j = Json::object();
  j["id"] = a.id;
  j["budget_id"] = a.budget_id;
  j["severity"] = to_string(a.severity);
  j["threshold"] = a.threshold;
  j["spend"] = cents(a.spend);
  j["message"] = a.message;
  j["ts_s"] = a.ts_s;
  j["acknowledged"] = a.acknowledged;
  return j;
}

Json to_json(const Recommendation& r) {
  Json j = Json::object();
  j["type"] = r.type;
  j["uid"] = r.uid;
  j["description"] = r.description;
  j["current_cost"] = cents(r.current_cost);
  j["projected_saving"] = cents(r.saving);
  j["saving_percent"] = r.saving_pct;
  j["confidence"] = r.confidence;
  return j;
}

// ---------------------------------------------------------------------------
CostEngine::CostEngine(CostEngineConfig cfg) : cfg_(std::move(cfg)) {
  // Default MI355X-fleet price table ($/GPU-hour; partition rates are a
  // proportional share of the on-demand GPU price: 1/2, 1/4, 1/8).
  auto add = [&](const std::string& t, double od, double spot, double res) {
    GpuPricing p;
    p.gpu_type = t;
    p.on_demand = od;
    p.spot = spot;
    p.reserved = res;
    p.partition["SPX"] = od;
    p.partition["DPX"] = od / 2;
    p.partition["QPX"] = od / 4;
    p.partition["CPX"] = od / 8;
    pricing_[t] = p;
  };
  add("amd-mi355x-288gb", 2.95, 1.18, 2.07);
  add("amd-mi325x-256gb", 2.45, 0.98, 1.72);
  add("amd-mi300x-192gb", 1.99, 0.80, 1.39);
  replay();
}

void CostEngine::set_pricing(const GpuPricing& p) {
  std::lock_guard<std::mutex> lk(mu_);
  pricing_[p.gpu_type] = p;
}

GpuPricing CostEngine::pricing(const std::string& gpu_type) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = pricing_.find(gpu_type);
  return it != pricing_.end() ? it->second : pricing_.at("amd-mi355x-288gb");
}

std::vector<GpuPricing> CostEngine::pricing_table() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<GpuPricing> out;
  for (const auto& kv : pricing_) out.push_back(kv.second);
  return out;
}

std::string CostEngine::start(const UsageRecord& r0, double now_s) {
  std::lock_guard<std::mutex> lk(mu_);
  if (r0.uid.empty()) return "uid required";
  if (active_.count(r0.uid)) return "usage already tracked for " + r0.uid;
  UsageRecord r = r0;
  if (r.gpu_type.empty()) r.gpu_type = "amd-mi355x-288gb";
  r.start_s = now_s;
  r.last_sample_s = now_s;
  r.journaled_s = now_s;
  active_[r.uid] = r;
  journal(r, "start");
  return "";
}

bool CostEngine::sample(const std::string& uid, double gfx, double mem, double now_s) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = active_.find(uid);
  if (it == active_.end()) return false;
  UsageRecord& r = it->second;
  const double dt = std::max(0.0, now_s - r.last_sample_s);
  r.gfx_integral += gfx * dt;
  r.mem_integral += mem * dt;
  r.sampled_s += dt;
  if (gfx < cfg_.idle_threshold_pct) r.idle_s += dt;
  r.peak_gfx = std::max(r.peak_gfx, gfx);
  r.peak_mem = std::max(r.peak_mem, mem);
  r.last_sample_s = now_s;
  // Checkpoint the running record (integrals included) at most once per
  // interval, so a controller restart / failover resumes it instead of
  // losing the metered time.
  if (now_s - r.journaled_s >= cfg_.journal_interval_s) {
    r.journaled_s = now_s;
    journal(r, "active");
  }
  return true;
}

double CostEngine::raw_cost(const UsageRecord& r) const {
  auto it = pricing_.find(r.gpu_type);
  const GpuPricing& p = it != pricing_.end() ? it->second : pricing_.at("amd-mi355x-288gb");
  double rate;
  if (!r.partition_mode.empty()) {
    auto pit = p.partition.find(r.partition_mode);
    rate = pit != p.partition.end() ? pit->second : p.on_demand;
  } else {
    switch (r.tier) {
      case PricingTier::Spot: rate = p.spot; break;
      case PricingTier::Reserved: rate = p.reserved; break;
      default: rate = p.on_demand;
    }
  }
  return rate * r.gpu_count * (r.duration_s / 3600.0);
}

double CostEngine::adjusted_cost(const UsageRecord& r) const {
  double c = r.raw_cost;
  if (r.duration_s < 60) return c;
  const double util = (r.avg_gfx() + r.avg_mem()) / 2.0;
  const double idle = r.duration_s > 0 ? r.idle_s / r.duration_s : 0.0;
  if (idle > 0.5) c *= 1.0 + idle * 0.1;
  if (util > 80) c *= 0.95;
  return cents(c);
}

void CostEngine::roll_period(Budget& b, double now_s) const {
  auto start_of = [&](double t) {
    std::time_t tt = static_cast<std::time_t>(t);
    std::tm tm{};
    gmtime_r(&tt, &tm);
    tm.tm_hour = tm.tm_min = tm.tm_sec = 0;
    if (b.period == BudgetPeriod::Weekly) tm.tm_mday -= (tm.tm_wday + 6) % 7;  // Monday
    if (b.period == BudgetPeriod::Monthly) tm.tm_mday = 1;
    return static_cast<double>(timegm(&tm));
  };
  auto end_of = [&](double s) {
    std::time_t tt = static_cast<std::time_t>(s);
    std::tm tm{};
    gmtime_r(&tt, &tm);
    if (b.period == BudgetPeriod::Daily) tm.tm_mday += 1;
    if (b.period == BudgetPeriod::Weekly) tm.tm_mday += 7;
    if (b.period == BudgetPeriod::Monthly) tm.tm_mon += 1;
    return static_cast<double>(timegm(&tm));
  };
  if (b.period_end_s == 0) {
    b.period_start_s = start_of(now_s);
    b.period_end_s = end_of(b.period_start_s);
    return;
  }
  if (now_s >= b.period_end_s) {
    b.period_start_s = start_of(now_s);
    b.period_end_s = end_of(b.period_start_s);
    b.spend = 0.0;  // new period
  }
}

bool CostEngine::applies(const Budget& b, const UsageRecord& r) const {
  switch (b.scope) {
    case BudgetScope::Namespace: return b.scope_id == r.ns;
    case BudgetScope::Team: return b.scope_id == r.team;
    case BudgetScope::Project: return b.scope_id == r.project;
    case BudgetScope::Cluster: return b.scope_id.empty() || b.scope_id == r.cluster;
  }
  return false;
}

void CostEngine::check_alerts(Budget& b, double now_s) {
  if (!b.alerts_enabled || b.limit <= 0) return;
  const double ratio = b.spend / b.limit;
  for (double th : b.thresholds) {
    if (ratio < th) continue;
    bool exists = false;
    for (const auto& a : alerts_)
      exists |= a.budget_id == b.id && a.threshold == th && a.ts_s >= b.period_start_s;
    if (exists) continue;
    BudgetAlert a;
    a.id = "alert-" + std::to_string(next_alert_++);
    a.budget_id = b.id;
    a.threshold = th;
    a.spend = b.spend;
    a.ts_s = now_s;
    a.severity = th >= 0.9 ? AlertSeverity::Critical : th >= 0.75 ? AlertSeverity::Warning
                                                                     : AlertSeverity::Info;
    char buf[256];
    std::snprintf(buf, sizeof buf, "Budget '%s' has reached %.0f%% of limit ($%.2f of $%.2f)",
                  b.name.c_str(), th * 100, b.spend, b.limit);
    a.message = buf;
    alerts_.push_back(a);
  }
}

bool CostEngine::finalize(const std::string& uid, double now_s, UsageRecord* out) {
  UsageRecord r;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = active_.find(uid);
    if (it == active_.end()) return false;
    r = it->second;
    active_.erase(it);
    r.end_s = now_s;
    r.duration_s = std::max(0.0, now_s - r.start_s);
    // Unsampled tail counts at the last known utilisation (no data = idle).
    if (r.sampled_s < r.duration_s) {
      const double tail = r.duration_s - r.sampled_s;
      if (r.sampled_s == 0) r.idle_s += tail;
      else {
        r.gfx_integral += r.avg_gfx() * tail;
        r.mem_integral += r.avg_mem() * tail;
      }
      r.sampled_s = r.duration_s;
    }
    r.raw_cost = raw_cost(r);
    r.adjusted_cost = adjusted_cost(r);
    r.finalized = true;
    for (auto& kv : budgets_) {
      Budget& b = kv.second;
      roll_period(b, now_s);
      if (applies(b, r)) {
        b.spend += r.adjusted_cost;
        check_alerts(b, now_s);
      }
    }
    done_.push_back(r);
    journal(r, "final");
  }
  if (hook_) hook_(r);
  if (out) *out = r;
  return true;
}

bool CostEngine::record(const std::string& uid, UsageRecord* out) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = active_.find(uid);
  if (it != active_.end()) {
    if (out) *out = it->second;
    return true;
  }
  for (auto rit = done_.rbegin(); rit != done_.rend(); ++rit)
    if (rit->uid == uid) {
      if (out) *out = *rit;
      return true;
    }
  return false;
}

std::string CostEngine::create_budget(const Budget& b0, double now_s) {
  if (b0.id.empty() && b0.name.empty()) return "budget id or name required";
  if (b0.limit <= 0) return "budget limit must be > 0";
  std::lock_guard<std::mutex> lk(mu_);
  Budget b = b0;
  if (b.id.empty()) b.id = b.name;
  if (b.thresholds.empty()) b.thresholds = cfg_.alert_thresholds;
  roll_period(b, now_s);
  // Spend so far in this period from finalized records.
  b.spend = 0;
  for (const auto& r : done_)
    if (r.end_s >= b.period_start_s && applies(b, r)) b.spend += r.adjusted_cost;
  budgets_[b.id] = b;
  check_alerts(budgets_[b.id], now_s);
  return "";
}

bool CostEngine::budget(const std::string& id, Budget* out, double now_s) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = budgets_.find(id);
  if (it == budgets_.end()) return false;
  roll_period(it->second, now_s);
  if (out) *out = it->second;
  return true;
}

std::vector<Budget> CostEngine::budgets(double now_s) {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<Budget> out;
  for (auto& kv : budgets_) {
    roll_period(kv.second, now_s);
    out.push_back(kv.second);
  }
  return out;
}

Admission CostEngine::admit(const std::string& ns, const std::string& team, const std::string& project,
                            double estimated_cost, double now_s) {
  Admission a;
  UsageRecord probe;
  probe.ns = ns;
  probe.team = team;
  probe.project = project;
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& kv : budgets_) {
    Budget& b = kv.second;
    roll_period(b, now_s);
    if (!applies(b, probe)) continue;
    // Committed spend of running workloads in scope, projected 1 h ahead.
    const double projected = b.spend + estimated_cost;
    if (projected <= b.limit) continue;
    if (b.enforcement == Enforcement::Block) {
      a.allowed = false;
      a.reason = "budget '" + b.name + "' would be exceeded (Block)";
      return a;
    }
    if (b.enforcement == Enforcement::Throttle) {
      a.throttled = true;
      a.reason = "budget '" + b.name + "' exceeded: throttled (lowest priority, preemptible)";
    }
  }
  return a;
}

std::vector<BudgetAlert> CostEngine::alerts(bool unack) const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<BudgetAlert> out;
  for (const auto& a : alerts_)
    if (!unack || !a.acknowledged) out.push_back(a);
  return out;
}

bool CostEngine::acknowledge(const std::string& id) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& a : alerts_)
    if (a.id == id) {
      a.acknowledged = true;
      return true;
    }
  return false;
}

bool CostEngine::in_scope(const UsageRecord& r, const std::string& scope, const std::string& id) const {
  if (scope.empty() || scope == "Cluster") return id.empty() || r.cluster == id;
  if (scope == "Namespace") return r.ns == id;
  if (scope == "Team") return r.team == id;
  if (scope == "Project") return r.project == id;
  return false;
}

Json CostEngine::summary(const std::string& scope, const std::string& id, double from_s,
                         double to_s) const {
  std::lock_guard<std::mutex> lk(mu_);
  double total = 0, hours = 0;
  std::map<std::string, double> by_type, by_workload, by_tier;
  int n = 0;
  for (const auto& r : done_) {
    if (!in_scope(r, scope, id)) continue;
    if (r.end_s < from_s || (to_s > 0 && r.start_s > to_s)) continue;
    ++n;
    total += r.adjusted_cost;
    hours += r.gpu_count * r.duration_s / 3600.0;
    by_type[r.gpu_type] += r.adjusted_cost;
    by_workload[r.uid] += r.adjusted_cost;
    by_tier[to_string(r.tier)] += r.adjusted_cost;
  }
  Json j = Json::object();
  j["scope"] = scope;
  j["scope_id"] = id;
  j["records"] = n;
  j["total_cost"] = cents(total);
  j["gpu_hours"] = hours;
  j["avg_cost_per_gpu_hour"] = hours > 0 ? total / hours : 0.0;
  auto m2j = [](const std::map<std::string, double>& m) {
    Json o = Json::object();
    for (const auto& kv : m) o[kv.first] = cents(kv.second);
    return o;
  };
  j["by_gpu_type"] = m2j(by_type);
  j["by_workload"] = m2j(by_workload);
  j["by_tier"] = m2j(by_tier);
  return j;
}

std::vector<Recommendation> CostEngine::recommendations(const std::string& scope,
                                                        const std::string& id) const {
  std::lock_guard<std::mutex> lk(mu_);
  struct Stats {
    double cost = 0, duration = 0, util = 0;
    int count = 0, gpus = 1;
    std::string type;
    PricingTier tier = PricingTier::OnDemand;
    bool partitioned = false;
  };
  std::map<std::string, Stats> by_uid;
  for (const auto& r : done_) {
    if (!in_scope(r, scope, id)) continue;
    Stats& s = by_uid[r.uid];
    s.cost += r.adjusted_cost;
    s.duration += r.duration_s;
    s.util = (s.util * s.count + r.avg_gfx()) / (s.count + 1);
    s.count++;
    s.type = r.gpu_type;
    s.gpus = r.gpu_count;
    s.tier = r.tier;
    s.partitioned = !r.partition_mode.empty();
  }
  std::vector<Recommendation> out;
  for (const auto& kv : by_uid) {
    const Stats& s = kv.second;
    if (cfg_.enable_spot && s.tier == PricingTier::OnDemand && !s.partitioned) {
      auto it = pricing_.find(s.type);
      if (it != pricing_.end()) {
        const double saving = (it->second.on_demand - it->second.spot) * s.duration / 3600.0 * s.gpus;
        if (saving > 10) {
          Recommendation r;
          r.type = "Spot";
          r.uid = kv.first;
          r.current_cost = s.cost;
          r.saving = saving;
          r.saving_pct = s.cost > 0 ? 100 * saving / s.cost : 0;
          r.description = "Switch to spot capacity for " + kv.first;
          r.confidence = 0.8;
          out.push_back(r);
        }
      }
    }
    if (cfg_.enable_rightsizing && s.util < 40 && !s.partitioned) {
      // A workload using < 40 % of a 256-CU GPU fits a QPX (1/4) or CPX (1/8)
      // compute partition; saving = the unused share of the GPU price.
      const bool cpx = s.util < 12.5;
      Recommendation r;
      r.type = "Rightsize";
      r.uid = kv.first;
      r.current_cost = s.cost;
      r.saving = s.cost * (cpx ? 7.0 / 8.0 : 3.0 / 4.0);
      r.saving_pct = cpx ? 87.5 : 75.0;
      char buf[200];
      std::snprintf(buf, sizeof buf, "Low utilization (%.0f%%) - run %s on a %s compute partition",
                    s.util, kv.first.c_str(), cpx ? "CPX (1/8 GPU)" : "QPX (1/4 GPU)");
      r.description = buf;
      r.confidence = 0.7;
      out.push_back(r);
    }
    if (s.util < 30 && s.count > 5) {
      Recommendation r;
      r.type = "Consolidate";
      r.uid = kv.first;
      r.current_cost = s.cost;
      r.saving = s.cost * 0.5;
      r.saving_pct = 50;
      char buf[160];
      std::snprintf(buf, sizeof buf, "Very low utilization (%.0f%%) - co-locate with other workloads",
                    s.util);
      r.description = buf;
      r.confidence = 0.6;
      out.push_back(r);
    }
  }
  std::sort(out.begin(), out.end(), [](const Recommendation& a, const Recommendation& b) {
    return a.saving > b.saving;
  });
  return out;
}

Json CostEngine::chargeback(const std::string& group_by, double from_s, double to_s) const {
  std::lock_guard<std::mutex> lk(mu_);
  struct Line {
    double cost = 0, gpu_hours = 0;
    int workloads = 0;
    std::map<std::string, double> by_type;
  };
  std::map<std::string, Line> lines;
  double total = 0;
  for (const auto& r : done_) {
    if (r.end_s < from_s || (to_s > 0 && r.start_s > to_s)) continue;
    std::string key = group_by == "team" ? r.team : group_by == "cluster" ? r.cluster
                                                  : group_by == "project" ? r.project
                                                                          : r.ns;
    if (key.empty()) key = "unassigned";
    Line& l = lines[key];
    l.cost += r.adjusted_cost;
    l.gpu_hours += r.gpu_count * r.duration_s / 3600.0;
    l.workloads++;
    l.by_type[r.gpu_type] += r.adjusted_cost;
    total += r.adjusted_cost;
  }
  Json j = Json::object();
  j["group_by"] = group_by;
  j["from_s"] = from_s;
  j["to_s"] = to_s;
  j["total_cost"] = cents(total);
  Json arr = Json::array();
  for (const auto& kv : lines) {
    Json e = Json::object();
    e["group"] = kv.first;
    e["cost"] = cents(kv.second.cost);
    e["gpu_hours"] = kv.second.gpu_hours;
    e["workloads"] = kv.second.workloads;
    e["share_percent"] = total > 0 ? 100.0 * kv.second.cost / total : 0.0;
    Json bt = Json::object();
    for (const auto& t : kv.second.by_type) bt[t.first] = cents(t.second);
    e["by_gpu_type"] = bt;
    arr.push_back(e);
  }
  j["lines"] = arr;
  return j;
}

double CostEngine::running_cost_per_hour() const {
  std::lock_guard<std::mutex> lk(mu_);
  double c = 0;
  for (const auto& kv : active_) {
    UsageRecord r = kv.second;
    r.duration_s = 3600.0;
    c += raw_cost(r);
  }
  return c;
}

// Caller holds mu_ (or runs single-threaded in the constructor).
// Journal lines: {"ev": "start" | "active" | "final", "record": {...}}.
void CostEngine::journal(const UsageRecord& r, const char* ev) {
  if (cfg_.journal_path.empty()) return;
  std::ofstream f(cfg_.journal_path, std::ios::app);
  if (!f) return;
  Json j = Json::object();
  j["ev"] = ev;
  j["record"] = to_json(r);
  f << j.dump() << "\n";
}

void CostEngine::replay() {
  if (cfg_.journal_path.empty()) return;
  std::ifstream f(cfg_.journal_path);
  std::string line;
  std::map<std::string, UsageRecord> open;  // latest start / checkpoint per uid
  while (std::getline(f, line)) {
    if (line.empty()) continue;
    try {
      Json j = Json::parse(line);
      const std::string ev = j.has("ev") ? j.get("ev").str() : "final";  // lines without an event tag are finals (older journals)
      UsageRecord r = usage_from_json(j.has("record") ? j.get("record") : j);
      if (ev == "final") {
        r.finalized = true;
        open.erase(r.uid);
        done_.push_back(r);
        ++replayed_;
      } else {
        r.finalized = false;
        open[r.uid] = r;
      }
    } catch (...) {
      // A torn final line (crash mid-write) is skipped, not fatal.
    }
  }
  // Resume running records: the time between their last checkpoint and the
  // next sample is metered at their last known utilisation by sample() /
  // finalize(), so a failover loses no metered time.
  for (auto& kv : open) {
    kv.second.journaled_s = kv.second.last_sample_s;
    active_[kv.first] = kv.second;
    ++resumed_;
  }
  // Compact: finals + the open records' latest state, atomically.
  const std::string tmp = cfg_.journal_path + ".compact";
  {
    std::ofstream o(tmp, std::ios::trunc);
    if (!o) return;
    for (const auto& r : done_) {
      Json j = Json::object();
      j["ev"] = "final";
      j["record"] = to_json(r);
      o << j.dump() << "\n";
    }
    for (const auto& kv : active_) {
      Json j = Json::object();
      j["ev"] = "active";
      j["record"] = to_json(kv.second);
      o << j.dump() << "\n";
    }
  }
  std::rename(tmp.c_str(), cfg_.journal_path.c_str());
}

}  // namespace kgwe
