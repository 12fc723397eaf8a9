// GPU cost engine (L6): pricing, metering, budgets with enforcement, alerts,
// summaries, optimisation recommendations and chargeback reports.
//
// Reference: src/api/cost_engine.go (pricing :72-96/:300-347, usage
// lifecycle :350-441, raw/adjusted cost :444-502, budgets/alerts :505-589,
// summary :592-670, recommendations :673-802, chargeback :829-912).
// Kept: tier pricing with per-partition rates, the adjusted-cost rules (<60 s
// no adjustment; idle ratio > 0.5 => x(1 + 0.1 idle); avg(gfx, mem) > 80 =>
// x0.95; round to cents), alert thresholds {0.5, 0.75, 0.9, 1.0} with
// severity >=0.9 Critical / >=0.75 Warning, recommendation rules (spot when
// saving > $10, rightsize when util < 40 %, consolidate when util < 30 % and
// > 5 records) and chargeback grouping.
// Fixed / added: Project and Cluster budget scopes match; budget periods roll
// over (Daily/Weekly/Monthly); enforcement is real (admit() => Block/Throttle);
// utilisation is time-weighted from samples instead of overwritten; starts,
// periodic checkpoints of RUNNING records and finals are journaled to an
// append-only JSONL file, replayed and compacted on start — finished records
// are restored and running ones resume metering (checkpoint/resume; the
// reference designed TimescaleDB for this, values.yaml:283-294, and kept
// everything in memory);
// MI355X prices with compute-partition (CPX/QPX/DPX) fractional rates.
#pragma once
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "json.h"

namespace kgwe {

enum class PricingTier { OnDemand, Spot, Reserved };
enum class BudgetScope { Namespace, Team, Project, Cluster };
enum class BudgetPeriod { Daily, Weekly, Monthly };
enum class Enforcement { Alert, Throttle, Block };
enum class AlertSeverity { Info, Warning, Critical };

const char* to_string(PricingTier t);
const char* to_string(BudgetScope s);
const char* to_string(BudgetPeriod p);
const char* to_string(Enforcement e);
const char* to_string(AlertSeverity s);
PricingTier tier_from(const std::string& s);
BudgetScope scope_from(const std::string& s);
BudgetPeriod period_from(const std::string& s);
Enforcement enforcement_from(const std::string& s);

struct GpuPricing {
  std::string gpu_type;
  double on_demand = 0, spot = 0, reserved = 0;        // $/GPU-hour
  std::map<std::string, double> partition;            // "CPX" -> $/slice-hour
};

struct UsageRecord {
  std::string uid, ns, team, project, cluster = "default", gpu_type, partition_mode;
  int gpu_count = 1;  // GPUs, or slices when partition_mode is set
  PricingTier tier = PricingTier::OnDemand;
  std::map<std::string, std::string> labels;
  double start_s = 0, end_s = 0, duration_s = 0;
  // Time-weighted utilisation integrals.
  double last_sample_s = 0, gfx_integral = 0, mem_integral = 0, idle_s = 0, sampled_s = 0;
  double peak_gfx = 0, peak_mem = 0;
  double journaled_s = 0;  // last journal checkpoint (not serialized)
  double raw_cost = 0, adjusted_cost = 0;
  bool finalized = false;

  double avg_gfx() const { return sampled_s > 0 ? gfx_integral / sampled_s : 0; }
  double avg_mem() const { return sampled_s > 0 ? mem_integral / sampled_s : 0; }
};
Json to_json(const UsageRecord& r);
UsageRecord usage_from_json(const Json& j);

struct Budget {
  std::string id, name;
  BudgetScope scope = BudgetScope::Namespace;
  std::string scope_id;
  double limit = 0, spend = 0;
  std::string currency = "USD";
  BudgetPeriod period = BudgetPeriod::Monthly;
  double period_start_s = 0, period_end_s = 0;
  bool alerts_enabled = true;
  std::vector<double> thresholds{0.5, 0.75, 0.9, 1.0};
  Enforcement enforcement = Enforcement::Alert;
};
Json to_json(const Budget& b);
Budget budget_from_json(const Json& j);

struct BudgetAlert {
  std::string id, budget_id, message;
  AlertSeverity severity = AlertSeverity::Info;
  double threshold = 0, spend = 0, ts_s = 0;
  bool acknowledged = false;
};
Json to_json(const BudgetAlert& a);

struct Recommendation {
  std::string type;  // Spot | Rightsize | Consolidate
  std::string uid, description;
  double current_cost = 0, saving = 0, saving_pct = 0, confidence = 0;
};
Json to_json(const Recommendation& r);

struct Admission {
  bool allowed = true;
  bool throttled = false;
  std::string reason;
};

struct CostEngineConfig {
  std::vector<double> alert_thresholds{0.5, 0.75, 0.9, 1.0};
  bool enable_spot = true;
  bool enable_rightsizing = true;
  double idle_threshold_pct = 5.0;  // gfx_activity below this counts as idle time
  std::string journal_path;         // "" = no persistence
  double journal_interval_s = 60.0; // running-record checkpoint period
};

class CostEngine {
 public:
  explicit CostEngine(CostEngineConfig cfg = {});

  void set_pricing(const GpuPricing& p);
  GpuPricing pricing(const std::string& gpu_type) const;
  std::vector<GpuPricing> pricing_table() const;

  std::string start(const UsageRecord& r, double now_s);  // "" = ok
  // One telemetry sample: gfx_activity %, memory used %.
  bool sample(const std::string& uid, double gfx_pct, double mem_pct, double now_s);
  bool finalize(const std::string& uid, double now_s, UsageRecord* out = nullptr);
  bool record(const std::string& uid, UsageRecord* out) const;

  double raw_cost(const UsageRecord& r) const;
  double adjusted_cost(const UsageRecord& r) const;

  std::string create_budget(const Budget& b, double now_s);
  bool budget(const std::string& id, Budget* out, double now_s);
  std::vector<Budget> budgets(double now_s);
  Admission admit(const std::string& ns, const std::string& team, const std::string& project,
                  double estimated_cost, double now_s);

  std::vector<BudgetAlert> alerts(bool unacknowledged_only = false) const;
  bool acknowledge(const std::string& alert_id);

  Json summary(const std::string& scope, const std::string& scope_id, double from_s, double to_s) const;
  std::vector<Recommendation> recommendations(const std::string& scope, const std::string& scope_id) const;
  Json chargeback(const std::string& group_by, double from_s, double to_s) const;
  // Cost of currently running (not finalized) workloads per hour.
  double running_cost_per_hour() const;

  // Metrics hook (wired to the Prometheus registry by the service layer).
  void set_cost_hook(std::function<void(const UsageRecord&)> f) { hook_ = std::move(f); }
  size_t replayed() const { return replayed_; }
  size_t resumed() const { return resumed_; }  // running records restored from the journal

 private:
  bool in_scope(const UsageRecord& r, const std::string& scope, const std::string& id) const;
  bool applies(const Budget& b, const UsageRecord& r) const;
  void roll_period(Budget& b, double now_s) const;
  void check_alerts(Budget& b, double now_s);
  void journal(const UsageRecord& r, const char* ev);
  void replay();

  CostEngineConfig cfg_;
  mutable std::mutex mu_;
  std::map<std::string, GpuPricing> pricing_;
  std::map<std::string, UsageRecord> active_;
  std::vector<UsageRecord> done_;
  std::map<std::string, Budget> budgets_;
  std::vector<BudgetAlert> alerts_;
  int next_alert_ = 1;
  size_t replayed_ = 0;
  size_t resumed_ = 0;
  std::function<void(const UsageRecord&)> hook_;
};

}  // namespace kgwe
