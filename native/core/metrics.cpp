#include "metrics.h"

#include <cmath>
#include <cstdio>
#include <stdexcept>

namespace kgwe {

std::string prom_escape(const std::string& v) {
  std::string o;
  o.reserve(v.size());
  for (char c : v) {
    if (c == '\\') o += "\\\\";
    else if (c == '"') o += "\\\"";
    else if (c == '\n') o += "\\n";
    else o.push_back(c);
  }
  return o;
}

std::string prom_number(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  char buf[40];
  if (v == std::floor(v) && std::fabs(v) < 1e15) std::snprintf(buf, sizeof buf, "%.0f", v);
  else std::snprintf(buf, sizeof buf, "%.17g", v);
  return buf;
}

void MetricRegistry::declare(const std::string& name, MetricType type, const std::string& help,
                             const std::vector<std::string>& label_names,
                             const std::vector<double>& buckets) {
  std::lock_guard<std::mutex> lk(mu_);
  Family& f = fams_[name];
  f.type = type;
  f.help = help;
  f.labels = label_names;
  f.buckets = buckets;
}

MetricRegistry::Family* MetricRegistry::find(const std::string& name) {
  auto it = fams_.find(name);
  if (it == fams_.end()) throw std::runtime_error("unknown metric family " + name);
  return &it->second;
}

MetricRegistry::Family* MetricRegistry::find_mut(const std::string& name) {
  Family* f = find(name);
  if (f->frozen) {
    f->series = *f->frozen;
    f->frozen.reset();
  }
  return f;
}

void MetricRegistry::set(const std::string& name, const Labels& lv, double v) {
  std::lock_guard<std::mutex> lk(mu_);
  Family* f = find_mut(name);
  if (lv.size() != f->labels.size()) throw std::runtime_error("label arity mismatch for " + name);
  f->series[lv].value = v;
}

void MetricRegistry::add(const std::string& name, const Labels& lv, double v) {
  std::lock_guard<std::mutex> lk(mu_);
  Family* f = find_mut(name);
  if (lv.size() != f->labels.size()) throw std::runtime_error("label arity mismatch for " + name);
  if (f->type == MetricType::Counter && v < 0) throw std::runtime_error("counter decrement: " + name);
  f->series[lv].value += v;
}

void MetricRegistry::observe(const std::string& name, const Labels& lv, double v) {
  std::lock_guard<std::mutex> lk(mu_);
  Family* f = find_mut(name);
  if (f->type != MetricType::Histogram) throw std::runtime_error("not a histogram: " + name);
  if (lv.size() != f->labels.size()) throw std::runtime_error("label arity mismatch for " + name);
  Series& s = f->series[lv];
  if (s.bucket_counts.size() != f->buckets.size()) s.bucket_counts.assign(f->buckets.size(), 0.0);
  for (size_t i = 0; i < f->buckets.size(); ++i)
    if (v <= f->buckets[i]) {
      s.bucket_counts[i] += 1;
      break;
    }
  s.sum += v;
  s.count += 1;
}

void MetricRegistry::remove(const std::string& name, const Labels& lv) {
  std::lock_guard<std::mutex> lk(mu_);
  find_mut(name)->series.erase(lv);
}

void MetricRegistry::clear(const std::string& name) {
  std::lock_guard<std::mutex> lk(mu_);
  Family* f = find(name);
  f->series.clear();
  f->frozen.reset();
  f->blocks.reset();
}

double MetricRegistry::value(const std::string& name, const Labels& lv) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = fams_.find(name);
  if (it == fams_.end()) return 0.0;
  const SeriesMap& m = it->second.frozen ? *it->second.frozen : it->second.series;
  auto s = m.find(lv);
  if (s == m.end()) {
    if (it->second.blocks)
      for (const auto& b : *it->second.blocks)
        for (const auto& e : *b.second)
          if (e.first == lv) return e.second;
    return 0.0;
  }
  return it->second.type == MetricType::Histogram ? static_cast<double>(s->second.count) : s->second.value;
}

bool MetricRegistry::has(const std::string& name) const {
  std::lock_guard<std::mutex> lk(mu_);
  return fams_.count(name) > 0;
}

std::vector<std::string> MetricRegistry::families() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::string> out;
  for (const auto& kv : fams_) out.push_back(kv.first);
  return out;
}

static std::string label_str(const std::vector<std::string>& names, const std::vector<std::string>& vals,
                             const std::string& extra_k = "", const std::string& extra_v = "") {
  if (names.empty() && extra_k.empty()) return "";
  std::string o = "{";
  bool first = true;
  for (size_t i = 0; i < names.size(); ++i) {
    if (!first) o += ",";
    first = false;
    o += names[i] + "=\"" + prom_escape(vals[i]) + "\"";
  }
  if (!extra_k.empty()) {
    if (!first) o += ",";
    o += extra_k + "=\"" + extra_v + "\"";
  }
  return o + "}";
}

void MetricRegistry::commit(GaugeBatch&& batch) {
  std::vector<size_t> arity;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : batch.fams_) arity.push_back(find(kv.first)->labels.size());
  }
  for (const auto& kv : batch.blocks_) {  // arity of block series, checked off the lock
    size_t want = 0;
    {
      std::lock_guard<std::mutex> lk(mu_);
      want = find(kv.first)->labels.size();
    }
    for (const auto& b : kv.second)
      for (const auto& e : *b.second)
        if (e.first.size() != want) throw std::runtime_error("label arity mismatch for " + kv.first);
  }
  std::vector<std::pair<std::string, std::shared_ptr<const SeriesMap>>> staged;
  staged.reserve(batch.fams_.size());
  size_t i = 0;
  for (auto& kv : batch.fams_) {
    auto series = std::make_shared<SeriesMap>();
    auto& m = kv.second;
    while (!m.empty()) {  // already sorted: move each key to the end, no re-sort, no copy
      auto nh = m.extract(m.begin());
      if (nh.key().size() != arity[i]) throw std::runtime_error("label arity mismatch for " + kv.first);
      Series sr;
      sr.value = nh.mapped();
      series->emplace_hint(series->end(), std::move(nh.key()), std::move(sr));
    }
    ++i;
    staged.emplace_back(kv.first, std::move(series));
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& st : staged) {
      Family* f = find(st.first);
      f->frozen.swap(st.second);  // old snapshot freed below, off the lock
      f->series.clear();
      auto bi = batch.blocks_.find(st.first);
      if (bi != batch.blocks_.end()) f->blocks = std::make_shared<const BlockMap>(std::move(bi->second));
      else f->blocks.reset();
    }
  }
}

std::string MetricRegistry::expose() const {
  std::map<std::string, Family> fams;
  {
    std::lock_guard<std::mutex> lk(mu_);
    fams = fams_;
  }
  std::string out;
  for (const auto& kv : fams) {
    const Family& f = kv.second;
    const SeriesMap& series = f.frozen ? *f.frozen : f.series;
    const char* t = f.type == MetricType::Counter ? "counter" : f.type == MetricType::Gauge ? "gauge"
                                                                                            : "histogram";
    out += "# HELP " + kv.first + " " + f.help + "\n";
    out += "# TYPE " + kv.first + " " + t + "\n";
    if (f.blocks)
      for (const auto& b : *f.blocks)
        for (const auto& e : *b.second)
          out += kv.first + label_str(f.labels, e.first) + " " + prom_number(e.second) + "\n";
    for (const auto& s : series) {
      if (f.type != MetricType::Histogram) {
        out += kv.first + label_str(f.labels, s.first) + " " + prom_number(s.second.value) + "\n";
        continue;
      }
      double cum = 0;
      for (size_t i = 0; i < f.buckets.size(); ++i) {
        cum += i < s.second.bucket_counts.size() ? s.second.bucket_counts[i] : 0;
        out += kv.first + "_bucket" + label_str(f.labels, s.first, "le", prom_number(f.buckets[i])) +
               " " + prom_number(cum) + "\n";
      }
      out += kv.first + "_bucket" + label_str(f.labels, s.first, "le", "+Inf") + " " +
             prom_number(static_cast<double>(s.second.count)) + "\n";
      out += kv.first + "_sum" + label_str(f.labels, s.first) + " " + prom_number(s.second.sum) + "\n";
      out += kv.first + "_count" + label_str(f.labels, s.first) + " " +
             prom_number(static_cast<double>(s.second.count)) + "\n";
    }
  }
  return out;
}

void MetricRegistry::declare_kgwe_families() {
  const std::vector<double> lat{1, 2.5, 5, 10, 25, 50, 85, 100, 250, 500, 1000, 2500, 5000};
  const std::vector<double> dur{60, 300, 900, 1800, 3600, 7200, 14400, 28800, 86400};
  using M = MetricType;
  // Scheduling
  declare("kgwe_scheduling_latency_ms", M::Histogram, "Pod-create to bind scheduling latency (ms)", {}, lat);
  declare("kgwe_scheduling_attempts_total", M::Counter, "Scheduling attempts", {});
  declare("kgwe_scheduling_successes_total", M::Counter, "Successful placements", {});
  declare("kgwe_scheduling_failures_total", M::Counter, "Failed placements", {"reason"});
  declare("kgwe_topology_optimal_placements_total", M::Counter, "Placements with topology score >= 80", {});
  declare("kgwe_preemptions_total", M::Counter, "Workloads preempted", {});
  declare("kgwe_preemptions_deferred_total", M::Counter,
          "Preemption requests not served: told to wait for a near completion (wait) or over the rate window (rate)",
          {"reason"});
  // Devices
  declare("kgwe_gpu_count", M::Gauge, "GPUs discovered", {"node"});
  declare("kgwe_gpu_utilization_percent", M::Gauge, "GPU utilization (amd-smi gfx_activity %)",
          {"gpu_uuid", "node", "model"});
  declare("kgwe_gpu_gfx_activity_percent", M::Gauge, "GFX engine activity %", {"gpu_uuid", "node"});
  declare("kgwe_gpu_umc_activity_percent", M::Gauge, "Memory controller activity %", {"gpu_uuid", "node"});
  declare("kgwe_gpu_memory_used_bytes", M::Gauge, "HBM used bytes", {"gpu_uuid", "node"});
  declare("kgwe_gpu_memory_total_bytes", M::Gauge, "HBM total bytes", {"gpu_uuid", "node"});
  declare("kgwe_gpu_temperature_celsius", M::Gauge, "Hotspot temperature", {"gpu_uuid", "node"});
  declare("kgwe_gpu_power_watts", M::Gauge, "Socket power", {"gpu_uuid", "node"});
  declare("kgwe_gpu_health_status", M::Gauge, "1 healthy, 0.5 degraded, 0 unhealthy", {"gpu_uuid", "node"});
  declare("kgwe_gpu_hbm_bandwidth_gbps", M::Gauge, "Measured HBM copy bandwidth (HIP probe)", {"gpu_uuid", "node"});
  declare("kgwe_gpu_ecc_errors_total", M::Gauge, "ECC error counts", {"gpu_uuid", "node", "type"});
  declare("kgwe_gpu_retired_pages", M::Gauge, "HBM pages retired / pending retirement",
          {"gpu_uuid", "node", "state"});
  declare("kgwe_gpu_xgmi_errors", M::Gauge, "xGMI error state (0 none, 1 error, 2 multiple)",
          {"gpu_uuid", "node"});
  declare("kgwe_gpu_cper_records", M::Gauge, "CPER error records since the agent started, by severity",
          {"gpu_uuid", "node", "severity"});
  declare("kgwe_gpu_throttle_active", M::Gauge, "Active throttle / violation reasons",
          {"gpu_uuid", "node", "reason"});
  // Partitions (MIG analogue)
  declare("kgwe_gpu_partition_mode", M::Gauge, "1 for the active compute/memory partition mode",
          {"gpu_uuid", "node", "compute", "memory"});
  declare("kgwe_partition_instance_count", M::Gauge, "Partition slices", {"gpu_uuid", "node", "mode"});
  declare("kgwe_partition_instance_utilization_percent", M::Gauge, "Slices in use %", {"node", "mode"});
  declare("kgwe_partition_allocations_total", M::Counter, "Slice allocations", {"mode"});
  declare("kgwe_partition_releases_total", M::Counter, "Slice releases", {"mode"});
  declare("kgwe_partition_reconfigurations_total", M::Counter, "Partition mode switches", {"node", "result"});
  declare("kgwe_partition_migrations_total", M::Counter, "Slices moved by partition consolidation", {});
  declare("kgwe_gpu_share_clients", M::Gauge, "Co-located / time-sliced clients per GPU",
          {"gpu_uuid", "node", "method"});
  // Interconnect
  declare("kgwe_xgmi_bandwidth_gbps", M::Gauge, "xGMI link bandwidth (measured, else rated)",
          {"gpu_uuid_1", "gpu_uuid_2", "node"});
  declare("kgwe_xgmi_link_status", M::Gauge, "1 up, 0 down", {"gpu_uuid_1", "gpu_uuid_2", "node"});
  declare("kgwe_pcie_bandwidth_gbps", M::Gauge, "PCIe bandwidth", {"gpu_uuid", "node"});
  declare("kgwe_topology_score", M::Gauge, "Node topology quality score (0-100)", {"node"});
  // Cost
  declare("kgwe_gpu_cost_total_dollars", M::Counter, "Accumulated GPU cost", {"namespace", "team"});
  declare("kgwe_gpu_cost_per_hour_dollars", M::Gauge, "Running GPU cost per hour", {"namespace"});
  declare("kgwe_budget_utilization_percent", M::Gauge, "Budget spend / limit %", {"budget_id", "scope"});
  declare("kgwe_cost_savings_recommended_dollars", M::Gauge, "Projected savings from recommendations", {"type"});
  // Workloads
  declare("kgwe_active_workloads", M::Gauge, "Active workloads", {"namespace", "workload_type"});
  declare("kgwe_workload_duration_seconds", M::Histogram, "Workload run time", {"workload_type"}, dur);
  declare("kgwe_workload_queue_depth", M::Gauge, "Pods filtered and not yet bound", {});
  declare("kgwe_controller_errors_total", M::Counter, "Exceptions in the controller's periodic steps",
          {"step"});
}

}  // namespace kgwe
