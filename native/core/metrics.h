// Prometheus metric registry + text exposition (format 0.0.4).
//
// Reference: src/monitoring/prometheus_exporter.go (primitives :135-238,
// 27 kgwe_* families :256-411, exposition :542-629).  Fixed: label SETS are
// kept per series (the reference collapsed them into one composite
// `label="node/uuid"`, :614-616, breaking the Grafana `node=~"$node"` filter),
// histogram `le` values are formatted exactly (not "%f", :598), every family is
// exposed (WorkloadDuration was never written), and the recorders are actually
// called by the scheduler / cost engine / agent.
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace kgwe {

enum class MetricType { Counter, Gauge, Histogram };

class GaugeBatch;

class MetricRegistry {
 public:
  using Labels = std::vector<std::string>;  // values, in the family's label order

  void declare(const std::string& name, MetricType type, const std::string& help,
               const std::vector<std::string>& label_names,
               const std::vector<double>& buckets = {});
  void set(const std::string& name, const Labels& lv, double v);
  void add(const std::string& name, const Labels& lv, double v = 1.0);
  void observe(const std::string& name, const Labels& lv, double v);
  void remove(const std::string& name, const Labels& lv);
  void clear(const std::string& name);  // drop all series of a family
  double value(const std::string& name, const Labels& lv) const;
  bool has(const std::string& name) const;
  // Render under a copy: the lock is held only for the copy, so counters
  // bumped by the scheduling path never wait on text formatting.
  std::string expose() const;
  std::vector<std::string> families() const;
  // Replace every family named in the batch with exactly the batch's series
  // (atomically per family: a scrape never sees a half-refreshed family).
  void commit(GaugeBatch&& batch);

  // The kgwe_* families (reference names kept; NVLink -> xGMI, MIG -> partition,
  // plus xGMI link status, partition mode and gfx activity gauges).
  void declare_kgwe_families();

 private:
  struct Series {
    double value = 0.0;
    std::vector<double> bucket_counts;  // histogram: per-bucket (non-cumulative)
    double sum = 0.0;
    uint64_t count = 0;
  };
  using SeriesMap = std::map<Labels, Series>;

 public:
  // Gauge series grouped in immutable blocks (one per source object, e.g. a
  // node): a refresh re-uses the block of every source that did not change,
  // so its cost — and its allocator churn — follows the changes, not the
  // fleet size.
  using Block = std::vector<std::pair<Labels, double>>;
  using BlockMap = std::map<std::string, std::shared_ptr<const Block>>;

 private:
  struct Family {
    MetricType type;
    std::string help;
    std::vector<std::string> labels;
    std::vector<double> buckets;
    SeriesMap series;
    // Committed by a GaugeBatch: immutable and shared with in-flight scrapes,
    // so expose() copies a pointer under the lock, not 10^5 series.  A later
    // set()/add() on the family copies it back into `series` (copy-on-write).
    std::shared_ptr<const SeriesMap> frozen;
    std::shared_ptr<const BlockMap> blocks;  // committed gauge blocks, beside `frozen`
  };
  Family* find(const std::string& name);
  Family* find_mut(const std::string& name);  // find + thaw a committed family
  mutable std::mutex mu_;
  std::map<std::string, Family> fams_;
};

// Gauge values staged off-lock by a periodic refresh (Platform::tick), then
// swapped in with MetricRegistry::commit.
class GaugeBatch {
 public:
  void set(const std::string& name, MetricRegistry::Labels lv, double v) { fams_[name][std::move(lv)] = v; }
  void add(const std::string& name, MetricRegistry::Labels lv, double v) { fams_[name][std::move(lv)] += v; }
  void touch(const std::string& name) { fams_[name]; }  // replace even when it ends up empty
  // Series of `name` that come as one shared block per source `key`.
  void block(const std::string& name, const std::string& key, std::shared_ptr<const MetricRegistry::Block> b) {
    fams_[name];
    blocks_[name][key] = std::move(b);
  }

 private:
  friend class MetricRegistry;
  std::map<std::string, std::map<MetricRegistry::Labels, double>> fams_;
  std::map<std::string, MetricRegistry::BlockMap> blocks_;
};

std::string prom_escape(const std::string& v);
std::string prom_number(double v);

}  // namespace kgwe
