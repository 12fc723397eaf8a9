// kgwe data model (L1): MI355X devices, xGMI links, compute/memory partitions,
// node and cluster topology snapshots.
//
// Parity map to the reference's Go types (src/discovery/types.go):
//   GPUDevice (:11-47)        -> GpuDevice
//   GPUMemory (:62-80)        -> memory_total_mb / memory_used_mb / hbm_bw_gbps
//   DeviceTopology (:116-131) -> numa_node, cpu_affinity, pcie, links
//   NVLinkInfo (:134-146)     -> XgmiLink (per peer, measured + rated GB/s)
//   MIGConfiguration (:167-230) -> PartitionConfig (SPX/DPX/QPX/CPX x NPS)
//   GPUUtilization (:242-266) -> Utilization (gfx_activity, umc_activity, ...)
//   GPUHealth (:269-321)      -> Health (RAS/ECC, xGMI errors, throttle)
//   NodeTopology (:351-366)   -> NodeTopology
//   ClusterTopology (:336-348)-> ClusterTopology (immutable snapshot)
// Everything is MI355X vocabulary: no NVLink / NVSwitch / MIG / NVML fields.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "json.h"

namespace kgwe {

enum class HealthStatus { Healthy, Degraded, Unhealthy, Unknown };
enum class LinkType { XGMI, PCIE, Unknown };
enum class ComputePartition { SPX, DPX, TPX, QPX, CPX };
enum class MemoryPartition { NPS1, NPS2, NPS4, NPS8 };

const char* to_string(HealthStatus s);
const char* to_string(LinkType t);
const char* to_string(ComputePartition p);
const char* to_string(MemoryPartition p);
HealthStatus health_from(const std::string& s);
LinkType link_from(const std::string& s);
ComputePartition compute_partition_from(const std::string& s);
MemoryPartition memory_partition_from(const std::string& s);
int partition_count(ComputePartition p);  // SPX 1, DPX 2, TPX 3, QPX 4, CPX 8

struct XgmiLink {
  std::string peer_uuid;
  LinkType type = LinkType::XGMI;
  int hops = 1;
  double rated_gbps = 153.6;   // per-direction rated xGMI link bandwidth
  double measured_gbps = 0.0;  // from the HIP pull probe (0 = not measured)
  bool up = true;
  // Effective bandwidth used by scorers: measured when available, else rated.
  double effective_gbps() const { return measured_gbps > 0 ? measured_gbps : rated_gbps; }
};

struct PcieInfo {
  std::string bdf;
  std::string switch_id;
  int generation = 5;
  int width = 16;
  double bandwidth_gbps = 63.0;  // Gen5 x16
};

struct Utilization {
  double gfx_activity = 0.0;  // % — THE "GPU utilisation" on MI355X
  double umc_activity = 0.0;  // % memory controller busy
  double memory_used_pct = 0.0;
  double power_w = 0.0;
  double temperature_c = 0.0;
  double gfx_clock_mhz = 0.0;
};

struct Health {
  HealthStatus status = HealthStatus::Healthy;
  std::vector<std::string> reasons;
  int64_t ecc_correctable = 0;
  int64_t ecc_uncorrectable = 0;
  int64_t ecc_deferred = 0;
  int xgmi_errors = 0;
  int xgmi_links_down = 0;          // amdsmi_get_gpu_xgmi_link_status: links reported DOWN
  int64_t retired_pages = 0;        // HBM pages retired (amdsmi_get_gpu_bad_page_info)
  int64_t pending_retired_pages = 0;  // marked bad, retired at the next reset
  std::vector<std::string> throttle_reasons;  // active violations: prochot, socket/vr/hbm thermal, ppt
  // CPER (Common Platform Error Record) entries the driver cached for this
  // GPU since the agent started (amdsmi_get_gpu_cper_entries), by severity.
  int64_t cper_fatal = 0;
  int64_t cper_uncorrected = 0;   // non-fatal uncorrected
  int64_t cper_corrected = 0;     // non-fatal corrected
  // Measured-performance degradation reported by the node agent's probes
  // (e.g. HBM copy rate well below the node median).
  bool perf_degraded = false;
  std::string perf_reason;
  bool pinned = false;              // status set by an operator / fault injection: policy leaves it
};

// Health policy shared by every HAL backend (reference GPUHealth,
// src/discovery/types.go:269-321; it only consumed `Healthy`).  Derives
// status + reasons from the raw RAS / xGMI / throttle signals:
//   Unhealthy: uncorrectable ECC, retired pages >= kRetiredPageLimit, or a
//              FATAL CPER record
//   Degraded : deferred ECC, correctable-ECC storm, pages pending retirement,
//              xGMI errors, non-fatal uncorrected CPER records, a corrected-
//              CPER storm, probe-measured performance degradation
//   reason only: xGMI links down (the group search drops the link, not the
//              GPU) and active throttling (prochot, PPT power, socket / VR /
//              HBM thermal — a GPU at full load routinely sits at its cap).
constexpr int64_t kRetiredPageLimit = 64;
constexpr int64_t kCorrectableStorm = 1000;
constexpr int64_t kCperCorrectedStorm = 100;
void apply_health_policy(Health& h, int links_down_in_topology = 0);

// One schedulable slice of a partitioned GPU (CPX: 8 per GPU, one per XCD).
struct PartitionInstance {
  std::string id;  // "<gpu uuid>/p<index>"
  int index = 0;
  int cu_count = 256;
  double memory_gb = 288.0;
  bool in_use = false;
  std::string owner;  // workload uid
};

struct PartitionConfig {
  ComputePartition compute = ComputePartition::SPX;
  MemoryPartition memory = MemoryPartition::NPS1;
  bool switching = false;  // reconfiguration in flight (drain -> switch)
  std::vector<PartitionInstance> instances;
};

struct GpuDevice {
  std::string uuid;
  int index = 0;
  std::string node;
  std::string model = "AMD Instinct MI355X";
  std::string arch = "gfx950";
  int cu_count = 256;
  int xcd_count = 8;
  double memory_total_gb = 288.0;
  double memory_used_gb = 0.0;
  double hbm_rated_gbps = 8000.0;
  double hbm_measured_gbps = 0.0;
  double peak_bf16_tflops = 2500.0;
  int numa_node = 0;
  int socket = 0;
  PcieInfo pcie;
  std::vector<XgmiLink> links;
  PartitionConfig partition;
  Utilization util;
  Health health;

  double memory_free_gb() const { return memory_total_gb - memory_used_gb; }
  const XgmiLink* link_to(const std::string& peer) const;
  bool healthy() const { return health.status == HealthStatus::Healthy; }
};

struct NodeTopology {
  std::string name;
  std::map<std::string, std::string> labels;
  std::vector<std::pair<std::string, std::string>> taints;  // key=value:effect
  std::vector<GpuDevice> gpus;
  int numa_nodes = 2;
  int cpu_sockets = 2;
  bool xgmi_fully_connected = true;
  int64_t updated_ns = 0;
  // Dense pairwise link tables by GPU POSITION in `gpus` (index_links): the
  // scheduler's group search reads these instead of resolving links by uuid.
  std::vector<float> link_bw;    // [G*G] effective xGMI GB/s, else PCIe fallback
  std::vector<uint8_t> link_up;  // [G*G] 1 = xGMI link up both ways
  uint64_t topo_fp = 0;          // fingerprint of links / NUMA / switches / health

  const GpuDevice* gpu(const std::string& uuid) const;
  GpuDevice* gpu(const std::string& uuid);
  int position(const GpuDevice* g) const { return static_cast<int>(g - gpus.data()); }
};

// Build NodeTopology::link_bw / link_up / topo_fp from the GPUs' links.
void index_links(NodeTopology& n);

// Copy-on-write node map of a cluster snapshot.  Every publish builds a new
// ClusterTopology from the previous one; with nodes held by shared pointer,
// that copy is O(nodes) pointer copies and only the changed nodes are cloned
// (a deep copy of 1,250 nodes cost ~30 ms per partition switch and made
// adding N nodes O(N^2)).  Reads look like std::map<std::string,
// NodeTopology>: `kv.first`, `kv.second.gpus`, `it->second`, find / at /
// count; writes go through set / mut / erase.
class NodeMap {
 public:
  using Ptr = std::shared_ptr<NodeTopology>;
  using Base = std::map<std::string, Ptr>;
  struct Entry {
    const std::string& first;
    const NodeTopology& second;
  };
  class const_iterator {
   public:
    const_iterator() = default;
    explicit const_iterator(Base::const_iterator it) : it_(it) {}
    Entry operator*() const { return Entry{it_->first, *it_->second}; }
    struct Arrow {
      Entry e;
      const Entry* operator->() const { return &e; }
    };
    Arrow operator->() const { return Arrow{**this}; }
    const_iterator& operator++() {
      ++it_;
      return *this;
    }
    bool operator==(const const_iterator& o) const { return it_ == o.it_; }
    bool operator!=(const const_iterator& o) const { return it_ != o.it_; }
    const Ptr& ptr() const { return it_->second; }

   private:
    Base::const_iterator it_;
  };

  const_iterator begin() const { return const_iterator(m_.begin()); }
  const_iterator end() const { return const_iterator(m_.end()); }
  const_iterator find(const std::string& k) const { return const_iterator(m_.find(k)); }
  size_t size() const { return m_.size(); }
  bool empty() const { return m_.empty(); }
  size_t count(const std::string& k) const { return m_.count(k); }
  const NodeTopology& at(const std::string& k) const { return *m_.at(k); }
  size_t erase(const std::string& k) { return m_.erase(k); }
  void set(const std::string& k, NodeTopology n) { m_[k] = std::make_shared<NodeTopology>(std::move(n)); }
  // A node this map owns alone (cloned first if a snapshot shares it).
  NodeTopology& mut(const std::string& k) {
    Ptr& p = m_.at(k);
    if (p.use_count() > 1) p = std::make_shared<NodeTopology>(*p);
    return *p;
  }
  // Same object in both maps => the node did not change between them.
  bool same(const std::string& k, const NodeMap& other) const {
    auto a = m_.find(k), b = other.m_.find(k);
    return a != m_.end() && b != other.m_.end() && a->second == b->second;
  }

 private:
  Base m_;
};

struct ClusterTopology {
  NodeMap nodes;
  uint64_t generation = 0;
  int64_t updated_ns = 0;
  int total_gpus() const;
};

using TopologySnapshot = std::shared_ptr<const ClusterTopology>;

// JSON <-> model (fixture format == snapshot export format).
GpuDevice gpu_from_json(const Json& j, const std::string& node);
Json to_json(const GpuDevice& g);
NodeTopology node_from_json(const Json& j);
Json to_json(const NodeTopology& n);
Json to_json(const ClusterTopology& c);

int64_t now_ns();

}  // namespace kgwe
