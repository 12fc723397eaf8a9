// Discovery service (L2): per-node HAL providers -> immutable cluster snapshot.
//
// Reference behaviour (src/discovery/discovery.go): a cache of the cluster
// topology refreshed every 30 s plus node-watch events (:170-183, :561-613),
// a topology-hint scorer (:222-559) and a 100-slot event channel (:112-125).
// MI355X-native redesign:
//   * the new snapshot is built OFF-lock and published with an atomic
//     shared_ptr swap, so schedulers never block on a refresh (the reference
//     held the write lock for the whole refresh, discovery.go:290-319);
//   * every node has its own HAL (real amd-smi agent or fixture), instead of
//     querying one local NVML handle for every node (discovery.go:323,334);
//   * node agents may also PUSH their topology (upsert_node), which is how a
//     real multi-node cluster feeds the controller;
//   * events go to a bounded ring that drops the oldest entry instead of
//     blocking the producer; HealthChanged / LinkDown are actually emitted.
#pragma once
#include <functional>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hal.h"
#include "model.h"

namespace kgwe {

enum class TopologyEventType { NodeAdded, NodeRemoved, NodeUpdated, HealthChanged, LinkDown,
                               LinkUp, PartitionChanged };
const char* to_string(TopologyEventType t);

struct TopologyEvent {
  TopologyEventType type;
  std::string node;
  std::string gpu;
  std::string detail;
  int64_t ts_ns;
};

struct HintRequest {
  int gpu_count = 1;
  double min_memory_gb = 0.0;
  std::string arch;
  bool prefer_xgmi = true;
  bool prefer_same_numa = true;
};

struct TopologyHint {
  std::string node;
  std::vector<std::string> gpus;
  int score = 0;
  double bandwidth_gbps = 0.0;  // mean pairwise effective bandwidth of the group
  std::vector<std::string> reasons;
};

class DiscoveryService {
 public:
  explicit DiscoveryService(int refresh_interval_ms = 30000, size_t event_capacity = 1024);
  ~DiscoveryService();

  void add_node(const std::string& name, std::shared_ptr<Hal> hal);
  void remove_node(const std::string& name);
  // Push path: a node agent reports its discovered topology.
  void upsert_node(const NodeTopology& node);

  // Full refresh: discover every HAL-backed node off-lock, then publish.
  void refresh();
  // Re-discover one HAL-backed node (e.g. after a partition switch).
  bool refresh_node(const std::string& name);
  // Telemetry-only refresh of the HAL-backed nodes (cheap, periodic).
  void refresh_telemetry();
  void start();
  void stop();

  TopologySnapshot snapshot() const;
  bool node(const std::string& name, NodeTopology* out) const;
  bool gpu(const std::string& uuid, GpuDevice* out) const;
  std::shared_ptr<Hal> hal(const std::string& node) const;
  // Agent-pushed nodes have no local HAL: partition switches on them go
  // through this actuator (the controller's authenticated call to the node
  // agent's SetPartition), and the pushed topology is updated on success.
  // Signature: (node, gpu uuid, compute mode or "", memory mode or "") -> error.
  using RemoteActuator = std::function<std::string(const std::string&, const std::string&,
                                                   const std::string&, const std::string&)>;
  void set_remote_actuator(RemoteActuator fn);
  // Pushed-node helpers for the remote HAL.
  bool pushed_node(const std::string& name, NodeTopology* out) const;
  std::string actuate_remote(const std::string& node, const std::string& gpu, const std::string& compute,
                             const std::string& memory);

  std::vector<TopologyHint> hints(const HintRequest& req, size_t max_results = 3) const;

  std::vector<TopologyEvent> drain_events(size_t max = 0);
  uint64_t events_dropped() const { return dropped_.load(); }
  uint64_t generation() const;

 private:
  void publish(std::shared_ptr<ClusterTopology> next, const TopologySnapshot& prev);
  void emit(TopologyEvent e);
  void loop();

  mutable std::mutex hal_mu_;
  std::map<std::string, std::shared_ptr<Hal>> hals_;
  std::map<std::string, NodeTopology> pushed_;
  RemoteActuator actuator_;

  std::shared_ptr<const ClusterTopology> snap_;  // accessed with std::atomic_load/store
  std::mutex publish_mu_;                        // serialises writers only

  mutable std::mutex ev_mu_;
  std::deque<TopologyEvent> events_;
  size_t ev_cap_;
  std::atomic<uint64_t> dropped_{0};

  int interval_ms_;
  std::thread thread_;
  std::mutex run_mu_;
  std::condition_variable run_cv_;
  bool running_ = false;
};

}  // namespace kgwe
