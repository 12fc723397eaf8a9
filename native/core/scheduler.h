// Topology-aware GPU scheduler core (L5) for MI355X clusters.
//
// Reference: src/scheduler/scheduler.go (Schedule :114-179, filter :206-241,
// scorers :244-578, ledger :625-727, preemption :730-790, metrics :805-819)
// and src/scheduler/types.go (workload/decision/config types).
//
// Capabilities kept: filter -> score (topology / resource / balance, weighted
// 40/35/25, +10 optimizer-hint bonus) -> try nodes best-first -> record;
// release; preemption; gang groups; metrics and events.  Defects fixed:
//   * reserve = ONE critical section (re-check + record): no double
//     allocation under concurrent Schedule calls (reference TOCTOU :630/:696);
//   * p99 comes from a real latency histogram, not a running max (:818);
//   * preemption respects priority and `preemptible`, picks the cheapest
//     victim SET on one node, and retries once (no unbounded recursion :759);
//   * every requirement is enforced in the filter: nodeSelector, required
//     node affinity, taints/tolerations, excludeNodes, co-location and
//     anti-affinity, minMemoryGB, minBandwidthGBps, arch (k GPUs of it, not
//     "any"), xGMIRequired as a hard constraint;
//   * events go to a bounded ring (never blocks), metrics are lock-consistent.
// MI355X-first scoring: an 8xMI355X node is an all-to-all
// xGMI mesh, so every k-subset is pairwise equivalent under the reference's
// clique search; the native scorer ranks groups by MEASURED link bandwidth
// (degraded/down links), NUMA/socket compactness and fragmentation (largest
// free group left behind).  The reference formulas are kept as
// ScoringMode::Compat for A/B comparison.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "rwlock.h"
#include "discovery.h"
#include "histogram.h"
#include "model.h"

namespace kgwe {

enum class TopologyPreference { None, XgmiOptimal, XgmiRequired, SameNUMA, SamePCIeSwitch };
enum class WorkloadType { Training, Inference, Batch, Interactive, Development, Unknown };
enum class DistributionStrategy { None, DataParallel, ModelParallel, PipelineParallel, Hybrid,
                                  FSDP, DeepSpeed, ContextParallel, ExpertParallel };
enum class CommBackend { RCCL, Gloo, MPI };
enum class ScoringMode { Xgmi, Compat };
// GPU sharing without compute partitions (reference MPS / time-slicing,
// src/sharing/mig_controller.go:545-857).  Partition = a CPX/QPX/DPX slice,
// held through the partition fields of the request instead.
enum class SharingMethod { None, Partition, CoLocate, TimeSlice };
const char* to_string(SharingMethod m);
SharingMethod sharing_method_from(const std::string& s);

const char* to_string(TopologyPreference p);
const char* to_string(WorkloadType t);
const char* to_string(DistributionStrategy s);
const char* to_string(CommBackend b);
TopologyPreference topology_preference_from(const std::string& s);
WorkloadType workload_type_from(const std::string& s);
DistributionStrategy strategy_from(const std::string& s);
CommBackend backend_from(const std::string& s);

struct Toleration {
  std::string key, op = "Equal", value, effect;
};

struct AffinityTerm {
  std::string key, op;  // In, NotIn, Exists, DoesNotExist, Gt, Lt
  std::vector<std::string> values;
  int weight = 0;       // preferred terms only
};

struct WorkloadRequest {
  std::string uid, name, ns = "default", team, project;
  int gpu_count = 1;
  double min_memory_gb = 0.0;
  double min_bandwidth_gbps = 0.0;
  TopologyPreference topology = TopologyPreference::None;
  std::string arch, model;
  // Partition (compute-partition slice) request instead of whole GPUs.
  bool partition = false;
  ComputePartition partition_mode = ComputePartition::CPX;
  int partition_count = 0;
  bool partition_memory_set = false;  // gpuRequirements.partition.memoryMode given
  MemoryPartition partition_memory = MemoryPartition::NPS1;
  WorkloadType type = WorkloadType::Training;
  std::string framework = "PyTorch";
  DistributionStrategy strategy = DistributionStrategy::None;
  CommBackend backend = CommBackend::RCCL;
  int world_size = 0;
  int64_t priority = 0;
  bool preemptible = true;
  std::map<std::string, std::string> node_selector;
  std::vector<AffinityTerm> required_affinity;
  std::vector<AffinityTerm> preferred_affinity;
  std::vector<Toleration> tolerations;
  std::vector<std::string> exclude_nodes;
  std::vector<std::string> colocate_with;
  std::vector<std::string> anti_affinity_with;
  std::string gang;
  int gang_size = 0;
  // Co-located / time-sliced share of ONE whole SPX GPU (no partition
  // switch): a disjoint CU range (HSA_CU_MASK) plus an HBM cap per client.
  SharingMethod sharing = SharingMethod::None;
  double share_cu_percent = 0.0;   // 0 = policy default
  double share_memory_gb = 0.0;    // 0 = no cap
  // Clients of one share group (same model, one serving process) hold ONE CU
  // range and ONE HBM cap on a GPU between them: the first is the group's
  // leader (runs the server), the rest are members that connect to it.
  std::string share_group;
  double max_latency_ms = 0.0;
  std::vector<std::string> preferred_nodes;  // optimizer hint (+10 bonus)
  // How long the workload is expected to hold its GPUs (spec
  // expectedDurationSeconds, pod annotation kgwe.amd.com/expected-duration-seconds
  // or spec.activeDeadlineSeconds); 0 = unknown (the scheduler's learned
  // per-type mean is used once it has enough samples).
  double expected_duration_s = 0.0;
};

WorkloadRequest workload_from_json(const Json& j);
Json to_json(const WorkloadRequest& w);

struct NodeScore {
  std::string node;
  int total = 0, topology = 0, resource = 0, balance = 0, affinity = 0;
  std::vector<std::string> gpus;        // selected whole GPUs
  std::vector<std::string> partitions;  // selected partition slices
  std::string shared_gpu;               // sharing requests: the GPU to join
  int cu_begin = 0, cu_end = 0;
  double bandwidth_gbps = 0.0;
  std::vector<std::string> reasons;
};

struct Allocation {
  std::string uid, node, ns, team, gang;
  int gang_size = 0;
  std::vector<std::string> gpus;
  std::vector<std::string> partitions;
  // Sharing: the one GPU co-located / time-sliced with other clients.
  SharingMethod sharing = SharingMethod::None;
  std::string shared_gpu;
  int cu_begin = 0, cu_end = 0;  // [begin, end) of the GPU's CUs (CoLocate)
  double share_memory_gb = 0.0;
  std::string share_group;       // "" = a share of its own
  bool share_leader = false;     // first client of its group on the GPU (holds the range and the cap)
  std::string share_leader_uid;  // the group's leader (itself for the leader)
  WorkloadType type = WorkloadType::Training;
  int64_t priority = 0;
  bool preemptible = true;
  bool gang_pending = false;  // reserved, waiting for the rest of its gang
  int64_t allocated_ns = 0;
  int64_t expected_end_ns = 0;  // 0 = unknown
  double bandwidth_gbps = 0.0;
};

struct Decision {
  bool ok = false;
  std::string status;  // Scheduled | Waiting (gang) | Unschedulable
  std::string uid, node;
  std::vector<std::string> gpus, partitions;
  std::string shared_gpu;
  SharingMethod sharing = SharingMethod::None;
  int cu_begin = 0, cu_end = 0;
  double share_memory_gb = 0.0;
  std::string share_group, share_leader_uid;  // group shares: who runs the group's server
  bool share_leader = false;
  int score = 0;
  double bandwidth_gbps = 0.0;
  double latency_ms = 0.0;
  std::vector<std::string> reasons;
  std::vector<std::string> preempted;
  std::map<std::string, std::string> failed_nodes;  // node -> reason
};

Json to_json(const Decision& d);
Json to_json(const Allocation& a);
Allocation allocation_from_json(const Json& j);

struct SchedulerConfig {
  int topology_weight = 40, resource_weight = 35, balance_weight = 25;
  bool enable_preemption = true;
  bool enable_gang = true;
  int gang_timeout_ms = 30000;
  int max_attempts = 3;           // nodes tried best-first per Schedule
  ScoringMode mode = ScoringMode::Xgmi;
  bool pack = true;                // xGMI mode: best-fit across nodes (false = spread)
  double rated_link_gbps = 153.6;  // MI355X xGMI per-link (normalisation)
  double degraded_link_ratio = 0.7;  // measured/rated below this => degraded link
  size_t event_capacity = 4096;
  size_t exhaustive_limit = 4096;  // max combinations enumerated per node
  // Sharing policy (reference MPSControllerConfig, mig_controller.go:559-581).
  int max_share_clients = 8;          // co-located clients per GPU
  double default_cu_percent = 12.5;   // one XCD (32 of 256 CUs)
  int max_timeslice_replicas = 4;
  int max_group_clients = 32;         // members of one share group on a GPU
  // Preemption policy.  Victims are planned exactly only on the K nodes a
  // cheap per-node estimate ranks best; an allocation expected to finish
  // within the wait window is not a victim, and a request whose room such
  // allocations will free waits for them instead (up to max wait; requests at
  // or above the urgent priority never wait); victims per sliding window are
  // capped at a percentage of the placements in it (plus a small burst).
  int preemption_candidate_nodes = 8;
  double preemption_wait_window_s = 30.0;   // 0 = never prefer waiting
  double preemption_max_wait_s = 120.0;
  int64_t preemption_urgent_priority = 1000000;
  double preemption_max_rate_percent = 4.0;  // 0 = no cap
  int preemption_window_s = 300;
  int preemption_burst = 8;
};

enum class SchedEventType { Scheduled, Failed, Released, Preempted, GangReady, GangTimeout, Migrated };
struct SchedEvent {
  SchedEventType type;
  std::string uid, node, detail;
  int64_t ts_ns;
};
const char* to_string(SchedEventType t);

struct SchedulerMetrics {
  uint64_t attempts = 0, scheduled = 0, failed = 0, topology_optimal = 0, preemptions = 0,
           releases = 0, gang_timeouts = 0,
           preemptions_deferred_wait = 0,   // requests told to wait for a near completion
           preemptions_rate_limited = 0;    // requests refused by the window cap
  double avg_latency_ms = 0.0, p50_ms = 0.0, p90_ms = 0.0, p99_ms = 0.0, max_ms = 0.0;
  size_t active_allocations = 0, allocated_gpus = 0, allocated_partitions = 0, shared_gpus = 0,
         share_clients = 0;
};

class Scheduler {
 public:
  Scheduler(std::shared_ptr<DiscoveryService> disc, SchedulerConfig cfg = {});

  // Full pipeline: filter -> score -> reserve best-first (-> preempt).
  Decision schedule(const WorkloadRequest& w);
  // All-or-nothing placement of a whole gang (controller path).
  std::vector<Decision> schedule_gang(const std::vector<WorkloadRequest>& members);

  // Extender building blocks (kube-scheduler extender verbs).
  std::map<std::string, std::string> filter(const WorkloadRequest& w,
                                            const std::vector<std::string>& nodes,
                                            std::vector<std::string>* passed);
  std::vector<NodeScore> prioritize(const WorkloadRequest& w, const std::vector<std::string>& nodes);
  // The two sweeps as the extender serves them: per candidate, the filter
  // verdict ("" = passes) / the total score, with no per-node allocation on a
  // cache hit (see NodeCache below).  (*why)[i] / (*totals)[i] belong to nodes[i].
  void filter_verdicts(const WorkloadRequest& w, const std::vector<std::string>& nodes,
                       std::vector<std::string>* why);
  void prioritize_totals(const WorkloadRequest& w, const std::vector<std::string>& nodes,
                         std::vector<int>* totals);
  // Reserve on a given node (bind verb); honours gangs (may return Waiting).
  Decision bind(const WorkloadRequest& w, const std::string& node);
  // Extender preempt verb: for the best candidate nodes (at most
  // preemption_candidate_nodes of them), the cheapest victim set that makes
  // room for `w` (empty = fits as is; absent = impossible, or preemption is
  // deferred by the wait / rate policy).  Dry run; the cheapest returned plan
  // is charged to the rate window.
  std::map<std::string, std::vector<std::string>> preemption_plans(const WorkloadRequest& w,
                                                                   const std::vector<std::string>& nodes);
  void count_preemptions(size_t n);  // victims evicted by kube-scheduler after a dry-run plan (statistics)
  // Permit-stage check for a gang member: "Allow" | "Wait" | "Reject".
  std::string permit(const std::string& uid);

  bool release(const std::string& uid);
  // Explicit share placement (SharingManager / tests): a client slot for the
  // sharing request `w` on GPU `gpu` of `node`.
  Decision reserve_share(const WorkloadRequest& w, const std::string& node, const std::string& gpu);
  // Move one partition slice of `uid` to another free slice (consolidation).
  // Atomic under the ledger lock; false if `to` is no longer free.
  bool migrate_partition(const std::string& uid, const std::string& from, const std::string& to);
  void expire_gangs();  // release timed-out gang reservations
  // Restore the ledger (controller restart: rebuilt from pod annotations).
  bool restore(const Allocation& a);

  // True when the GPU, any of its partition slices or a share of it is held
  // in the ledger.
  bool gpu_busy(const GpuDevice& g) const;
  // Ledger view of one node for the partition controller's capacity planning,
  // memoised like the filter verdicts (same validity key): bit p of idle_mask
  // = GPU at position p is healthy, not switching, unreserved (whole, slices,
  // shares, fence), reports no busy slice and < 5 % gfx activity;
  // free_slices[p] = its slices that are neither in use nor reserved.
  struct NodeSummary {
    uint64_t idle_mask = 0;
    std::vector<uint8_t> free_slices;
  };
  NodeSummary node_summary(const NodeTopology& n) const;
  // Share clients currently on a GPU (CoLocate / TimeSlice).
  int share_clients(const std::string& gpu_uuid) const;
  // Members of `uid`'s share group left on its GPU (uid itself excluded), and
  // whether uid is the group's leader: what a release has to tell the controller.
  std::vector<std::string> share_group_peers(const std::string& uid, bool* leader) const;
  // Partition-switch fence: atomically (under the ledger lock) check that no
  // whole-GPU or slice reservation holds `gpu_uuid` and bar new ones until
  // unfence_gpu.  Closes the window between the controller's idle check and
  // the mode switch, during which a scheduler thread working from an older
  // snapshot could otherwise reserve the GPU (or a slice of it).
  bool fence_gpu(const std::string& gpu_uuid, const std::string& node = "");
  void unfence_gpu(const std::string& gpu_uuid, const std::string& node = "");
  // Consolidation donor: no NEW slice reservations on the GPU (existing ones
  // stay until their pods are evicted); whole-GPU requests never land on a
  // partitioned GPU anyway.
  void set_draining(const std::string& gpu_uuid, const std::string& node, bool on);
  std::vector<std::string> draining() const;
  // Cordon: no new placements on the node (NotReady / draining); existing
  // allocations are untouched.
  void set_cordon(const std::string& node, bool on);
  std::vector<std::string> cordoned() const;
  std::vector<Allocation> allocations() const;
  bool allocation(const std::string& uid, Allocation* out) const;
  SchedulerMetrics metrics() const;
  const LatencyHistogram& latency() const { return latency_; }
  void record_latency_ms(double ms) { latency_.record_ms(ms); }
  std::vector<SchedEvent> drain_events(size_t max = 0);
  const SchedulerConfig& config() const { return cfg_; }
  void set_config(const SchedulerConfig& c);
  std::shared_ptr<DiscoveryService> discovery() const { return disc_; }

  // Exposed for tests / the optimizer: score one node for a request.
  NodeScore score_node(const NodeTopology& n, const WorkloadRequest& w) const;
  std::string eligible(const NodeTopology& n, const WorkloadRequest& w) const;  // "" = ok
  std::string admissible(const NodeTopology& n, const WorkloadRequest& w) const;  // eligible() minus capacity

 private:
  struct Ctx;  // per-call view of the ledger for one node
  std::vector<const GpuDevice*> free_gpus(const NodeTopology& n, const WorkloadRequest& w) const;
  std::vector<const PartitionInstance*> free_partitions(const NodeTopology& n,
                                                        const WorkloadRequest& w,
                                                        std::vector<std::string>* gpu_of) const;
  int topology_score(const NodeTopology& n, const std::vector<const GpuDevice*>& avail,
                     const WorkloadRequest& w, std::vector<std::string>* sel, double* bw,
                     bool* clique) const;
  int topology_search(const NodeTopology& n, const std::vector<const GpuDevice*>& avail,
                      const WorkloadRequest& w, std::vector<std::string>* sel, double* bw, bool* clique) const;
  int topology_score_compat(const NodeTopology& n, const std::vector<const GpuDevice*>& avail,
                            const WorkloadRequest& w, std::vector<std::string>* sel) const;
  int resource_score(const std::vector<const GpuDevice*>& avail, const WorkloadRequest& w) const;
  int balance_score(const NodeTopology& n, int requested) const;
  // Sharing requests: best-fit GPU on the node + CU range; false if none.
  bool pick_share(const NodeTopology& n, const WorkloadRequest& w, NodeScore* s) const;
  bool share_fits(const GpuDevice& g, const WorkloadRequest& w, int* cu_begin, int* cu_end) const;
  bool reserve_locked(const WorkloadRequest& w, const NodeScore& s, bool gang_pending);
  void erase_locked(std::unordered_map<std::string, Allocation>::iterator it);
  using PreemptCost = std::tuple<int64_t, size_t, size_t>;  // (sum of victim priorities, victims, GPUs)
  struct PreemptPlan {
    std::string node;
    std::vector<std::string> victims;
    PreemptCost cost{0, 0, 0};
  };
  bool try_preempt(const WorkloadRequest& w, const TopologySnapshot& snap, Decision* d);
  // Exact plans on the best candidate nodes (see SchedulerConfig).  With
  // `commit` the cheapest plan's victims are erased under the same exclusive
  // lock hold that validated it, and only that plan is returned.
  std::vector<PreemptPlan> select_preemption(const WorkloadRequest& w, const TopologySnapshot& snap,
                                             const std::vector<std::string>* nodes, bool commit);
  bool plan_node_preemption(const WorkloadRequest& w, const NodeTopology& n, int64_t protect_until_ns,
                            std::vector<std::string>* victims, PreemptCost* cost);
  // Shared lock.  Cheap upper-bound estimate for one node: false if even
  // evicting every eligible victim cannot make room; *wait = the room will be
  // freed by allocations expected to finish before `soon_ns`.
  bool estimate_node_preemption(const WorkloadRequest& w, const NodeTopology& n, int64_t now, int64_t soon_ns,
                                PreemptCost* cost, bool* wait) const;
  bool near_completion(const Allocation& a, int64_t now, int64_t soon_ns) const;
  void index_alloc_locked(const Allocation& a);
  int64_t expected_end_locked(const WorkloadRequest& w, int64_t start_ns) const;
  // Rate window (stat_mu_): victims still allowed now; charge() books them.
  int preemption_budget_locked(int64_t now);
  void note_placement();
  void emit(SchedEvent e);
  double bandwidth_of(const NodeTopology& n, const std::vector<std::string>& gpus) const;

  std::shared_ptr<DiscoveryService> disc_;
  SchedulerConfig cfg_;

  mutable RwLock mu_;  // guards the ledger below (writer-preferring)
  std::unordered_map<std::string, Allocation> allocs_;
  std::unordered_map<std::string, std::string> gpu_owner_;   // gpu uuid -> uid
  std::unordered_map<std::string, std::string> part_owner_;  // partition id -> uid
  struct SharedGpu {
    SharingMethod method = SharingMethod::None;
    std::vector<std::string> clients;  // uids
  };
  std::unordered_map<std::string, SharedGpu> shared_;        // gpu uuid -> clients
  std::set<std::string> fenced_;                             // GPUs mid partition switch
  std::set<std::string> draining_gpus_;                      // consolidation donors: no new slices
  mutable std::mutex cordon_mu_;
  std::set<std::string> cordoned_;
  bool gpu_has_slice_owner_locked(const std::string& gpu_uuid) const;
  std::unordered_map<std::string, int> node_gpus_used_;      // node -> allocated GPUs
  std::unordered_map<std::string, std::vector<std::string>> node_allocs_;  // node -> uids on it
  // Learned mean lifetime per workload type (released allocations only), for
  // allocations that do not say how long they expect to run.
  struct Lifetime {
    double mean_s = 0.0;
    uint64_t n = 0;
  };
  Lifetime lifetimes_[8];
  struct Gang {
    int size = 0;
    std::set<std::string> members;
    int64_t first_ns = 0;
    bool ready = false;
  };
  std::map<std::string, Gang> gangs_;

  // Per-node memo of filter verdicts and scores.  A node's verdict for a
  // request depends on the node's topology object, the ledger entries on that
  // node and the request's placement-relevant fields; between two scheduling
  // cycles almost no node changes, so a 500-candidate sweep is ~500 lookups
  // instead of 500 x (8 GPUs x 3 ledger probes + group search).  Entries are
  // keyed by the request signature and validated against the node's ledger
  // epoch (bumped under the exclusive ledger lock by every change on that
  // node), the topology object and a global generation (cordon, config,
  // fences without a node).  Advisory only: bind() re-checks under the lock.
  struct NodeCacheEntry {
    uint64_t sig = 0, epoch = 0, gen = 0;
    const NodeTopology* topo = nullptr;
    int64_t topo_ns = 0;
    bool has_why = false, has_total = false, has_summary = false;
    NodeSummary summary;
    std::string why;
    int total = 0;
    uint64_t used = 0;
  };
  struct NodeCache {
    std::mutex mu;
    std::atomic<uint64_t> epoch{0};
    std::vector<NodeCacheEntry> entries;
    uint64_t clock = 0;
  };
  NodeCache& cache_of(const std::string& node) const;
  void touch_node(const std::string& node);  // caller holds mu_ exclusively
  // 0 = not cacheable (verdict depends on other nodes' ledger entries).
  static uint64_t request_signature(const WorkloadRequest& w);
  const std::string& eligible_cached(const NodeTopology& n, const WorkloadRequest& w, uint64_t sig,
                                     std::string* scratch) const;
  int total_cached(const NodeTopology& n, const WorkloadRequest& w, uint64_t sig) const;
  mutable std::shared_mutex cache_map_mu_;
  mutable std::unordered_map<std::string, std::unique_ptr<NodeCache>> node_cache_;
  std::atomic<uint64_t> global_gen_{1};

  mutable std::mutex stat_mu_;
  SchedulerMetrics stats_;
  struct RateBucket {
    int64_t sec = 0;
    uint32_t placed = 0, victims = 0;
  };
  std::deque<RateBucket> rate_;                              // one bucket per second with activity
  std::unordered_map<std::string, int64_t> preempt_wait_;    // uid -> first time it was told to wait
  LatencyHistogram latency_;

  mutable std::mutex ev_mu_;
  std::deque<SchedEvent> events_;
};

}  // namespace kgwe
