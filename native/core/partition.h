// MI355X compute/memory-partition controller (replaces the reference's MIG
// controller, src/sharing/mig_controller.go:16-542).
//
// MI355X partitions are HOMOGENEOUS per GPU: a compute mode (SPX = 1 x 256
// CUs, DPX = 2 x 128, QPX = 4 x 64, CPX = 8 x 32, one slice per XCD) applies
// to the whole device, a mode switch needs the GPU idle, and the memory mode
// (NPS1 / NPS2) constrains which compute modes are valid.  So unlike MIG's
// per-slot profiles, the planner reasons at GPU-mode granularity:
//   * ensure_capacity(mode, n): free slices of `mode` first (best fit), then
//     convert idle SPX GPUs, preferring nodes that already run that mode
//     (consolidation) — drain -> switch -> re-advertise;
//   * strategies (PartitionStrategy CRD, the MIGStrategy analogue,
//     gpuworkload-crd.yaml:248-366): validated mode distribution, rebalanced
//     onto idle GPUs only;
//   * every reconfiguration is an Operation with a state machine
//     (Pending -> Draining -> Switching -> Completed | Failed), actuated
//     through the node's HAL (amd-smi set_gpu_compute_partition), dry-run
//     capable (the gpurun box is non-root, settings are read-only).
// The reference's allocation path could never succeed (both lookup helpers
// were stubs that always errored, mig_controller.go:340-415); here slice
// allocation is done by the scheduler ledger and this controller only
// manages capacity.
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <unordered_set>
#include <vector>

#include "discovery.h"
#include "scheduler.h"

namespace kgwe {

struct PartitionStrategy {
  std::string name;
  std::map<std::string, std::string> node_selector;
  std::string gpu_model;
  double min_memory_gb = 0.0;
  std::map<ComputePartition, double> distribution;  // fraction of matching GPUs
  MemoryPartition memory = MemoryPartition::NPS1;
  bool allow_dynamic = true;
  int rebalance_interval_s = 300;
  double min_utilization = 0.3;  // slices of a mode below this use may shrink
  int priority = 0;
};

// MI355X memory modes: NPS1 with any compute mode; NPS2 needs the compute
// partitions to split evenly over the two memory domains (DPX / QPX / CPX).
bool valid_mode_combo(ComputePartition c, MemoryPartition m);
std::string validate_strategy(const PartitionStrategy& s);  // "" = valid
PartitionStrategy strategy_from_json(const Json& j);
Json to_json(const PartitionStrategy& s);

enum class OpState { Pending, Draining, Switching, Completed, Failed };
const char* to_string(OpState s);

struct PartitionOp {
  std::string id, node, gpu, reason, error;
  ComputePartition from = ComputePartition::SPX, to = ComputePartition::SPX;
  MemoryPartition mem_to = MemoryPartition::NPS1;
  OpState state = OpState::Pending;
  bool dry_run = false;
  int64_t created_ns = 0, finished_ns = 0;
};
Json to_json(const PartitionOp& op);

// One slice moved by consolidation: `uid` leaves `from` for `to`.
struct PartitionMove {
  std::string uid, from, to, node_from, node_to;
};
Json to_json(const PartitionMove& m);

// Consolidating rebalance (reference MIGController.Rebalance, a no-op there:
// src/sharing/mig_controller.go:480-512; minUtilizationThreshold, CRD
// gpuworkload-crd.yaml:248-366).
struct ConsolidationPolicy {
  double below = 0.75;         // a partitioned GPU with slice occupancy < this is a donor
  double after_s = 120.0;      // ... once it has stayed below for this long (hysteresis)
  double cooldown_s = 3600.0;  // a workload is migrated at most once per cooldown
};

struct PartitionMetrics {
  struct Mode {
    int gpus = 0, slices = 0, slices_in_use = 0;
  };
  std::map<std::string, Mode> modes;
  int ops_total = 0, ops_failed = 0, ops_pending = 0;
  double slice_utilization = 0.0;  // in-use / total over partitioned GPUs
};

class PartitionController {
 public:
  PartitionController(std::shared_ptr<DiscoveryService> disc, std::shared_ptr<Scheduler> sched,
                      bool dry_run = false);

  std::string register_strategy(const PartitionStrategy& s);  // "" = ok
  bool remove_strategy(const std::string& name);
  std::vector<PartitionStrategy> strategies() const;

  // Plan (and unless plan_only, execute) conversions so that `count` free
  // slices of `mode` exist.  Returns the operations (possibly empty).
  // `memory` (optional): the NPS mode the slices must have; converted GPUs
  // are switched to it too.
  // `within` (optional): only count and convert GPUs on these nodes — the
  // extender passes the pod's candidate nodes, so capacity appears where
  // kube-scheduler can actually bind.
  std::vector<PartitionOp> ensure_capacity(ComputePartition mode, int count, bool plan_only = false,
                                           const MemoryPartition* memory = nullptr,
                                           const std::unordered_set<std::string>* within = nullptr);
  // Move idle GPUs toward a strategy's distribution.
  std::vector<PartitionOp> rebalance(const std::string& strategy, bool plan_only = false);
  // Return idle partitioned GPUs with no slice in use back to SPX.
  std::vector<PartitionOp> reclaim_idle(bool plan_only = false);
  // Hysteresis variant driven by the housekeeping tick (reference: the MIG
  // controller's auto-rebalance, src/sharing/mig_controller.go:39-69): a
  // partitioned GPU returns to SPX only after it has stayed idle for
  // `min_idle_s`, so a burst of partition pods does not thrash modes.
  std::vector<PartitionOp> reclaim_idle_after(double now_s, double min_idle_s);

  // Empty under-used partitioned GPUs: move their preemptible inference
  // slices onto the fullest GPUs of the same mode (only when a donor can be
  // emptied completely), then switch the emptied GPU back to SPX.
  // move_in_ledger: true -> the ledger moves the slices itself (simulation /
  // direct API); false -> only plan: the controller evicts the pods (the
  // recreated pods are packed onto the fuller GPUs by best fit) and the
  // emptied donors are reclaimed on the next call.
  std::vector<PartitionMove> consolidate(double now_s, const ConsolidationPolicy& pol,
                                         bool move_in_ledger);
  int migrations() const;

  std::vector<PartitionOp> operations() const;
  PartitionMetrics metrics() const;
  void set_dry_run(bool d) { dry_run_ = d; }

 private:
  bool gpu_idle(const GpuDevice& g) const;
  PartitionOp execute(const std::string& node, const GpuDevice& g, ComputePartition to,
                      const std::string& reason, bool plan_only, const MemoryPartition* mem_to = nullptr);
  int free_slices(const ClusterTopology& c, ComputePartition mode, const MemoryPartition* memory = nullptr,
                  const std::unordered_set<std::string>* within = nullptr) const;

  std::shared_ptr<DiscoveryService> disc_;
  std::shared_ptr<Scheduler> sched_;
  bool dry_run_;
  mutable std::mutex mu_;
  std::map<std::string, PartitionStrategy> strategies_;
  std::map<std::string, double> idle_since_;  // partitioned GPU uuid -> first idle tick
  std::map<std::string, double> low_since_;   // partitioned GPU uuid -> first under-used tick
  std::map<std::string, double> migrated_at_; // workload uid -> last migration
  std::set<std::string> draining_;            // donors emptied by consolidation
  std::map<std::string, double> draining_since_;
  int migrations_ = 0;
  std::vector<PartitionOp> ops_;
  int next_op_ = 1;
};

// ---------------------------------------------------------------------------
// GPU sharing (reference src/sharing/mig_controller.go:545-857: MPS controller
// + GPUSharingManager).  ROCm has no MPS daemon; the MI355X-native equivalent
// of MPS's active-thread percentage is CU masking: each co-located client gets
// a DISJOINT range of compute units through HSA_CU_MASK, plus an HBM cap.
// The CU ranges live in the scheduler LEDGER (Scheduler::shared_), so a GPU
// with co-located clients is never handed out whole or partitioned, and a
// whole / partitioned GPU never takes a client — one lock, no second book.
// SharingManager is the policy + explicit-placement facade over it.
// ---------------------------------------------------------------------------
struct SharingRequest {
  std::string uid, ns = "default", team;
  WorkloadType type = WorkloadType::Inference;
  bool require_isolation = false;
  bool prefer_partition = false;
  SharingMethod method = SharingMethod::None;  // None: decided by policy
  ComputePartition partition_mode = ComputePartition::CPX;
  double cu_percent = 0.0;   // 0: scheduler default (one XCD)
  double memory_gb = 0.0;
  std::string node, gpu;  // target GPU for co-location / time-slicing
};

struct SharingAllocation {
  std::string uid, node, gpu;
  SharingMethod method = SharingMethod::None;
  int cu_begin = 0, cu_end = 0;  // [begin, end) for CoLocate
  double memory_gb = 0.0;
  int gpu_index = 0;
  std::map<std::string, std::string> env;  // injected into the pod
};
Json to_json(const SharingAllocation& a);

// Container environment of a share: device visibility, HSA_CU_MASK (device-
// local index 0 after HIP/ROCR_VISIBLE_DEVICES), memory cap as a fraction of
// the GPU's HBM (KGWE_GPU_MEMORY_FRACTION, applied by kgwe.launch /
// kgwe.utils.sharing through torch.cuda.set_per_process_memory_fraction).
std::map<std::string, std::string> share_env(SharingMethod m, int gpu_index, int cu_begin, int cu_end,
                                             double memory_gb, double gpu_memory_gb);

struct SharingPolicy {
  std::map<WorkloadType, SharingMethod> by_type;
};

class SharingManager {
 public:
  SharingManager(std::shared_ptr<DiscoveryService> disc, std::shared_ptr<Scheduler> sched,
                 SharingPolicy policy = {});
  SharingMethod decide(const SharingRequest& r) const;
  // Partition method returns method=Partition and leaves slice choice to the
  // scheduler; CoLocate / TimeSlice reserve a client slot on r.gpu in the
  // scheduler ledger.  error set on failure.
  SharingAllocation allocate(const SharingRequest& r, std::string* error);
  bool release(const std::string& uid);
  std::vector<SharingAllocation> allocations() const;
  int clients_on(const std::string& gpu) const;

 private:
  SharingAllocation from_alloc(const Allocation& a) const;
  std::shared_ptr<DiscoveryService> disc_;
  std::shared_ptr<Scheduler> sched_;
  SharingPolicy policy_;
};

}  // namespace kgwe
