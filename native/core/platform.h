// The kgwe control plane wired end to end, with the kube-scheduler EXTENDER
// wire contract handled natively (JSON in -> JSON out).
//
// Reference: the extender contract exists only as configuration
// (deploy/helm/kgwe/templates/scheduler-configmap.yaml:61-79: verbs filter /
// prioritize / bind, weight 100, nodeCacheCapable false, managed resources);
// no server, no glue and no constructor calls exist.  Here:
//   filter      ExtenderArgs          -> ExtenderFilterResult
//                 (+ budget admission, + partition auto-provisioning — the
//                  designed PreBind "KGWEMIGProvisioning" plugin)
//   prioritize  ExtenderArgs          -> HostPriorityList (0..10)
//   bind        ExtenderBindingArgs   -> ExtenderBindingResult + the placement
//                 (GPUs / slices, RCCL-over-xGMI rank env, CU masks) that the
//                 Python shell writes to the apiserver (Binding + annotations);
//                 starts cost metering (the designed PostBind
//                 "KGWECostTracking" plugin) and records metrics.
// The HTTP socket handling lives in the Python shell (kgwe/extender); every
// byte of request parsing, scoring and response building is here.
#pragma once
#include <atomic>
#include <memory>
#include <string>

#include "cost.h"
#include "discovery.h"
#include "metrics.h"
#include "partition.h"
#include "scheduler.h"

namespace kgwe {

struct PlatformConfig {
  SchedulerConfig sched;
  CostEngineConfig cost;
  bool partition_dry_run = false;
  bool auto_provision_partitions = true;
  // Idle partitioned GPUs go back to SPX after this many seconds (<0: never).
  double partition_reclaim_idle_s = 60.0;
  bool enforce_budgets = true;
  int master_port = 29500;
  std::string gpu_resource = "amd.com/gpu";
  // Node directory (a hostPath shared by the share pods of a node) where a
  // share group's leader puts its serving socket.
  std::string share_socket_dir = "/run/kgwe/share";
  ConsolidationPolicy consolidate;
};

// Pod (core/v1 JSON) -> workload request.  Sources, in order: annotation
// kgwe.amd.com/workload (a GPUWorkload spec), amd.com/gpu limits,
// amd.com/gpu-<mode> partition resources, kgwe.amd.com/* annotations,
// spec.priority / nodeSelector / tolerations / nodeAffinity.
WorkloadRequest workload_from_pod(const Json& pod, const std::string& gpu_resource = "amd.com/gpu");

// RCCL-over-xGMI rank environment for a placement.
std::map<std::string, std::string> rccl_env(const WorkloadRequest& w, const Decision& d,
                                            const NodeTopology& node, int master_port,
                                            const std::string& master_addr = "");

class Platform {
 public:
  explicit Platform(PlatformConfig cfg = {});

  std::shared_ptr<DiscoveryService> discovery() { return disc_; }
  std::shared_ptr<Scheduler> scheduler() { return sched_; }
  std::shared_ptr<PartitionController> partitions() { return part_; }
  std::shared_ptr<SharingManager> sharing() { return share_; }
  std::shared_ptr<CostEngine> cost() { return cost_; }
  std::shared_ptr<MetricRegistry> metrics() { return reg_; }

  // Extender verbs (bodies are JSON text).
  std::string filter(const std::string& body);
  std::string prioritize(const std::string& body);
  // ExtenderPreemptionArgs -> ExtenderPreemptionResult (nodeNameToMetaVictims):
  // the victims kube-scheduler should evict per node so the pod fits on
  // kgwe's terms (whole gangs, share clients, priorities, preemptible).
  std::string preempt(const std::string& body);
  // Returns {"result": ExtenderBindingResult, "placement": {...}}.
  std::string bind(const std::string& body, const std::string& pod_json = "");
  // bind() plus what a serving shell needs to act on the result without
  // re-parsing it.  `waiting`: the pod is a gang member whose GPUs are
  // reserved but whose gang is not complete yet (the scheduler framework's
  // Permit "Wait"); calling bind again once the gang is ready returns ok.
  struct BindOutcome {
    std::string json;   // what bind() returns
    bool ok = false;    // bound: placement is final
    bool waiting = false;
    bool unknown_pod = false;  // no filter call seen for this pod (and no pod_json)
    std::string uid, ns, name, node, gang, error;
  };
  BindOutcome bind_outcome(const std::string& body, const std::string& pod_json = "");

  // Direct API (controller / optimizer / tests).
  std::string schedule(const std::string& workload_json);
  std::string release(const std::string& uid, double now_s);
  void observe_pod_latency_ms(double ms);
  // Pod create -> bind latency (the KPI; reference docs/PRD.md:440), fed by
  // bind() itself from the pod's creation stamp or its first filter call.
  const LatencyHistogram& pod_latency() const { return pod_latency_; }
  // Pods seen by filter and not yet bound / released (kgwe_workload_queue_depth).
  size_t queue_depth() const;
  // Consolidating partition rebalance; JSON list of moves.  move_in_ledger:
  // see PartitionController::consolidate.  The moved workloads' cost records
  // keep running (same uid); pods must be restarted on their new slice.
  std::string consolidate_partitions(double now_s, bool move_in_ledger);

  // Periodic sweep: gang timeouts, cost samples from telemetry, gauges.
  void tick(double now_s);
  std::string expose_metrics();

  // Remember the pod object for a uid between filter and bind (the bind
  // request only carries name/namespace/uid/node).
  void remember_pod(const std::string& uid, const WorkloadRequest& w, double created_s = 0.0);

 private:
  std::string placement_json(const WorkloadRequest& w, const Decision& d);
  void refresh_gauges(double now_s);

  PlatformConfig cfg_;
  std::shared_ptr<DiscoveryService> disc_;
  std::shared_ptr<Scheduler> sched_;
  std::shared_ptr<PartitionController> part_;
  std::shared_ptr<SharingManager> share_;
  std::shared_ptr<CostEngine> cost_;
  std::shared_ptr<MetricRegistry> reg_;
  mutable std::mutex pods_mu_;
  std::map<std::string, WorkloadRequest> pods_;  // uid -> request (filter -> bind)
  std::map<std::string, std::string> name_to_uid_;
  // uid -> (monotonic first-seen ns, wall-clock creation stamp or 0) for
  // pods not yet bound: the latency origin and the queue.
  std::map<std::string, std::pair<int64_t, double>> pending_;
  // preempt(): victim uid -> (its gang's members on other nodes, plan time).
  std::map<std::string, std::pair<std::vector<std::string>, int64_t>> gang_peers_;
  LatencyHistogram pod_latency_;
  // tick() refreshes gauges at most at a 10 % duty cycle: at 10,000 GPUs a
  // refresh is ~0.5 s of CPU, and a scrape refreshes them anyway.
  std::atomic<int64_t> gauges_next_ns_{0};
  // Per-node gauge blocks of the last refresh, re-used while the node's
  // topology object is the same one (nothing about it changed).
  struct NodeGauges {
    const NodeTopology* topo = nullptr;
    int64_t updated_ns = 0;
    std::map<std::string, std::shared_ptr<const MetricRegistry::Block>> blocks;
  };
  std::mutex gauges_mu_;
  std::map<std::string, NodeGauges> node_gauges_;
};

}  // namespace kgwe
