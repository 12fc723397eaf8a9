// Hardware abstraction layer (L0): the device side of topology discovery.
//
// Replaces the reference's NVMLClient interface, which had ZERO
// implementations (src/discovery/discovery.go:35-71).  Two backends:
//   * AmdSmiHal — libamd_smi (dlopen'ed at run time, so the core also loads
//     on hosts without the driver): enumeration, xGMI link type / hops /
//     min-max bandwidth, NUMA affinity, gfx/umc activity, VRAM, ECC, compute
//     and memory partition get/set.
//   * FakeHal — JSON fixtures (8xMI355X full mesh, degraded link, CPX GPU,
//     unhealthy GPU, 2-socket NUMA...) with fault injection for tests.
#pragma once
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "model.h"

namespace kgwe {

class Hal {
 public:
  virtual ~Hal() = default;
  virtual std::string backend() const = 0;
  // Full node discovery: devices, links, partitions, telemetry, health.
  virtual NodeTopology discover(const std::string& node_name) = 0;
  // Cheap telemetry refresh (utilisation / memory / health) of known devices.
  virtual void refresh_telemetry(NodeTopology& node) = 0;
  // Partition actuation; returns "" on success, else an error string.
  virtual std::string set_compute_partition(const std::string& gpu_uuid,
                                            ComputePartition mode) = 0;
  virtual std::string set_memory_partition(const std::string& gpu_uuid,
                                           MemoryPartition mode) = 0;
};

// Re-slice one GPU's partition instances for a new compute mode (one slice
// per partition, CUs and HBM split evenly) — what a successful switch does to
// the device model, whoever actuated it.
void apply_compute_partition(GpuDevice& g, ComputePartition mode);

class FakeHal : public Hal {
 public:
  explicit FakeHal(const Json& node_fixture);
  static std::unique_ptr<FakeHal> from_file(const std::string& path);
  std::string backend() const override { return "fake"; }
  NodeTopology discover(const std::string& node_name) override;
  void refresh_telemetry(NodeTopology& node) override;
  std::string set_compute_partition(const std::string& gpu_uuid, ComputePartition mode) override;
  std::string set_memory_partition(const std::string& gpu_uuid, MemoryPartition mode) override;

  // Fault / state injection (tests, chaos drills).
  void set_link_up(const std::string& a, const std::string& b, bool up);
  void set_health(const std::string& gpu, HealthStatus s, const std::string& reason);  // pinned
  // Raw RAS / xGMI / throttle signals (keys of the fixture "health" object);
  // status is re-derived by apply_health_policy.  Chaos drills: ECC storms,
  // page retirement, xGMI error bursts.
  void set_health_signals(const std::string& gpu, const Json& signals);
  void set_util(const std::string& gpu, double gfx_activity, double mem_used_gb);
  void set_measured_link(const std::string& a, const std::string& b, double gbps);
  Json fixture() const;
  int partition_switches() const { return switches_; }

 private:
  mutable std::mutex mu_;
  NodeTopology node_;
  int switches_ = 0;
};

// Builders for the standard fixtures (also written to tests/fixtures/*.json).
Json make_mi355x_node_fixture(const std::string& name, int n_gpus = 8, int numa_nodes = 2,
                              const std::string& prefix = "");

class AmdSmiHal : public Hal {
 public:
  AmdSmiHal();
  ~AmdSmiHal() override;
  bool ok() const { return ok_; }
  const std::string& error() const { return err_; }
  std::string backend() const override { return "amdsmi"; }
  NodeTopology discover(const std::string& node_name) override;
  void refresh_telemetry(NodeTopology& node) override;
  std::string set_compute_partition(const std::string& gpu_uuid, ComputePartition mode) override;
  std::string set_memory_partition(const std::string& gpu_uuid, MemoryPartition mode) override;

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
  bool ok_ = false;
  std::string err_;
};

}  // namespace kgwe
