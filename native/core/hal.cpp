#include "hal.h"

#include <array>

#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <vector>
#include <sstream>

#include <amd_smi/amdsmi.h>

namespace kgwe {

// ---------------------------------------------------------------------------
// Fixtures
// ---------------------------------------------------------------------------
Json make_mi355x_node_fixture(const std::string& name, int n_gpus, int numa_nodes,
                              const std::string& prefix) {
  Json node = Json::object();
  node["name"] = name;
  Json labels = Json::object();
  labels["kubernetes.io/hostname"] = name;
  labels["amd.com/gpu.product"] = "MI355X";
  labels["amd.com/gpu.family"] = "CDNA4";
  labels["amd.com/gpu.count"] = std::to_string(n_gpus);
  node["labels"] = labels;
  node["numa_nodes"] = numa_nodes;
  node["cpu_sockets"] = numa_nodes;
  Json gpus = Json::array();
  auto uuid = [&](int i) {
    char buf[96];
    std::snprintf(buf, sizeof buf, "GPU-%s%s-%02d", prefix.c_str(), name.c_str(), i);
    return std::string(buf);
  };
  for (int i = 0; i < n_gpus; ++i) {
    Json g = Json::object();
    g["uuid"] = uuid(i);
    g["index"] = i;
    g["numa_node"] = numa_nodes > 0 ? i * numa_nodes / n_gpus : 0;
    g["socket"] = numa_nodes > 0 ? i * numa_nodes / n_gpus : 0;
    Json pc = Json::object();
    char bdf[32];
    std::snprintf(bdf, sizeof bdf, "0000:%02x:00.0", 0x05 + i * 0x10);
    pc["bdf"] = bdf;
    pc["switch_id"] = "sw" + std::to_string(i / 2);
    g["pcie"] = pc;
    Json links = Json::array();
    for (int j = 0; j < n_gpus; ++j) {
      if (j == i) continue;
      Json l = Json::object();
      l["peer"] = uuid(j);
      l["type"] = "XGMI";
      l["hops"] = 1;
      l["rated_gbps"] = 153.6;
      links.push_back(l);
    }
    g["links"] = links;
    Json pj = Json::object();
    pj["compute"] = "SPX";
    pj["memory"] = "NPS1";
    g["partition"] = pj;
    gpus.push_back(g);
  }
  node["gpus"] = gpus;
  return node;
}

// ---------------------------------------------------------------------------
// FakeHal
// ---------------------------------------------------------------------------
FakeHal::FakeHal(const Json& node_fixture) : node_(node_from_json(node_fixture)) {}

std::unique_ptr<FakeHal> FakeHal::from_file(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open fixture " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return std::make_unique<FakeHal>(Json::parse(ss.str()));
}

NodeTopology FakeHal::discover(const std::string& node_name) {
  std::lock_guard<std::mutex> lk(mu_);
  NodeTopology n = node_;
  if (!node_name.empty() && node_name != n.name) {
    n.name = node_name;
    for (auto& g : n.gpus) g.node = node_name;
  }
  n.updated_ns = now_ns();
  return n;
}

void FakeHal::refresh_telemetry(NodeTopology& node) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& g : node.gpus) {
    const GpuDevice* src = node_.gpu(g.uuid);
    if (!src) continue;
    g.util = src->util;
    g.memory_used_gb = src->memory_used_gb;
    g.health = src->health;
    g.links = src->links;
    g.partition = src->partition;
  }
  node.updated_ns = now_ns();
}

std::string FakeHal::set_compute_partition(const std::string& gpu_uuid, ComputePartition mode) {
  std::lock_guard<std::mutex> lk(mu_);
  GpuDevice* g = node_.gpu(gpu_uuid);
  if (!g) return "unknown gpu " + gpu_uuid;
  for (const auto& pi : g->partition.instances)
    if (pi.in_use) return "gpu busy: partition " + pi.id + " in use by " + pi.owner;
  if (mode == ComputePartition::TPX) return "TPX not supported on MI355X (8 XCDs)";
  apply_compute_partition(*g, mode);
  ++switches_;
  return "";
}

void apply_compute_partition(GpuDevice& g, ComputePartition mode) {
  g.partition.compute = mode;
  g.partition.instances.clear();
  const int np = partition_count(mode);
  for (int i = 0; i < np; ++i) {
    PartitionInstance pi;
    pi.index = i;
    pi.id = g.uuid + "/p" + std::to_string(i);
    pi.cu_count = g.cu_count / np;
    pi.memory_gb = g.memory_total_gb / np;
    g.partition.instances.push_back(pi);
  }
}

std::string FakeHal::set_memory_partition(const std::string& gpu_uuid, MemoryPartition mode) {
  std::lock_guard<std::mutex> lk(mu_);
  GpuDevice* g = node_.gpu(gpu_uuid);
  if (!g) return "unknown gpu " + gpu_uuid;
  if (mode == MemoryPartition::NPS4 || mode == MemoryPartition::NPS8)
    return std::string(to_string(mode)) + " not supported on MI355X";
  g->partition.memory = mode;
  ++switches_;
  return "";
}

void FakeHal::set_link_up(const std::string& a, const std::string& b, bool up) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& g : node_.gpus) {
    if (g.uuid != a && g.uuid != b) continue;
    for (auto& l : g.links)
      if (l.peer_uuid == (g.uuid == a ? b : a)) l.up = up;
  }
}

void FakeHal::set_health(const std::string& gpu, HealthStatus s, const std::string& reason) {
  std::lock_guard<std::mutex> lk(mu_);
  GpuDevice* g = node_.gpu(gpu);
  if (!g) return;
  g->health.status = s;
  g->health.pinned = true;
  g->health.reasons.clear();
  if (!reason.empty()) g->health.reasons.push_back(reason);
}

void FakeHal::set_health_signals(const std::string& gpu, const Json& j) {
  std::lock_guard<std::mutex> lk(mu_);
  GpuDevice* g = node_.gpu(gpu);
  if (!g) return;
  Health& h = g->health;
  h.ecc_correctable = j.get("ecc_correctable").as_int(h.ecc_correctable);
  h.ecc_uncorrectable = j.get("ecc_uncorrectable").as_int(h.ecc_uncorrectable);
  h.ecc_deferred = j.get("ecc_deferred").as_int(h.ecc_deferred);
  h.xgmi_errors = static_cast<int>(j.get("xgmi_errors").as_int(h.xgmi_errors));
  h.xgmi_links_down = static_cast<int>(j.get("xgmi_links_down").as_int(h.xgmi_links_down));
  h.retired_pages = j.get("retired_pages").as_int(h.retired_pages);
  h.pending_retired_pages = j.get("pending_retired_pages").as_int(h.pending_retired_pages);
  h.cper_fatal = j.get("cper_fatal").as_int(h.cper_fatal);
  h.cper_uncorrected = j.get("cper_uncorrected").as_int(h.cper_uncorrected);
  h.cper_corrected = j.get("cper_corrected").as_int(h.cper_corrected);
  if (j.get("throttle").is_array()) {
    h.throttle_reasons.clear();
    for (const auto& t : j.get("throttle").items()) h.throttle_reasons.push_back(t.str());
  }
  h.pinned = false;
  int down = 0;
  for (const auto& l : g->links) down += !l.up;
  apply_health_policy(h, down);
}

void FakeHal::set_util(const std::string& gpu, double gfx, double mem_used_gb) {
  std::lock_guard<std::mutex> lk(mu_);
  GpuDevice* g = node_.gpu(gpu);
  if (!g) return;
  g->util.gfx_activity = gfx;
  g->memory_used_gb = mem_used_gb;
  g->util.memory_used_pct = 100.0 * mem_used_gb / g->memory_total_gb;
}

void FakeHal::set_measured_link(const std::string& a, const std::string& b, double gbps) {
  std::lock_guard<std::mutex> lk(mu_);
  GpuDevice* g = node_.gpu(a);
  if (!g) return;
  for (auto& l : g->links)
    if (l.peer_uuid == b) l.measured_gbps = gbps;
}

Json FakeHal::fixture() const {
  std::lock_guard<std::mutex> lk(mu_);
  return to_json(node_);
}

// ---------------------------------------------------------------------------
// AmdSmiHal — libamd_smi resolved with dlopen/dlsym
// ---------------------------------------------------------------------------
struct AmdSmiHal::Impl {
  void* so = nullptr;
#define KGWE_SMI_FN(name) decltype(&::name) name = nullptr;
  KGWE_SMI_FN(amdsmi_init)
  KGWE_SMI_FN(amdsmi_shut_down)
  KGWE_SMI_FN(amdsmi_get_socket_handles)
  KGWE_SMI_FN(amdsmi_get_processor_handles)
  KGWE_SMI_FN(amdsmi_get_gpu_device_bdf)
  KGWE_SMI_FN(amdsmi_get_gpu_device_uuid)
  KGWE_SMI_FN(amdsmi_topo_get_link_type)
  KGWE_SMI_FN(amdsmi_topo_get_numa_node_number)
  KGWE_SMI_FN(amdsmi_get_minmax_bandwidth_between_processors)
  KGWE_SMI_FN(amdsmi_get_gpu_activity)
  KGWE_SMI_FN(amdsmi_get_gpu_vram_usage)
  KGWE_SMI_FN(amdsmi_get_gpu_total_ecc_count)
  KGWE_SMI_FN(amdsmi_get_gpu_compute_partition)
  KGWE_SMI_FN(amdsmi_set_gpu_compute_partition)
  KGWE_SMI_FN(amdsmi_get_gpu_memory_partition)
  KGWE_SMI_FN(amdsmi_set_gpu_memory_partition)
  KGWE_SMI_FN(amdsmi_get_temp_metric)
  KGWE_SMI_FN(amdsmi_get_power_info)
  // optional (older libamd_smi builds may lack them): resolved without failing
  KGWE_SMI_FN(amdsmi_gpu_xgmi_error_status)
  KGWE_SMI_FN(amdsmi_get_gpu_xgmi_link_status)
  KGWE_SMI_FN(amdsmi_get_gpu_bad_page_info)
  KGWE_SMI_FN(amdsmi_get_violation_status)
  KGWE_SMI_FN(amdsmi_get_gpu_cper_entries)
#undef KGWE_SMI_FN
  std::vector<amdsmi_processor_handle> handles;
  std::vector<std::string> uuids;
  // CPER: per-GPU read cursor and cumulative counts by severity (the driver
  // keeps a ring of records; the cursor walks it once).
  std::vector<uint64_t> cper_cursor;
  std::vector<std::array<int64_t, 3>> cper_counts;
  std::vector<uint8_t> cper_primed;  // first read only advances the cursor past history
};

AmdSmiHal::AmdSmiHal() : impl_(new Impl) {
  const char* names[] = {"libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so"};
  for (const char* n : names) {
    impl_->so = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (impl_->so) break;
  }
  if (!impl_->so) {
    err_ = "libamd_smi not found";
    return;
  }
#define KGWE_SMI_SYM(name)                                                      \
  impl_->name = reinterpret_cast<decltype(impl_->name)>(dlsym(impl_->so, #name)); \
  if (!impl_->name) {                                                            \
    err_ = "missing symbol " #name;                                              \
    return;                                                                      \
  }
  KGWE_SMI_SYM(amdsmi_init)
  KGWE_SMI_SYM(amdsmi_shut_down)
  KGWE_SMI_SYM(amdsmi_get_socket_handles)
  KGWE_SMI_SYM(amdsmi_get_processor_handles)
  KGWE_SMI_SYM(amdsmi_get_gpu_device_bdf)
  KGWE_SMI_SYM(amdsmi_get_gpu_device_uuid)
  KGWE_SMI_SYM(amdsmi_topo_get_link_type)
  KGWE_SMI_SYM(amdsmi_topo_get_numa_node_number)
  KGWE_SMI_SYM(amdsmi_get_minmax_bandwidth_between_processors)
  KGWE_SMI_SYM(amdsmi_get_gpu_activity)
  KGWE_SMI_SYM(amdsmi_get_gpu_vram_usage)
  KGWE_SMI_SYM(amdsmi_get_gpu_total_ecc_count)
  KGWE_SMI_SYM(amdsmi_get_gpu_compute_partition)
  KGWE_SMI_SYM(amdsmi_set_gpu_compute_partition)
  KGWE_SMI_SYM(amdsmi_get_gpu_memory_partition)
  KGWE_SMI_SYM(amdsmi_set_gpu_memory_partition)
  KGWE_SMI_SYM(amdsmi_get_temp_metric)
  KGWE_SMI_SYM(amdsmi_get_power_info)
#undef KGWE_SMI_SYM
#define KGWE_SMI_OPT(name) \
  impl_->name = reinterpret_cast<decltype(impl_->name)>(dlsym(impl_->so, #name));
  KGWE_SMI_OPT(amdsmi_gpu_xgmi_error_status)
  KGWE_SMI_OPT(amdsmi_get_gpu_xgmi_link_status)
  KGWE_SMI_OPT(amdsmi_get_gpu_bad_page_info)
  KGWE_SMI_OPT(amdsmi_get_violation_status)
  KGWE_SMI_OPT(amdsmi_get_gpu_cper_entries)
#undef KGWE_SMI_OPT
  if (impl_->amdsmi_init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) {
    err_ = "amdsmi_init failed (no amdgpu driver?)";
    return;
  }
  uint32_t nsock = 0;
  if (impl_->amdsmi_get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS) {
    err_ = "amdsmi_get_socket_handles failed";
    return;
  }
  std::vector<amdsmi_socket_handle> socks(nsock);
  impl_->amdsmi_get_socket_handles(&nsock, socks.data());
  for (auto s : socks) {
    uint32_t np = 0;
    if (impl_->amdsmi_get_processor_handles(s, &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> ph(np);
    impl_->amdsmi_get_processor_handles(s, &np, ph.data());
    for (auto h : ph) impl_->handles.push_back(h);
  }
  for (size_t i = 0; i < impl_->handles.size(); ++i) {
    char buf[128] = {0};
    unsigned int len = sizeof buf;
    std::string u;
    if (impl_->amdsmi_get_gpu_device_uuid(impl_->handles[i], &len, buf) == AMDSMI_STATUS_SUCCESS)
      u = buf;
    if (u.empty()) u = "GPU-amdsmi-" + std::to_string(i);
    impl_->uuids.push_back(u);
  }
  impl_->cper_cursor.assign(impl_->handles.size(), 0);
  impl_->cper_counts.assign(impl_->handles.size(), {0, 0, 0});
  impl_->cper_primed.assign(impl_->handles.size(), 0);
  ok_ = true;
}

AmdSmiHal::~AmdSmiHal() {
  if (ok_ && impl_->amdsmi_shut_down) impl_->amdsmi_shut_down();
  if (impl_->so) dlclose(impl_->so);
}

NodeTopology AmdSmiHal::discover(const std::string& node_name) {
  NodeTopology n;
  n.name = node_name;
  if (!ok_) return n;
  auto& I = *impl_;
  int max_numa = 0;
  for (size_t i = 0; i < I.handles.size(); ++i) {
    GpuDevice g;
    g.uuid = I.uuids[i];
    g.index = static_cast<int>(i);
    g.node = node_name;
    amdsmi_bdf_t bdf;
    std::memset(&bdf, 0, sizeof bdf);
    if (I.amdsmi_get_gpu_device_bdf(I.handles[i], &bdf) == AMDSMI_STATUS_SUCCESS) {
      char b[32];
      std::snprintf(b, sizeof b, "%04x:%02x:%02x.%x", static_cast<unsigned>(bdf.domain_number),
                    static_cast<unsigned>(bdf.bus_number), static_cast<unsigned>(bdf.device_number),
                    static_cast<unsigned>(bdf.function_number));
      g.pcie.bdf = b;
    }
    uint32_t numa = 0;
    if (I.amdsmi_topo_get_numa_node_number(I.handles[i], &numa) == AMDSMI_STATUS_SUCCESS) {
      g.numa_node = static_cast<int>(numa);
      g.socket = g.numa_node;
      if (g.numa_node > max_numa) max_numa = g.numa_node;
    }
    char part[64] = {0};
    if (I.amdsmi_get_gpu_compute_partition(I.handles[i], part, sizeof part) == AMDSMI_STATUS_SUCCESS)
      g.partition.compute = compute_partition_from(part);
    char mpart[64] = {0};
    if (I.amdsmi_get_gpu_memory_partition(I.handles[i], mpart, sizeof mpart) == AMDSMI_STATUS_SUCCESS)
      g.partition.memory = memory_partition_from(mpart);
    const int np = partition_count(g.partition.compute);
    for (int p = 0; p < np; ++p) {
      PartitionInstance pi;
      pi.index = p;
      pi.id = g.uuid + "/p" + std::to_string(p);
      pi.cu_count = g.cu_count / np;
      pi.memory_gb = g.memory_total_gb / np;
      g.partition.instances.push_back(pi);
    }
    for (size_t j = 0; j < I.handles.size(); ++j) {
      if (j == i) continue;
      XgmiLink l;
      l.peer_uuid = I.uuids[j];
      uint64_t hops = 0;
      amdsmi_link_type_t t;
      if (I.amdsmi_topo_get_link_type(I.handles[i], I.handles[j], &hops, &t) == AMDSMI_STATUS_SUCCESS) {
        l.type = t == AMDSMI_LINK_TYPE_XGMI ? LinkType::XGMI
                 : t == AMDSMI_LINK_TYPE_PCIE ? LinkType::PCIE
                                              : LinkType::Unknown;
        l.hops = static_cast<int>(hops);
      }
      uint64_t mn = 0, mx = 0;
      if (I.amdsmi_get_minmax_bandwidth_between_processors(I.handles[i], I.handles[j], &mn, &mx) ==
              AMDSMI_STATUS_SUCCESS &&
          mx > 0)
        l.rated_gbps = static_cast<double>(mx) / 1000.0;  // MB/s -> GB/s
      g.links.push_back(l);
    }
    n.gpus.push_back(g);
  }
  n.numa_nodes = max_numa + 1;
  n.cpu_sockets = n.numa_nodes;
  refresh_telemetry(n);
  bool full = n.gpus.size() > 1;
  for (const auto& a : n.gpus)
    for (const auto& l : a.links)
      if (l.type != LinkType::XGMI || !l.up) full = false;
  n.xgmi_fully_connected = full;
  return n;
}

void AmdSmiHal::refresh_telemetry(NodeTopology& n) {
  if (!ok_) return;
  auto& I = *impl_;
  for (auto& g : n.gpus) {
    if (g.index < 0 || g.index >= static_cast<int>(I.handles.size())) continue;
    auto h = I.handles[g.index];
    amdsmi_engine_usage_t eu;
    std::memset(&eu, 0, sizeof eu);
    if (I.amdsmi_get_gpu_activity(h, &eu) == AMDSMI_STATUS_SUCCESS) {
      g.util.gfx_activity = eu.gfx_activity;
      g.util.umc_activity = eu.umc_activity;
    }
    amdsmi_vram_usage_t vu;
    std::memset(&vu, 0, sizeof vu);
    if (I.amdsmi_get_gpu_vram_usage(h, &vu) == AMDSMI_STATUS_SUCCESS) {
      if (vu.vram_total > 0) g.memory_total_gb = vu.vram_total / 1024.0;
      g.memory_used_gb = vu.vram_used / 1024.0;
      g.util.memory_used_pct = vu.vram_total ? 100.0 * vu.vram_used / vu.vram_total : 0.0;
    }
    amdsmi_error_count_t ec;
    std::memset(&ec, 0, sizeof ec);
    if (I.amdsmi_get_gpu_total_ecc_count(h, &ec) == AMDSMI_STATUS_SUCCESS) {
      // Seen on MI355X hosts without RAS access (containers): SUCCESS with
      // the struct left as-is, i.e. uninitialised stack words (~1e14).  Any
      // count beyond 2^40 is not a real error count: ignore the reading
      // instead of declaring the GPU Unhealthy.
      constexpr uint64_t kImplausible = 1ull << 40;
      if (ec.correctable_count < kImplausible && ec.uncorrectable_count < kImplausible &&
          ec.deferred_count < kImplausible) {
        g.health.ecc_correctable = static_cast<int64_t>(ec.correctable_count);
        g.health.ecc_uncorrectable = static_cast<int64_t>(ec.uncorrectable_count);
        g.health.ecc_deferred = static_cast<int64_t>(ec.deferred_count);
      }
    }
    int64_t temp = 0;
    if (I.amdsmi_get_temp_metric(h, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &temp) ==
        AMDSMI_STATUS_SUCCESS)
      g.util.temperature_c = static_cast<double>(temp);
    amdsmi_power_info_t pw;
    std::memset(&pw, 0, sizeof pw);
    if (I.amdsmi_get_power_info(h, &pw) == AMDSMI_STATUS_SUCCESS)
      g.util.power_w = static_cast<double>(pw.current_socket_power ? pw.current_socket_power
                                                                   : pw.average_socket_power);
    if (I.amdsmi_gpu_xgmi_error_status) {
      amdsmi_xgmi_status_t xs;
      if (I.amdsmi_gpu_xgmi_error_status(h, &xs) == AMDSMI_STATUS_SUCCESS)
        g.health.xgmi_errors = xs == AMDSMI_XGMI_STATUS_NO_ERRORS ? 0
                               : xs == AMDSMI_XGMI_STATUS_ERROR   ? 1
                                                                  : 2;
    }
    if (I.amdsmi_get_gpu_xgmi_link_status) {
      amdsmi_xgmi_link_status_t ls;
      std::memset(&ls, 0, sizeof ls);
      if (I.amdsmi_get_gpu_xgmi_link_status(h, &ls) == AMDSMI_STATUS_SUCCESS) {
        int down = 0;
        for (uint32_t k = 0; k < ls.total_links && k < AMDSMI_MAX_NUM_XGMI_LINKS; ++k)
          down += ls.status[k] == AMDSMI_XGMI_LINK_DOWN;
        g.health.xgmi_links_down = down;
      }
    }
    if (I.amdsmi_get_gpu_bad_page_info) {
      uint32_t np = 0;
      if (I.amdsmi_get_gpu_bad_page_info(h, &np, nullptr) == AMDSMI_STATUS_SUCCESS) {
        std::vector<amdsmi_retired_page_record_t> rec(np);
        int64_t retired = 0, pending = 0;
        if (np && I.amdsmi_get_gpu_bad_page_info(h, &np, rec.data()) == AMDSMI_STATUS_SUCCESS)
          for (uint32_t k = 0; k < np; ++k) {
            retired += rec[k].status == AMDSMI_MEM_PAGE_STATUS_RESERVED;
            pending += rec[k].status == AMDSMI_MEM_PAGE_STATUS_PENDING;
          }
        g.health.retired_pages = retired;
        g.health.pending_retired_pages = pending;
      }
    }
    if (I.amdsmi_get_violation_status) {
      // ~100 KB (per-XCP x XCC arrays): heap, not the agent thread's stack.
      auto vs = std::make_unique<amdsmi_violation_status_t>();
      std::memset(vs.get(), 0, sizeof *vs);
      g.health.throttle_reasons.clear();
      if (I.amdsmi_get_violation_status(h, vs.get()) == AMDSMI_STATUS_SUCCESS) {
        auto on = [](uint8_t v) { return v == 1; };  // 0xff = unsupported
        if (on(vs->active_prochot_thrm)) g.health.throttle_reasons.push_back("prochot");
        if (on(vs->active_ppt_pwr)) g.health.throttle_reasons.push_back("ppt_power");
        if (on(vs->active_socket_thrm)) g.health.throttle_reasons.push_back("socket_thermal");
        if (on(vs->active_vr_thrm)) g.health.throttle_reasons.push_back("vr_thermal");
        if (on(vs->active_hbm_thrm)) g.health.throttle_reasons.push_back("hbm_thermal");
      }
    }
    if (I.amdsmi_get_gpu_cper_entries) {
      // New records since the last read (bounded: at most 8 x 64 per refresh).
      constexpr uint32_t kMask = (1u << AMDSMI_CPER_SEV_NON_FATAL_UNCORRECTED) | (1u << AMDSMI_CPER_SEV_FATAL) |
                                 (1u << AMDSMI_CPER_SEV_NON_FATAL_CORRECTED);
      std::vector<char> data(64 * 1024);
      std::vector<amdsmi_cper_hdr_t*> hdrs(64, nullptr);
      auto& counts = I.cper_counts[g.index];
      // Records cached before this agent started (an error the GPU was reset
      // from, possibly days ago) are skipped: the first read only moves the
      // cursor to the end of the ring.
      const bool count_them = I.cper_primed[g.index] != 0;
      for (int round = 0; round < (count_them ? 8 : 1024); ++round) {
        uint64_t size = data.size(), count = hdrs.size();
        const amdsmi_status_t st = I.amdsmi_get_gpu_cper_entries(h, kMask, data.data(), &size, hdrs.data(), &count,
                                                                 &I.cper_cursor[g.index]);
        if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_MORE_DATA) break;
        for (uint64_t k = 0; k < count && k < hdrs.size(); ++k) {
          if (!hdrs[k]) continue;
          const int sev = static_cast<int>(hdrs[k]->error_severity);
          if (count_them && sev >= 0 && sev < 3) ++counts[sev];
        }
        if (st != AMDSMI_STATUS_MORE_DATA || count == 0) break;
      }
      I.cper_primed[g.index] = 1;
      g.health.cper_uncorrected = counts[AMDSMI_CPER_SEV_NON_FATAL_UNCORRECTED];
      g.health.cper_fatal = counts[AMDSMI_CPER_SEV_FATAL];
      g.health.cper_corrected = counts[AMDSMI_CPER_SEV_NON_FATAL_CORRECTED];
    }
    if (!g.health.pinned) {
      int down = 0;
      for (const auto& l : g.links) down += !l.up;
      apply_health_policy(g.health, down);
    }
  }
  n.updated_ns = now_ns();
}

std::string AmdSmiHal::set_compute_partition(const std::string& gpu_uuid, ComputePartition mode) {
  if (!ok_) return err_;
  auto& I = *impl_;
  for (size_t i = 0; i < I.uuids.size(); ++i) {
    if (I.uuids[i] != gpu_uuid) continue;
    amdsmi_compute_partition_type_t t = AMDSMI_COMPUTE_PARTITION_SPX;
    switch (mode) {
      case ComputePartition::SPX: t = AMDSMI_COMPUTE_PARTITION_SPX; break;
      case ComputePartition::DPX: t = AMDSMI_COMPUTE_PARTITION_DPX; break;
      case ComputePartition::TPX: t = AMDSMI_COMPUTE_PARTITION_TPX; break;
      case ComputePartition::QPX: t = AMDSMI_COMPUTE_PARTITION_QPX; break;
      case ComputePartition::CPX: t = AMDSMI_COMPUTE_PARTITION_CPX; break;
    }
    amdsmi_status_t st = I.amdsmi_set_gpu_compute_partition(I.handles[i], t);
    return st == AMDSMI_STATUS_SUCCESS ? "" : "amdsmi_set_gpu_compute_partition status " +
                                                   std::to_string(static_cast<int>(st));
  }
  return "unknown gpu " + gpu_uuid;
}

std::string AmdSmiHal::set_memory_partition(const std::string& gpu_uuid, MemoryPartition mode) {
  if (!ok_) return err_;
  auto& I = *impl_;
  for (size_t i = 0; i < I.uuids.size(); ++i) {
    if (I.uuids[i] != gpu_uuid) continue;
    amdsmi_memory_partition_type_t t = AMDSMI_MEMORY_PARTITION_NPS1;
    if (mode == MemoryPartition::NPS2) t = AMDSMI_MEMORY_PARTITION_NPS2;
    if (mode == MemoryPartition::NPS4) t = AMDSMI_MEMORY_PARTITION_NPS4;
    if (mode == MemoryPartition::NPS8) t = AMDSMI_MEMORY_PARTITION_NPS8;
    amdsmi_status_t st = I.amdsmi_set_gpu_memory_partition(I.handles[i], t);
    return st == AMDSMI_STATUS_SUCCESS ? "" : "amdsmi_set_gpu_memory_partition status " +
                                                   std::to_string(static_cast<int>(st));
  }
  return "unknown gpu " + gpu_uuid;
}

}  // namespace kgwe
