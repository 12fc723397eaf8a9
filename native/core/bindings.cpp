// pybind11 module `_kgwe_core`: the C++ control plane exposed to the Python
// service shells (extender HTTP server, controller, node agent, optimizer).
// The boundary is JSON text both ways, so the shells never hold C++ objects
// beyond the Platform handle and the GIL is released for every hot call.
#include <pybind11/pybind11.h>
#include <pybind11/functional.h>
#include <pybind11/stl.h>

#include "cost.h"
#include "extender_scan.h"
#include "hal.h"
#include "histogram.h"
#include "http_client.h"
#include "http_server.h"
#include "platform.h"

namespace py = pybind11;
using namespace kgwe;

namespace {

PlatformConfig config_from_json(const std::string& s) {
  PlatformConfig c;
  if (s.empty()) return c;
  Json j = Json::parse(s);
  const Json& sc = j.get("scheduler");
  c.sched.topology_weight = static_cast<int>(sc.get("topologyWeight").as_int(c.sched.topology_weight));
  c.sched.resource_weight = static_cast<int>(sc.get("resourceWeight").as_int(c.sched.resource_weight));
  c.sched.balance_weight = static_cast<int>(sc.get("balanceWeight").as_int(c.sched.balance_weight));
  c.sched.enable_preemption = sc.get("enablePreemption").as_bool(c.sched.enable_preemption);
  c.sched.enable_gang = sc.get("enableGangScheduling").as_bool(c.sched.enable_gang);
  c.sched.gang_timeout_ms = static_cast<int>(sc.get("gangTimeoutMs").as_int(c.sched.gang_timeout_ms));
  c.sched.max_attempts = static_cast<int>(sc.get("maxSchedulingAttempts").as_int(c.sched.max_attempts));
  c.sched.mode = sc.get("scoring").str("xgmi") == "compat" ? ScoringMode::Compat : ScoringMode::Xgmi;
  c.sched.rated_link_gbps = sc.get("ratedLinkGBps").as_number(c.sched.rated_link_gbps);
  c.sched.pack = sc.get("placement").str("pack") != "spread";
  const Json& cc = j.get("cost");
  c.cost.journal_path = cc.get("journalPath").str();
  c.cost.journal_interval_s = cc.get("journalIntervalSeconds").as_number(c.cost.journal_interval_s);
  c.cost.enable_spot = cc.get("enableSpotOptimization").as_bool(true);
  c.cost.enable_rightsizing = cc.get("enableRightsizing").as_bool(true);
  c.partition_dry_run = j.get("partitionDryRun").as_bool(false);
  c.auto_provision_partitions = j.get("autoProvisionPartitions").as_bool(true);
  c.partition_reclaim_idle_s = j.get("partitionReclaimIdleSeconds").as_number(c.partition_reclaim_idle_s);
  c.enforce_budgets = j.get("enforceBudgets").as_bool(true);
  c.master_port = static_cast<int>(j.get("masterPort").as_int(29500));
  c.gpu_resource = j.get("gpuResource").str("amd.com/gpu");
  c.share_socket_dir = j.get("shareSocketDir").str(c.share_socket_dir);
  c.consolidate.below = j.get("partitionConsolidateBelow").as_number(c.consolidate.below);
  c.consolidate.after_s = j.get("partitionConsolidateAfterSeconds").as_number(c.consolidate.after_s);
  c.consolidate.cooldown_s = j.get("migrationCooldownSeconds").as_number(c.consolidate.cooldown_s);
  c.sched.max_share_clients = static_cast<int>(sc.get("maxShareClients").as_int(c.sched.max_share_clients));
  c.sched.max_group_clients = static_cast<int>(sc.get("maxGroupClients").as_int(c.sched.max_group_clients));
  c.sched.preemption_candidate_nodes =
      static_cast<int>(sc.get("preemptionCandidateNodes").as_int(c.sched.preemption_candidate_nodes));
  c.sched.preemption_wait_window_s = sc.get("preemptionWaitWindowSeconds").as_number(c.sched.preemption_wait_window_s);
  c.sched.preemption_max_wait_s = sc.get("preemptionMaxWaitSeconds").as_number(c.sched.preemption_max_wait_s);
  c.sched.preemption_urgent_priority =
      sc.get("preemptionUrgentPriority").as_int(c.sched.preemption_urgent_priority);
  c.sched.preemption_max_rate_percent =
      sc.get("preemptionMaxRatePercent").as_number(c.sched.preemption_max_rate_percent);
  c.sched.preemption_window_s = static_cast<int>(sc.get("preemptionWindowSeconds").as_int(c.sched.preemption_window_s));
  c.sched.preemption_burst = static_cast<int>(sc.get("preemptionBurst").as_int(c.sched.preemption_burst));
  c.sched.default_cu_percent = sc.get("defaultCuPercent").as_number(c.sched.default_cu_percent);
  return c;
}

template <class T>
std::string list_json(const std::vector<T>& v) {
  Json a = Json::array();
  for (const auto& x : v) a.push_back(to_json(x));
  return a.dump();
}

Json metrics_json(const SchedulerMetrics& m) {
  Json j = Json::object();
  j["attempts"] = m.attempts;
  j["scheduled"] = m.scheduled;
  j["failed"] = m.failed;
  j["topology_optimal"] = m.topology_optimal;
  j["preemptions"] = m.preemptions;
  j["preemptions_deferred_wait"] = m.preemptions_deferred_wait;
  j["preemptions_rate_limited"] = m.preemptions_rate_limited;
  j["releases"] = m.releases;
  j["gang_timeouts"] = m.gang_timeouts;
  j["avg_latency_ms"] = m.avg_latency_ms;
  j["p50_ms"] = m.p50_ms;
  j["p90_ms"] = m.p90_ms;
  j["p99_ms"] = m.p99_ms;
  j["max_ms"] = m.max_ms;
  j["active_allocations"] = static_cast<int64_t>(m.active_allocations);
  j["allocated_gpus"] = static_cast<int64_t>(m.allocated_gpus);
  j["allocated_partitions"] = static_cast<int64_t>(m.allocated_partitions);
  j["shared_gpus"] = static_cast<int64_t>(m.shared_gpus);
  j["share_clients"] = static_cast<int64_t>(m.share_clients);
  return j;
}

struct PyPlatform {
  std::shared_ptr<Platform> p;
  std::map<std::string, std::shared_ptr<FakeHal>> fakes;
  std::mutex mu;

  explicit PyPlatform(const std::string& cfg) : p(std::make_shared<Platform>(config_from_json(cfg))) {}

  FakeHal& fake(const std::string& node) {
    std::lock_guard<std::mutex> lk(mu);
    auto it = fakes.find(node);
    if (it == fakes.end()) throw std::runtime_error("no fake HAL for node " + node);
    return *it->second;
  }
};

// The native extender server with its Python-side hooks.  Hooks run on the
// server's worker threads: each takes the GIL for the call only.
struct PyHttpServer {
  std::shared_ptr<ExtenderHttpServer> srv;
  // Hook objects are shared with the server's std::functions and must die
  // under the GIL.
  struct Hook {
    py::object fn;
    ~Hook() {
      py::gil_scoped_acquire g;
      fn = py::object();
    }
  };

  PyHttpServer(PyPlatform& p, const std::string& host, int port, const std::string& prefix, int workers,
               int gang_hold_ms) {
    ExtenderHttpServer::Options o;
    o.host = host;
    o.port = port;
    o.prefix = prefix;
    o.workers = workers;
    o.gang_hold_ms = gang_hold_ms;
    srv = std::make_shared<ExtenderHttpServer>(p.p, o);
  }

  void set_bind_sink(py::object fn) {
    auto h = std::make_shared<Hook>();
    h->fn = std::move(fn);
    srv->set_bind_sink([h](const std::string& args, const std::string& result) {
      py::gil_scoped_acquire g;
      try {
        return h->fn(py::bytes(args), py::bytes(result)).cast<std::string>();
      } catch (py::error_already_set& e) {
        std::string what = e.what();
        e.restore();
        PyErr_Clear();
        return what.empty() ? std::string("bind sink failed") : what;
      }
    });
  }

  void set_pod_lookup(py::object fn) {
    auto h = std::make_shared<Hook>();
    h->fn = std::move(fn);
    srv->set_pod_lookup([h](const std::string& ns, const std::string& name) {
      py::gil_scoped_acquire g;
      try {
        return h->fn(ns, name).cast<std::string>();
      } catch (py::error_already_set& e) {
        e.restore();
        PyErr_Clear();
        return std::string();
      }
    });
  }

  void set_fallback(py::object fn) {
    auto h = std::make_shared<Hook>();
    h->fn = std::move(fn);
    srv->set_fallback([h](const HttpRequest& rq) {
      HttpResponse r;
      py::gil_scoped_acquire g;
      try {
        py::tuple t = h->fn(rq.method, rq.path, py::bytes(rq.body), rq.authorization).cast<py::tuple>();
        r.code = t[0].cast<int>();
        r.body = t[1].cast<std::string>();
        if (t.size() > 2) r.ctype = t[2].cast<std::string>();
      } catch (py::error_already_set& e) {
        r.code = 500;
        r.body = std::string("{\"error\":\"") + json_escape(e.what()) + "\"}";
        e.restore();
        PyErr_Clear();
      }
      return r;
    });
  }
};

}  // namespace

PYBIND11_MODULE(_kgwe_core, m) {
  m.doc() = "kgwe MI355X control-plane core (C++17)";

  m.def("make_fixture", [](const std::string& name, int n, int numa, const std::string& prefix) {
    return make_mi355x_node_fixture(name, n, numa, prefix).dump();
  }, py::arg("name"), py::arg("n_gpus") = 8, py::arg("numa_nodes") = 2, py::arg("prefix") = "");

  m.def("amdsmi_discover", [](const std::string& node) {
    AmdSmiHal h;
    Json j = Json::object();
    j["ok"] = h.ok();
    j["error"] = h.error();
    if (h.ok()) j["node"] = to_json(h.discover(node));
    return j.dump();
  }, py::arg("node") = "local", py::call_guard<py::gil_scoped_release>());

  m.def("amdsmi_set_partition", [](const std::string& gpu, const std::string& compute,
                                   const std::string& memory) {
    AmdSmiHal h;
    if (!h.ok()) return std::string("amd-smi unavailable: ") + h.error();
    std::string err;
    if (!memory.empty()) err = h.set_memory_partition(gpu, memory_partition_from(memory));
    if (err.empty() && !compute.empty()) err = h.set_compute_partition(gpu, compute_partition_from(compute));
    return err;
  }, py::arg("gpu"), py::arg("compute"), py::arg("memory") = "",
     py::call_guard<py::gil_scoped_release>());

  m.def("workload_from_pod", [](const std::string& pod) {
    return to_json(workload_from_pod(Json::parse(pod))).dump();
  });
  m.def("workload_normalize", [](const std::string& wl) {
    return to_json(workload_from_json(Json::parse(wl))).dump();
  });
  m.def("json_roundtrip", [](const std::string& s) { return Json::parse(s).dump(); });
  m.def("scan_node_names", [](const std::string& s) {
    std::vector<std::string> names;
    if (!scan_node_names(s, &names)) throw std::runtime_error("not an ExtenderArgs / FilterResult document");
    return names;
  }, py::call_guard<py::gil_scoped_release>());

  py::class_<LatencyHistogram>(m, "LatencyHistogram")
      .def(py::init<>())
      .def("record_ms", &LatencyHistogram::record_ms)
      .def("quantile_ms", &LatencyHistogram::quantile_ms)
      .def("cumulative_le_ms", &LatencyHistogram::cumulative_le_ms)
      .def("count", &LatencyHistogram::count)
      .def("mean_ms", &LatencyHistogram::mean_ms)
      .def("max_ms", &LatencyHistogram::max_ms)
      .def("reset", &LatencyHistogram::reset);

  py::class_<PyPlatform>(m, "Platform")
      .def(py::init<const std::string&>(), py::arg("config_json") = "")
      // ---- topology / discovery
      .def("add_fake_node", [](PyPlatform& s, const std::string& fixture) {
        Json j = Json::parse(fixture);
        auto hal = std::make_shared<FakeHal>(j);
        const std::string name = j.get("name").str();
        {
          std::lock_guard<std::mutex> lk(s.mu);
          s.fakes[name] = hal;
        }
        s.p->discovery()->add_node(name, hal);
        return name;
      }, py::call_guard<py::gil_scoped_release>())
      .def("add_amdsmi_node", [](PyPlatform& s, const std::string& name) {
        auto hal = std::make_shared<AmdSmiHal>();
        if (!hal->ok()) throw std::runtime_error("amd-smi unavailable: " + hal->error());
        s.p->discovery()->add_node(name, hal);
        return name;
      }, py::call_guard<py::gil_scoped_release>())
      .def("upsert_node", [](PyPlatform& s, const std::string& node_json) {
        s.p->discovery()->upsert_node(node_from_json(Json::parse(node_json)));
      }, py::call_guard<py::gil_scoped_release>())
      .def("remove_node", [](PyPlatform& s, const std::string& n) { s.p->discovery()->remove_node(n); }, py::call_guard<py::gil_scoped_release>())
      .def("set_cordon", [](PyPlatform& s, const std::string& n, bool on) { s.p->scheduler()->set_cordon(n, on); }, py::call_guard<py::gil_scoped_release>())
      .def("cordoned", [](PyPlatform& s) { return s.p->scheduler()->cordoned(); })
      .def("refresh", [](PyPlatform& s) { s.p->discovery()->refresh(); },
           py::call_guard<py::gil_scoped_release>())
      .def("refresh_telemetry", [](PyPlatform& s) { s.p->discovery()->refresh_telemetry(); },
           py::call_guard<py::gil_scoped_release>())
      .def("snapshot_json", [](PyPlatform& s) { return to_json(*s.p->discovery()->snapshot()).dump(); }, py::call_guard<py::gil_scoped_release>())
      .def("node_json", [](PyPlatform& s, const std::string& n) {
        NodeTopology t;
        if (!s.p->discovery()->node(n, &t)) return std::string("null");
        return to_json(t).dump();
      }, py::call_guard<py::gil_scoped_release>())
      .def("generation", [](PyPlatform& s) { return s.p->discovery()->generation(); })
      .def("topology_events_json", [](PyPlatform& s) {
        Json a = Json::array();
        for (const auto& e : s.p->discovery()->drain_events()) {
          Json j = Json::object();
          j["type"] = to_string(e.type);
          j["node"] = e.node;
          j["gpu"] = e.gpu;
          j["detail"] = e.detail;
          a.push_back(j);
        }
        return a.dump();
      }, py::call_guard<py::gil_scoped_release>())
      .def("hints_json", [](PyPlatform& s, int count, double min_mem, const std::string& arch) {
        HintRequest r;
        r.gpu_count = count;
        r.min_memory_gb = min_mem;
        r.arch = arch;
        Json a = Json::array();
        for (const auto& h : s.p->discovery()->hints(r)) {
          Json j = Json::object();
          j["node"] = h.node;
          j["score"] = h.score;
          j["bandwidth_gbps"] = h.bandwidth_gbps;
          Json g = Json::array();
          for (const auto& x : h.gpus) g.push_back(x);
          j["gpus"] = g;
          Json rs = Json::array();
          for (const auto& x : h.reasons) rs.push_back(x);
          j["reasons"] = rs;
          a.push_back(j);
        }
        return a.dump();
      }, py::arg("count"), py::arg("min_memory_gb") = 0.0, py::arg("arch") = "", py::call_guard<py::gil_scoped_release>())
      // ---- fault injection on fake nodes
      .def("fake_set_link_up", [](PyPlatform& s, const std::string& node, const std::string& a,
                                  const std::string& b, bool up) {
        s.fake(node).set_link_up(a, b, up);
        s.p->discovery()->refresh_node(node);
      }, py::call_guard<py::gil_scoped_release>())
      .def("fake_set_health", [](PyPlatform& s, const std::string& node, const std::string& gpu,
                                 const std::string& status, const std::string& reason) {
        s.fake(node).set_health(gpu, health_from(status), reason);
        s.p->discovery()->refresh_node(node);
      }, py::call_guard<py::gil_scoped_release>())
      .def("fake_set_health_signals", [](PyPlatform& s, const std::string& node, const std::string& gpu,
                                         const std::string& js) {
        s.fake(node).set_health_signals(gpu, Json::parse(js));
        s.p->discovery()->refresh_node(node);
      }, py::call_guard<py::gil_scoped_release>())
      .def("fake_set_util", [](PyPlatform& s, const std::string& node, const std::string& gpu,
                               double gfx, double mem_gb) {
        s.fake(node).set_util(gpu, gfx, mem_gb);
        s.p->discovery()->refresh_node(node);
      }, py::call_guard<py::gil_scoped_release>())
      .def("fake_set_measured_link", [](PyPlatform& s, const std::string& node, const std::string& a,
                                        const std::string& b, double gbps) {
        s.fake(node).set_measured_link(a, b, gbps);
        s.p->discovery()->refresh_node(node);
      }, py::call_guard<py::gil_scoped_release>())
      .def("fake_partition_switches", [](PyPlatform& s, const std::string& node) {
        return s.fake(node).partition_switches();
      }, py::call_guard<py::gil_scoped_release>())
      // ---- extender verbs
      .def("filter", [](PyPlatform& s, const std::string& b) { return s.p->filter(b); },
           py::call_guard<py::gil_scoped_release>())
      // bytes in / bytes out (the HTTP shell: no UTF-8 decode / encode of
      // multi-megabyte ExtenderArgs with full Node objects)
      .def("filter_bytes", [](PyPlatform& s, const py::bytes& b) {
        std::string in = b;
        std::string out;
        {
          py::gil_scoped_release nogil;
          out = s.p->filter(in);
        }
        return py::bytes(out);
      })
      .def("prioritize_bytes", [](PyPlatform& s, const py::bytes& b) {
        std::string in = b;
        std::string out;
        {
          py::gil_scoped_release nogil;
          out = s.p->prioritize(in);
        }
        return py::bytes(out);
      })
      .def("preempt", [](PyPlatform& s, const std::string& b) { return s.p->preempt(b); },
           py::call_guard<py::gil_scoped_release>())
      .def("count_preemptions", [](PyPlatform& s, size_t n) {
        s.p->scheduler()->count_preemptions(n);
        s.p->metrics()->add("kgwe_preemptions_total", {}, static_cast<double>(n));
      })
      .def("prioritize", [](PyPlatform& s, const std::string& b) { return s.p->prioritize(b); },
           py::call_guard<py::gil_scoped_release>())
      .def("bind", [](PyPlatform& s, const std::string& b, const std::string& pod) { return s.p->bind(b, pod); },
           py::arg("body"), py::arg("pod_json") = "", py::call_guard<py::gil_scoped_release>())
      .def("observe_pod_latency_ms", [](PyPlatform& s, double ms) { s.p->observe_pod_latency_ms(ms); })
      // ---- scheduler direct API
      .def("schedule", [](PyPlatform& s, const std::string& w) { return s.p->schedule(w); },
           py::call_guard<py::gil_scoped_release>())
      .def("schedule_gang", [](PyPlatform& s, const std::string& arr) {
        std::vector<WorkloadRequest> ws;
        const Json parsed = Json::parse(arr);  // keep alive: items() is a reference into it
        for (const auto& j : parsed.items()) ws.push_back(workload_from_json(j));
        return list_json(s.p->scheduler()->schedule_gang(ws));
      }, py::call_guard<py::gil_scoped_release>())
      .def("release", [](PyPlatform& s, const std::string& uid, double now) { return s.p->release(uid, now); }, py::call_guard<py::gil_scoped_release>())
      .def("permit", [](PyPlatform& s, const std::string& uid) { return s.p->scheduler()->permit(uid); }, py::call_guard<py::gil_scoped_release>())
      .def("restore_allocation", [](PyPlatform& s, const std::string& js) {
        return s.p->scheduler()->restore(allocation_from_json(Json::parse(js)));
      }, py::call_guard<py::gil_scoped_release>())
      .def("allocations_json", [](PyPlatform& s) { return list_json(s.p->scheduler()->allocations()); }, py::call_guard<py::gil_scoped_release>())
      .def("scheduler_metrics_json", [](PyPlatform& s) { return metrics_json(s.p->scheduler()->metrics()).dump(); }, py::call_guard<py::gil_scoped_release>())
      .def("latency_quantile_ms", [](PyPlatform& s, double q) { return s.p->scheduler()->latency().quantile_ms(q); })
      .def("scheduler_events_json", [](PyPlatform& s) {
        Json a = Json::array();
        for (const auto& e : s.p->scheduler()->drain_events()) {
          Json j = Json::object();
          j["type"] = to_string(e.type);
          j["uid"] = e.uid;
          j["node"] = e.node;
          j["detail"] = e.detail;
          a.push_back(j);
        }
        return a.dump();
      }, py::call_guard<py::gil_scoped_release>())
      .def("score_node_json", [](PyPlatform& s, const std::string& node, const std::string& w) {
        NodeTopology n;
        if (!s.p->discovery()->node(node, &n)) return std::string("null");
        WorkloadRequest r = workload_from_json(Json::parse(w));
        std::string why = s.p->scheduler()->eligible(n, r);
        NodeScore sc = s.p->scheduler()->score_node(n, r);
        Json j = Json::object();
        j["node"] = node;
        j["eligible"] = why.empty();
        j["reason"] = why;
        j["total"] = sc.total;
        j["topology"] = sc.topology;
        j["resource"] = sc.resource;
        j["balance"] = sc.balance;
        j["bandwidth_gbps"] = sc.bandwidth_gbps;
        Json g = Json::array();
        for (const auto& x : sc.gpus) g.push_back(x);
        j["gpus"] = g;
        Json p = Json::array();
        for (const auto& x : sc.partitions) p.push_back(x);
        j["partitions"] = p;
        return j.dump();
      }, py::call_guard<py::gil_scoped_release>())
      // ---- partitions
      .def("register_strategy", [](PyPlatform& s, const std::string& js) {
        return s.p->partitions()->register_strategy(strategy_from_json(Json::parse(js)));
      }, py::call_guard<py::gil_scoped_release>())
      .def("strategies_json", [](PyPlatform& s) { return list_json(s.p->partitions()->strategies()); }, py::call_guard<py::gil_scoped_release>())
      .def("ensure_partitions", [](PyPlatform& s, const std::string& mode, int count, bool plan_only,
                                   const std::string& memory) {
        MemoryPartition m = memory_partition_from(memory.empty() ? "NPS1" : memory);
        return list_json(s.p->partitions()->ensure_capacity(compute_partition_from(mode), count, plan_only,
                                                            memory.empty() ? nullptr : &m));
      }, py::arg("mode"), py::arg("count"), py::arg("plan_only") = false, py::arg("memory") = "", py::call_guard<py::gil_scoped_release>())
      .def("rebalance", [](PyPlatform& s, const std::string& name, bool plan_only) {
        return list_json(s.p->partitions()->rebalance(name, plan_only));
      }, py::arg("name"), py::arg("plan_only") = false, py::call_guard<py::gil_scoped_release>())
      .def("reclaim_idle_partitions", [](PyPlatform& s, bool plan_only) {
        return list_json(s.p->partitions()->reclaim_idle(plan_only));
      }, py::arg("plan_only") = false, py::call_guard<py::gil_scoped_release>())
      .def("reclaim_idle_after", [](PyPlatform& s, double now, double min_idle_s) {
        return list_json(s.p->partitions()->reclaim_idle_after(now, min_idle_s));
      }, py::call_guard<py::gil_scoped_release>())
      .def("set_partition_actuator", [](PyPlatform& s, DiscoveryService::RemoteActuator fn) {
        s.p->discovery()->set_remote_actuator(std::move(fn));
      })
      .def("draining_gpus", [](PyPlatform& s) { return s.p->scheduler()->draining(); })
      .def("consolidate_partitions", [](PyPlatform& s, double now, bool plan_only) {
        return s.p->consolidate_partitions(now, !plan_only);
      }, py::arg("now"), py::arg("plan_only") = true, py::call_guard<py::gil_scoped_release>())
      .def("pod_latency_quantile_ms", [](PyPlatform& s, double q) { return s.p->pod_latency().quantile_ms(q); })
      .def("pod_latency_count", [](PyPlatform& s) { return s.p->pod_latency().count(); })
      .def("queue_depth", [](PyPlatform& s) { return s.p->queue_depth(); })
      .def("count_error", [](PyPlatform& s, const std::string& step) {
        s.p->metrics()->add("kgwe_controller_errors_total", {step}, 1.0);
      })
      .def("partition_ops_json", [](PyPlatform& s) { return list_json(s.p->partitions()->operations()); }, py::call_guard<py::gil_scoped_release>())
      .def("partition_metrics_json", [](PyPlatform& s) {
        PartitionMetrics pm = s.p->partitions()->metrics();
        Json j = Json::object();
        Json modes = Json::object();
        for (const auto& kv : pm.modes) {
          Json mj = Json::object();
          mj["gpus"] = kv.second.gpus;
          mj["slices"] = kv.second.slices;
          mj["slices_in_use"] = kv.second.slices_in_use;
          modes[kv.first] = mj;
        }
        j["modes"] = modes;
        j["slice_utilization"] = pm.slice_utilization;
        j["ops_total"] = pm.ops_total;
        j["ops_failed"] = pm.ops_failed;
        j["ops_pending"] = pm.ops_pending;
        j["migrations"] = s.p->partitions()->migrations();
        return j.dump();
      }, py::call_guard<py::gil_scoped_release>())
      // ---- sharing
      .def("share_allocate", [](PyPlatform& s, const std::string& js) {
        Json j = Json::parse(js);
        SharingRequest r;
        r.uid = j.get("uid").str();
        r.ns = j.get("namespace").str("default");
        r.team = j.get("team").str();
        r.method = sharing_method_from(j.get("method").str("None"));
        r.type = workload_type_from(j.get("type").str("Inference"));
        r.require_isolation = j.get("requireIsolation").as_bool(false);
        r.prefer_partition = j.get("preferPartition").as_bool(false);
        r.partition_mode = compute_partition_from(j.get("partitionMode").str("CPX"));
        r.cu_percent = j.get("cuPercent").as_number(0.0);
        r.memory_gb = j.get("memoryGB").as_number(0.0);
        r.node = j.get("node").str();
        r.gpu = j.get("gpu").str();
        std::string err;
        SharingAllocation a = s.p->sharing()->allocate(r, &err);
        Json out = to_json(a);
        out["error"] = err;
        return out.dump();
      }, py::call_guard<py::gil_scoped_release>())
      .def("share_release", [](PyPlatform& s, const std::string& uid) { return s.p->sharing()->release(uid); }, py::call_guard<py::gil_scoped_release>())
      .def("share_allocations_json", [](PyPlatform& s) { return list_json(s.p->sharing()->allocations()); }, py::call_guard<py::gil_scoped_release>())
      // ---- cost
      .def("cost_start", [](PyPlatform& s, const std::string& js, double now) {
        return s.p->cost()->start(usage_from_json(Json::parse(js)), now);
      }, py::call_guard<py::gil_scoped_release>())
      .def("cost_sample", [](PyPlatform& s, const std::string& uid, double gfx, double mem, double now) {
        return s.p->cost()->sample(uid, gfx, mem, now);
      }, py::call_guard<py::gil_scoped_release>())
      .def("cost_finalize", [](PyPlatform& s, const std::string& uid, double now) {
        UsageRecord r;
        if (!s.p->cost()->finalize(uid, now, &r)) return std::string("null");
        return to_json(r).dump();
      }, py::call_guard<py::gil_scoped_release>())
      .def("cost_record_json", [](PyPlatform& s, const std::string& uid) {
        UsageRecord r;
        if (!s.p->cost()->record(uid, &r)) return std::string("null");
        return to_json(r).dump();
      }, py::call_guard<py::gil_scoped_release>())
      .def("create_budget", [](PyPlatform& s, const std::string& js, double now) {
        return s.p->cost()->create_budget(budget_from_json(Json::parse(js)), now);
      }, py::call_guard<py::gil_scoped_release>())
      .def("budgets_json", [](PyPlatform& s, double now) { return list_json(s.p->cost()->budgets(now)); }, py::call_guard<py::gil_scoped_release>())
      .def("alerts_json", [](PyPlatform& s, bool unack) { return list_json(s.p->cost()->alerts(unack)); },
           py::arg("unacknowledged_only") = false, py::call_guard<py::gil_scoped_release>())
      .def("acknowledge_alert", [](PyPlatform& s, const std::string& id) { return s.p->cost()->acknowledge(id); }, py::call_guard<py::gil_scoped_release>())
      .def("cost_summary_json", [](PyPlatform& s, const std::string& scope, const std::string& id, double from,
                                   double to) { return s.p->cost()->summary(scope, id, from, to).dump(); }, py::call_guard<py::gil_scoped_release>())
      .def("recommendations_json", [](PyPlatform& s, const std::string& scope, const std::string& id) {
        return list_json(s.p->cost()->recommendations(scope, id));
      }, py::call_guard<py::gil_scoped_release>())
      .def("chargeback_json", [](PyPlatform& s, const std::string& by, double from, double to) {
        return s.p->cost()->chargeback(by, from, to).dump();
      }, py::call_guard<py::gil_scoped_release>())
      .def("admit", [](PyPlatform& s, const std::string& ns, const std::string& team, const std::string& project,
                       double est, double now) {
        Admission a = s.p->cost()->admit(ns, team, project, est, now);
        Json j = Json::object();
        j["allowed"] = a.allowed;
        j["throttled"] = a.throttled;
        j["reason"] = a.reason;
        return j.dump();
      }, py::call_guard<py::gil_scoped_release>())
      .def("pricing_json", [](PyPlatform& s) {
        Json a = Json::array();
        for (const auto& p : s.p->cost()->pricing_table()) {
          Json j = Json::object();
          j["gpu_type"] = p.gpu_type;
          j["on_demand"] = p.on_demand;
          j["spot"] = p.spot;
          j["reserved"] = p.reserved;
          Json pt = Json::object();
          for (const auto& kv : p.partition) pt[kv.first] = kv.second;
          j["partition"] = pt;
          a.push_back(j);
        }
        return a.dump();
      }, py::call_guard<py::gil_scoped_release>())
      .def("set_pricing", [](PyPlatform& s, const std::string& js) {
        Json j = Json::parse(js);
        GpuPricing p;
        p.gpu_type = j.get("gpu_type").str();
        p.on_demand = j.get("on_demand").as_number();
        p.spot = j.get("spot").as_number();
        p.reserved = j.get("reserved").as_number();
        for (const auto& kv : j.get("partition").fields()) p.partition[kv.first] = kv.second.as_number();
        s.p->cost()->set_pricing(p);
      }, py::call_guard<py::gil_scoped_release>())
      .def("cost_replayed", [](PyPlatform& s) { return s.p->cost()->replayed(); })
      .def("cost_resumed", [](PyPlatform& s) { return s.p->cost()->resumed(); })
      // ---- metrics / housekeeping
      .def("tick", [](PyPlatform& s, double now) { s.p->tick(now); }, py::call_guard<py::gil_scoped_release>())
      .def("expose_metrics", [](PyPlatform& s) { return s.p->expose_metrics(); },
           py::call_guard<py::gil_scoped_release>())
      .def("metric_value", [](PyPlatform& s, const std::string& name, const std::vector<std::string>& labels) {
        return s.p->metrics()->value(name, labels);
      }, py::call_guard<py::gil_scoped_release>())
      .def("metric_families", [](PyPlatform& s) { return s.p->metrics()->families(); }, py::call_guard<py::gil_scoped_release>());

  py::class_<PyHttpServer>(m, "HttpServer")
      .def(py::init<PyPlatform&, const std::string&, int, const std::string&, int, int>(), py::arg("platform"),
           py::arg("host") = "0.0.0.0", py::arg("port") = 8080, py::arg("prefix") = "", py::arg("workers") = 0,
           py::arg("gang_hold_ms") = 25000)
      .def("start", [](PyHttpServer& s) {
        const std::string err = s.srv->start();
        if (!err.empty()) throw std::runtime_error(err);
      }, py::call_guard<py::gil_scoped_release>())
      .def("stop", [](PyHttpServer& s) { s.srv->stop(); }, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", [](PyHttpServer& s) { return s.srv->port(); })
      .def("set_ready", [](PyHttpServer& s, bool r) { s.srv->set_ready(r); })
      .def("set_verbs_via_fallback", [](PyHttpServer& s, bool v) { s.srv->set_verbs_via_fallback(v); })
      .def("set_bind_sink", &PyHttpServer::set_bind_sink)
      .def("set_pod_lookup", &PyHttpServer::set_pod_lookup)
      .def("set_fallback", &PyHttpServer::set_fallback)
      .def("parked", [](PyHttpServer& s) { return s.srv->parked(); })
      .def("stats_json", [](PyHttpServer& s) { return s.srv->stats_json(); },
           py::call_guard<py::gil_scoped_release>());

  // Keep-alive extender client of the scheduler stand-in.  `parts` are bytes
  // objects sent back to back as the body (no join); the GIL is released for
  // the round trip.  post() -> (status, bytes); post_names() -> (status, names
  // of the Node items / nodenames in the reply) without building the reply in
  // Python.
  py::class_<HttpClient>(m, "HttpClient")
      .def(py::init<std::string, int, double>(), py::arg("host"), py::arg("port"), py::arg("timeout_s") = 30.0)
      .def("post", [](HttpClient& c, const std::string& path, const py::list& parts) {
        std::vector<std::string_view> views;
        for (const auto& h : parts) {
          char* p = nullptr;
          Py_ssize_t n = 0;
          if (PyBytes_AsStringAndSize(h.ptr(), &p, &n) != 0) throw py::error_already_set();
          views.emplace_back(p, static_cast<size_t>(n));
        }
        std::string body;
        int status;
        {
          py::gil_scoped_release nogil;
          status = c.post(path, views, &body);
        }
        return py::make_tuple(status, py::bytes(body));
      })
      .def("post_names", [](HttpClient& c, const std::string& path, const py::list& parts) {
        std::vector<std::string_view> views;
        for (const auto& h : parts) {
          char* p = nullptr;
          Py_ssize_t n = 0;
          if (PyBytes_AsStringAndSize(h.ptr(), &p, &n) != 0) throw py::error_already_set();
          views.emplace_back(p, static_cast<size_t>(n));
        }
        std::string body;
        std::vector<std::string> names;
        int status;
        bool ok;
        {
          py::gil_scoped_release nogil;
          status = c.post(path, views, &body);
          ok = scan_node_names(body, &names);
        }
        if (!ok) throw std::runtime_error("reply is not an ExtenderFilterResult: " + body.substr(0, 200));
        return py::make_tuple(status, names);
      });
}
