// Native unit + concurrency tests for the C++ platform core (the reference's
// `go test -race` role: Makefile:79-85).  Plain asserts, no framework; one
// binary per build flavour (plain, -fsanitize=thread, -fsanitize=address,
// undefined), driven by tests/test_native_core.py.
//
// The reference's only race tooling is `go test -race` with no tests to run
// (Makefile:81, .github/workflows/ci.yaml:91) while its ledger re-checks and
// records under separate lock acquisitions (src/scheduler/scheduler.go:630-640,
// 695-707).  The stress cases below drive schedule / release / extender
// filter+bind / topology refresh / telemetry / partition reclaim / metrics
// exposition from many threads at once and check the ledger invariants
// (no GPU or slice ever has two owners, everything is released at the end);
// under TSan any unsynchronised access fails the run.
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <random>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "cost.h"
#include "discovery.h"
#include "hal.h"
#include "histogram.h"
#include "http_client.h"
#include "http_server.h"
#include "metrics.h"
#include "partition.h"
#include "platform.h"
#include "scheduler.h"

using namespace kgwe;

static int g_failures = 0;
#define CHECK(cond)                                                                      \
  do {                                                                                   \
    if (!(cond)) {                                                                       \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond);     \
      ++g_failures;                                                                      \
    }                                                                                    \
  } while (0)

static std::shared_ptr<Platform> make_platform(int nodes, PlatformConfig cfg = {}) {
  auto p = std::make_shared<Platform>(cfg);
  for (int i = 0; i < nodes; ++i) {
    std::string name = "n" + std::to_string(i);
    p->discovery()->add_node(name, std::make_shared<FakeHal>(make_mi355x_node_fixture(name, 8, 2)));
  }
  p->discovery()->refresh();
  return p;
}

static WorkloadRequest gpus(const std::string& uid, int n, bool xgmi = true) {
  WorkloadRequest w;
  w.uid = w.name = uid;
  w.gpu_count = n;
  w.topology = xgmi && n > 1 ? TopologyPreference::XgmiOptimal : TopologyPreference::None;
  return w;
}

static WorkloadRequest slice(const std::string& uid) {
  WorkloadRequest w;
  w.uid = w.name = uid;
  w.gpu_count = 0;
  w.partition = true;
  w.partition_mode = ComputePartition::CPX;
  w.partition_count = 1;
  w.type = WorkloadType::Inference;
  return w;
}

static WorkloadRequest share(const std::string& uid) {
  WorkloadRequest w;
  w.uid = w.name = uid;
  w.gpu_count = 1;
  w.sharing = SharingMethod::CoLocate;
  w.share_cu_percent = 12.5;
  w.share_memory_gb = 30.0;
  w.type = WorkloadType::Inference;
  return w;
}

// Ledger invariant: every GPU / slice has at most one owner, no GPU is held
// whole while any of its slices is held, a shared GPU is neither held whole
// nor sliced, and co-located clients of one GPU have disjoint CU ranges.
static bool ledger_consistent(Scheduler& s, size_t* n_gpus = nullptr) {
  std::set<std::string> seen, whole, sliced;
  std::map<std::string, std::vector<std::pair<int, int>>> shared;
  size_t total = 0;
  for (const auto& a : s.allocations()) {
    if (!a.shared_gpu.empty()) {
      shared[a.shared_gpu].emplace_back(a.cu_begin, a.cu_end);
      ++total;
    }
    for (const auto& g : a.gpus) {
      if (!seen.insert(g).second) return false;
      whole.insert(g);
      ++total;
    }
    for (const auto& p : a.partitions) {
      if (!seen.insert(p).second) return false;
      sliced.insert(p.substr(0, p.rfind("/p")));
      ++total;
    }
  }
  for (const auto& g : sliced)
    if (whole.count(g)) return false;
  for (auto& kv : shared) {
    if (whole.count(kv.first) || sliced.count(kv.first)) return false;
    std::sort(kv.second.begin(), kv.second.end());
    for (size_t i = 1; i < kv.second.size(); ++i)
      if (kv.second[i].first < kv.second[i - 1].second) return false;  // overlapping CU masks
  }
  if (n_gpus) *n_gpus = total;
  return true;
}

// Platform path (auto-provisions partitions) for a one-slice CPX request,
// in GPUWorkload shape.
static bool platform_schedule(Platform& p, const WorkloadRequest& w) {
  const std::string body = "{\"metadata\":{\"name\":\"" + w.name + "\",\"uid\":\"" + w.uid +
                           "\"},\"spec\":{\"workloadType\":\"Inference\",\"gpuRequirements\":"
                           "{\"count\":0,\"partition\":{\"mode\":\"CPX\",\"count\":1}}}}";
  return Json::parse(p.schedule(body)).get("ok").as_bool(false);
}

static void test_topology_fixture() {
  NodeTopology n = node_from_json(make_mi355x_node_fixture("a", 8, 2));
  CHECK(n.gpus.size() == 8);
  CHECK(n.xgmi_fully_connected);
  for (const auto& g : n.gpus) CHECK(g.links.size() == 7);
  Json round = to_json(n);
  NodeTopology m = node_from_json(round);
  CHECK(m.gpus.size() == 8 && m.gpus[3].uuid == n.gpus[3].uuid);
}

static void test_schedule_whole_node_and_numa() {
  auto p = make_platform(1);
  Scheduler& s = *p->scheduler();
  Decision d = s.schedule(gpus("two", 2));
  CHECK(d.ok);
  Allocation a;
  CHECK(s.allocation("two", &a) && a.gpus.size() == 2);
  NodeTopology n;
  CHECK(p->discovery()->node("n0", &n));
  CHECK(n.gpu(a.gpus[0])->numa_node == n.gpu(a.gpus[1])->numa_node);  // one NUMA domain
  CHECK(!s.schedule(gpus("eight", 8)).ok);  // only 6 free
  CHECK(s.release("two"));
  CHECK(s.schedule(gpus("eight", 8)).ok);
  CHECK(s.release("eight"));
  CHECK(s.allocations().empty());
}

static void test_health_policy() {
  Health h;
  h.ecc_uncorrectable = 1;
  apply_health_policy(h);
  CHECK(h.status == HealthStatus::Unhealthy);
  Health d;
  d.pending_retired_pages = 2;
  apply_health_policy(d);
  CHECK(d.status == HealthStatus::Degraded);
  Health l;
  apply_health_policy(l, 1);  // a down link is a reason, not a status change
  CHECK(l.status == HealthStatus::Healthy && l.reasons.size() == 1);
}

static void test_histogram_quantile_not_max() {
  LatencyHistogram hist;
  for (int i = 0; i < 990; ++i) hist.record_ms(1.0);
  for (int i = 0; i < 10; ++i) hist.record_ms(500.0);
  CHECK(hist.quantile_ms(0.99) < 2.0);  // the reference's "P99" would be 500
  CHECK(hist.max_ms() >= 499.0);
}

static void test_cost_math() {
  CostEngine c;
  UsageRecord r;
  r.uid = "job";
  r.ns = "ml";
  r.gpu_count = 8;
  CHECK(c.start(r, 0.0).empty());
  for (int i = 1; i <= 10; ++i) CHECK(c.sample("job", 95.0, 90.0, 360.0 * i));
  UsageRecord out;
  CHECK(c.finalize("job", 3600.0, &out));
  const double price = c.pricing(out.gpu_type).on_demand;
  CHECK(std::fabs(out.raw_cost - 8 * price) < 0.01);
  CHECK(out.adjusted_cost <= out.raw_cost);  // >80 % utilisation: efficiency discount
}

static void test_metrics_exposition_labels() {
  MetricRegistry reg;
  reg.declare("kgwe_test_gauge", MetricType::Gauge, "help", {"node", "gpu_uuid"});
  reg.set("kgwe_test_gauge", {"n\"0", "GPU-1"}, 3.0);
  std::string text = reg.expose();
  CHECK(text.find("# TYPE kgwe_test_gauge gauge") != std::string::npos);
  CHECK(text.find("kgwe_test_gauge{node=\"n\\\"0\",gpu_uuid=\"GPU-1\"} 3") != std::string::npos);
}

// Copy-on-write snapshots: a publish shares every untouched node with the
// previous snapshot, clones only what it writes, and readers holding the old
// snapshot keep seeing the old node.
static void test_nodemap_copy_on_write() {
  ClusterTopology a;
  a.nodes.set("n0", node_from_json(make_mi355x_node_fixture("n0", 8, 2)));
  a.nodes.set("n1", node_from_json(make_mi355x_node_fixture("n1", 8, 2)));
  ClusterTopology b(a);
  CHECK(b.nodes.same("n0", a.nodes) && b.nodes.same("n1", a.nodes));
  b.nodes.mut("n1").gpus[0].health.status = HealthStatus::Unhealthy;
  CHECK(b.nodes.same("n0", a.nodes));
  CHECK(!b.nodes.same("n1", a.nodes));
  CHECK(a.nodes.at("n1").gpus[0].health.status == HealthStatus::Healthy);
  CHECK(b.nodes.at("n1").gpus[0].health.status == HealthStatus::Unhealthy);
  int seen = 0;
  for (const auto& kv : b.nodes) seen += static_cast<int>(kv.second.gpus.size());
  CHECK(seen == 16 && b.total_gpus() == 16);
  CHECK(b.nodes.find("n0")->second.name == "n0" && b.nodes.find("nx") == b.nodes.end());
  b.nodes.erase("n0");
  CHECK(b.nodes.size() == 1 && a.nodes.size() == 2);
}

// Committed gauge families are shared snapshots: a scrape taken before a
// commit keeps its view; set() after a commit thaws the family.
static void test_metrics_commit_snapshot() {
  MetricRegistry reg;
  reg.declare("kgwe_g", MetricType::Gauge, "help", {"node"});
  GaugeBatch b1;
  b1.set("kgwe_g", {"a"}, 1.0);
  b1.set("kgwe_g", {"b"}, 2.0);
  reg.commit(std::move(b1));
  CHECK(reg.value("kgwe_g", {"b"}) == 2.0);
  GaugeBatch b2;
  b2.set("kgwe_g", {"c"}, 3.0);
  reg.commit(std::move(b2));
  CHECK(reg.value("kgwe_g", {"a"}) == 0.0 && reg.value("kgwe_g", {"c"}) == 3.0);
  reg.set("kgwe_g", {"d"}, 4.0);
  CHECK(reg.value("kgwe_g", {"c"}) == 3.0 && reg.value("kgwe_g", {"d"}) == 4.0);
  CHECK(reg.expose().find("kgwe_g{node=\"d\"} 4") != std::string::npos);
}

static void test_partition_binpack() {
  auto p = make_platform(1);
  std::set<std::string> gpus_used;
  for (int i = 0; i < 8; ++i) {
    CHECK(platform_schedule(*p, slice("s" + std::to_string(i))));  // auto-provisions CPX
    Allocation a;
    if (p->scheduler()->allocation("s" + std::to_string(i), &a) && a.partitions.size() == 1)
      gpus_used.insert(a.partitions[0].substr(0, a.partitions[0].rfind("/p")));
    else
      CHECK(false);
  }
  CHECK(gpus_used.size() == 1);  // one GPU split 8-way
  CHECK(p->partitions()->metrics().slice_utilization == 1.0);
}

// Many threads: schedule / release whole-GPU and slice workloads while
// other threads refresh topology, tick telemetry + reclaim, and scrape.
static void test_concurrent_ledger_stress(int threads, int iters) {
  PlatformConfig cfg;
  cfg.partition_reclaim_idle_s = 0.0;  // reclaim races with slice placement
  auto p = make_platform(4, cfg);
  Scheduler& s = *p->scheduler();
  std::atomic<bool> stop{false};
  std::atomic<int> violations{0}, scheduled{0};
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      std::mt19937 rng(1234 + t);
      std::vector<std::string> mine;
      for (int i = 0; i < iters; ++i) {
        const std::string uid = "t" + std::to_string(t) + "-" + std::to_string(i);
        const int kind = static_cast<int>(rng() % 6);
        WorkloadRequest w = kind == 4 ? slice(uid) : kind == 5 ? share(uid) : gpus(uid, 1 << (rng() % 3));
        Decision d;
        if (kind == 3) {  // extender path: filter -> bind on the first passing node
          std::vector<std::string> nodes = {"n0", "n1", "n2", "n3"}, passed;
          s.filter(w, nodes, &passed);
          if (!passed.empty()) d = s.bind(w, passed[rng() % passed.size()]);
        } else if (kind == 4) {  // platform path: may convert an idle GPU to CPX
          d.ok = platform_schedule(*p, w);
        } else {
          d = s.schedule(w);
        }
        if (d.ok) {
          mine.push_back(uid);
          ++scheduled;
        }
        if (mine.size() > 3 || (rng() % 3 == 0 && !mine.empty())) {
          const size_t k = rng() % mine.size();
          if (!s.release(mine[k])) ++violations;
          mine.erase(mine.begin() + static_cast<long>(k));
        }
        if (!ledger_consistent(s)) ++violations;
      }
      for (const auto& u : mine) s.release(u);
    });
  std::thread refresher([&] {
    while (!stop.load()) {
      p->discovery()->refresh();
      p->discovery()->refresh_telemetry();
    }
  });
  std::thread ticker([&] {
    double now = 0;
    while (!stop.load()) p->tick(now += 1.0);
  });
  std::thread consolidator([&] {  // moves slices in the ledger under everyone's feet
    ConsolidationPolicy pol;
    pol.after_s = 0;
    pol.cooldown_s = 0;
    double now = 0;
    while (!stop.load()) (void)p->partitions()->consolidate(now += 1.0, pol, true);
  });
  std::thread scraper([&] {
    while (!stop.load()) {
      (void)p->expose_metrics();
      (void)p->partitions()->metrics();
      (void)s.metrics();
      (void)s.drain_events();
    }
  });
  for (auto& th : pool) th.join();
  stop = true;
  refresher.join();
  ticker.join();
  consolidator.join();
  scraper.join();
  size_t held = 0;
  CHECK(violations.load() == 0);
  CHECK(scheduled.load() > threads * iters / 4);
  CHECK(ledger_consistent(s, &held));
  CHECK(held == 0);
  CHECK(s.allocations().empty());
  std::printf("  stress: %d threads x %d iters, %d scheduled\n", threads, iters, scheduled.load());
}

// Preemption from many threads on a full fleet: planning walks the ledger
// under the shared lock while binds, releases and other preemptions take the
// exclusive one.  Non-preemptible work must survive everything.
static void test_concurrent_preemption(int threads, int iters) {
  PlatformConfig cfg;
  cfg.sched.preemption_wait_window_s = 0.0;
  cfg.sched.preemption_max_rate_percent = 0.0;  // no cap: as many preemptions as the load asks for
  cfg.sched.preemption_candidate_nodes = 3;
  auto p = make_platform(12, cfg);
  Scheduler& s = *p->scheduler();
  std::set<std::string> pinned;
  for (int n = 0; n < 12; ++n) {
    WorkloadRequest keep = gpus("keep" + std::to_string(n), 2, false);
    keep.preemptible = false;
    keep.priority = 1;
    keep.node_selector["kubernetes.io/hostname"] = "n" + std::to_string(n);
    CHECK(s.schedule(keep).ok);
    pinned.insert(keep.uid);
    for (int k = 0; k < 3; ++k) {
      WorkloadRequest low = gpus("low" + std::to_string(n) + "-" + std::to_string(k), 2, false);
      low.priority = 1 + k;
      low.node_selector = keep.node_selector;
      CHECK(s.schedule(low).ok);
    }
  }
  std::atomic<int> violations{0}, preempted{0}, placed{0};
  std::vector<std::thread> pool;
  std::vector<std::string> all_nodes;
  for (int n = 0; n < 12; ++n) all_nodes.push_back("n" + std::to_string(n));
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      std::mt19937 rng(99 + t);
      std::vector<std::string> mine;
      for (int i = 0; i < iters; ++i) {
        const std::string uid = "hi" + std::to_string(t) + "-" + std::to_string(i);
        WorkloadRequest w = gpus(uid, 1 << (rng() % 3), false);
        w.priority = 100 + static_cast<int>(rng() % 50);
        if (rng() % 4 == 0) {  // the extender's dry run
          for (const auto& kv : s.preemption_plans(w, all_nodes))
            for (const auto& v : kv.second)
              if (pinned.count(v)) ++violations;
          continue;
        }
        Decision d = s.schedule(w);
        for (const auto& v : d.preempted) {
          ++preempted;
          if (pinned.count(v)) ++violations;
        }
        if (d.ok) {
          ++placed;
          mine.push_back(uid);
        }
        if (mine.size() > 2) {
          if (!s.release(mine.front())) {
            // released behind our back = preempted by a higher priority: fine
          }
          mine.erase(mine.begin());
        }
        if (!ledger_consistent(s)) ++violations;
      }
      for (const auto& u : mine) (void)s.release(u);
    });
  for (auto& th : pool) th.join();
  CHECK(violations.load() == 0);
  CHECK(preempted.load() > 0 && placed.load() > 0);
  for (const auto& k : pinned) CHECK(s.allocation(k, nullptr));  // never evicted
  CHECK(ledger_consistent(s));
  CHECK(s.metrics().preemptions >= static_cast<uint64_t>(preempted.load()));
  std::printf("  preemption: %d threads x %d iters, %d placed, %d victims\n", threads, iters, placed.load(),
              preempted.load());
}

// The native extender server under concurrent keep-alive clients: filter,
// prioritize and bind over real sockets, a gang whose members' binds are held
// until the last one arrives, and a clean stop with connections open.
static void test_http_server_verbs_and_gang_hold(int clients, int iters) {
  auto p = make_platform(4);
  ExtenderHttpServer::Options opt;
  opt.host = "127.0.0.1";
  opt.port = 0;
  opt.workers = 4;
  opt.gang_hold_ms = 5000;
  ExtenderHttpServer srv(p, opt);
  std::atomic<int> sunk{0};
  srv.set_bind_sink([&](const std::string&, const std::string&) {
    ++sunk;
    return std::string();
  });
  CHECK(srv.start().empty());
  const int port = srv.port();
  CHECK(port > 0);
  auto pod = [](const std::string& name, int gpus_n, const std::string& gang, int gang_size) {
    std::string ann = "\"kgwe.amd.com/topology\":\"None\"";
    if (!gang.empty())
      ann += ",\"kgwe.amd.com/gang\":\"" + gang + "\",\"kgwe.amd.com/gang-size\":\"" + std::to_string(gang_size) + "\"";
    return "{\"metadata\":{\"name\":\"" + name + "\",\"namespace\":\"t\",\"uid\":\"u-" + name +
           "\",\"annotations\":{" + ann + "}},\"spec\":{\"containers\":[{\"resources\":{\"limits\":{\"amd.com/gpu\":\"" +
           std::to_string(gpus_n) + "\"}}}]}}";
  };
  const std::string names = "[\"n0\",\"n1\",\"n2\",\"n3\"]";
  std::atomic<int> bad{0}, bound{0};
  // A scheduling cycle as kube-scheduler runs it; a bind that lost a race for
  // the node's GPUs ("insufficient free GPUs") is retried like a requeued pod.
  std::function<bool(HttpClient&, const std::string&, int, const std::string&, int, int)> one_pod;
  one_pod = [&](HttpClient& c, const std::string& name, int n, const std::string& gang, int gsize, int tries) {
    std::string body, out;
    body = "{\"pod\":" + pod(name, n, gang, gsize) + ",\"nodenames\":" + names + "}";
    if (c.post("/filter", {body}, &out) != 200) return ++bad, false;
    Json f = Json::parse(out);
    const auto& passed = f.get("nodenames").items();
    if (passed.empty()) {
      if (!gang.empty()) std::fprintf(stderr, "  gang member %s: no node passed: %s\n", name.c_str(), out.c_str());
      return false;
    }
    if (c.post("/prioritize", {body}, &out) != 200 || Json::parse(out).items().size() != 4) return ++bad, false;
    const std::string node = passed[std::hash<std::string>{}(name) % passed.size()].str();
    body = "{\"podName\":\"" + name + "\",\"podNamespace\":\"t\",\"podUID\":\"u-" + name + "\",\"node\":\"" + node + "\"}";
    if (c.post("/bind", {body}, &out) != 200) return ++bad, false;
    const std::string err = Json::parse(out).get("error").str();
    if (!err.empty()) {
      if (err.find("insufficient") != std::string::npos && tries > 1) return one_pod(c, name, n, gang, gsize, tries - 1);
      if (!gang.empty()) std::fprintf(stderr, "  gang member %s: bind answered %s\n", name.c_str(), out.c_str());
      return false;
    }
    ++bound;
    return true;
  };
  std::vector<std::thread> pool;
  for (int t = 0; t < clients; ++t)
    pool.emplace_back([&, t] {
      HttpClient c("127.0.0.1", port, 10.0);
      for (int i = 0; i < iters; ++i) {
        const std::string name = "p" + std::to_string(t) + "-" + std::to_string(i);
        if (one_pod(c, name, 1, "", 0, 1)) (void)p->release("u-" + name, 0.0);
      }
    });
  // meanwhile: a gang of 4 whose members arrive 30 ms apart; every bind must
  // come back OK, the early ones only after the last member's bind
  std::vector<std::thread> gang;
  std::atomic<int> gang_ok{0};
  std::vector<double> done_ms(4, 0.0);
  const auto t0 = std::chrono::steady_clock::now();
  for (int m = 0; m < 4; ++m)
    gang.emplace_back([&, m] {
      std::this_thread::sleep_for(std::chrono::milliseconds(30 * m));
      HttpClient c("127.0.0.1", port, 10.0);
      if (one_pod(c, "g" + std::to_string(m), 2, "ring", 4, 5)) ++gang_ok;
      done_ms[m] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
  for (auto& th : gang) th.join();
  for (auto& th : pool) th.join();
  CHECK(bad.load() == 0);
  CHECK(gang_ok.load() == 4);
  CHECK(done_ms[0] >= 85.0);  // held until the member that arrived at 90 ms
  CHECK(bound.load() >= 4 && sunk.load() == bound.load());
  CHECK(srv.parked() == 0);
  const Json st = Json::parse(srv.stats_json());
  CHECK(st.get("gang_binds_held").as_int(0) >= 3);
  CHECK(st.get("verbs").get("filter").get("count").as_int(0) >= clients * iters);
  HttpClient idle("127.0.0.1", port, 5.0);  // an open keep-alive connection at stop
  std::string out;
  CHECK(idle.post("/filter", {"{\"pod\":" + pod("z", 1, "", 0) + ",\"nodenames\":" + names + "}"}, &out) == 200);
  srv.stop();
  for (int m = 0; m < 4; ++m) (void)p->release("u-g" + std::to_string(m), 0.0);
  CHECK(ledger_consistent(*p->scheduler()));
  std::printf("  http: %d clients x %d pods + gang of 4 (held %.0f ms), %d binds\n", clients, iters, done_ms[0],
              bound.load());
}

// Hostile input on the extender port: truncated and oversized requests, bad
// chunk framing, binary garbage, pipelined requests, clients that vanish mid
// request.  The server may answer 400 or close, never crash or wedge; a
// well-formed request afterwards must still be served.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

static int raw_connect(int port) {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  timeval tv{2, 0};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
    close(fd);
    return -1;
  }
  return fd;
}

static std::string raw_exchange(int port, const std::string& bytes, bool half_close = true) {
  int fd = raw_connect(port);
  if (fd < 0) return "<connect failed>";
  size_t off = 0;
  while (off < bytes.size()) {
    ssize_t n = send(fd, bytes.data() + off, bytes.size() - off, MSG_NOSIGNAL);
    if (n <= 0) break;
    off += static_cast<size_t>(n);
  }
  if (half_close) shutdown(fd, SHUT_WR);
  std::string out;
  char buf[4096];
  for (;;) {
    ssize_t n = recv(fd, buf, sizeof buf, 0);
    if (n <= 0) break;
    out.append(buf, static_cast<size_t>(n));
    if (out.size() > (1u << 20)) break;
  }
  close(fd);
  return out;
}

static void test_http_server_hostile_input() {
  auto p = make_platform(2);
  ExtenderHttpServer::Options opt;
  opt.host = "127.0.0.1";
  opt.port = 0;
  opt.workers = 3;
  opt.max_body = 1 << 16;
  ExtenderHttpServer srv(p, opt);
  CHECK(srv.start().empty());
  const int port = srv.port();
  const std::string good_body = "{\"pod\":{\"metadata\":{\"name\":\"a\",\"uid\":\"ua\"},\"spec\":{\"containers\":[{\"resources\":"
                                "{\"limits\":{\"amd.com/gpu\":\"1\"}}}]}},\"nodenames\":[\"n0\",\"n1\"]}";
  auto post = [&](const std::string& path, const std::string& body) {
    return "POST " + path + " HTTP/1.1\r\nHost: x\r\nContent-Length: " + std::to_string(body.size()) +
           "\r\nConnection: close\r\n\r\n" + body;
  };
  auto status = [](const std::string& r) { return r.size() > 12 ? std::atoi(r.c_str() + 9) : 0; };
  std::vector<std::string> hostile = {
      "",                                                             // connect and leave
      "GARBAGE\r\n\r\n",                                            // no request line
      "POST /filter HTTP/1.1\r\nContent-Length: 100\r\n\r\n{\"pod\":",   // body cut short
      "POST /filter HTTP/1.1\r\nContent-Length: 99999999999\r\n\r\n",   // over max_body
      "POST /filter HTTP/1.1\r\nContent-Length: -5\r\n\r\nxx",
      "POST /filter HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nZZZ\r\nabc\r\n0\r\n\r\n",  // bad chunk size
      "POST /filter HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nffffffffffffffff\r\n",      // absurd chunk
      post("/filter", "{not json"),
      post("/filter", "[]"),
      post("/bind", "{\"podName\":5}"),
      post("/preempt", "{\"pod\":null,\"nodeNameToMetaVictims\":7}"),
      post("/prioritize", std::string(60000, '[')),                      // deep nesting
      "POST /" + std::string(70000, 'a') + " HTTP/1.1\r\n\r\n",          // header past the limit
      std::string("POST /filter HTTP/1.1\r\nContent-Length: 4\r\n\r\n\0\xff\xfe\x01", 47),
  };
  std::mt19937 rng(7);
  for (int i = 0; i < 40; ++i) {  // random bytes, some after a plausible request line
    std::string g(rng() % 600, '\0');
    for (auto& ch : g) ch = static_cast<char>(rng());
    hostile.push_back(i % 2 ? "POST /filter HTTP/1.1\r\n" + g : g);
  }
  for (const auto& h : hostile) {
    const std::string r = raw_exchange(port, h);
    const int st = status(r);
    CHECK(r.empty() || st == 200 || st == 400 || st == 404 || st == 413 || st == 500);
  }
  // 200 replies to hostile JSON carry an error, not a placement
  CHECK(raw_exchange(port, post("/filter", "{not json")).find("rror") != std::string::npos);
  // two pipelined requests on one connection, both answered in order
  const std::string keep = "POST /filter HTTP/1.1\r\nContent-Length: " + std::to_string(good_body.size()) + "\r\n\r\n" + good_body;
  const std::string two = raw_exchange(port, keep + post("/prioritize", good_body));
  size_t first = two.find("HTTP/1.1 200"), second = two.find("HTTP/1.1 200", first + 1);
  CHECK(first != std::string::npos && second != std::string::npos);
  CHECK(two.find("nodenames") != std::string::npos && two.find("\"host\"") != std::string::npos);
  // the server is still healthy
  const std::string ok = raw_exchange(port, post("/filter", good_body));
  CHECK(status(ok) == 200 && ok.find("\"n0\"") != std::string::npos);
  srv.stop();
  std::printf("  http hostile input: %zu cases survived\n", hostile.size());
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 400;
  test_topology_fixture();
  test_schedule_whole_node_and_numa();
  test_health_policy();
  test_histogram_quantile_not_max();
  test_cost_math();
  test_metrics_exposition_labels();
  test_partition_binpack();
  test_nodemap_copy_on_write();
  test_metrics_commit_snapshot();
  test_concurrent_ledger_stress(8, iters);
  test_concurrent_preemption(6, std::max(40, iters / 4));
  test_http_server_verbs_and_gang_hold(6, std::max(20, iters / 10));
  test_http_server_hostile_input();
  if (g_failures) {
    std::fprintf(stderr, "%d check(s) failed\n", g_failures);
    return 1;
  }
  std::printf("core_tests: all passed\n");
  return 0;
}
