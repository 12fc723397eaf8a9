// Native HTTP/1.1 server for the kube-scheduler EXTENDER verbs.
//
// The reference declares the extender contract only as configuration
// (deploy/helm/kgwe/templates/scheduler-configmap.yaml:61-79: urlPrefix on
// the controller service :8080, verbs filter / prioritize / bind, 30 s
// httpTimeout) and a Permit plugin "KGWEGangScheduling" next to a Reserve
// plugin "KGWEReservation" (:38-41,57-60); nothing serves either.  Here the
// verbs are served from C++ straight into `Platform`: one epoll thread
// watches keep-alive connections (EPOLLONESHOT), a worker pool reads the
// request, runs the verb and writes the reply.  No Python object is touched on
// filter / prioritize / preempt; bind calls one registered sink (the
// apiserver Binding write, which lives with the cluster credentials).
//
// Gang Permit: a gang member's bind reserves its GPUs and, while the gang is
// incomplete, the REQUEST IS HELD (the connection is parked, no worker
// blocks).  When the last member's bind arrives every held bind is finished
// and answered; when the gang reservation times out every held bind is
// answered with an error and the reservations are gone.  A held request is
// answered with a retryable error after `gang_hold_ms` at the latest, below
// kube-scheduler's extender httpTimeout.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "histogram.h"
#include "platform.h"

namespace kgwe {

struct HttpRequest {
  std::string method, path, query, body;
  std::string authorization;  // the Authorization header's value, if any
};

struct HttpResponse {
  int code = 200;
  std::string ctype = "application/json";
  std::string body;
};

class ExtenderHttpServer {
 public:
  struct Options {
    std::string host = "0.0.0.0";
    int port = 8080;             // 0: pick a free port
    std::string prefix;          // urlPrefix of the extender verbs
    int workers = 0;             // 0: min(16, max(4, hardware threads))
    size_t max_body = 256u << 20;
    int gang_hold_ms = 25000;    // a parked gang bind is answered by then
    int idle_timeout_s = 300;    // keep-alive connections idle longer are closed
  };
  // Apiserver write of a successful bind (Binding + placement annotations).
  // Arguments: the ExtenderBindingArgs body and bind()'s JSON.  Returns ""
  // or an error; on an error the reservation is released and the verb fails.
  using BindSink = std::function<std::string(const std::string&, const std::string&)>;
  // Pod object (JSON) of namespace/name, "" if unknown: the extender
  // restarted between a pod's filter and its bind.
  using PodLookup = std::function<std::string(const std::string&, const std::string&)>;
  // Every request that is not a native route (webhooks, agent pushes, debug).
  using Fallback = std::function<HttpResponse(const HttpRequest&)>;

  ExtenderHttpServer(std::shared_ptr<Platform> platform, Options opt);
  ~ExtenderHttpServer();
  ExtenderHttpServer(const ExtenderHttpServer&) = delete;
  ExtenderHttpServer& operator=(const ExtenderHttpServer&) = delete;

  // Binds and listens; "" or the error.  Handlers must be set before start().
  std::string start();
  void stop();
  int port() const { return port_; }
  const std::string& host() const { return opt_.host; }

  void set_bind_sink(BindSink f) { sink_ = std::move(f); }
  void set_pod_lookup(PodLookup f) { lookup_ = std::move(f); }
  void set_fallback(Fallback f) { fallback_ = std::move(f); }
  void set_ready(bool r) { ready_.store(r); }
  // Route the verbs through the fallback too (a shell that wraps every verb
  // in trace spans).
  void set_verbs_via_fallback(bool v) { verbs_via_fallback_.store(v); }

  // {"verbs": {verb: {count, p50_ms, p99_ms, mean_ms, max_ms}}, "connections",
  //  "requests", "parked", "gang_binds_held", "gang_binds_timed_out"}.
  // Verb times run from the request's last byte read to the reply's last byte
  // written; a held gang bind counts under "bind_held" instead of "bind".
  std::string stats_json() const;
  const LatencyHistogram& verb_histogram(const std::string& verb) const;
  size_t parked() const;

 private:
  struct Conn;
  struct Parked;
  using ConnPtr = std::shared_ptr<Conn>;

  void loop();
  void worker();
  void post(std::function<void()> fn);
  void on_readable(const ConnPtr& c);
  // Parses as much as is buffered; true when a full request is in `req`.
  bool parse(Conn& c, HttpRequest* req, bool* bad);
  // Handles one request; false when the connection was parked (no reply yet).
  bool dispatch(const ConnPtr& c, HttpRequest& req, int64_t t_read_ns);
  bool handle_bind(const ConnPtr& c, const std::string& body, int64_t t_read_ns, bool held);
  void finish_gang(const std::string& gang);
  void sweep_parked();
  bool reply(const ConnPtr& c, const HttpResponse& r);
  bool reply_json(const ConnPtr& c, const std::string& body) {
    HttpResponse r;
    r.body = body;
    return reply(c, r);
  }
  void rearm(const ConnPtr& c);
  void close_conn(const ConnPtr& c);
  void record(const char* verb, int64_t t0_ns);

  std::shared_ptr<Platform> plat_;
  Options opt_;
  BindSink sink_;
  PodLookup lookup_;
  Fallback fallback_;
  std::atomic<bool> ready_{true};
  std::atomic<bool> verbs_via_fallback_{false};
  std::atomic<bool> stop_{false};
  bool started_ = false;
  int listen_fd_ = -1, epoll_fd_ = -1, wake_fd_ = -1, port_ = 0;
  std::thread loop_thread_;
  std::vector<std::thread> workers_;
  std::mutex q_mu_;
  std::condition_variable q_cv_;
  std::deque<std::function<void()>> q_;
  mutable std::mutex conns_mu_;
  std::unordered_map<int, ConnPtr> conns_;
  mutable std::mutex park_mu_;
  std::map<std::string, std::vector<Parked>> parked_;  // gang -> held binds
  std::atomic<uint64_t> requests_{0}, held_total_{0}, held_timeouts_{0};
  LatencyHistogram h_filter_, h_prioritize_, h_bind_, h_bind_held_, h_preempt_, h_other_;
};

}  // namespace kgwe
