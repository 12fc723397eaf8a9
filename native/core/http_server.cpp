#include "http_server.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>

namespace kgwe {

namespace {

int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

double wall_now_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

const char* reason_of(int code) {
  switch (code) {
    case 200: return "OK";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 413: return "Payload Too Large";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    default: return "Status";
  }
}

bool ieq(const char* a, size_t n, const char* lit) {
  const size_t m = std::strlen(lit);
  if (n != m) return false;
  for (size_t i = 0; i < n; ++i)
    if (std::tolower(static_cast<unsigned char>(a[i])) != lit[i]) return false;
  return true;
}

std::string lower(std::string s) {
  for (auto& ch : s) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
  return s;
}

std::string error_json(const std::string& msg) { return "{\"error\":\"" + json_escape(msg) + "\"}"; }

constexpr size_t kMaxHeader = 64 * 1024;
constexpr int kArmed = 0, kOwned = 1, kParked = 2;

}  // namespace

struct ExtenderHttpServer::Conn {
  int fd = -1;
  std::atomic<int> state{kOwned};
  std::atomic<int64_t> last_ns{0};
  // request being read
  std::string hdr;  // bytes up to the end of the headers (and whatever followed)
  bool have_hdr = false;
  std::string method, target, authorization;
  bool keep_alive = true, chunked = false;
  size_t content_length = 0, body_got = 0;
  std::string body;
  std::string chunk_raw;  // undecoded chunked body
  bool dead = false;      // a write failed: close instead of re-arming
};

struct ExtenderHttpServer::Parked {
  ConnPtr conn;
  std::string body;  // ExtenderBindingArgs
  std::string uid;
  int64_t deadline_ns = 0;
  int64_t t_read_ns = 0;
};

ExtenderHttpServer::ExtenderHttpServer(std::shared_ptr<Platform> platform, Options opt)
    : plat_(std::move(platform)), opt_(std::move(opt)) {
  while (!opt_.prefix.empty() && opt_.prefix.back() == '/') opt_.prefix.pop_back();
  if (opt_.workers <= 0) {
    const unsigned hw = std::thread::hardware_concurrency();
    opt_.workers = static_cast<int>(std::min(16u, std::max(4u, hw)));
  }
}

ExtenderHttpServer::~ExtenderHttpServer() { stop(); }

std::string ExtenderHttpServer::start() {
  if (started_) return "";
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE | AI_NUMERICSERV;
  addrinfo* res = nullptr;
  const std::string port = std::to_string(opt_.port);
  const char* host = opt_.host.empty() ? nullptr : opt_.host.c_str();
  if (int rc = getaddrinfo(host, port.c_str(), &hints, &res)) return std::string("getaddrinfo: ") + gai_strerror(rc);
  std::string err = "no address to bind";
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    int fd = socket(ai->ai_family, ai->ai_socktype | SOCK_NONBLOCK | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) {
      err = std::string("socket: ") + std::strerror(errno);
      continue;
    }
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (bind(fd, ai->ai_addr, ai->ai_addrlen) != 0 || listen(fd, 1024) != 0) {
      err = std::string("bind/listen ") + opt_.host + ":" + port + ": " + std::strerror(errno);
      close(fd);
      continue;
    }
    sockaddr_storage ss{};
    socklen_t sl = sizeof ss;
    getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &sl);
    port_ = ntohs(ss.ss_family == AF_INET6 ? reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port
                                           : reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
    listen_fd_ = fd;
    break;
  }
  freeaddrinfo(res);
  if (listen_fd_ < 0) return err;
  epoll_fd_ = epoll_create1(EPOLL_CLOEXEC);
  wake_fd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = listen_fd_;
  epoll_ctl(epoll_fd_, EPOLL_CTL_ADD, listen_fd_, &ev);
  ev.data.fd = wake_fd_;
  epoll_ctl(epoll_fd_, EPOLL_CTL_ADD, wake_fd_, &ev);
  stop_.store(false);
  started_ = true;
  for (int i = 0; i < opt_.workers; ++i) workers_.emplace_back([this] { worker(); });
  loop_thread_ = std::thread([this] { loop(); });
  return "";
}

void ExtenderHttpServer::stop() {
  if (!started_) return;
  started_ = false;
  stop_.store(true);
  uint64_t one = 1;
  if (write(wake_fd_, &one, sizeof one) < 0) {
  }
  if (loop_thread_.joinable()) loop_thread_.join();
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    q_cv_.notify_all();
  }
  for (auto& t : workers_)
    if (t.joinable()) t.join();
  workers_.clear();
  {
    std::lock_guard<std::mutex> lk(park_mu_);
    parked_.clear();
  }
  {
    std::lock_guard<std::mutex> lk(conns_mu_);
    for (auto& kv : conns_) close(kv.first);
    conns_.clear();
  }
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    q_.clear();
  }
  close(listen_fd_);
  close(epoll_fd_);
  close(wake_fd_);
  listen_fd_ = epoll_fd_ = wake_fd_ = -1;
}

void ExtenderHttpServer::post(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    q_.push_back(std::move(fn));
  }
  q_cv_.notify_one();
}

void ExtenderHttpServer::worker() {
  for (;;) {
    std::function<void()> fn;
    {
      std::unique_lock<std::mutex> lk(q_mu_);
      q_cv_.wait(lk, [this] { return stop_.load() || !q_.empty(); });
      if (stop_.load()) return;
      fn = std::move(q_.front());
      q_.pop_front();
    }
    fn();
  }
}

void ExtenderHttpServer::loop() {
  std::vector<epoll_event> evs(256);
  int64_t next_sweep = mono_ns(), next_idle = mono_ns();
  while (!stop_.load()) {
    const int n = epoll_wait(epoll_fd_, evs.data(), static_cast<int>(evs.size()), 50);
    if (n < 0 && errno != EINTR) break;
    for (int i = 0; i < n; ++i) {
      const int fd = evs[i].data.fd;
      if (fd == wake_fd_) continue;
      if (fd == listen_fd_) {
        for (;;) {
          int cfd = accept4(listen_fd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (cfd < 0) break;
          int one = 1;
          setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
          auto c = std::make_shared<Conn>();
          c->fd = cfd;
          c->last_ns.store(mono_ns());
          c->state.store(kArmed);
          {
            std::lock_guard<std::mutex> lk(conns_mu_);
            conns_[cfd] = c;
          }
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP | EPOLLONESHOT;
          ev.data.fd = cfd;
          epoll_ctl(epoll_fd_, EPOLL_CTL_ADD, cfd, &ev);
        }
        continue;
      }
      ConnPtr c;
      {
        std::lock_guard<std::mutex> lk(conns_mu_);
        auto it = conns_.find(fd);
        if (it != conns_.end()) c = it->second;
      }
      if (!c) continue;
      int armed = kArmed;
      if (!c->state.compare_exchange_strong(armed, kOwned)) continue;
      post([this, c] { on_readable(c); });
    }
    const int64_t now = mono_ns();
    if (now >= next_sweep) {
      sweep_parked();
      next_sweep = now + 50 * 1000000LL;
    }
    if (now >= next_idle && opt_.idle_timeout_s > 0) {
      next_idle = now + 5 * 1000000000LL;
      std::vector<ConnPtr> idle;
      {
        std::lock_guard<std::mutex> lk(conns_mu_);
        for (auto& kv : conns_)
          if (kv.second->state.load() == kArmed &&
              now - kv.second->last_ns.load() > static_cast<int64_t>(opt_.idle_timeout_s) * 1000000000LL)
            idle.push_back(kv.second);
      }
      for (auto& c : idle) {
        int armed = kArmed;  // armed and no event consumed by this thread: nobody owns it
        if (c->state.compare_exchange_strong(armed, kOwned)) close_conn(c);
      }
    }
  }
}

void ExtenderHttpServer::rearm(const ConnPtr& c) {
  c->last_ns.store(mono_ns());
  c->state.store(kArmed);
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP | EPOLLONESHOT;
  ev.data.fd = c->fd;
  if (epoll_ctl(epoll_fd_, EPOLL_CTL_MOD, c->fd, &ev) != 0) {
    int armed = kArmed;
    if (c->state.compare_exchange_strong(armed, kOwned)) close_conn(c);
  }
}

void ExtenderHttpServer::close_conn(const ConnPtr& c) {
  if (c->fd < 0) return;
  epoll_ctl(epoll_fd_, EPOLL_CTL_DEL, c->fd, nullptr);
  {
    std::lock_guard<std::mutex> lk(conns_mu_);
    conns_.erase(c->fd);
  }
  close(c->fd);
  c->fd = -1;
}

// Decodes a complete chunked body out of `raw` (sets *done); false on a
// malformed stream.
static bool dechunk(const std::string& raw, std::string* out, bool* done, size_t* used) {
  size_t p = 0;
  out->clear();
  *done = false;
  for (;;) {
    const size_t eol = raw.find("\r\n", p);
    if (eol == std::string::npos) return true;
    char* endp = nullptr;
    const unsigned long long n = std::strtoull(raw.c_str() + p, &endp, 16);
    if (endp == raw.c_str() + p) return false;
    const size_t data = eol + 2;
    if (n == 0) {  // last chunk; trailers end with an empty line
      const size_t fin = raw.find("\r\n", data);
      if (fin == std::string::npos) return true;
      if (fin != data) {
        const size_t te = raw.find("\r\n\r\n", data);
        if (te == std::string::npos) return true;
        *used = te + 4;
      } else {
        *used = data + 2;
      }
      *done = true;
      return true;
    }
    if (raw.size() < data + n + 2) return true;
    out->append(raw, data, n);
    p = data + n + 2;
  }
}

bool ExtenderHttpServer::parse(Conn& c, HttpRequest* req, bool* bad) {
  if (!c.have_hdr) {
    const size_t end = c.hdr.find("\r\n\r\n");
    if (end == std::string::npos) {
      if (c.hdr.size() > kMaxHeader) *bad = true;
      return false;
    }
    const size_t l0 = c.hdr.find("\r\n");
    const std::string line = c.hdr.substr(0, l0);
    const size_t s1 = line.find(' '), s2 = line.rfind(' ');
    if (s1 == std::string::npos || s2 == s1) {
      *bad = true;
      return false;
    }
    c.method = line.substr(0, s1);
    c.target = line.substr(s1 + 1, s2 - s1 - 1);
    c.keep_alive = line.compare(s2 + 1, std::string::npos, "HTTP/1.0") != 0;
    c.chunked = false;
    c.content_length = 0;
    c.authorization.clear();
    bool expect = false;
    size_t p = l0 + 2;
    while (p < end) {
      size_t e = c.hdr.find("\r\n", p);
      if (e == std::string::npos || e > end) e = end;
      const size_t colon = c.hdr.find(':', p);
      if (colon != std::string::npos && colon < e) {
        size_t v = colon + 1;
        while (v < e && (c.hdr[v] == ' ' || c.hdr[v] == '\t')) ++v;
        const char* name = c.hdr.data() + p;
        const size_t nlen = colon - p;
        const std::string val = c.hdr.substr(v, e - v);
        if (ieq(name, nlen, "content-length")) c.content_length = std::strtoull(val.c_str(), nullptr, 10);
        else if (ieq(name, nlen, "transfer-encoding")) c.chunked = lower(val).find("chunked") != std::string::npos;
        else if (ieq(name, nlen, "connection")) {
          const std::string lv = lower(val);
          if (lv.find("close") != std::string::npos) c.keep_alive = false;
          else if (lv.find("keep-alive") != std::string::npos) c.keep_alive = true;
        } else if (ieq(name, nlen, "expect")) expect = lower(val).find("100-continue") != std::string::npos;
        else if (ieq(name, nlen, "authorization")) c.authorization = val;
      }
      p = e + 2;
    }
    if (c.content_length > opt_.max_body) {
      *bad = true;
      return false;
    }
    std::string rest = c.hdr.substr(end + 4);
    c.hdr.clear();
    c.have_hdr = true;
    c.body_got = 0;
    c.body.clear();
    c.chunk_raw.clear();
    if (c.chunked) {
      c.chunk_raw = std::move(rest);
    } else {
      c.body.resize(c.content_length);
      const size_t take = std::min(rest.size(), c.content_length);
      std::memcpy(&c.body[0], rest.data(), take);
      c.body_got = take;
      if (rest.size() > take) c.hdr.assign(rest, take, std::string::npos);  // a pipelined request
    }
    if (expect && (c.chunked || c.body_got < c.content_length)) {
      static const char k100[] = "HTTP/1.1 100 Continue\r\n\r\n";
      if (send(c.fd, k100, sizeof k100 - 1, MSG_NOSIGNAL) < 0) {
      }
    }
  }
  if (c.chunked) {
    bool done = false;
    size_t used = 0;
    std::string out;
    if (!dechunk(c.chunk_raw, &out, &done, &used) || c.chunk_raw.size() > opt_.max_body) {
      *bad = true;
      return false;
    }
    if (!done) return false;
    c.hdr.assign(c.chunk_raw, used, std::string::npos);
    c.chunk_raw.clear();
    c.body = std::move(out);
  } else if (c.body_got < c.content_length) {
    return false;
  }
  req->method = c.method;
  const size_t q = c.target.find('?');
  req->path = c.target.substr(0, q);
  req->query = q == std::string::npos ? "" : c.target.substr(q + 1);
  req->body = std::move(c.body);
  req->authorization = c.authorization;
  c.body.clear();
  c.have_hdr = false;
  return true;
}

void ExtenderHttpServer::on_readable(const ConnPtr& c) {
  char tmp[16384];
  for (;;) {
    HttpRequest req;
    bool bad = false;
    const bool full = parse(*c, &req, &bad);
    if (bad) {
      HttpResponse r;
      r.code = 400;
      r.body = error_json("bad request");
      c->keep_alive = false;
      reply(c, r);
      close_conn(c);
      return;
    }
    if (full) {
      requests_.fetch_add(1, std::memory_order_relaxed);
      if (!dispatch(c, req, mono_ns())) return;  // parked: whoever finishes it continues
      if (req.body.capacity() > c->body.capacity()) {  // keep the (multi-MB) buffer for the next request
        req.body.clear();
        c->body.swap(req.body);
      }
      if (!c->keep_alive || c->dead) {
        close_conn(c);
        return;
      }
      continue;
    }
    ssize_t r;
    const bool in_body = c->have_hdr && !c->chunked;
    if (in_body) r = recv(c->fd, &c->body[c->body_got], c->content_length - c->body_got, 0);
    else r = recv(c->fd, tmp, sizeof tmp, 0);
    if (r > 0) {
      if (in_body) c->body_got += static_cast<size_t>(r);
      else (c->have_hdr ? c->chunk_raw : c->hdr).append(tmp, static_cast<size_t>(r));
      continue;
    }
    if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)) {
      close_conn(c);
      return;
    }
    if (errno == EINTR) continue;
    if (c->have_hdr) {  // a body is streaming in: wait for it here
      pollfd pf{c->fd, POLLIN, 0};
      if (poll(&pf, 1, 20) > 0) continue;
    }
    rearm(c);
    return;
  }
}

bool ExtenderHttpServer::reply(const ConnPtr& c, const HttpResponse& r) {
  char head[256];
  const int hn = std::snprintf(head, sizeof head,
                               "HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %zu\r\nConnection: %s\r\n\r\n",
                               r.code, reason_of(r.code), r.ctype.c_str(), r.body.size(),
                               c->keep_alive ? "keep-alive" : "close");
  iovec iov[2] = {{head, static_cast<size_t>(hn)}, {const_cast<char*>(r.body.data()), r.body.size()}};
  int idx = 0;
  const int64_t give_up = mono_ns() + 30LL * 1000000000LL;
  while (idx < 2) {
    if (iov[idx].iov_len == 0) {
      ++idx;
      continue;
    }
    msghdr mh{};
    mh.msg_iov = &iov[idx];
    mh.msg_iovlen = static_cast<size_t>(2 - idx);
    ssize_t w = sendmsg(c->fd, &mh, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        pollfd pf{c->fd, POLLOUT, 0};
        if (mono_ns() < give_up && poll(&pf, 1, 1000) >= 0) continue;
      }
      c->dead = true;
      return false;
    }
    size_t left = static_cast<size_t>(w);
    while (idx < 2 && left > 0) {
      const size_t take = std::min(left, iov[idx].iov_len);
      iov[idx].iov_base = static_cast<char*>(iov[idx].iov_base) + take;
      iov[idx].iov_len -= take;
      left -= take;
      if (iov[idx].iov_len == 0) ++idx;
    }
  }
  return true;
}

void ExtenderHttpServer::record(const char* verb, int64_t t0_ns) {
  const uint64_t us = static_cast<uint64_t>(std::max<int64_t>(0, (mono_ns() - t0_ns) / 1000));
  LatencyHistogram* h = &h_other_;
  switch (verb[0]) {
    case 'f': h = &h_filter_; break;
    case 'b': h = std::strcmp(verb, "bind") == 0 ? &h_bind_ : &h_bind_held_; break;
    case 'p': h = verb[2] == 'i' ? &h_prioritize_ : &h_preempt_; break;
    default: break;
  }
  h->record_us(us);
}

bool ExtenderHttpServer::dispatch(const ConnPtr& c, HttpRequest& req, int64_t t_read_ns) {
  const std::string& path = req.path;
  if (req.method == "POST" && !verbs_via_fallback_.load() && path.size() > opt_.prefix.size() &&
      path.compare(0, opt_.prefix.size(), opt_.prefix) == 0 && path[opt_.prefix.size()] == '/') {
    const std::string verb = path.substr(opt_.prefix.size() + 1);
    const bool is_filter = verb == "filter", is_prio = verb == "prioritize", is_pre = verb == "preempt";
    if (is_filter || is_prio || is_pre) {
      std::string out;
      try {
        out = is_filter ? plat_->filter(req.body) : is_prio ? plat_->prioritize(req.body) : plat_->preempt(req.body);
      } catch (const std::exception& e) {
        out = error_json(e.what());
      }
      reply_json(c, out);
      record(verb.c_str(), t_read_ns);
      return true;
    }
    if (verb == "bind") return handle_bind(c, req.body, t_read_ns, false);
  }
  if (req.method == "GET" || req.method == "HEAD") {
    HttpResponse r;
    r.ctype = "text/plain";
    if (path == "/healthz" || path == "/health") {
      r.body = "ok";
      reply(c, r);
      return true;
    }
    if (path == "/readyz") {
      // Only the lease holder is Ready, so the Service routes extender verbs
      // and agent pushes to the one replica whose ledger is authoritative.
      if (ready_.load()) r.body = "ok";
      else {
        r.code = 503;
        r.body = "standby";
      }
      reply(c, r);
      return true;
    }
    if (path == "/metrics") {
      r.ctype = "text/plain; version=0.0.4";
      r.body = plat_->expose_metrics();
      reply(c, r);
      record("other", t_read_ns);
      return true;
    }
  }
  HttpResponse r;
  if (fallback_) {
    try {
      r = fallback_(req);
    } catch (const std::exception& e) {
      r.code = 500;
      r.body = error_json(e.what());
    }
  } else {
    r.code = 404;
    r.body = "{\"error\":\"not found\"}";
  }
  reply(c, r);
  record("other", t_read_ns);
  return true;
}

bool ExtenderHttpServer::handle_bind(const ConnPtr& c, const std::string& body, int64_t t_read_ns, bool held) {
  Platform::BindOutcome bo;
  try {
    bo = plat_->bind_outcome(body);
    if (bo.unknown_pod && lookup_) {  // the extender restarted between this pod's verbs
      const std::string pod = lookup_(bo.ns, bo.name);
      if (!pod.empty()) bo = plat_->bind_outcome(body, pod);
    }
  } catch (const std::exception& e) {
    bo = Platform::BindOutcome();
    bo.error = e.what();
  }
  if (bo.waiting && !held && opt_.gang_hold_ms > 0) {
    Parked p;
    p.conn = c;
    p.body = body;
    p.uid = bo.uid;
    p.t_read_ns = t_read_ns;
    p.deadline_ns = mono_ns() + static_cast<int64_t>(opt_.gang_hold_ms) * 1000000LL;
    c->state.store(kParked);
    {
      std::lock_guard<std::mutex> lk(park_mu_);
      parked_[bo.gang].push_back(std::move(p));
    }
    held_total_.fetch_add(1, std::memory_order_relaxed);
    // The gang's last member may have completed it between our bind and the
    // parking: then nobody will come for this request.
    if (plat_->scheduler()->permit(bo.uid) != "Allow") return false;
    bool mine = false;
    {
      std::lock_guard<std::mutex> lk(park_mu_);
      auto it = parked_.find(bo.gang);
      if (it != parked_.end()) {
        auto& v = it->second;
        for (auto pi = v.begin(); pi != v.end(); ++pi)
          if (pi->conn == c) {
            v.erase(pi);
            mine = true;
            break;
          }
        if (v.empty()) parked_.erase(it);
      }
    }
    if (!mine) return false;  // the completing bind took it
    c->state.store(kOwned);
    return handle_bind(c, body, t_read_ns, true);
  }
  std::string out = "{}";
  if (bo.ok) {
    // Held members first: their apiserver writes then run beside this one.
    if (!bo.gang.empty()) finish_gang(bo.gang);
    if (sink_) {
      std::string err;
      try {
        err = sink_(body, bo.json);
      } catch (const std::exception& e) {
        err = e.what();
      }
      if (!err.empty()) {
        try {
          plat_->release(bo.uid, wall_now_s());
        } catch (...) {
        }
        out = error_json("binding failed: " + err);
      }
    }
  } else {
    out = error_json(bo.error.empty() ? "bind failed" : bo.error);
  }
  reply_json(c, out);
  record(held ? "bind_held" : "bind", t_read_ns);
  return true;
}

void ExtenderHttpServer::finish_gang(const std::string& gang) {
  std::vector<Parked> take;
  {
    std::lock_guard<std::mutex> lk(park_mu_);
    auto it = parked_.find(gang);
    if (it == parked_.end()) return;
    take = std::move(it->second);
    parked_.erase(it);
  }
  for (auto& p : take) {
    ConnPtr c = p.conn;
    std::string body = std::move(p.body);
    const int64_t t0 = p.t_read_ns;
    c->state.store(kOwned);
    post([this, c, body, t0] {
      handle_bind(c, body, t0, true);
      if (!c->keep_alive || c->dead) close_conn(c);
      else on_readable(c);
    });
  }
}

void ExtenderHttpServer::sweep_parked() {
  {
    std::lock_guard<std::mutex> lk(park_mu_);
    if (parked_.empty()) return;
  }
  // Gang reservations older than the gang timeout are dropped here as well
  // as in the platform's tick, so a held bind hears of it within one sweep.
  plat_->scheduler()->expire_gangs();
  std::vector<std::pair<Parked, int>> out;  // 0: hold expired, 1: gang gone, 2: gang ready
  const int64_t now = mono_ns();
  {
    std::lock_guard<std::mutex> lk(park_mu_);
    for (auto it = parked_.begin(); it != parked_.end();) {
      auto& v = it->second;
      for (auto pi = v.begin(); pi != v.end();) {
        const std::string verdict = plat_->scheduler()->permit(pi->uid);
        int why = -1;
        if (verdict == "Reject") why = 1;
        else if (verdict == "Allow") why = 2;
        else if (now >= pi->deadline_ns) why = 0;
        if (why >= 0) {
          out.emplace_back(std::move(*pi), why);
          pi = v.erase(pi);
        } else {
          ++pi;
        }
      }
      it = v.empty() ? parked_.erase(it) : std::next(it);
    }
  }
  for (auto& pw : out) {
    ConnPtr c = pw.first.conn;
    std::string body = std::move(pw.first.body);
    const int64_t t0 = pw.first.t_read_ns;
    const int why = pw.second;
    c->state.store(kOwned);
    if (why != 2) held_timeouts_.fetch_add(1, std::memory_order_relaxed);
    post([this, c, body, t0, why] {
      if (why == 2) {
        handle_bind(c, body, t0, true);
      } else {
        reply_json(c, error_json(why == 1 ? "gang timed out: reservation released"
                                          : "gang still waiting for members"));
        record("bind_held", t0);
      }
      if (!c->keep_alive || c->dead) close_conn(c);
      else on_readable(c);
    });
  }
}

size_t ExtenderHttpServer::parked() const {
  std::lock_guard<std::mutex> lk(park_mu_);
  size_t n = 0;
  for (const auto& kv : parked_) n += kv.second.size();
  return n;
}

const LatencyHistogram& ExtenderHttpServer::verb_histogram(const std::string& verb) const {
  if (verb == "filter") return h_filter_;
  if (verb == "prioritize") return h_prioritize_;
  if (verb == "bind") return h_bind_;
  if (verb == "bind_held") return h_bind_held_;
  if (verb == "preempt") return h_preempt_;
  return h_other_;
}

std::string ExtenderHttpServer::stats_json() const {
  Json verbs = Json::object();
  for (const char* v : {"filter", "prioritize", "bind", "bind_held", "preempt", "other"}) {
    const LatencyHistogram& h = verb_histogram(v);
    if (h.count() == 0) continue;
    Json j = Json::object();
    j["count"] = static_cast<int64_t>(h.count());
    j["p50_ms"] = h.quantile_ms(0.50);
    j["p99_ms"] = h.quantile_ms(0.99);
    j["mean_ms"] = h.mean_ms();
    j["max_ms"] = h.max_ms();
    verbs[v] = j;
  }
  Json out = Json::object();
  out["verbs"] = verbs;
  {
    std::lock_guard<std::mutex> lk(conns_mu_);
    out["connections"] = static_cast<int64_t>(conns_.size());
  }
  out["requests"] = static_cast<int64_t>(requests_.load());
  out["parked"] = static_cast<int64_t>(parked());
  out["gang_binds_held"] = static_cast<int64_t>(held_total_.load());
  out["gang_binds_timed_out"] = static_cast<int64_t>(held_timeouts_.load());
  out["workers"] = static_cast<int64_t>(opt_.workers);
  return out.dump();
}

}  // namespace kgwe
