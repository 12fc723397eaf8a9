#include "http_client.h"

#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace kgwe {

HttpClient::HttpClient(std::string host, int port, double timeout_s)
    : host_(std::move(host)), port_(port), timeout_s_(timeout_s) {}

HttpClient::~HttpClient() { close_(); }

void HttpClient::close_() {
  if (fd_ >= 0) close(fd_);
  fd_ = -1;
  buf_.clear();
}

bool HttpClient::connect_() {
  close_();
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  if (getaddrinfo(host_.c_str(), std::to_string(port_).c_str(), &hints, &res) != 0) return false;
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    int fd = socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    timeval tv{};
    tv.tv_sec = static_cast<time_t>(timeout_s_);
    tv.tv_usec = static_cast<suseconds_t>((timeout_s_ - static_cast<double>(tv.tv_sec)) * 1e6);
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    if (connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) {
      fd_ = fd;
      break;
    }
    close(fd);
  }
  freeaddrinfo(res);
  return fd_ >= 0;
}

bool HttpClient::send_all(const std::string& head, const std::vector<std::string_view>& parts) {
  std::vector<iovec> iov;
  iov.reserve(parts.size() + 1);
  iov.push_back({const_cast<char*>(head.data()), head.size()});
  for (const auto& p : parts)
    if (!p.empty()) iov.push_back({const_cast<char*>(p.data()), p.size()});
  size_t idx = 0;
  while (idx < iov.size()) {
    msghdr mh{};
    mh.msg_iov = &iov[idx];
    mh.msg_iovlen = std::min<size_t>(iov.size() - idx, 1024);
    ssize_t w = sendmsg(fd_, &mh, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    size_t left = static_cast<size_t>(w);
    while (idx < iov.size() && left > 0) {
      const size_t take = std::min(left, iov[idx].iov_len);
      iov[idx].iov_base = static_cast<char*>(iov[idx].iov_base) + take;
      iov[idx].iov_len -= take;
      left -= take;
      if (iov[idx].iov_len == 0) ++idx;
    }
    while (idx < iov.size() && iov[idx].iov_len == 0) ++idx;
  }
  return true;
}

bool HttpClient::read_reply(int* status, std::string* body, bool* got_any) {
  std::string& b = buf_;
  size_t hend;
  char tmp[16384];
  while ((hend = b.find("\r\n\r\n")) == std::string::npos) {
    ssize_t r = recv(fd_, tmp, sizeof tmp, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    *got_any = true;
    b.append(tmp, static_cast<size_t>(r));
    if (b.size() > (1u << 20)) return false;
  }
  *status = std::atoi(b.c_str() + b.find(' ') + 1);
  size_t clen = 0;
  bool close_after = false;
  size_t p = b.find("\r\n") + 2;
  while (p < hend) {
    size_t e = b.find("\r\n", p);
    if (e == std::string::npos || e > hend) e = hend;
    std::string line = b.substr(p, e - p);
    for (auto& ch : line) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
    if (line.compare(0, 15, "content-length:") == 0) clen = std::strtoull(line.c_str() + 15, nullptr, 10);
    else if (line.compare(0, 11, "connection:") == 0 && line.find("close") != std::string::npos) close_after = true;
    p = e + 2;
  }
  const size_t have = b.size() - (hend + 4);
  body->clear();
  body->resize(clen);
  const size_t take = std::min(have, clen);
  std::memcpy(&(*body)[0], b.data() + hend + 4, take);
  std::string rest = have > take ? b.substr(hend + 4 + take) : std::string();
  size_t got = take;
  while (got < clen) {
    ssize_t r = recv(fd_, &(*body)[got], clen - got, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    got += static_cast<size_t>(r);
  }
  b = std::move(rest);
  if (close_after) close_();
  return true;
}

int HttpClient::post(const std::string& path, const std::vector<std::string_view>& parts, std::string* body) {
  size_t n = 0;
  for (const auto& p : parts) n += p.size();
  const std::string head = "POST " + path + " HTTP/1.1\r\nHost: " + host_ + ":" + std::to_string(port_) +
                           "\r\nContent-Type: application/json\r\nContent-Length: " + std::to_string(n) +
                           "\r\nConnection: keep-alive\r\n\r\n";
  for (int attempt = 0; attempt < 2; ++attempt) {
    const bool fresh = fd_ < 0;
    if (fresh && !connect_()) throw std::runtime_error("connect " + host_ + ":" + std::to_string(port_) + " failed");
    int status = 0;
    bool got_any = false;
    if (send_all(head, parts) && read_reply(&status, body, &got_any)) return status;
    close_();
    // A kept-alive connection the server closed while idle: retry once on a
    // new one, unless part of a reply had already arrived.
    if (fresh || got_any) break;
  }
  throw std::runtime_error("POST " + path + " to " + host_ + ":" + std::to_string(port_) + " failed");
}

}  // namespace kgwe
