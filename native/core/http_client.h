// Minimal blocking HTTP/1.1 keep-alive client (POST only): what a compiled
// kube-scheduler's extender client does, for the scheduler stand-in and the
// benchmarks.  The request body is written from several buffers with one
// gather write (ExtenderArgs = prefix + cached Node objects + suffix are never
// joined), the reply is read into one buffer.
#pragma once
#include <string>
#include <string_view>
#include <vector>

namespace kgwe {

class HttpClient {
 public:
  HttpClient(std::string host, int port, double timeout_s = 30.0);
  ~HttpClient();
  HttpClient(const HttpClient&) = delete;
  HttpClient& operator=(const HttpClient&) = delete;

  // POST `parts` (concatenated) to `path`; returns the status code and fills
  // *body.  Throws std::runtime_error on a transport failure (after one
  // reconnect-and-retry when a kept-alive connection turned out closed).
  int post(const std::string& path, const std::vector<std::string_view>& parts, std::string* body);

 private:
  bool connect_();
  void close_();
  bool send_all(const std::string& head, const std::vector<std::string_view>& parts);
  bool read_reply(int* status, std::string* body, bool* got_any);

  std::string host_;
  int port_;
  double timeout_s_;
  int fd_ = -1;
  std::string buf_;  // bytes read past the previous reply (none with a well-behaved server)
};

}  // namespace kgwe
