// Native HTTP/1.1 keep-alive load generator for the Seldon predict() endpoint
// (bench/rest_native.py): `conns` connections, one request in flight on each, the same
// POST body repeated for `seconds`; returns throughput and latency percentiles.  A Python
// client tops out far below what the native server sustains, so the measurement is native too.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct C {
  int fd = -1;
  std::string in;
  size_t sent = 0;
  int64_t t0 = 0;
};

}  // namespace

namespace {

struct Result {
  std::vector<float> lat;
  uint64_t errors = 0;
  int64_t last_done = 0;
  bool ok = true;
};

void run_conns(const std::string& req, const char* host, int port, int nconn, int64_t start, int64_t end, Result* res) {
  const int efd = epoll_create1(0);
  std::vector<C> cs(nconn);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = inet_addr(host);
  for (int i = 0; i < nconn; ++i) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) { ::close(fd); res->ok = false; break; }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    cs[i].fd = fd;
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u32 = (uint32_t)i;
    epoll_ctl(efd, EPOLL_CTL_ADD, fd, &ev);
  }
  res->lat.reserve(1 << 20);
  res->last_done = start;
  auto send_req = [&](C& c) {
    c.t0 = now_ns();
    size_t off = 0;
    while (off < req.size()) {
      const ssize_t w = ::send(c.fd, req.data() + off, req.size() - off, MSG_NOSIGNAL);
      if (w <= 0) return false;
      off += (size_t)w;
    }
    return true;
  };
  if (res->ok)
    for (auto& c : cs) send_req(c);
  std::vector<epoll_event> evs(1024);
  char buf[65536];
  while (res->ok && now_ns() < end) {
    const int n = epoll_wait(efd, evs.data(), (int)evs.size(), 100);
    for (int i = 0; i < n; ++i) {
      C& c = cs[evs[i].data.u32];
      const ssize_t r = ::recv(c.fd, buf, sizeof buf, 0);
      if (r <= 0) { ++res->errors; continue; }
      c.in.append(buf, (size_t)r);
      for (;;) {
        const size_t he = c.in.find("\r\n\r\n");
        if (he == std::string::npos) break;
        const char* cl = strcasestr(c.in.c_str(), "content-length:");
        const size_t blen = cl ? (size_t)std::strtoull(cl + 15, nullptr, 10) : 0;
        if (c.in.size() < he + 4 + blen) break;
        if (std::strncmp(c.in.c_str(), "HTTP/1.1 200", 12) != 0) ++res->errors;
        c.in.erase(0, he + 4 + blen);
        const int64_t t = now_ns();
        res->lat.push_back((float)((t - c.t0) * 1e-3));
        res->last_done = t;
        if (t < end) send_req(c);
      }
    }
  }
  for (auto& c : cs) if (c.fd >= 0) ::close(c.fd);
  ::close(efd);
}

}  // namespace

// `nconn` connections spread over `threads` client threads (threads <= 0: one per 64 conns).
extern "C" int ccfd_http_load(const char* host, int port, const char* path, const char* body, int body_len,
                              int nconn, double seconds, double* out, int threads) {
  char hdr[512];
  const int hn = std::snprintf(hdr, sizeof hdr,
                               "POST %s HTTP/1.1\r\nHost: %s\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n",
                               path, host, body_len);
  std::string req(hdr, hn);
  req.append(body, body_len);
  if (threads <= 0) threads = std::max(1, std::min(16, (nconn + 63) / 64));
  threads = std::min(threads, nconn);
  const int64_t start = now_ns(), end = start + (int64_t)(seconds * 1e9);
  std::vector<Result> rs(threads);
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) {
    const int nc = nconn / threads + (t < nconn % threads ? 1 : 0);
    th.emplace_back(run_conns, std::cref(req), host, port, nc, start, end, &rs[t]);
  }
  for (auto& x : th) x.join();
  std::vector<float> lat;
  uint64_t errors = 0;
  int64_t last_done = start;
  for (auto& r : rs) {
    if (!r.ok) return -1;
    lat.insert(lat.end(), r.lat.begin(), r.lat.end());
    errors += r.errors;
    last_done = std::max(last_done, r.last_done);
  }
  const double el = (last_done - start) * 1e-9;
  std::sort(lat.begin(), lat.end());
  auto pct = [&](double q) { return lat.empty() ? 0.0 : (double)lat[std::min(lat.size() - 1, (size_t)(q * lat.size()))]; };
  out[0] = el > 0 ? lat.size() / el : 0.0;
  out[1] = pct(0.50);
  out[2] = pct(0.99);
  out[3] = (double)errors;
  out[4] = (double)lat.size();
  return 0;
}
