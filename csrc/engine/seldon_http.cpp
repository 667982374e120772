// Native Seldon v0.1 REST front end (the reference's model endpoint: deploy/model/
// modelfull.json:37-44, POST {SELDON_URL}/{SELDON_ENDPOINT} from deploy/router.yaml:65-68,
// README.md:379 for the KIE `predict` default).
//
// One epoll thread per server speaks HTTP/1.1 keep-alive.  Every predict request that is
// complete after one wake-up is parsed straight into a shared row block and the whole block is
// scored with ONE call -- the GPU engine's synchronous path (H2D, fused kernel, D2H) or a
// caller-supplied scorer -- so concurrent clients are batched dynamically without any timer:
// the batch is simply whatever arrived while the previous batch was on the GPU.  Responses
// are formatted in C++; /prometheus and /metrics are rendered by a callback (the Python
// exporter with the reference metric names), health routes answer locally.
//
// Protocol (contracts/seldon.py): request {"data":{"names":[..],"ndarray":[[..],..]}} or
// {"data":{"tensor":{"shape":[n,30],"values":[..]}}}; response {"meta":{..},"data":{"names":
// ["proba_0","proba_1"],"ndarray":[[p0,p1],..]}} (tensor in, tensor out).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>
#include <fcntl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../include/ccfd_abi.h"
#include "json_num.h"

extern "C" int ccfd_engine_score_sync(void* eng, const float* x, int32_t n, float* proba_out, uint8_t* route_out);

namespace {

constexpr int kF = CCFD_N_FEATURES;
constexpr int kLatBuckets = 32;               // upper bounds supplied by the caller (seconds)
constexpr size_t kMaxBody = 64u << 20;        // 413 above this (a predict body is ~1 KB per row)
constexpr int64_t kMaxRows = 1 << 24;         // tensor shape entries above this are invalid
constexpr size_t kMaxHeader = 64u << 10;      // a request head longer than this closes the connection

typedef int (*score_fn)(const float* rows, int32_t n, float* proba, void* ctx);
typedef int32_t (*render_fn)(char* buf, int32_t cap, void* ctx);

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// ------------------------------------------------------------------ minimal JSON reader
struct Cur {
  const char* p;
  const char* e;
  void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; }
  bool eat(char c) { ws(); if (p < e && *p == c) { ++p; return true; } return false; }
  bool peek(char c) { ws(); return p < e && *p == c; }
};

bool parse_num(Cur& c, float* out) {
  c.ws();
  double d;
  if (!ccfd::json::parse_number(c.p, c.e, &d)) return false;
  *out = (float)d;                  // decimal -> double -> float, as json.loads + float32 in Python
  return true;
}

bool parse_str(Cur& c, std::string* out) {
  if (!c.eat('"')) return false;
  const char* b = c.p;
  while (c.p < c.e && *c.p != '"') { if (*c.p == '\\') ++c.p; ++c.p; }
  if (c.p >= c.e) return false;
  if (out) out->assign(b, c.p - b);
  ++c.p;
  return true;
}

bool skip_val(Cur& c, int depth = 0) {
  if (depth > 32) return false;
  c.ws();
  if (c.p >= c.e) return false;
  if (*c.p == '"') return parse_str(c, nullptr);
  if (*c.p == '{' || *c.p == '[') {
    const char close = *c.p == '{' ? '}' : ']';
    const bool obj = *c.p == '{';
    ++c.p;
    if (c.eat(close)) return true;
    for (;;) {
      if (obj) { if (!parse_str(c, nullptr) || !c.eat(':')) return false; }
      if (!skip_val(c, depth + 1)) return false;
      if (c.eat(',')) continue;
      return c.eat(close);
    }
  }
  while (c.p < c.e && *c.p != ',' && *c.p != '}' && *c.p != ']') ++c.p;   // number / literal
  return true;
}

// flat array of numbers -> out; returns count or -1
int parse_num_array(Cur& c, std::vector<float>& out) {
  if (!c.eat('[')) return -1;
  int n = 0;
  if (c.eat(']')) return 0;
  for (;;) {
    float v;
    if (!parse_num(c, &v)) return -1;
    out.push_back(v);
    ++n;
    if (c.eat(',')) continue;
    return c.eat(']') ? n : -1;
  }
}

int feature_col(const std::string& k) {
  if (k == "Time") return 0;
  if (k == "Amount") return kF - 1;
  if ((k.size() == 2 || k.size() == 3) && k[0] == 'V') {
    int v = 0;
    for (size_t i = 1; i < k.size(); ++i) { if (!std::isdigit((unsigned char)k[i])) return -1; v = v * 10 + (k[i] - '0'); }
    return (v >= 1 && v <= 28) ? v : -1;
  }
  return -1;
}

// Parse a Seldon request body; appends n rows x 30 to `rows`.  Returns n or -1 (err set).
int parse_seldon(const char* b, size_t len, std::vector<float>& rows, bool* tensor, std::string* err) {
  Cur c{b, b + len};
  std::vector<float> vals;
  std::vector<std::string> names;
  int shape0 = -1, shape1 = -1, ncols = -1, nrows = 0;
  bool have = false;
  *tensor = false;
  if (!c.eat('{')) { *err = "invalid JSON"; return -1; }
  bool found_data = false;
  while (!c.peek('}')) {
    std::string key;
    if (!parse_str(c, &key) || !c.eat(':')) { *err = "invalid JSON"; return -1; }
    if (key != "data") { if (!skip_val(c)) { *err = "invalid JSON"; return -1; } }
    else {
      found_data = true;
      if (!c.eat('{')) { *err = "'data' must be an object"; return -1; }
      while (!c.peek('}')) {
        std::string k2;
        if (!parse_str(c, &k2) || !c.eat(':')) { *err = "invalid JSON"; return -1; }
        if (k2 == "names") {
          if (!c.eat('[')) { *err = "names must be an array"; return -1; }
          if (!c.eat(']')) for (;;) {
            std::string nm;
            if (!parse_str(c, &nm)) { *err = "invalid names"; return -1; }
            names.push_back(nm);
            if (c.eat(',')) continue;
            if (!c.eat(']')) { *err = "invalid names"; return -1; }
            break;
          }
        } else if (k2 == "ndarray") {
          if (!c.eat('[')) { *err = "ndarray must be an array"; return -1; }
          if (c.peek('[')) {                       // [[..],[..]]
            for (;;) {
              const int m = parse_num_array(c, vals);
              if (m < 0) { *err = "ndarray rows must be numbers"; return -1; }
              if (ncols < 0) ncols = m;
              else if (m != ncols) { *err = "ragged ndarray"; return -1; }
              ++nrows;
              if (c.eat(',')) continue;
              if (!c.eat(']')) { *err = "invalid ndarray"; return -1; }
              break;
            }
          } else {                                  // one flat row: [x0, x1, ...]
            int m = 0;
            if (!c.eat(']')) for (;;) {
              float v;
              if (!parse_num(c, &v)) { *err = "invalid ndarray"; return -1; }
              vals.push_back(v);
              ++m;
              if (c.eat(',')) continue;
              if (!c.eat(']')) { *err = "invalid ndarray"; return -1; }
              break;
            }
            ncols = m; nrows = 1;
          }
          have = true;
        } else if (k2 == "tensor") {
          *tensor = true;
          if (!c.eat('{')) { *err = "tensor must be an object"; return -1; }
          while (!c.peek('}')) {
            std::string k3;
            if (!parse_str(c, &k3) || !c.eat(':')) { *err = "invalid JSON"; return -1; }
            if (k3 == "shape") {
              std::vector<float> sh;
              if (parse_num_array(c, sh) < 1) { *err = "invalid shape"; return -1; }
              // range-check before the float->int conversion (no UB on 1e300 / NaN / -5)
              for (double d : sh)
                if (!(d >= 0.0 && d <= (double)kMaxRows) || d != (double)(int64_t)d) { *err = "invalid shape"; return -1; }
              shape0 = (int)sh[0]; shape1 = sh.size() > 1 ? (int)sh[1] : 1;
            } else if (k3 == "values") {
              if (parse_num_array(c, vals) < 0) { *err = "invalid values"; return -1; }
            } else if (!skip_val(c)) { *err = "invalid JSON"; return -1; }
            if (!c.eat(',')) break;
          }
          if (!c.eat('}')) { *err = "invalid tensor"; return -1; }
          if (shape0 < 0 || (int64_t)shape0 * shape1 != (int64_t)vals.size()) { *err = "tensor shape/values mismatch"; return -1; }
          if (shape1 == 1 && shape0 == kF) { shape1 = kF; shape0 = 1; }
          nrows = shape0; ncols = shape1;
          have = true;
        } else if (!skip_val(c)) { *err = "invalid JSON"; return -1; }
        if (!c.eat(',')) break;
      }
      if (!c.eat('}')) { *err = "invalid data object"; return -1; }
    }
    if (!c.eat(',')) break;
  }
  if (!found_data) { *err = "request must carry a 'data' object"; return -1; }
  if (!have) { *err = "data must contain 'ndarray' or 'tensor'"; return -1; }
  if (ncols != kF) { *err = "expected 30 features"; return -1; }
  // named columns in another order are re-ordered to Time, V1..V28, Amount
  int perm[kF];
  bool reorder = false;
  if ((int)names.size() == kF) {
    bool ok = true;
    for (int j = 0; j < kF; ++j) { perm[j] = feature_col(names[j]); if (perm[j] < 0) ok = false; if (perm[j] != j) reorder = true; }
    if (!ok) reorder = false;
  }
  const size_t base = rows.size();
  rows.resize(base + (size_t)nrows * kF);
  float* dst = rows.data() + base;
  for (int r = 0; r < nrows; ++r)
    for (int j = 0; j < kF; ++j) dst[(size_t)r * kF + (reorder ? perm[j] : j)] = vals[(size_t)r * kF + j];
  return nrows;
}

// ------------------------------------------------------------------ server
struct Pending {
  int fd;
  size_t row0;
  int nrows;
  bool tensor;
  bool close_after;
  int64_t t0;
};

struct Conn {
  std::string in;
  std::string out;
  size_t out_off = 0;
  bool closing = false;
  // a predict is being scored: later pipelined requests stay buffered until its response
  // is queued, so responses leave in request order (HTTP/1.1 pipelining)
  bool predict_pending = false;
  bool peer_closed = false;    // peer half-closed: answer what is buffered, then drop
  bool parsed_all = false;     // the last parse consumed every complete request in `in`
};

constexpr int kNStatus = 4;

struct Stats {
  std::atomic<uint64_t> count[kNStatus];          // 200, 4xx (not 401), 401, 5xx
  std::atomic<uint64_t> sum_ns[kNStatus];
  std::atomic<uint64_t> hist[kNStatus][kLatBuckets + 1];
  std::atomic<uint64_t> rows, batches, model_ns;
  std::atomic<uint64_t> last_bits[4];             // proba_1, Amount, V17, V10 (f32 bits)
};

struct Server {
  int lfd = -1, efd = -1, port = 0;
  std::thread th;
  std::atomic<bool> stop{false};
  void* engine = nullptr;
  score_fn scorer = nullptr;
  void* score_ctx = nullptr;
  render_fn render = nullptr;
  void* render_ctx = nullptr;
  std::string model, token;
  int max_batch = 65536;
  double bounds[kLatBuckets];
  int nbounds = 0;
  Stats* stp = nullptr;                           // shared by the workers of one server group
  std::unordered_map<int, Conn> conns;
  uint64_t puid = 0;                              // worker index in the top byte

  int status_idx(int code) { return code == 200 ? 0 : code == 401 ? 2 : code >= 500 ? 3 : 1; }
  void observe(int code, int64_t dt_ns) {
    const int s = status_idx(code);
    stp->count[s].fetch_add(1, std::memory_order_relaxed);
    stp->sum_ns[s].fetch_add((uint64_t)dt_ns, std::memory_order_relaxed);
    const double sec = dt_ns * 1e-9;
    int b = 0;
    while (b < nbounds && sec > bounds[b]) ++b;
    stp->hist[s][b].fetch_add(1, std::memory_order_relaxed);
  }

  void queue(int fd, int code, const char* ctype, const std::string& body, bool close_after) {
    auto it = conns.find(fd);
    if (it == conns.end()) return;
    char hdr[256];
    const char* reason = code == 200 ? "OK" : code == 400 ? "Bad Request" : code == 401 ? "Unauthorized" :
                         code == 404 ? "Not Found" : code == 413 ? "Payload Too Large" :
                         code == 500 ? "Internal Server Error" : code == 503 ? "Service Unavailable" : "Error";
    const int n = std::snprintf(hdr, sizeof hdr, "HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %zu\r\n%s\r\n",
                                code, reason, ctype, body.size(), close_after ? "Connection: close\r\n" : "");
    it->second.out.append(hdr, n);
    it->second.out.append(body);
    if (close_after) it->second.closing = true;
  }

  static std::string error_json(int code, const std::string& why) {
    std::string s = "{\"status\":{\"code\":" + std::to_string(code) + ",\"info\":\"";
    for (char ch : why) s += (ch == '"' || ch == '\\') ? ' ' : ch;
    return s + "\",\"reason\":\"MICROSERVICE_BAD_DATA\",\"status\":\"FAILURE\"}}";
  }

  void flush(int fd) {
    auto it = conns.find(fd);
    if (it == conns.end()) return;
    Conn& c = it->second;
    while (c.out_off < c.out.size()) {
      const ssize_t w = ::send(fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
      if (w > 0) { c.out_off += (size_t)w; continue; }
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        epoll_event ev{};
        ev.events = c.peer_closed ? EPOLLOUT : (EPOLLIN | EPOLLOUT);
        ev.data.fd = fd;
        epoll_ctl(efd, EPOLL_CTL_MOD, fd, &ev);
        return;
      }
      drop(fd);
      return;
    }
    c.out.clear();
    c.out_off = 0;
    if (c.closing || (c.peer_closed && !c.predict_pending && c.parsed_all)) { drop(fd); return; }
    epoll_event ev{};
    ev.events = c.peer_closed ? 0u : (uint32_t)EPOLLIN;   // EOF stays readable: stop polling it
    ev.data.fd = fd;
    epoll_ctl(efd, EPOLL_CTL_MOD, fd, &ev);
  }

  void drop(int fd) {
    epoll_ctl(efd, EPOLL_CTL_DEL, fd, nullptr);
    ::close(fd);
    conns.erase(fd);
  }

  static bool ieq_prefix(const char* a, const char* lit) {
    for (; *lit; ++a, ++lit)
      if (std::tolower((unsigned char)*a) != *lit) return false;
    return true;
  }

  // Parse every complete request buffered on fd.  Predict requests append rows to `rows`.
  void parse_requests(int fd, std::vector<float>& rows, std::vector<Pending>& pend) {
    Conn& c = conns[fd];
    size_t off = 0;
    for (;;) {
      if (c.predict_pending) break;                          // keep response order
      const size_t hend = c.in.find("\r\n\r\n", off);
      if (hend == std::string::npos) {
        if (c.in.size() - off > kMaxHeader) { c.closing = true; off = c.in.size(); }
        break;
      }
      const char* h = c.in.data() + off;
      const char* he = c.in.data() + hend;
      // request line
      const char* sp1 = static_cast<const char*>(std::memchr(h, ' ', he - h));
      if (!sp1) { c.closing = true; break; }
      const char* sp2 = static_cast<const char*>(std::memchr(sp1 + 1, ' ', he - sp1 - 1));
      if (!sp2) { c.closing = true; break; }
      const std::string method(h, sp1 - h);
      std::string path(sp1 + 1, sp2 - sp1 - 1);
      const size_t q = path.find('?');
      std::string query = q == std::string::npos ? "" : path.substr(q + 1);
      if (q != std::string::npos) path.resize(q);
      size_t clen = 0;
      bool close_after = false, authed = token.empty();
      for (const char* line = static_cast<const char*>(std::memchr(h, '\n', he - h)); line && line < he;) {
        ++line;
        const char* eol = static_cast<const char*>(std::memchr(line, '\n', he - line + 1));
        if (!eol) eol = he;
        if (ieq_prefix(line, "content-length:")) clen = (size_t)std::strtoull(line + 15, nullptr, 10);
        else if (ieq_prefix(line, "connection:") && std::strstr(std::string(line, eol - line).c_str(), "close"))
          close_after = true;
        else if (!authed && ieq_prefix(line, "authorization:")) {
          std::string v(line + 14, eol - line - 14);
          while (!v.empty() && (v.back() == '\r' || v.back() == ' ')) v.pop_back();
          while (!v.empty() && v.front() == ' ') v.erase(v.begin());
          authed = v == "Bearer " + token;
        }
        line = eol < he ? eol : nullptr;
      }
      if (!authed && !query.empty() && query.find("access_token=" + token) != std::string::npos) authed = true;
      const size_t body0 = hend + 4;
      if (clen > kMaxBody) {                                 // never buffer an unbounded body
        queue(fd, 413, "application/json", error_json(413, "request body too large"), true);
        off = c.in.size();
        break;
      }
      if (c.in.size() < body0 + clen) break;                 // body not complete yet
      const char* body = c.in.data() + body0;
      const int64_t t0 = now_ns();
      off = body0 + clen;
      if (method == "POST" && (path == "/api/v0.1/predictions" || path == "/api/v1.0/predictions" ||
                               path == "/predict" || path == "/api/v0.1/predict")) {
        if (!authed) { observe(401, now_ns() - t0); queue(fd, 401, "application/json", error_json(401, "unauthorized"), close_after); continue; }
        bool tensor = false;
        std::string err;
        const size_t r0 = rows.size();
        const int n = parse_seldon(body, clen, rows, &tensor, &err);
        if (n < 0) {
          rows.resize(r0);
          observe(400, now_ns() - t0);
          queue(fd, 400, "application/json", error_json(400, err), close_after);
          continue;
        }
        pend.push_back(Pending{fd, r0 / kF, n, tensor, close_after, t0});
        c.predict_pending = true;
      } else if (method == "GET" && (path == "/prometheus" || path == "/metrics")) {
        std::string text;
        if (render) {
          text.resize(1 << 20);
          const int32_t m = render(&text[0], (int32_t)text.size(), render_ctx);
          text.resize(m > 0 ? (size_t)m : 0);
        }
        queue(fd, 200, "text/plain; version=0.0.4; charset=utf-8", text, close_after);
      } else if (method == "GET" && (path == "/health/ping" || path == "/ping" || path == "/live" || path == "/ready" ||
                                     path == "/health/status")) {
        queue(fd, 200, "application/json", "{\"status\":\"ok\",\"model\":\"" + model + "\",\"server\":\"native\"}", close_after);
      } else {
        queue(fd, 404, "application/json", error_json(404, "not found"), close_after);
      }
      if (c.closing) break;
    }
    c.in.erase(0, off);
    c.parsed_all = !c.predict_pending;
  }

  void respond(const std::vector<Pending>& pend, const std::vector<float>& rows, const std::vector<float>& proba,
               int64_t model_ns) {
    std::string body;
    char num[96];
    for (const Pending& p : pend) {
      body.clear();
      body += "{\"meta\":{\"puid\":\"";
      std::snprintf(num, sizeof num, "%016llx", (unsigned long long)++puid);
      body += num;
      body += "\",\"tags\":{},\"routing\":{},\"requestPath\":{\"" + model + "\":\"" + model + "\"}},\"data\":{\"names\":[\"proba_0\",\"proba_1\"],";
      if (p.tensor) {
        body += "\"tensor\":{\"shape\":[" + std::to_string(p.nrows) + ",2],\"values\":[";
        for (int r = 0; r < p.nrows; ++r) {
          const float v = proba[p.row0 + r];
          std::snprintf(num, sizeof num, "%s%.7g,%.7g", r ? "," : "", 1.0 - (double)v, (double)v);
          body += num;
        }
        body += "]}}}";
      } else {
        body += "\"ndarray\":[";
        for (int r = 0; r < p.nrows; ++r) {
          const float v = proba[p.row0 + r];
          std::snprintf(num, sizeof num, "%s[%.7g,%.7g]", r ? "," : "", 1.0 - (double)v, (double)v);
          body += num;
        }
        body += "]}}";
      }
      queue(p.fd, 200, "application/json", body, p.close_after);
      observe(200, now_ns() - p.t0);
    }
    const Pending* lp = nullptr;                            // last request with rows (n may be 0)
    for (const Pending& p : pend) if (p.nrows > 0) lp = &p;
    if (lp) {
      const Pending& l = *lp;
      const float* x = rows.data() + (l.row0 + l.nrows - 1) * kF;
      const float last[4] = {proba[l.row0 + l.nrows - 1], x[kF - 1], x[17], x[10]};
      for (int i = 0; i < 4; ++i) { uint32_t b; std::memcpy(&b, &last[i], 4); stp->last_bits[i].store(b, std::memory_order_relaxed); }
      stp->model_ns.fetch_add((uint64_t)model_ns, std::memory_order_relaxed);
    }
  }

  void loop() {
    std::vector<epoll_event> evs(512);
    std::vector<float> rows, proba;
    std::vector<uint8_t> route;
    std::vector<Pending> pend;
    std::vector<int> touched, deferred;
    char buf[65536];
    while (!stop.load(std::memory_order_relaxed)) {
      // connections holding pipelined requests behind an answered predict are parsed
      // without waiting for new bytes (level-triggered epoll will not fire for them)
      const int n = epoll_wait(efd, evs.data(), (int)evs.size(), deferred.empty() ? 50 : 0);
      rows.clear();
      pend.clear();
      touched.clear();
      for (int fd : deferred) {
        auto it = conns.find(fd);
        if (it == conns.end()) continue;
        parse_requests(fd, rows, pend);
        if (it->second.peer_closed && !it->second.predict_pending && it->second.out.empty()) { drop(fd); continue; }
        touched.push_back(fd);
      }
      deferred.clear();
      for (int i = 0; i < n; ++i) {
        const int fd = evs[i].data.fd;
        if (fd == lfd) {
          for (;;) {
            const int cfd = ::accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK);
            if (cfd < 0) break;
            int one = 1;
            setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
            epoll_event ev{};
            ev.events = EPOLLIN;
            ev.data.fd = cfd;
            epoll_ctl(efd, EPOLL_CTL_ADD, cfd, &ev);
            conns.emplace(cfd, Conn{});
          }
          continue;
        }
        if (evs[i].events & EPOLLOUT) flush(fd);
        if (!(evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR))) continue;
        bool dead = false;
        for (;;) {
          const ssize_t r = ::recv(fd, buf, sizeof buf, 0);
          if (r > 0) { conns[fd].in.append(buf, (size_t)r); if ((size_t)r < sizeof buf) break; continue; }
          if (r == 0) dead = true;
          else if (errno != EAGAIN && errno != EWOULDBLOCK) dead = true;
          break;
        }
        if (conns.count(fd)) {
          Conn& c = conns[fd];
          if (dead) c.peer_closed = true;
          parse_requests(fd, rows, pend);
          touched.push_back(fd);
          if (dead) {
            if (c.out.empty() && !c.predict_pending) { drop(fd); continue; }
            epoll_event ev{};
            ev.events = c.out.empty() ? 0u : (uint32_t)EPOLLOUT;
            ev.data.fd = fd;
            epoll_ctl(efd, EPOLL_CTL_MOD, fd, &ev);
          }
        }
      }
      if (!pend.empty()) {
        // dynamic batch: everything that arrived during the previous GPU call, one score
        const int total = (int)(rows.size() / kF);
        proba.resize(total);
        route.resize(total);
        const int64_t m0 = now_ns();
        int rc = 0;
        for (int b0 = 0; b0 < total && rc == 0; b0 += max_batch) {
          const int nb = std::min(max_batch, total - b0);
          rc = scorer ? scorer(rows.data() + (size_t)b0 * kF, nb, proba.data() + b0, score_ctx)
                      : ccfd_engine_score_sync(engine, rows.data() + (size_t)b0 * kF, nb, proba.data() + b0,
                                               route.data() + b0);
        }
        stp->rows.fetch_add((uint64_t)total, std::memory_order_relaxed);
        stp->batches.fetch_add(1, std::memory_order_relaxed);
        if (rc != 0) {
          for (const Pending& p : pend) { observe(500, now_ns() - p.t0); queue(p.fd, 500, "application/json", error_json(500, "scoring failed"), true); }
        } else {
          respond(pend, rows, proba, now_ns() - m0);
        }
      }
      for (const Pending& p : pend) {
        auto it = conns.find(p.fd);
        if (it == conns.end()) continue;
        it->second.predict_pending = false;
        if (!it->second.in.empty() && !it->second.closing) deferred.push_back(p.fd);
        else it->second.parsed_all = true;
      }
      for (int fd : touched)
        if (conns.count(fd) && !conns[fd].out.empty()) flush(fd);
    }
    for (auto& kv : conns) ::close(kv.first);
    conns.clear();
  }
};

struct Group {
  std::vector<Server*> workers;
  Stats st;
  int port = 0;
};

}  // namespace

extern "C" {

// Start a server on host:port (port 0 = ephemeral) with `n_workers` epoll threads sharing the
// port (SO_REUSEPORT: the kernel spreads connections).  Scoring: worker i calls engine
// `engines[i]` (a ccfd engine over f32 rows; engines are not shared between threads) or, if
// non-null, `scorer(rows, n, proba, ctx)`.  `render` fills the /prometheus body.  `bounds`:
// latency histogram upper bounds in seconds (<= 32).
void* ccfd_seldon_http_start(const char* host, int port, void** engines, int n_workers, void* scorer, void* score_ctx,
                             void* render, void* render_ctx, const char* model, const char* token, int max_batch,
                             const double* bounds, int nbounds) {
  if (n_workers < 1 || (!scorer && !engines)) return nullptr;
  auto* g = new Group();
  for (int i = 0; i < kNStatus; ++i) {
    g->st.count[i] = 0; g->st.sum_ns[i] = 0;
    for (int b = 0; b <= kLatBuckets; ++b) g->st.hist[i][b] = 0;
  }
  g->st.rows = 0; g->st.batches = 0; g->st.model_ns = 0;
  for (int i = 0; i < 4; ++i) g->st.last_bits[i] = 0;
  for (int w = 0; w < n_workers; ++w) {
    auto* s = new Server();
    s->engine = engines ? engines[w] : nullptr;
    s->scorer = reinterpret_cast<score_fn>(scorer);
    s->score_ctx = score_ctx;
    s->render = reinterpret_cast<render_fn>(render);
    s->render_ctx = render_ctx;
    s->model = model ? model : "modelfull";
    s->token = token ? token : "";
    s->max_batch = max_batch > 0 ? max_batch : 65536;
    s->nbounds = std::min(std::max(nbounds, 0), kLatBuckets);
    for (int i = 0; i < s->nbounds; ++i) s->bounds[i] = bounds[i];
    s->stp = &g->st;
    s->puid = (uint64_t)w << 56;
    s->lfd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK, 0);
    int one = 1;
    setsockopt(s->lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    setsockopt(s->lfd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)(w == 0 ? port : g->port));
    a.sin_addr.s_addr = (host && *host && std::strcmp(host, "0.0.0.0")) ? inet_addr(host) : INADDR_ANY;
    if ((!s->engine && !s->scorer) || ::bind(s->lfd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 ||
        ::listen(s->lfd, 1024) != 0) {
      ::close(s->lfd);
      delete s;
      for (Server* o : g->workers) { o->stop.store(true); o->th.join(); ::close(o->efd); ::close(o->lfd); delete o; }
      delete g;
      return nullptr;
    }
    if (w == 0) {
      socklen_t al = sizeof a;
      getsockname(s->lfd, reinterpret_cast<sockaddr*>(&a), &al);
      g->port = ntohs(a.sin_port);
    }
    s->port = g->port;
    s->efd = epoll_create1(0);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = s->lfd;
    epoll_ctl(s->efd, EPOLL_CTL_ADD, s->lfd, &ev);
    s->th = std::thread([s] { s->loop(); });
    g->workers.push_back(s);
  }
  return g;
}

// Fuzz / test entry: parse a Seldon request body; returns rows or -1.
int64_t ccfd_seldon_parse_fuzz(const char* buf, int64_t len, float* rows_out, int64_t max_rows) {
  std::vector<float> rows;
  bool tensor = false;
  std::string err;
  const int n = parse_seldon(buf, (size_t)len, rows, &tensor, &err);
  if (n > 0 && rows_out) std::memcpy(rows_out, rows.data(), sizeof(float) * (size_t)std::min<int64_t>(n, max_rows) * kF);
  return n;
}

int ccfd_seldon_http_port(void* h) { return h ? static_cast<Group*>(h)->port : -1; }

// stats: [count x4, sum_ns x4, rows, batches, model_ns, last_bits x4, hist 4 x (32+1)] (u64);
// status order 200, 4xx (not 401), 401, 5xx
int ccfd_seldon_http_stats(void* h, uint64_t* out) {
  if (!h) return -1;
  Stats& st = static_cast<Group*>(h)->st;
  int k = 0;
  for (int i = 0; i < kNStatus; ++i) out[k++] = st.count[i].load();
  for (int i = 0; i < kNStatus; ++i) out[k++] = st.sum_ns[i].load();
  out[k++] = st.rows.load();
  out[k++] = st.batches.load();
  out[k++] = st.model_ns.load();
  for (int i = 0; i < 4; ++i) out[k++] = st.last_bits[i].load();
  for (int i = 0; i < kNStatus; ++i)
    for (int b = 0; b <= kLatBuckets; ++b) out[k++] = st.hist[i][b].load();
  return k;
}

void ccfd_seldon_http_stop(void* h) {
  if (!h) return;
  Group* g = static_cast<Group*>(h);
  for (Server* s : g->workers) s->stop.store(true);
  for (Server* s : g->workers) {
    if (s->th.joinable()) s->th.join();
    ::close(s->efd);
    ::close(s->lfd);
    delete s;
  }
  delete g;
}

}  // extern "C"
