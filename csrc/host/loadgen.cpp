// Open-loop HTTP/1.1 load generator (bench/bench_serve.py): request i is due at
// t0 + i / qps on keep-alive connection i % C, whatever happened to earlier requests; latency is
// measured from that SCHEDULED time, so a stalled server shows up as latency instead of as a
// slower send rate (no coordinated omission).  A few epoll threads drive all connections; a
// connection carries one request at a time, so requests due on a busy connection wait and that
// wait is counted.
#include "kmls/loadgen.hpp"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace kmls {

namespace {

using Clock = std::chrono::steady_clock;

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

struct LConn {
  int fd = -1;
  int idx = 0;          // connection index c: carries requests c, c + C, c + 2C, ...
  int64_t next_k = 0;   // next request of this connection (global index c + k * C)
  bool busy = false;
  int64_t sched = 0;    // scheduled time of the request in flight
  int64_t sent_at = 0;
  std::string out;
  size_t out_off = 0;
  std::string in;
};

int connect_to(const std::string& host, int port) {
  const int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, IPPROTO_TCP);
  if (fd < 0) return -1;
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
    ::close(fd);
    return -1;
  }
  if (::connect(fd, (sockaddr*)&a, sizeof a) != 0) {
    ::close(fd);
    return -1;
  }
  const int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
  return fd;
}

// complete response at the front of `in`: returns its length (0: incomplete), status in *st
size_t response_len(const std::string& in, int* st, bool* close) {
  const size_t he = in.find("\r\n\r\n");
  if (he == std::string::npos) return 0;
  *st = 0;
  if (in.size() >= 12) *st = std::atoi(in.c_str() + 9);
  size_t clen = 0;
  *close = false;
  size_t p = in.find("\r\n") + 2;
  while (p < he) {
    const size_t e = in.find("\r\n", p);
    std::string line = in.substr(p, e - p);
    for (auto& ch : line) ch = (char)std::tolower((unsigned char)ch);
    if (line.rfind("content-length:", 0) == 0) clen = (size_t)std::strtoull(line.c_str() + 15, nullptr, 10);
    if (line.rfind("connection:", 0) == 0 && line.find("close") != std::string::npos) *close = true;
    p = e + 2;
  }
  const size_t total = he + 4 + clen;
  return in.size() >= total ? total : 0;
}

}  // namespace

LoadResult run_loadgen(const std::string& host, int port, const std::vector<std::string>& requests,
                       double qps, double duration_s, int connections, int threads,
                       double drain_s) {
  if (requests.empty() || qps <= 0 || duration_s <= 0) throw std::invalid_argument("loadgen: bad args");
  const int C = std::max(1, connections);
  const int T = std::max(1, std::min(threads, C));
  const int64_t n_total = (int64_t)(qps * duration_s);
  const double period_ns = 1e9 / qps;
  LoadResult res;
  res.offered = n_total;
  std::vector<std::vector<int64_t>> lat((size_t)T), lag((size_t)T), at((size_t)T);
  std::vector<int64_t> errors((size_t)T, 0), done((size_t)T, 0), sent((size_t)T, 0);
  // connect everything first, then start the clock
  std::vector<LConn> conns((size_t)C);
  for (int c = 0; c < C; ++c) {
    conns[(size_t)c].idx = c;
    conns[(size_t)c].fd = connect_to(host, port);
    if (conns[(size_t)c].fd < 0) {
      for (auto& x : conns)
        if (x.fd >= 0) ::close(x.fd);
      throw std::runtime_error("loadgen: cannot connect to " + host + ":" + std::to_string(port));
    }
  }
  const int64_t t0 = now_ns() + 20'000'000;  // 20 ms to let every thread reach its loop
  const int64_t t_end = t0 + (int64_t)(duration_s * 1e9);
  const int64_t t_stop = t_end + (int64_t)(drain_s * 1e9);
  auto sched_of = [&](int64_t i) { return t0 + (int64_t)((double)i * period_ns); };

  auto worker = [&](int t) {
    const int ep = epoll_create1(EPOLL_CLOEXEC);
    std::vector<LConn*> mine;
    for (int c = t; c < C; c += T) {
      LConn* x = &conns[(size_t)c];
      mine.push_back(x);
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.ptr = x;
      epoll_ctl(ep, EPOLL_CTL_ADD, x->fd, &ev);
    }
    auto& L = lat[(size_t)t];
    auto& G = lag[(size_t)t];
    auto& A = at[(size_t)t];
    L.reserve((size_t)(n_total / T + 16));
    char buf[65536];
    epoll_event evs[64];
    while (true) {
      const int64_t now = now_ns();
      bool pending = false;
      int64_t next_due = INT64_MAX;
      for (LConn* x : mine) {
        const int64_t i = x->idx + x->next_k * C;
        if (!x->busy && i < n_total) {
          const int64_t s = sched_of(i);
          if (s <= now) {
            x->out = requests[(size_t)(i % (int64_t)requests.size())];
            x->out_off = 0;
            x->busy = true;
            x->sched = s;
            x->sent_at = now;
            ++sent[(size_t)t];
            while (x->out_off < x->out.size()) {
              const ssize_t n = ::send(x->fd, x->out.data() + x->out_off, x->out.size() - x->out_off, MSG_NOSIGNAL);
              if (n > 0) x->out_off += (size_t)n;
              else if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) std::this_thread::yield();
              else break;
            }
          } else {
            next_due = std::min(next_due, s);
          }
        }
        if (x->busy || i < n_total) pending = true;
      }
      if (!pending || now > t_stop) break;
      // wait for responses, at most until the next request is due
      int64_t wait_ns = next_due == INT64_MAX ? 1'000'000 : std::max<int64_t>(0, next_due - now_ns());
      wait_ns = std::min<int64_t>(wait_ns, 1'000'000);
      timespec ts{0, (long)wait_ns};
      const int n = epoll_pwait2(ep, evs, 64, &ts, nullptr);
      const int64_t tr = now_ns();
      for (int e = 0; e < n; ++e) {
        LConn* x = (LConn*)evs[e].data.ptr;
        while (true) {
          const ssize_t r = ::recv(x->fd, buf, sizeof buf, 0);
          if (r > 0) {
            x->in.append(buf, (size_t)r);
            continue;
          }
          break;
        }
        int st = 0;
        bool cl = false;
        size_t len;
        while (x->busy && (len = response_len(x->in, &st, &cl)) > 0) {
          x->in.erase(0, len);
          L.push_back(tr - x->sched);
          G.push_back(x->sent_at - x->sched);
          A.push_back(x->sched - t0);
          if (st != 200) ++errors[(size_t)t];
          ++done[(size_t)t];
          x->busy = false;
          x->next_k += 1;
          if (cl) {  // server closed the keep-alive connection: reconnect
            epoll_ctl(ep, EPOLL_CTL_DEL, x->fd, nullptr);
            ::close(x->fd);
            x->fd = connect_to(host, port);
            if (x->fd >= 0) {
              epoll_event ev{};
              ev.events = EPOLLIN;
              ev.data.ptr = x;
              epoll_ctl(ep, EPOLL_CTL_ADD, x->fd, &ev);
            }
          }
        }
      }
    }
    ::close(ep);
  };
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back(worker, t);
  for (auto& x : th) x.join();
  for (auto& x : conns)
    if (x.fd >= 0) ::close(x.fd);
  for (int t = 0; t < T; ++t) {
    res.lat_ns.insert(res.lat_ns.end(), lat[(size_t)t].begin(), lat[(size_t)t].end());
    res.lag_ns.insert(res.lag_ns.end(), lag[(size_t)t].begin(), lag[(size_t)t].end());
    res.at_ns.insert(res.at_ns.end(), at[(size_t)t].begin(), at[(size_t)t].end());
    res.errors += errors[(size_t)t];
    res.completed += done[(size_t)t];
    res.sent += sent[(size_t)t];
  }
  res.duration_s = duration_s;
  return res;
}

}  // namespace kmls
