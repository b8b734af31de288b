// Native HTTP/1.1 serving front (kmls/http_front.hpp has the design notes).
//
// Reference behaviour kept on the native route (rest_api/app/main.py:176-187, 205-254):
//   present seeds in request order -> max-merge -> stable sort desc -> top K (C++ RuleIndex or
//   the HIP matcher); no seed known -> the static fallback; response body
//   {"songs": [...], "model_date": <marker>, "version": VERSION} byte-identical to FastAPI's
//   JSONResponse (json.dumps(ensure_ascii=False, separators=(",", ":"))).
// Anything the native route does not answer goes to the FastAPI app unchanged.
#include "kmls/http_front.hpp"
#include "../kernels/kernels.hpp"  // kServeMaxSeeds / kServeWaveMerge (the loop router)

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cctype>
#include <condition_variable>
#include <cstring>
#include <ctime>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "kmls/gpu.hpp"

namespace kmls {

// ------------------------------------------------------------------------------------------
// JSON helpers

void json_escape_append(std::string& out, const std::string& s) {
  static const char* hex = "0123456789abcdef";
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          out += "\\u00";
          out.push_back(hex[c >> 4]);
          out.push_back(hex[c & 15]);
        } else {
          out.push_back((char)c);
        }
    }
  }
  out.push_back('"');
}

namespace {

enum class BodyParse { Ok, Empty, Invalid };

struct JsonCursor {
  const char* p;
  const char* e;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
};

bool utf8_append(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back((char)cp);
  } else if (cp < 0x800) {
    out.push_back((char)(0xC0 | (cp >> 6)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    if (cp >= 0xD800 && cp <= 0xDFFF) return false;  // lone surrogate: Python cannot encode it
    out.push_back((char)(0xE0 | (cp >> 12)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else if (cp <= 0x10FFFF) {
    out.push_back((char)(0xF0 | (cp >> 18)));
    out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    return false;
  }
  return true;
}

// length of a valid UTF-8 sequence starting at p (0: invalid)
int utf8_len(const unsigned char* p, const unsigned char* e) {
  const unsigned c = p[0];
  if (c < 0x80) return 1;
  int n;
  uint32_t cp;
  if ((c & 0xE0) == 0xC0) { n = 2; cp = c & 0x1F; }
  else if ((c & 0xF0) == 0xE0) { n = 3; cp = c & 0x0F; }
  else if ((c & 0xF8) == 0xF0) { n = 4; cp = c & 0x07; }
  else return 0;
  if (e - p < n) return 0;
  for (int i = 1; i < n; ++i) {
    if ((p[i] & 0xC0) != 0x80) return 0;
    cp = (cp << 6) | (p[i] & 0x3F);
  }
  if ((n == 2 && cp < 0x80) || (n == 3 && cp < 0x800) || (n == 4 && cp < 0x10000) ||
      cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF))
    return 0;
  return n;
}

int hexv(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

bool parse_string(JsonCursor& j, std::string* out) {
  if (j.p >= j.e || *j.p != '"') return false;
  ++j.p;
  while (j.p < j.e) {
    const unsigned char c = (unsigned char)*j.p;
    if (c == '"') {
      ++j.p;
      return true;
    }
    if (c < 0x20) return false;  // strict json: raw control characters are an error
    if (c == '\\') {
      if (j.e - j.p < 2) return false;
      const char x = j.p[1];
      j.p += 2;
      char lit = 0;
      switch (x) {
        case '"': lit = '"'; break;
        case '\\': lit = '\\'; break;
        case '/': lit = '/'; break;
        case 'b': lit = '\b'; break;
        case 'f': lit = '\f'; break;
        case 'n': lit = '\n'; break;
        case 'r': lit = '\r'; break;
        case 't': lit = '\t'; break;
        case 'u': {
          auto read4 = [&](uint32_t& v) {
            if (j.e - j.p < 4) return false;
            v = 0;
            for (int i = 0; i < 4; ++i) {
              const int h = hexv(j.p[i]);
              if (h < 0) return false;
              v = v * 16 + (uint32_t)h;
            }
            j.p += 4;
            return true;
          };
          uint32_t cp;
          if (!read4(cp)) return false;
          if (cp >= 0xD800 && cp <= 0xDBFF) {  // high surrogate: needs its low half
            if (j.e - j.p < 6 || j.p[0] != '\\' || j.p[1] != 'u') return false;
            j.p += 2;
            uint32_t lo;
            if (!read4(lo) || lo < 0xDC00 || lo > 0xDFFF) return false;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          if (out) {
            if (!utf8_append(*out, cp)) return false;
          } else if (cp >= 0xD800 && cp <= 0xDFFF) {
            return false;
          }
          continue;
        }
        default: return false;
      }
      if (out) out->push_back(lit);
      continue;
    }
    const int n = utf8_len((const unsigned char*)j.p, (const unsigned char*)j.e);
    if (!n) return false;
    if (out) out->append(j.p, (size_t)n);
    j.p += n;
  }
  return false;
}

bool skip_value(JsonCursor& j, int depth);

bool skip_number(JsonCursor& j) {
  const char* s = j.p;
  if (j.p < j.e && *j.p == '-') ++j.p;
  if (j.p >= j.e) return false;
  if (*j.p == '0') {
    ++j.p;
  } else if (*j.p >= '1' && *j.p <= '9') {
    while (j.p < j.e && *j.p >= '0' && *j.p <= '9') ++j.p;
  } else {
    return false;
  }
  if (j.p < j.e && *j.p == '.') {
    ++j.p;
    if (j.p >= j.e || *j.p < '0' || *j.p > '9') return false;
    while (j.p < j.e && *j.p >= '0' && *j.p <= '9') ++j.p;
  }
  if (j.p < j.e && (*j.p == 'e' || *j.p == 'E')) {
    ++j.p;
    if (j.p < j.e && (*j.p == '+' || *j.p == '-')) ++j.p;
    if (j.p >= j.e || *j.p < '0' || *j.p > '9') return false;
    while (j.p < j.e && *j.p >= '0' && *j.p <= '9') ++j.p;
  }
  return j.p > s;
}

bool skip_lit(JsonCursor& j, const char* lit) {
  const size_t n = std::strlen(lit);
  if ((size_t)(j.e - j.p) < n || std::memcmp(j.p, lit, n) != 0) return false;
  j.p += n;
  return true;
}

bool skip_value(JsonCursor& j, int depth) {
  if (depth > 64) return false;
  j.ws();
  if (j.p >= j.e) return false;
  switch (*j.p) {
    case '"': return parse_string(j, nullptr);
    case '{': {
      ++j.p;
      j.ws();
      if (j.p < j.e && *j.p == '}') { ++j.p; return true; }
      while (true) {
        j.ws();
        if (!parse_string(j, nullptr)) return false;
        j.ws();
        if (j.p >= j.e || *j.p != ':') return false;
        ++j.p;
        if (!skip_value(j, depth + 1)) return false;
        j.ws();
        if (j.p < j.e && *j.p == ',') { ++j.p; continue; }
        if (j.p < j.e && *j.p == '}') { ++j.p; return true; }
        return false;
      }
    }
    case '[': {
      ++j.p;
      j.ws();
      if (j.p < j.e && *j.p == ']') { ++j.p; return true; }
      while (true) {
        if (!skip_value(j, depth + 1)) return false;
        j.ws();
        if (j.p < j.e && *j.p == ',') { ++j.p; continue; }
        if (j.p < j.e && *j.p == ']') { ++j.p; return true; }
        return false;
      }
    }
    case 't': return skip_lit(j, "true");
    case 'f': return skip_lit(j, "false");
    case 'n': return skip_lit(j, "null");
    default: return skip_number(j);
  }
}

// {"songs": [str, ...], ...}: Ok (non-empty list of strings), Empty, or Invalid (anything
// FastAPI answers with 422/400 of its own: not JSON, not an object, no "songs", non-strings)
BodyParse parse_songs(const std::string& body, std::vector<std::string>& songs) {
  JsonCursor j{body.data(), body.data() + body.size()};
  j.ws();
  if (j.p >= j.e || *j.p != '{') return BodyParse::Invalid;
  ++j.p;
  bool have = false, valid = false;
  j.ws();
  if (j.p < j.e && *j.p == '}') {
    ++j.p;
  } else {
    while (true) {
      j.ws();
      std::string key;
      if (!parse_string(j, &key)) return BodyParse::Invalid;
      j.ws();
      if (j.p >= j.e || *j.p != ':') return BodyParse::Invalid;
      ++j.p;
      j.ws();
      if (key == "songs") {  // json.loads keeps the LAST duplicate key
        have = true;
        songs.clear();
        valid = false;
        if (j.p < j.e && *j.p == '[') {
          ++j.p;
          j.ws();
          valid = true;
          if (j.p < j.e && *j.p == ']') {
            ++j.p;
          } else {
            while (true) {
              j.ws();
              if (j.p < j.e && *j.p == '"') {
                std::string s;
                if (!parse_string(j, &s)) return BodyParse::Invalid;
                songs.push_back(std::move(s));
              } else {
                valid = false;  // not a string: pydantic rejects it (422)
                if (!skip_value(j, 1)) return BodyParse::Invalid;
              }
              j.ws();
              if (j.p < j.e && *j.p == ',') { ++j.p; continue; }
              if (j.p < j.e && *j.p == ']') { ++j.p; break; }
              return BodyParse::Invalid;
            }
          }
        } else if (!skip_value(j, 0)) {
          return BodyParse::Invalid;
        }
      } else if (!skip_value(j, 0)) {
        return BodyParse::Invalid;
      }
      j.ws();
      if (j.p < j.e && *j.p == ',') { ++j.p; continue; }
      if (j.p < j.e && *j.p == '}') { ++j.p; break; }
      return BodyParse::Invalid;
    }
  }
  j.ws();
  if (j.p != j.e || !have || !valid) return BodyParse::Invalid;
  return songs.empty() ? BodyParse::Empty : BodyParse::Ok;
}

// ------------------------------------------------------------------------------------------
// CPython's Mersenne Twister + Random.sample, bit-exact

struct PyMT {
  uint32_t mt[624];
  int mti = 625;
  void init_genrand(uint32_t s) {
    mt[0] = s;
    for (mti = 1; mti < 624; ++mti)
      mt[mti] = 1812433253u * (mt[mti - 1] ^ (mt[mti - 1] >> 30)) + (uint32_t)mti;
  }
  void init_by_array(const uint32_t* key, int len) {
    init_genrand(19650218u);
    int i = 1, j = 0;
    for (int k = std::max(624, len); k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      ++i;
      ++j;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
      if (j >= len) j = 0;
    }
    for (int k = 623; k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      ++i;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
    }
    mt[0] = 0x80000000u;
    mti = 624;
  }
  uint32_t next() {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    if (mti >= 624) {
      int kk = 0;
      for (; kk < 624 - 397; ++kk) {
        const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
      }
      for (; kk < 623; ++kk) {
        const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
      }
      const uint32_t y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
      mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
      mti = 0;
    }
    uint32_t y = mt[mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  uint32_t randbelow(uint32_t n) {  // Random._randbelow_with_getrandbits, n <= 2^32 - 1
    int k = 0;
    for (uint32_t x = n; x; x >>= 1) ++k;  // n.bit_length()
    uint32_t r = next() >> (32 - k);
    while (r >= n) r = next() >> (32 - k);
    return r;
  }
};

}  // namespace

std::vector<int> python_random_sample(uint64_t seed, int n, int k) {
  PyMT g;
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  g.init_by_array(key, (seed >> 32) ? 2 : 1);
  std::vector<int> out;
  if (n <= 0 || k <= 0) return out;
  k = std::min(k, n);
  out.resize((size_t)k);
  int setsize = 21;
  if (k > 5) setsize += (int)std::pow(4.0, std::ceil(std::log(k * 3.0) / std::log(4.0)));
  if (n <= setsize) {
    std::vector<int> pool((size_t)n);
    for (int i = 0; i < n; ++i) pool[(size_t)i] = i;
    for (int i = 0; i < k; ++i) {
      const int j = (int)g.randbelow((uint32_t)(n - i));
      out[(size_t)i] = pool[(size_t)j];
      pool[(size_t)j] = pool[(size_t)(n - i - 1)];
    }
  } else {
    std::vector<int> sel;
    for (int i = 0; i < k; ++i) {
      int j = (int)g.randbelow((uint32_t)n);
      while (std::find(sel.begin(), sel.end(), j) != sel.end()) j = (int)g.randbelow((uint32_t)n);
      sel.push_back(j);
      out[(size_t)i] = j;
    }
  }
  return out;
}

uint64_t fallback_seed(std::vector<std::string> seeds) {
  std::sort(seeds.begin(), seeds.end());  // UTF-8 byte order == code point order
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < seeds.size(); ++i) {
    if (i) h = (h ^ 0x1fu) * 0x100000001b3ull;
    for (unsigned char c : seeds[i]) h = (h ^ c) * 0x100000001b3ull;
  }
  return h;
}

// ------------------------------------------------------------------------------------------
// server

namespace {

constexpr uint64_t kListenId = 0, kEventId = 1;
constexpr size_t kMaxHeader = 64 << 10, kMaxBody = 16 << 20;

const char* reason(int status) {
  switch (status) {
    case 100: return "Continue";
    case 200: return "OK";
    case 201: return "Created";
    case 204: return "No Content";
    case 301: return "Moved Permanently";
    case 302: return "Found";
    case 304: return "Not Modified";
    case 307: return "Temporary Redirect";
    case 308: return "Permanent Redirect";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 413: return "Request Entity Too Large";
    case 422: return "Unprocessable Entity";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
  }
  return "";
}

std::string lower(std::string s) {
  for (char& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t')) ++a;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t')) --b;
  return s.substr(a, b - a);
}

struct Request {
  std::string method, target, path, query, version;
  std::vector<std::pair<std::string, std::string>> headers;
  std::string body;
  bool keep_alive = true;
  bool json = false;
};

struct Conn {
  int fd = -1;
  uint64_t id = 0;
  std::string in;
  size_t in_off = 0;
  std::string out;
  size_t out_off = 0;
  bool busy = false;         // one request answered asynchronously (GPU batch / FastAPI)
  bool close_after = false;  // close once `out` is flushed
  bool head = false;         // the request in flight is a HEAD
  bool sent_continue = false;
  bool want_out = false;     // EPOLLOUT registered
  std::string peer;
  int peer_port = 0;
};

struct Outgoing {
  uint64_t conn;
  std::string bytes;
  bool close;
};

}  // namespace

struct GpuJob {
  int worker;
  uint64_t conn;
  bool keep_alive;
  std::shared_ptr<const FrontModel> model;
  std::vector<int32_t> ids;
  std::vector<std::string> seeds;  // for the fallback
};

struct HttpFront::Impl {
  HttpFront* self;
  int k = 10;
  std::string version_json;
  int batch_max = 256, batch_wait_us = 100;
  std::atomic<bool> running{false};
  std::shared_ptr<const FrontModel> model;  // std::atomic_load / atomic_store
  // the model replaced by the last set_model, kept alive until the next one: otherwise the last
  // reference could drop on the GPU worker or an I/O worker, which would then run the old GPU
  // index's destructor (loop pause, hipFree device syncs, ~0.1 s) while requests queue behind it
  // (measured: 105 ms p99 in the reload window with the serving loop)
  std::shared_ptr<const FrontModel> retired;
  std::mutex retire_mu;
  struct Worker {
    int epfd = -1, lfd = -1, efd = -1;
    std::thread th;
    std::mutex mu;
    std::vector<Outgoing> outbox;
    std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns;
    uint64_t next_id = 2;
  };
  std::vector<std::unique_ptr<Worker>> workers;
  // slow path (FastAPI)
  std::mutex slow_mu;
  std::deque<SlowRequest> slow_q;
  // GPU batcher
  std::thread gpu_th;
  std::mutex gpu_mu;
  std::condition_variable gpu_cv;
  std::deque<GpuJob> gpu_q;
  std::atomic<int> gpu_pending{0};
  // stats
  std::atomic<uint64_t> st_requests{0}, st_native{0}, st_fallback{0}, st_slow{0},
      st_gpu_batches{0}, st_gpu_queries{0}, st_conns{0}, st_in{0}, st_out{0}, st_gpu_loop{0},
      st_gpu_loop_refused{0};

  // ---- response building ----
  // Date header cache: per calling thread (I/O threads, the GPU batcher and respond() all build
  // responses; a per-worker cache written from several of them would race)
  const char* date_hdr(Worker&) {
    thread_local time_t date_t = 0;
    thread_local char date[64] = {0};
    const time_t now = std::time(nullptr);
    if (now != date_t) {
      struct tm g;
      gmtime_r(&now, &g);
      std::strftime(date, sizeof date, "%a, %d %b %Y %H:%M:%S GMT", &g);
      date_t = now;
    }
    return date;
  }
  std::string json_response(Worker& w, const std::string& body, bool keep_alive) {
    std::string r;
    r.reserve(body.size() + 160);
    r += "HTTP/1.1 200 OK\r\ndate: ";
    r += date_hdr(w);
    r += "\r\nserver: kmls\r\ncontent-length: ";
    r += std::to_string(body.size());
    r += "\r\ncontent-type: application/json\r\n";
    if (!keep_alive) r += "connection: close\r\n";
    r += "\r\n";
    r += body;
    return r;
  }
  std::string songs_body(const FrontModel& m, const int32_t* ids, int n) {
    std::string b = "{\"songs\":[";
    for (int i = 0; i < n; ++i) {
      if (i) b.push_back(',');
      b += m.names_json[(size_t)ids[i]];
    }
    b += "],\"model_date\":";
    b += m.marker_json;
    b += ",\"version\":";
    b += version_json;
    b += "}";
    return b;
  }
  std::string fallback_body(const FrontModel& m, const std::vector<std::string>& seeds) {
    const std::vector<int> pick =
        python_random_sample(fallback_seed(seeds), (int)m.best_json.size(), k);
    std::string b = "{\"songs\":[";
    for (size_t i = 0; i < pick.size(); ++i) {
      if (i) b.push_back(',');
      b += m.best_json[(size_t)pick[i]];
    }
    b += "],\"model_date\":";
    b += m.marker_json;
    b += ",\"version\":";
    b += version_json;
    b += "}";
    return b;
  }

  // ---- worker side ----
  void post(int wi, uint64_t conn, std::string bytes, bool close) {
    Worker& w = *workers[(size_t)wi];
    {
      std::lock_guard<std::mutex> lk(w.mu);
      w.outbox.push_back(Outgoing{conn, std::move(bytes), close});
    }
    const uint64_t one = 1;
    (void)!write(w.efd, &one, 8);
  }

  void close_conn(Worker& w, Conn& c) {
    epoll_ctl(w.epfd, EPOLL_CTL_DEL, c.fd, nullptr);
    ::close(c.fd);
    w.conns.erase(c.id);  // destroys c
  }

  // returns false when the connection was closed
  bool flush(Worker& w, Conn& c) {
    while (c.out_off < c.out.size()) {
      const ssize_t n = ::send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
      if (n > 0) {
        c.out_off += (size_t)n;
        st_out += (uint64_t)n;
        continue;
      }
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        if (!c.want_out) {
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP;
          ev.data.u64 = c.id;
          epoll_ctl(w.epfd, EPOLL_CTL_MOD, c.fd, &ev);
          c.want_out = true;
        }
        return true;
      }
      close_conn(w, c);
      return false;
    }
    c.out.clear();
    c.out_off = 0;
    if (c.want_out) {
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = c.id;
      epoll_ctl(w.epfd, EPOLL_CTL_MOD, c.fd, &ev);
      c.want_out = false;
    }
    if (c.close_after && !c.busy) {
      close_conn(w, c);
      return false;
    }
    return true;
  }

  // 1: request parsed into r; 0: need more bytes; -1: protocol error (connection closed)
  int parse_request(Worker& w, Conn& c, Request& r) {
    const char* base = c.in.data() + c.in_off;
    const size_t avail = c.in.size() - c.in_off;
    const char* hend = (const char*)memmem(base, avail, "\r\n\r\n", 4);
    if (!hend) {
      if (avail > kMaxHeader) return -1;
      return 0;
    }
    const size_t hlen = (size_t)(hend - base) + 4;
    // request line
    const char* le = (const char*)memmem(base, hlen, "\r\n", 2);
    std::string line(base, (size_t)(le - base));
    const size_t s1 = line.find(' '), s2 = line.rfind(' ');
    if (s1 == std::string::npos || s2 == s1) return -1;
    r.method = line.substr(0, s1);
    r.target = line.substr(s1 + 1, s2 - s1 - 1);
    r.version = line.substr(s2 + 1);
    if (r.version != "HTTP/1.1" && r.version != "HTTP/1.0") return -1;
    const size_t q = r.target.find('?');
    r.path = r.target.substr(0, q);
    r.query = q == std::string::npos ? "" : r.target.substr(q + 1);
    r.keep_alive = r.version == "HTTP/1.1";
    // headers
    int64_t clen = -1;
    bool chunked = false, expect = false;
    const char* p = le + 2;
    const char* hstop = base + hlen - 2;
    while (p < hstop) {
      const char* e = (const char*)memmem(p, (size_t)(hstop - p) + 2, "\r\n", 2);
      if (!e) return -1;
      const char* colon = (const char*)memchr(p, ':', (size_t)(e - p));
      if (!colon) return -1;
      std::string name = lower(std::string(p, (size_t)(colon - p)));
      std::string val = trim(std::string(colon + 1, (size_t)(e - colon - 1)));
      if (name == "content-length") {
        char* endp = nullptr;
        const long long v = std::strtoll(val.c_str(), &endp, 10);
        if (!endp || *endp || v < 0 || (clen >= 0 && clen != v)) return -1;
        clen = v;
      } else if (name == "transfer-encoding") {
        if (lower(val).find("chunked") != std::string::npos) chunked = true;
      } else if (name == "connection") {
        const std::string v = lower(val);
        if (v.find("close") != std::string::npos) r.keep_alive = false;
        else if (v.find("keep-alive") != std::string::npos) r.keep_alive = true;
      } else if (name == "expect") {
        expect = lower(val) == "100-continue";
      } else if (name == "content-type") {
        const std::string v = lower(val);
        const std::string mt = trim(v.substr(0, v.find(';')));
        r.json = mt == "application/json";
      }
      r.headers.emplace_back(std::move(name), std::move(val));
      p = e + 2;
    }
    // body (both framings at once is a request-smuggling vector: refuse it)
    if (chunked && clen >= 0) return -1;
    size_t consumed = hlen;
    if (chunked) {
      size_t pos = hlen;
      std::string body;
      while (true) {
        const char* ce = (const char*)memmem(base + pos, avail - pos, "\r\n", 2);
        if (!ce) goto need_more;
        const std::string hx(base + pos, (size_t)(ce - (base + pos)));
        // chunk-size: 1-16 hex digits, optionally followed by ";ext" (no sign, no blanks, no
        // overflow), and never more than what is left of the body budget
        size_t nd = 0;
        unsigned long long sz = 0;
        while (nd < hx.size() && std::isxdigit((unsigned char)hx[nd])) {
          if (nd == 16) return -1;
          const char ch = hx[nd];
          sz = (sz << 4) | (unsigned long long)(ch <= '9' ? ch - '0' : (ch | 0x20) - 'a' + 10);
          ++nd;
        }
        if (nd == 0 || (nd < hx.size() && hx[nd] != ';')) return -1;
        if (sz > kMaxBody - body.size()) return -1;
        pos = (size_t)(ce - base) + 2;
        if (sz == 0) {  // trailers until an empty line
          const char* te = (const char*)memmem(base + pos, avail - pos, "\r\n", 2);
          while (te && te != base + pos) {
            pos = (size_t)(te - base) + 2;
            te = (const char*)memmem(base + pos, avail - pos, "\r\n", 2);
          }
          if (!te) goto need_more;
          pos += 2;
          break;
        }
        if (avail - pos < sz || avail - pos - sz < 2) goto need_more;
        if (base[pos + sz] != '\r' || base[pos + sz + 1] != '\n') return -1;
        body.append(base + pos, (size_t)sz);
        pos += (size_t)sz + 2;
      }
      r.body = std::move(body);
      consumed = pos;
    } else if (clen > 0) {
      if ((size_t)clen > kMaxBody) return -1;
      if (avail - hlen < (size_t)clen) goto need_more;
      r.body.assign(base + hlen, (size_t)clen);
      consumed = hlen + (size_t)clen;
    }
    c.in_off += consumed;
    c.sent_continue = false;
    if (c.in_off == c.in.size()) {
      c.in.clear();
      c.in_off = 0;
    }
    return 1;
  need_more:
    if (expect && !c.sent_continue) {
      c.out += "HTTP/1.1 100 Continue\r\n\r\n";
      c.sent_continue = true;
    }
    (void)w;
    return 0;
  }

  void to_slow(Worker& w, int wi, Conn& c, Request& r) {
    SlowRequest s;
    s.token = ((uint64_t)wi << 56) | c.id;
    s.method = std::move(r.method);
    s.path = std::move(r.path);
    s.query = std::move(r.query);
    s.http_version = r.version == "HTTP/1.0" ? "1.0" : "1.1";
    s.headers = std::move(r.headers);
    s.body = std::move(r.body);
    s.client_host = c.peer;
    s.client_port = c.peer_port;
    c.busy = true;
    c.close_after = c.close_after || !r.keep_alive;
    ++st_slow;
    {
      std::lock_guard<std::mutex> lk(slow_mu);
      slow_q.push_back(std::move(s));
    }
    const uint64_t one = 1;
    (void)!write(self->slow_efd_, &one, 8);
    (void)w;
  }

  void handle(Worker& w, int wi, Conn& c, Request& r) {
    ++st_requests;
    c.head = r.method == "HEAD";
    std::shared_ptr<const FrontModel> m = std::atomic_load(&model);
    if (r.method != "POST" || r.path != "/api/recommend/" || !r.json || !m || m->best_json.empty()) {
      to_slow(w, wi, c, r);
      return;
    }
    std::vector<std::string> seeds;
    if (parse_songs(r.body, seeds) != BodyParse::Ok) {
      to_slow(w, wi, c, r);
      return;
    }
    std::vector<int32_t> ids(seeds.size());
    for (size_t i = 0; i < seeds.size(); ++i) {
      auto it = m->name_to_id.find(seeds[i]);
      ids[i] = it == m->name_to_id.end() ? -1 : it->second;
    }
    bool to_gpu = false;
    if (m->gpu && m->gpu_min_merge >= 0) {  // the serving loop: by the query's merged size
      if ((int)ids.size() <= kern::kServeMaxSeeds) {
        const int64_t merged = m->gpu->merged_size(ids.data(), (int64_t)ids.size());
        to_gpu = merged >= m->gpu_min_merge && merged <= kern::kServeWaveMerge && merged > 0;
      }
    } else if (m->gpu && m->gpu_min_batch > 0) {
      to_gpu = m->gpu_min_batch == 1 ||
               gpu_pending.load(std::memory_order_relaxed) + 1 >= m->gpu_min_batch;
    }
    int32_t out[256];
    const int kk = std::min(k, 256);
    if (to_gpu && m->gpu_min_merge >= 0) {
      // the persistent serving kernel answers on THIS I/O thread (each caller gets its own
      // request slot, answered by its own workgroup): no hop to the GPU thread and back
      const int64_t qp[2] = {0, (int64_t)ids.size()};
      int32_t on = -3;
      bool ok = false;
      try {
        ok = m->gpu->query_loop(qp, 1, ids.data(), kk, out, &on);
      } catch (...) {
        ok = false;
      }
      int n = on;
      if (ok) {
        ++st_gpu_loop;
        ++st_gpu_batches;
        ++st_gpu_queries;
      } else {
        ++st_gpu_loop_refused;
      }
      if (!ok || n == -2) n = m->index->query(ids.data(), (int)ids.size(), kk, out, nullptr);
      std::string body;
      if (n < 0) {
        body = fallback_body(*m, seeds);
        ++st_fallback;
      } else {
        body = songs_body(*m, out, n);
      }
      ++st_native;
      c.out += json_response(w, body, r.keep_alive);
      if (!r.keep_alive) c.close_after = true;
      return;
    }
    if (to_gpu) {
      c.busy = true;
      c.close_after = c.close_after || !r.keep_alive;
      ++gpu_pending;
      {
        std::lock_guard<std::mutex> lk(gpu_mu);
        gpu_q.push_back(GpuJob{wi, c.id, r.keep_alive, m, std::move(ids), std::move(seeds)});
      }
      gpu_cv.notify_one();
      return;
    }
    const int n = m->index->query(ids.data(), (int)ids.size(), kk, out, nullptr);
    std::string body;
    if (n < 0) {
      body = fallback_body(*m, seeds);
      ++st_fallback;
    } else {
      body = songs_body(*m, out, n);
    }
    ++st_native;
    c.out += json_response(w, body, r.keep_alive);
    if (!r.keep_alive) c.close_after = true;
  }

  // parse and answer every complete request in the buffer (stops at an async one)
  bool pump(Worker& w, int wi, Conn& c) {
    while (!c.busy && !c.close_after) {
      Request r;
      int st = -1;
      try {  // a malformed request closes its own connection, never the I/O thread
        st = parse_request(w, c, r);
      } catch (const std::exception&) {
        st = -1;
      }
      if (st > 0) {
        const size_t out0 = c.out.size();
        try {
          handle(w, wi, c, r);
        } catch (const std::exception&) {
          // handle() failed after the parse: if it already queued the request (busy) or wrote
          // its answer, that path owns the connection's response — close without a second one
          if (c.busy || c.out.size() != out0) {
            c.close_after = true;
            break;
          }
          st = -1;
        }
      }
      if (st < 0) {
        c.out += "HTTP/1.1 400 Bad Request\r\ncontent-length: 0\r\nconnection: close\r\n\r\n";
        c.close_after = true;
        break;
      }
      if (st == 0) break;
    }
    return flush(w, c);
  }

  void on_readable(Worker& w, int wi, Conn& c) {
    char buf[65536];
    bool eof = false;
    while (true) {
      const ssize_t n = ::recv(c.fd, buf, sizeof buf, 0);
      if (n > 0) {
        if (c.in_off > (1 << 20)) {
          c.in.erase(0, c.in_off);
          c.in_off = 0;
        }
        c.in.append(buf, (size_t)n);
        st_in += (uint64_t)n;
        continue;
      }
      if (n == 0) eof = true;
      else if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
      break;
    }
    const uint64_t id = c.id;
    if (!pump(w, wi, c)) return;
    if (eof) {
      auto it = w.conns.find(id);
      if (it == w.conns.end()) return;
      Conn& cc = *it->second;
      if (cc.busy) cc.close_after = true;  // answer the request in flight, then close
      else close_conn(w, cc);
    }
  }

  void on_outbox(Worker& w, int wi) {
    uint64_t v;
    (void)!read(w.efd, &v, 8);
    std::vector<Outgoing> items;
    {
      std::lock_guard<std::mutex> lk(w.mu);
      items.swap(w.outbox);
    }
    for (auto& o : items) {
      auto it = w.conns.find(o.conn);
      if (it == w.conns.end()) continue;  // the client went away
      Conn& c = *it->second;
      c.out += o.bytes;
      c.busy = false;
      if (o.close) c.close_after = true;
      pump(w, wi, c);
    }
  }

  void accept_all(Worker& w) {
    while (true) {
      sockaddr_storage ss{};
      socklen_t sl = sizeof ss;
      const int fd = ::accept4(w.lfd, (sockaddr*)&ss, &sl, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      const int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      c->id = w.next_id++;
      char host[INET6_ADDRSTRLEN] = {0};
      if (ss.ss_family == AF_INET) {
        auto* a = (sockaddr_in*)&ss;
        inet_ntop(AF_INET, &a->sin_addr, host, sizeof host);
        c->peer_port = ntohs(a->sin_port);
      } else if (ss.ss_family == AF_INET6) {
        auto* a = (sockaddr_in6*)&ss;
        inet_ntop(AF_INET6, &a->sin6_addr, host, sizeof host);
        c->peer_port = ntohs(a->sin6_port);
      }
      c->peer = host;
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = c->id;
      epoll_ctl(w.epfd, EPOLL_CTL_ADD, fd, &ev);
      ++st_conns;
      w.conns.emplace(c->id, std::move(c));
    }
  }

  void run_worker(int wi) {
    Worker& w = *workers[(size_t)wi];
    epoll_event evs[256];
    while (running.load(std::memory_order_relaxed)) {
      const int n = epoll_wait(w.epfd, evs, 256, 100);
      for (int i = 0; i < n; ++i) {
        const uint64_t id = evs[i].data.u64;
        if (id == kListenId) {
          accept_all(w);
          continue;
        }
        if (id == kEventId) {
          on_outbox(w, wi);
          continue;
        }
        auto it = w.conns.find(id);
        if (it == w.conns.end()) continue;
        Conn& c = *it->second;
        if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
          on_readable(w, wi, c);
          continue;
        }
        if (evs[i].events & EPOLLOUT) flush(w, c);
      }
    }
    for (auto& kv : w.conns) ::close(kv.second->fd);
    w.conns.clear();
  }

  // ---- GPU batcher: micro-batches requests of every connection into one HIP launch ----
  void run_gpu() {
    std::vector<GpuJob> batch;
    std::vector<int64_t> q_ptr;
    std::vector<int32_t> seeds, out_ids, out_n;
    while (true) {
      {
        std::unique_lock<std::mutex> lk(gpu_mu);
        gpu_cv.wait(lk, [&] { return !gpu_q.empty() || !running.load(); });
        if (gpu_q.empty() && !running.load()) return;
        // the serving loop answers a request in one round trip whatever the batch: no
        // micro-batching wait for it (that wait is for the per-batch launch path)
        const std::shared_ptr<const FrontModel> cur = std::atomic_load(&model);
        const bool loop_mode = cur && cur->gpu_min_merge >= 0;
        if ((int)gpu_q.size() < batch_max && batch_wait_us > 0 && !loop_mode) {
          gpu_cv.wait_for(lk, std::chrono::microseconds(batch_wait_us),
                          [&] { return (int)gpu_q.size() >= batch_max || !running.load(); });
        }
        const size_t take = std::min<size_t>(gpu_q.size(), (size_t)batch_max);
        batch.clear();
        for (size_t i = 0; i < take; ++i) {
          batch.push_back(std::move(gpu_q.front()));
          gpu_q.pop_front();
        }
      }
      // one launch per model generation in the batch (a reload may straddle it)
      size_t a = 0;
      while (a < batch.size()) {
        size_t b = a;
        while (b < batch.size() && batch[b].model == batch[a].model) ++b;
        const FrontModel& m = *batch[a].model;
        const int64_t B = (int64_t)(b - a);
        q_ptr.assign((size_t)B + 1, 0);
        seeds.clear();
        for (size_t i = a; i < b; ++i) {
          seeds.insert(seeds.end(), batch[i].ids.begin(), batch[i].ids.end());
          q_ptr[i - a + 1] = (int64_t)seeds.size();
        }
        out_ids.assign((size_t)B * (size_t)k, 0);
        out_n.assign((size_t)B, 0);
        bool ok = true;
        try {
          if (m.gpu_min_merge >= 0) {  // the persistent serving kernel (false: paused)
            ok = m.gpu->query_loop(q_ptr.data(), B, seeds.data(), k, out_ids.data(), out_n.data());
            if (ok) ++st_gpu_loop;
            else ++st_gpu_loop_refused;
          } else {
            m.gpu->query_batch(q_ptr.data(), B, seeds.data(), k, out_ids.data(), out_n.data());
          }
        } catch (...) {
          ok = false;
        }
        if (ok) {
          ++st_gpu_batches;
          st_gpu_queries += (uint64_t)B;
        }
        for (size_t i = a; i < b; ++i) {
          GpuJob& j = batch[i];
          const int64_t row = (int64_t)(i - a);
          int n = ok ? out_n[(size_t)row] : 0;
          std::vector<int32_t> cpu(256);
          const int32_t* ids = out_ids.data() + row * k;
          if (!ok || n == -2) {  // HIP error / paused loop / long merge: the C++ matcher
            n = m.index->query(j.ids.data(), (int)j.ids.size(), std::min(k, 256), cpu.data(), nullptr);
            ids = cpu.data();
          }
          std::string body;
          if (n < 0) {
            body = fallback_body(m, j.seeds);
            ++st_fallback;
          } else {
            body = songs_body(m, ids, n);
          }
          ++st_native;
          Worker& w = *workers[(size_t)j.worker];
          std::string resp;
          {
            std::lock_guard<std::mutex> lk(w.mu);  // date cache is per worker
            resp = json_response(w, body, j.keep_alive);
          }
          post(j.worker, j.conn, std::move(resp), !j.keep_alive);
        }
        gpu_pending -= (int)B;
        a = b;
      }
    }
  }
};

HttpFront::HttpFront(const std::string& host, int port, int threads, int k,
                     const std::string& version, int batch_max, int batch_wait_us)
    : host_(host), port_(port), threads_(std::max(1, threads)) {
  impl_ = new Impl();
  impl_->self = this;
  impl_->k = std::max(1, std::min(k, 256));
  json_escape_append(impl_->version_json, version);
  impl_->batch_max = std::max(1, batch_max);
  impl_->batch_wait_us = std::max(0, batch_wait_us);
  slow_efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (slow_efd_ < 0) throw std::runtime_error("HttpFront: eventfd failed");
}

HttpFront::~HttpFront() {
  stop();
  if (slow_efd_ >= 0) ::close(slow_efd_);
  delete impl_;
}

void HttpFront::start() {
  if (impl_->running.load()) return;
  // resolve the bind address; port 0 = pick one (the first socket's port is then reused)
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE;
  addrinfo* res = nullptr;
  const std::string ps = std::to_string(port_);
  if (getaddrinfo(host_.empty() ? nullptr : host_.c_str(), ps.c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("HttpFront: cannot resolve " + host_);
  std::vector<int> lfds;
  for (int t = 0; t < threads_; ++t) {
    const int fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, IPPROTO_TCP);
    if (fd < 0) throw std::runtime_error("HttpFront: socket failed");
    const int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    sockaddr_storage ss{};
    std::memcpy(&ss, res->ai_addr, res->ai_addrlen);
    if (port_ != 0 || t > 0) {
      if (ss.ss_family == AF_INET) ((sockaddr_in*)&ss)->sin_port = htons((uint16_t)port_);
      else ((sockaddr_in6*)&ss)->sin6_port = htons((uint16_t)port_);
    }
    if (::bind(fd, (sockaddr*)&ss, res->ai_addrlen) != 0 || ::listen(fd, 4096) != 0) {
      const int e = errno;
      ::close(fd);
      for (int f : lfds) ::close(f);
      freeaddrinfo(res);
      throw std::runtime_error("HttpFront: bind/listen on " + host_ + ":" + std::to_string(port_) +
                               " failed: " + std::strerror(e));
    }
    if (port_ == 0) {
      sockaddr_storage got{};
      socklen_t gl = sizeof got;
      getsockname(fd, (sockaddr*)&got, &gl);
      port_ = ntohs(got.ss_family == AF_INET ? ((sockaddr_in*)&got)->sin_port
                                             : ((sockaddr_in6*)&got)->sin6_port);
    }
    lfds.push_back(fd);
  }
  freeaddrinfo(res);
  impl_->running = true;
  for (int t = 0; t < threads_; ++t) {
    auto w = std::make_unique<Impl::Worker>();
    w->lfd = lfds[(size_t)t];
    w->epfd = epoll_create1(EPOLL_CLOEXEC);
    w->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = kListenId;
    epoll_ctl(w->epfd, EPOLL_CTL_ADD, w->lfd, &ev);
    ev.data.u64 = kEventId;
    epoll_ctl(w->epfd, EPOLL_CTL_ADD, w->efd, &ev);
    impl_->workers.push_back(std::move(w));
  }
  for (int t = 0; t < threads_; ++t)
    impl_->workers[(size_t)t]->th = std::thread([this, t] { impl_->run_worker(t); });
  impl_->gpu_th = std::thread([this] { impl_->run_gpu(); });
}

void HttpFront::stop() {
  if (!impl_ || !impl_->running.exchange(false)) return;
  impl_->gpu_cv.notify_all();
  if (impl_->gpu_th.joinable()) impl_->gpu_th.join();
  for (auto& w : impl_->workers) {
    if (w->th.joinable()) w->th.join();
    ::close(w->lfd);
    ::close(w->epfd);
    ::close(w->efd);
  }
  impl_->workers.clear();
}

void HttpFront::set_model(std::shared_ptr<const RuleIndex> index,
                          const std::vector<std::string>& names,
                          const std::vector<std::string>& best_names, const std::string* marker,
                          std::shared_ptr<gpu::GpuRuleIndex> gpu, int gpu_min_batch,
                          int gpu_min_merge) {
  KMLS_CHECK(index != nullptr, "set_model: no index");
  KMLS_CHECK((int64_t)names.size() == index->n_items(), "set_model: names != index items");
  auto m = std::make_shared<FrontModel>();
  m->index = std::move(index);
  m->names_json.reserve(names.size());
  m->name_to_id.reserve(names.size() * 2);
  for (size_t i = 0; i < names.size(); ++i) {
    std::string j;
    json_escape_append(j, names[i]);
    m->names_json.push_back(std::move(j));
    m->name_to_id.emplace(names[i], (int32_t)i);  // first occurrence wins (dict comprehension: last)
  }
  // name_to_id in Python ({n: i for i, n in enumerate(names)}) keeps the LAST id of a repeated
  // name: do the same
  for (size_t i = 0; i < names.size(); ++i) m->name_to_id[names[i]] = (int32_t)i;
  for (const auto& b : best_names) {
    std::string j;
    json_escape_append(j, b);
    m->best_json.push_back(std::move(j));
  }
  if (marker) json_escape_append(m->marker_json, *marker);
  else m->marker_json = "null";
  m->gpu = std::move(gpu);
  m->gpu_min_batch = m->gpu ? std::max(0, gpu_min_batch) : 0;
  m->gpu_min_merge = m->gpu ? gpu_min_merge : -1;
  std::shared_ptr<const FrontModel> cm = m;
  retire(std::atomic_exchange(&impl_->model, cm));
}

void HttpFront::clear_model() {
  std::shared_ptr<const FrontModel> none;
  retire(std::atomic_exchange(&impl_->model, none));
}

// Keep `prev` alive until the next swap; the model retired before it is released here, on the
// caller's (reload) thread.
void HttpFront::retire(std::shared_ptr<const FrontModel> prev) {
  std::shared_ptr<const FrontModel> old;
  {
    std::lock_guard<std::mutex> lk(impl_->retire_mu);
    old = std::move(impl_->retired);
    impl_->retired = std::move(prev);
  }
  old.reset();
}

bool HttpFront::next_slow(SlowRequest& out) {
  std::lock_guard<std::mutex> lk(impl_->slow_mu);
  if (impl_->slow_q.empty()) {
    uint64_t v;
    (void)!read(slow_efd_, &v, 8);  // drain the doorbell (non-blocking)
    return false;
  }
  out = std::move(impl_->slow_q.front());
  impl_->slow_q.pop_front();
  return true;
}

void HttpFront::respond(uint64_t token, int status,
                        const std::vector<std::pair<std::string, std::string>>& headers,
                        const std::string& body) {
  const int wi = (int)(token >> 56);
  const uint64_t conn = token & ((1ull << 56) - 1);
  if (wi < 0 || wi >= (int)impl_->workers.size()) return;
  Impl::Worker& w = *impl_->workers[(size_t)wi];
  bool close = false, has_len = false, has_date = false, has_server = false;
  std::string r = "HTTP/1.1 " + std::to_string(status) + " " + reason(status) + "\r\n";
  for (const auto& h : headers) {
    const std::string n = lower(h.first);
    if (n == "content-length") has_len = true;
    if (n == "date") has_date = true;
    if (n == "server") has_server = true;
    if (n == "connection" && lower(h.second).find("close") != std::string::npos) close = true;
    r += h.first;
    r += ": ";
    r += h.second;
    r += "\r\n";
  }
  {
    std::lock_guard<std::mutex> lk(w.mu);
    if (!has_date) {
      r += "date: ";
      r += impl_->date_hdr(w);
      r += "\r\n";
    }
  }
  if (!has_server) r += "server: kmls\r\n";
  if (!has_len) r += "content-length: " + std::to_string(body.size()) + "\r\n";
  r += "\r\n";
  r += body;  // (HEAD: Starlette already sent no body)
  impl_->post(wi, conn, std::move(r), close);
}

FrontStats HttpFront::stats() const {
  FrontStats s;
  s.requests = impl_->st_requests;
  s.native_ok = impl_->st_native;
  s.fallback = impl_->st_fallback;
  s.slow = impl_->st_slow;
  s.gpu_batches = impl_->st_gpu_batches;
  s.gpu_queries = impl_->st_gpu_queries;
  s.gpu_loop_batches = impl_->st_gpu_loop;
  s.gpu_loop_refused = impl_->st_gpu_loop_refused;
  s.connections = impl_->st_conns;
  s.bytes_in = impl_->st_in;
  s.bytes_out = impl_->st_out;
  return s;
}

}  // namespace kmls
