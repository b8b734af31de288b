// Native HTTP/1.1 serving front of the recommendation API (http_front.cpp).
//
// The reference serves POST /api/recommend/ from FastAPI on uvicorn with the C/Cython
// httptools + uvloop stack (fastapi[standard], rest_api/pyproject.toml:7-11; SURVEY §2.B "HTTP
// parse / event loop").  Neither is in this image, and pure-Python h11 parsing caps one process
// at a few thousand requests per second.  This front is the native replacement:
//   * N I/O threads, one SO_REUSEPORT listening socket + epoll loop each (the kernel spreads
//     connections), HTTP/1.1 keep-alive, pipelining-safe (one request in flight per connection);
//   * the hot route (POST /api/recommend/ with a well-formed {"songs": [str, ...]} body) is
//     answered natively: seed names -> ids, the C++ matcher or (micro-batched across connections)
//     the HIP matcher over the HBM rule index, the static fallback, and the exact JSON bytes
//     FastAPI would send ({"songs", "model_date", "version"}, json.dumps(ensure_ascii=False));
//   * EVERY other request (other routes, /docs, malformed or empty bodies, not-loaded model) is
//     handed to the FastAPI app itself (an asyncio loop in the same process drains a queue
//     signalled through an eventfd), so status codes, 422 bodies and headers stay FastAPI's.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "kmls/host.hpp"

namespace kmls {

namespace gpu { class GpuRuleIndex; }

// One immutable model generation (swapped atomically on hot reload).
struct FrontModel {
  std::shared_ptr<const RuleIndex> index;
  std::vector<std::string> names_json;  // item id -> name as a JSON string literal
  std::unordered_map<std::string, int32_t> name_to_id;
  std::vector<std::string> best_json;   // best-track names (fallback pool) as JSON literals
  std::string marker_json;              // model_date: JSON string literal or null
  std::shared_ptr<gpu::GpuRuleIndex> gpu;  // HBM index (optional)
  int gpu_min_batch = 0;                // batches >= this go to the GPU (0: never)
  // persistent serving kernel (gpu::GpuServeLoop): a query whose merged rows hold at least this
  // many entries (and fit the wave matcher) is answered by the loop, whatever the batch;
  // -1 = off (batch routing by gpu_min_batch)
  int gpu_min_merge = -1;
};

struct FrontStats {
  uint64_t requests = 0, native_ok = 0, fallback = 0, slow = 0, gpu_batches = 0,
           gpu_queries = 0, connections = 0, bytes_in = 0, bytes_out = 0;
  uint64_t gpu_loop_batches = 0, gpu_loop_refused = 0;  // (of gpu_batches) via the serving loop
};

struct SlowRequest {  // a request handed to the Python (FastAPI) side
  uint64_t token = 0;
  std::string method, path, query, http_version;
  std::vector<std::pair<std::string, std::string>> headers;  // names lower-cased
  std::string body;
  std::string client_host;
  int client_port = 0;
};

class HttpFront {
 public:
  // k: recommendations per response (K_BEST_TRACKS); version: the VERSION string
  HttpFront(const std::string& host, int port, int threads, int k, const std::string& version,
            int batch_max, int batch_wait_us);
  ~HttpFront();
  HttpFront(const HttpFront&) = delete;
  HttpFront& operator=(const HttpFront&) = delete;

  void start();
  void stop();
  int port() const { return port_; }

  // hot reload: build and publish a new model generation (the old one is released when the
  // last request that holds it finishes)
  void set_model(std::shared_ptr<const RuleIndex> index, const std::vector<std::string>& names,
                 const std::vector<std::string>& best_names, const std::string* marker,
                 std::shared_ptr<gpu::GpuRuleIndex> gpu, int gpu_min_batch,
                 int gpu_min_merge = -1);
  void clear_model();
  void retire(std::shared_ptr<const FrontModel> prev);  // (internal: deferred release)

  // Python side of the slow path: the eventfd becomes readable when requests are queued
  int slow_fd() const { return slow_efd_; }
  bool next_slow(SlowRequest& out);  // non-blocking; false when the queue is empty
  void respond(uint64_t token, int status, const std::vector<std::pair<std::string, std::string>>& headers,
               const std::string& body);
  FrontStats stats() const;

  struct Impl;

 private:
  std::string host_;
  int port_;
  int threads_;
  int slow_efd_ = -1;
  Impl* impl_ = nullptr;
};

// The static fallback pool sampler, bit-exact with CPython's random.Random(seed).sample(pool, k)
// (MT19937 init_by_array + _randbelow + sample's list/set branches), so the native front and the
// Python matcher return the same fallback list (serve/matcher.py: static_recommendation).
std::vector<int> python_random_sample(uint64_t seed, int n, int k);
// FNV-1a 64 of "\x1f".join(sorted(seeds)) (UTF-8): the fallback seed (serve/matcher.py)
uint64_t fallback_seed(std::vector<std::string> seeds);

// JSON string literal as json.dumps(s, ensure_ascii=False) writes it
void json_escape_append(std::string& out, const std::string& s);

}  // namespace kmls
