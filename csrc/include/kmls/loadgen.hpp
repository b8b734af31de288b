// Open-loop HTTP load generator (loadgen.cpp) for the serving benchmark.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace kmls {

struct LoadResult {
  std::vector<int64_t> lat_ns;  // completion - scheduled send time, per answered request
  std::vector<int64_t> lag_ns;  // actual - scheduled send time (client/connection backlog)
  std::vector<int64_t> at_ns;   // scheduled send time of each answered request, from the start
  int64_t offered = 0, sent = 0, completed = 0, errors = 0;  // errors: non-200 answers
  double duration_s = 0;
};

// requests: complete HTTP/1.1 request byte strings, used round robin
LoadResult run_loadgen(const std::string& host, int port, const std::vector<std::string>& requests,
                       double qps, double duration_s, int connections, int threads,
                       double drain_s = 5.0);

}  // namespace kmls
