// Optional roctx ranges: KMLS_ROCTX=1 loads the ROCm roctx library at first use
// and brackets the framework's phases (mining prologue / levels, rules, group-by), so a
// `rocprofv3 --marker-trace` timeline shows them over the kernels.  Off (or the library
// missing) → every call is a no-op branch.
#pragma once

namespace kmls {
namespace trace {

bool enabled();
void push(const char* name);
void pop();

struct Range {
  explicit Range(const char* name) { push(name); }
  ~Range() { pop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

}  // namespace trace
}  // namespace kmls
