// Test hooks: KMLS_TEST_HOOKS="name=value,name=value" forces a code path that production sizes
// never reach on the small test inputs (a fallback, a split, a tiny capacity).  One variable for
// all of them, read at the call (tests set it per case); unset = every hook returns its default.
#pragma once

#include <cstdlib>
#include <cstring>
#include <string>

namespace kmls {

inline long long test_hook(const char* name, long long dflt) {
  const char* e = std::getenv("KMLS_TEST_HOOKS");
  if (!e || !*e) return dflt;
  const size_t n = std::strlen(name);
  for (const char* p = e; *p;) {
    const char* end = std::strchr(p, ',');
    const size_t len = end ? (size_t)(end - p) : std::strlen(p);
    if (len > n + 1 && std::strncmp(p, name, n) == 0 && p[n] == '=')
      return std::atoll(std::string(p + n + 1, len - n - 1).c_str());
    if (!end) break;
    p = end + 1;
  }
  return dflt;
}

}  // namespace kmls
