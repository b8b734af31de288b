// roctx ranges through dlopen (no link-time dependency): see kmls/trace.hpp.
#include "kmls/trace.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <mutex>

namespace kmls {
namespace trace {
namespace {

using push_fn = int (*)(const char*);
using pop_fn = int (*)();

struct Roctx {
  push_fn push = nullptr;
  pop_fn pop = nullptr;
  Roctx() {
    const char* e = std::getenv("KMLS_ROCTX");
    if (!(e && e[0] == '1')) return;
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                            "libroctx64.so.4", "libroctx64.so"}) {
      void* h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
      if (!h) continue;
      push = (push_fn)dlsym(h, "roctxRangePushA");
      pop = (pop_fn)dlsym(h, "roctxRangePop");
      if (push && pop) return;
      push = nullptr;
      pop = nullptr;
    }
  }
};

const Roctx& lib() {
  static const Roctx r;
  return r;
}

}  // namespace

bool enabled() { return lib().push != nullptr; }
void push(const char* name) {
  if (const auto f = lib().push) f(name);
}
void pop() {
  if (const auto f = lib().pop) f();
}

}  // namespace trace
}  // namespace kmls
