// Emulator stand-in for the hipCUB device scans the kernels' host code calls (tests only): a
// serial host scan over the emulator's host-memory "device" buffers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace hipcub {
struct DeviceScan {
  template <typename In, typename Out>
  static hipError_t ExclusiveSum(void* tmp, size_t& bytes, In in, Out out, int n,
                                 hipStream_t = nullptr) {
    if (tmp == nullptr) {
      bytes = 16;
      return hipSuccess;
    }
    using T = typename std::remove_reference<decltype(*out)>::type;
    T run = 0;
    for (int i = 0; i < n; ++i) {
      const T v = (T)in[i];
      out[i] = run;
      run += v;
    }
    return hipSuccess;
  }
};
}  // namespace hipcub
