// Wave64 helpers shared by the CDNA4 kernels (device code).  Included with angle brackets so the
// CPU wave emulator (csrc/emu, tests only) can substitute its own definitions by include order.
#pragma once

#include <hip/hip_runtime.h>

namespace kmls {
namespace kern {

// A lane-varying zero: indices built from it are divergent, so the compiler emits vector loads.
// Data a wave writes with vector stores and reads back later in the same launch must not be read
// through the scalar cache, which vector stores do not update.
__device__ __forceinline__ unsigned vzero() {
  unsigned z = 0;
  asm volatile("" : "+v"(z));
  return z;
}

__device__ __forceinline__ unsigned long long bcast64(unsigned long long v, int src) {
  const unsigned lo = __shfl((unsigned)v, src, 64);
  const unsigned hi = __shfl((unsigned)(v >> 32), src, 64);
  return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ unsigned long long shfl_xor64(unsigned long long v, int m) {
  const unsigned lo = __shfl_xor((unsigned)v, m, 64);
  const unsigned hi = __shfl_xor((unsigned)(v >> 32), m, 64);
  return ((unsigned long long)hi << 32) | lo;
}

// (the builtin returns int: both halves go through unsigned, or the low half sign-extends)
__device__ __forceinline__ unsigned uni(unsigned v) {
  return (unsigned)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ unsigned long long uni64(unsigned long long v) {
  return ((unsigned long long)uni((unsigned)(v >> 32)) << 32) | uni((unsigned)v);
}

// Cross-wave hand-off (work queues inside one launch): loads that observe another CU's
// stores go to L2 (agent-scope atomic load, no stale vector-L1 line); the fence orders this
// wave's earlier stores before a later flag store (release) and invalidates L1 after a flag was
// seen (acquire).
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fence_agent() { __threadfence(); }
__device__ __forceinline__ void wait_short() { __builtin_amdgcn_s_sleep(8); }

}  // namespace kern
}  // namespace kmls
