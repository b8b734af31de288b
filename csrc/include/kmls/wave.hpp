// Wave64 helpers shared by the CDNA4 kernels (device code).  Included with angle brackets so the
// CPU wave emulator (csrc/emu, tests only) can substitute its own definitions by include order.
#pragma once

#include <hip/hip_runtime.h>

// Dynamic LDS of a kernel (`extern __shared__ T name[]`); the CPU wave emulator maps it to the
// launch's dynamic-LDS buffer.
#define KMLS_DYN_LDS(T, name) extern __shared__ T name[]

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

// A pointer the compiler must treat as GLOBAL memory (address space 1).  A row pointer rebuilt
// from an integer (a frame's block address) is otherwise generic, so its loads become flat_load:
// those count in lgkmcnt as well as vmcnt and may return out of order, so every later wait for
// an LDS result also waits for the row loads in flight.  Through a gptr they are global_load.
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ gptr<T> as_global(T* p) {
  return (gptr<T>)p;
}
template <typename T>
__device__ __forceinline__ gptr<T> as_global_addr(unsigned long long a) {
  return (gptr<T>)a;
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

// lane 0's value (uniform) whichever lanes are active
__device__ __forceinline__ unsigned lane0(unsigned v) {
  return (unsigned)__builtin_amdgcn_readlane((int)v, 0);
}
__device__ __forceinline__ unsigned long long lane0_64(unsigned long long v) {
  return ((unsigned long long)lane0((unsigned)(v >> 32)) << 32) | lane0((unsigned)v);
}

// (the builtin returns int: both halves go through unsigned, or the low half sign-extends)
__device__ __forceinline__ unsigned uni(unsigned v) {
  return (unsigned)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ unsigned long long uni64(unsigned long long v) {
  return ((unsigned long long)uni((unsigned)(v >> 32)) << 32) | uni((unsigned)v);
}

// Cross-wave hand-off inside one launch (work queues).  The 8 XCDs' L2 caches are not coherent
// with each other, and an agent-scope fence writes back / invalidates a whole L2, so hand-offs
// avoid fences: the producer writes the handed-over data with agent-scope (write-through)
// stores, waits for them to complete (wait_stores), then sets a flag with an atomic; the
// consumer reads the flag and the small descriptors with agent-scope loads.  Bulk data read
// afterwards with plain loads lives in 128-byte-aligned lines no wave of the launch has read
// before it was published, so no cache holds a stale copy of it.
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wait_stores() { __builtin_amdgcn_s_waitcnt(0); }
__device__ __forceinline__ void wait_short(unsigned n) {
  // s_sleep takes an immediate: a few fixed steps of backoff
  if (n < 4) __builtin_amdgcn_s_sleep(2);
  else if (n < 16) __builtin_amdgcn_s_sleep(16);
  else __builtin_amdgcn_s_sleep(127);
}

}  // namespace kern
}  // namespace kmls
