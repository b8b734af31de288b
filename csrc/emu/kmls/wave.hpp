// Emulator version of kmls/wave.hpp (csrc/emu/hip/hip_runtime.h): same helpers, no inline asm.
#pragma once

#include <hip/hip_runtime.h>

#define KMLS_DYN_LDS(T, name) T* name = (T*)emu::dyn_lds()

namespace kmls {
namespace kern {

inline unsigned vzero() { return 0u; }

template <typename T>
using gptr = T*;
template <typename T>
inline gptr<T> as_global(T* p) { return p; }
template <typename T>
inline gptr<T> as_global_addr(unsigned long long a) { return (T*)a; }

inline unsigned long long bcast64(unsigned long long v, int src) {
  return emu::xchg(v, src);
}
inline unsigned long long shfl_xor64(unsigned long long v, int m) {
  return emu::xchg(v, emu::tl->lane ^ m);
}
inline unsigned uni(unsigned v) { return (unsigned)__builtin_amdgcn_readfirstlane((int)v); }
inline unsigned lane0(unsigned v) { return (unsigned)emu::xchg((unsigned long long)v, 0); }
inline unsigned long long lane0_64(unsigned long long v) { return emu::xchg(v, 0); }
inline unsigned long long uni64(unsigned long long v) {
  return ((unsigned long long)uni((unsigned)(v >> 32)) << 32) | uni((unsigned)v);
}

inline unsigned long long ld_agent(const unsigned long long* p) { return __atomic_load_n(p, __ATOMIC_SEQ_CST); }
inline unsigned ld_agent(const unsigned* p) { return __atomic_load_n(p, __ATOMIC_SEQ_CST); }
inline void st_agent(unsigned long long* p, unsigned long long v) { __atomic_store_n(p, v, __ATOMIC_SEQ_CST); }
inline void st_agent(unsigned* p, unsigned v) { __atomic_store_n(p, v, __ATOMIC_SEQ_CST); }
inline void wait_stores() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }
inline void wait_short(unsigned) { std::this_thread::yield(); }

}  // namespace kern
}  // namespace kmls
