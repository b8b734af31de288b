// CPU wave emulator of the HIP subset the kmls kernels use (tests only; never part of _native).
//
// Every lane is a host thread; a workgroup's threads run together and blocks run one after the
// other, so `__shared__` becomes a function-static.  Cross-lane operations (__shfl*, __ballot,
// readfirstlane) exchange values through the wave's slots between two barriers, so the kernel's
// own source runs unchanged under AddressSanitizer/UBSan.  A cross-lane operation that not all 64
// lanes reach (divergent control flow around a wave op) is reported as a deadlock instead of
// hanging.  Host-side HIP runtime calls map to malloc/memcpy; streams are synchronous.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__ static

struct uint2 {  // HIP's vector types, as far as the shared headers name them
  unsigned int x, y;
};
inline uint2 make_uint2(unsigned int x, unsigned int y) { return uint2{x, y}; }
struct alignas(16) ulonglong2 {
  unsigned long long x, y;
};
struct alignas(16) int4 {
  int x, y, z, w;
};
inline int4 make_int4(int x, int y, int z, int w) { return int4{x, y, z, w}; }

struct dim3 {
  unsigned x, y, z;
  constexpr dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};

namespace emu {

struct Wave {
  std::mutex mu;
  std::condition_variable cv;
  int nlanes = 64;
  int arrived = 0;
  uint64_t gen = 0;
  uint64_t slot[64] = {0};
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t g = gen;
    if (++arrived == nlanes) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(30), [&] { return gen != g; })) {
      std::fprintf(stderr, "emu: wave deadlock (a cross-lane op not reached by every lane)\n");
      std::abort();
    }
  }
};

// the workgroup's barrier (__syncthreads): every live thread of the block; a finished thread
// leaves the count, so the others are not left waiting for it
struct Block {
  std::mutex mu;
  std::condition_variable cv;
  int alive = 0;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<unsigned char> dyn;  // the launch's dynamic LDS (extern __shared__)
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t g = gen;
    if (++arrived >= alive) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(60), [&] { return gen != g; })) {
      std::fprintf(stderr, "emu: block deadlock (a __syncthreads not reached by every thread)\n");
      std::abort();
    }
  }
  void leave() {
    std::unique_lock<std::mutex> lk(mu);
    alive -= 1;
    if (arrived > 0 && arrived >= alive) {
      arrived = 0;
      ++gen;
    }
    cv.notify_all();
  }
};

struct Lane {
  int lane = 0;
  Wave* wave = nullptr;
  Block* block = nullptr;
  dim3 tidx;
};

inline thread_local Lane* tl = nullptr;
inline dim3 g_block_idx, g_block_dim, g_grid_dim;

inline uint64_t xchg(uint64_t mine, int src) {
  Wave* w = tl->wave;
  w->slot[tl->lane] = mine;
  w->barrier();
  const uint64_t r = w->slot[src & 63];
  w->barrier();
  return r;
}

// returns int, as the builtin does (callers must not widen it with sign extension)
inline int readfirstlane(int v) { return (int)(uint32_t)xchg((uint32_t)v, 0); }

}  // namespace emu

#define threadIdx (emu::tl->tidx)
#define blockIdx (emu::g_block_idx)
#define blockDim (emu::g_block_dim)
#define gridDim (emu::g_grid_dim)

#define __builtin_amdgcn_readfirstlane(v) emu::readfirstlane(v)
namespace emu {
// the GPU executes a wave's memory operations in program order across its lanes; the emulator's
// lane threads synchronise at the kernel's wave barriers to model that
inline void wave_barrier() { tl->wave->barrier(); }
}  // namespace emu
#define __builtin_amdgcn_wave_barrier() emu::wave_barrier()

inline unsigned __shfl(unsigned v, int src, int = 64) { return (unsigned)emu::xchg(v, src); }
inline int __shfl(int v, int src, int = 64) { return (int)emu::xchg((uint32_t)v, src); }
inline long long __shfl(long long v, int src, int = 64) {
  return (long long)emu::xchg((uint64_t)v, src);
}
inline unsigned long long __shfl(unsigned long long v, int src, int = 64) {
  return emu::xchg(v, src);
}
inline void __syncthreads() { emu::tl->block->barrier(); }
namespace emu {
inline void* dyn_lds() { return tl->block->dyn.data(); }
}  // namespace emu
inline unsigned __shfl_up(unsigned v, unsigned delta, int = 64) {
  const int l = emu::tl->lane;
  const int src = l - (int)delta;
  return (unsigned)emu::xchg(v, src >= 0 ? src : l);
}
inline unsigned __shfl_xor(unsigned v, int m, int = 64) {
  return (unsigned)emu::xchg(v, emu::tl->lane ^ m);
}
inline unsigned long long __ballot(int pred) {
  emu::Wave* w = emu::tl->wave;
  w->slot[emu::tl->lane] = pred ? 1 : 0;
  w->barrier();
  unsigned long long m = 0;
  for (int i = 0; i < 64; ++i)
    if (w->slot[i]) m |= 1ull << i;
  w->barrier();
  return m;
}
// HIP's device min/max (the kernels call them unqualified)
template <typename A, typename B>
inline auto min(A a, B b) -> decltype(a < b ? a : b) { return a < b ? a : b; }
template <typename A, typename B>
inline auto max(A a, B b) -> decltype(a > b ? a : b) { return a > b ? a : b; }
inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
inline int __popc(unsigned x) { return __builtin_popcount(x); }
inline unsigned long long wall_clock64() {
  return (unsigned long long)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count() / 10;  // 100 MHz
}

template <typename T> inline T atomicAdd(T* p, T v) { return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
template <typename T> inline T atomicSub(T* p, T v) { return __atomic_fetch_sub(p, v, __ATOMIC_SEQ_CST); }
template <typename T> inline T atomicOr(T* p, T v) { return __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
template <typename T> inline T atomicXor(T* p, T v) { return __atomic_fetch_xor(p, v, __ATOMIC_SEQ_CST); }
template <typename T> inline T atomicExch(T* p, T v) { return __atomic_exchange_n(p, v, __ATOMIC_SEQ_CST); }
template <typename T> inline T atomicCAS(T* p, T cmp, T v) {
  __atomic_compare_exchange_n(p, &cmp, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
  return cmp;  // the old value (== the expected one on success)
}
template <typename T> inline T atomicMax(T* p, T v) {
  T old = __atomic_load_n(p, __ATOMIC_SEQ_CST);
  while (v > old && !__atomic_compare_exchange_n(p, &old, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
  }
  return old;
}
template <typename T> inline T atomicMin(T* p, T v) {
  T old = __atomic_load_n(p, __ATOMIC_SEQ_CST);
  while (v < old && !__atomic_compare_exchange_n(p, &old, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
  }
  return old;
}

// ---- host runtime subset ----
typedef int hipError_t;
typedef void* hipStream_t;
constexpr hipError_t hipSuccess = 0;
enum hipMemcpyKind { hipMemcpyHostToHost, hipMemcpyHostToDevice, hipMemcpyDeviceToHost,
                     hipMemcpyDeviceToDevice, hipMemcpyDefault };
enum hipDeviceAttribute_t { hipDeviceAttributeWallClockRate = 1 };
inline const char* hipGetErrorString(hipError_t) { return "emulator error"; }
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipMalloc(void** p, size_t n) {
  *p = std::malloc(std::max<size_t>(n, 1));
  if (!*p) return 2;
  std::memset(*p, 0xCD, n);  // device memory starts as garbage
  return hipSuccess;
}
inline hipError_t hipFree(void* p) { std::free(p); return hipSuccess; }
inline hipError_t hipHostMalloc(void** p, size_t n, unsigned = 0) { return hipMalloc(p, n); }
inline hipError_t hipHostFree(void* p) { std::free(p); return hipSuccess; }
inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t = nullptr) {
  if (n) std::memmove(d, s, n);
  return hipSuccess;
}
inline hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind k) { return hipMemcpyAsync(d, s, n, k); }
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t = nullptr) {
  std::memset(p, v, n);
  return hipSuccess;
}
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
constexpr unsigned hipHostMallocDefault = 0, hipHostMallocMapped = 2, hipHostMallocCoherent = 4;
enum hipFuncAttribute { hipFuncAttributeMaxDynamicSharedMemorySize = 8 };
inline hipError_t hipFuncSetAttribute(const void*, hipFuncAttribute, int) { return hipSuccess; }
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t, int) {
  *v = 100000;  // kHz of wall_clock64 above
  return hipSuccess;
}

// one workgroup at a time, every thread a host thread, grouped into waves of 64
template <typename K, typename... Args>
inline void hipLaunchKernelGGL(K kernel, dim3 grid, dim3 block, size_t shared, hipStream_t,
                               Args... args) {
  emu::g_grid_dim = grid;
  emu::g_block_dim = block;
  const unsigned nt = block.x;
  const unsigned nw = (nt + 63) / 64;
  for (unsigned by = 0; by < grid.y; ++by)
  for (unsigned bx = 0; bx < grid.x; ++bx) {
    emu::g_block_idx = dim3(bx, by);
    std::vector<emu::Wave> waves(nw);
    for (unsigned w = 0; w < nw; ++w) waves[w].nlanes = (int)std::min(64u, nt - 64 * w);
    emu::Block blk;
    blk.alive = (int)nt;
    blk.dyn.assign(std::max<size_t>(shared, 16), (unsigned char)0xCD);  // LDS starts as garbage
    std::vector<std::thread> th;
    th.reserve(nt);
    for (unsigned t = 0; t < nt; ++t) {
      th.emplace_back([&, t] {
        emu::Lane me;
        me.lane = (int)(t & 63);
        me.wave = &waves[t / 64];
        me.block = &blk;
        me.tidx = dim3(t);
        emu::tl = &me;
        kernel(args...);
        // a finished lane keeps answering its wave's barriers until every lane is done
        emu::Wave* w = me.wave;
        {
          std::unique_lock<std::mutex> lk(w->mu);
          w->nlanes -= 1;
          if (w->arrived >= w->nlanes && w->arrived > 0) {
            w->arrived = 0;
            ++w->gen;
          }
          w->cv.notify_all();
        }
        blk.leave();
      });
    }
    for (auto& x : th) x.join();
  }
}
