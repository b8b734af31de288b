// Item-sharded mining support (parallel/item_shard.py): each rank holds its item shard's bitmap
// rows over ALL transactions (1/N of the replicated bitmap); a batch of root classes is mined on
// the rows of every item compressed onto the union of the batch roots' transactions.
//
//   k_rows_union    mask[w] = OR of rows idx[0..n) at word w          (thread per word)
//   k_word_popc     cnt[w] = popcount(mask[w])                         (thread per word)
//   k_compact_rows  out[r] = rows[r] compressed onto mask (bit-gather)  (thread per nonzero
//                   mask word x row block; the compressed bits of word k land at bit offset
//                   off[k] of the output row, straddling at most two output words)
//
// The compress of one 64-bit word is the 6-round move-mask network (Hacker's Delight 7-4), the
// same primitive k_deep_root uses for its tid projection.  Two lanes can write into one output
// word (the tail of word k and the head of word k+1), so the stores are atomicOr into a zeroed
// output.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace kmls::kern {
namespace {

__device__ __forceinline__ unsigned long long compress64(unsigned long long x, unsigned long long m) {
  x &= m;
  unsigned long long mk = ~m << 1;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    unsigned long long mp = mk ^ (mk << 1);
    mp ^= mp << 2;
    mp ^= mp << 4;
    mp ^= mp << 8;
    mp ^= mp << 16;
    mp ^= mp << 32;
    const unsigned long long mv = mp & m;
    m = (m ^ mv) | (mv >> (1u << i));
    const unsigned long long t = x & mv;
    x = (x ^ t) | (t >> (1u << i));
    mk &= ~mp;
  }
  return x;
}

__global__ __launch_bounds__(256) void k_rows_union(const unsigned long long* rows, long long Wp,
                                                    const int32_t* idx, int n, long long W,
                                                    unsigned long long* mask) {
  for (long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x; w < W;
       w += (long long)gridDim.x * blockDim.x) {
    unsigned long long v = 0;
    for (int k = 0; k < n; ++k) v |= rows[(long long)idx[k] * Wp + w];
    mask[w] = v;
  }
}

__global__ __launch_bounds__(256) void k_word_popc(const unsigned long long* mask, long long W,
                                                   int32_t* cnt) {
  for (long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x; w < W;
       w += (long long)gridDim.x * blockDim.x)
    cnt[w] = __popcll(mask[w]);
}

// blockIdx.y strides the rows; each thread keeps its word's mask in registers across the rows
__global__ __launch_bounds__(256) void k_compact_rows(const unsigned long long* rows, long long R,
                                                      long long Wp_in,
                                                      const unsigned long long* mask,
                                                      const int64_t* nzw, const int64_t* off,
                                                      long long n_nz, unsigned long long* out,
                                                      long long Wp_out) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_nz) return;
  const long long w = nzw[k];
  const unsigned long long m = mask[w];
  const long long b = off[k];
  const long long q = b >> 6;
  const int sh = (int)(b & 63);
  const int n = __popcll(m);
  for (long long r = blockIdx.y; r < R; r += gridDim.y) {
    const unsigned long long x = compress64(rows[r * Wp_in + w], m);
    if (!x) continue;
    unsigned long long* o = out + r * Wp_out;
    atomicOr(o + q, x << sh);
    if (sh && sh + n > 64) atomicOr(o + q + 1, x >> (64 - sh));
  }
}

unsigned grid_for(long long n) {
  const long long g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : g > 65535 ? 65535 : g);
}

}  // namespace

void rows_union(const uint64_t* rows, int64_t Wp, const int32_t* idx, int n, int64_t W,
                uint64_t* mask, hipStream_t s) {
  if (W <= 0) return;
  hipLaunchKernelGGL(k_rows_union, dim3(grid_for(W)), dim3(256), 0, s,
                     (const unsigned long long*)rows, (long long)Wp, idx, n, (long long)W,
                     (unsigned long long*)mask);
}

void word_popc(const uint64_t* mask, int64_t W, int32_t* cnt, hipStream_t s) {
  if (W <= 0) return;
  hipLaunchKernelGGL(k_word_popc, dim3(grid_for(W)), dim3(256), 0, s,
                     (const unsigned long long*)mask, (long long)W, cnt);
}

void compact_rows(const uint64_t* rows, int64_t R, int64_t Wp_in, const uint64_t* mask,
                  const int64_t* nzw, const int64_t* off, int64_t n_nz, uint64_t* out,
                  int64_t Wp_out, hipStream_t s) {
  if (R <= 0 || n_nz <= 0) return;
  const unsigned gx = (unsigned)((n_nz + 255) / 256);
  const unsigned gy = (unsigned)(R < 64 ? R : 64);
  hipLaunchKernelGGL(k_compact_rows, dim3(gx, gy), dim3(256), 0, s,
                     (const unsigned long long*)rows, (long long)R, (long long)Wp_in,
                     (const unsigned long long*)mask, nzw, off, (long long)n_nz, (unsigned long long*)out,
                     (long long)Wp_out);
}

}  // namespace kmls::kern
