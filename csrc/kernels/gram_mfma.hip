// Level-2 co-occurrence GEMM on the matrix cores: G = A·Aᵀ over the transaction axis, with A
// the 0/1 one-hot matrix of frequent items stored as packed tid-bitmaps (SURVEY §2.C O8,
// BASELINE north star "MFMA int8 one-hot×one-hot co-occurrence GEMM for the first pass").
//
// v_mfma_i32_32x32x32_i8 (gfx950): lane l (r = l&31, h = l>>5) supplies A[row r][k = 16h + j]
// and B[k = 16h + j][col r], j = 0..15, as 16 int8 in 4 VGPRs; C/D (16 i32 / lane):
// col = l&31, row = (reg&3) + 8*(reg>>2) + 4*h.  Bits are unpacked to int8 in registers
// (each byte of bits → 8 int8 through an LDS lookup table), so HBM/L2 traffic stays at 1 bit
// per (item, transaction) — 8x fewer bytes than an int8 one-hot operand.
//
// Tiling: 256-thread block = 4 waves (2x2) → 128x128 output tile; each wave 64x64 = 2x2 MFMA
// tiles (4 accumulators, 64 AGPRs) so every unpacked fragment feeds 2 MFMAs.  Row words are
// read 32 B at a time per lane (4 words = 256 transactions = 8 K-steps of 32).  Only upper-
// triangular block tiles are launched (G is symmetric); blocks are remapped XCD-aware so the
// tiles of one tile-row share an XCD L2.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "kernels.hpp"

namespace kmls {
namespace kern {

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// 16 bits → 16 int8 {0,1} (k order = bit order) through a 256-entry byte → 8-bytes table in LDS:
// two ds_read_b64 per fragment instead of 12 VALU (PMC counters showed the arithmetic unpack at
// 15 VALU instructions per MFMA and the matrix cores 40 % busy; the table moves the expansion to
// the LDS pipe, well inside its budget at one fragment per 2 MFMAs)
__device__ __forceinline__ v4i unpack16(uint32_t bits, const uint2* __restrict__ lut) {
  const uint2 lo = lut[bits & 0xFFu], hi = lut[(bits >> 8) & 0xFFu];
  v4i r;
  r.x = (int)lo.x;
  r.y = (int)lo.y;
  r.z = (int)hi.x;
  r.w = (int)hi.y;
  return r;
}

__device__ __forceinline__ uint32_t nib(uint32_t x) { return (x * 0x00204081u) & 0x01010101u; }

constexpr int kTile = 128;
constexpr int64_t kStripe = 16;  // words per split-K stripe

__global__ __launch_bounds__(256) void k_pair_gram_mfma(const unsigned long long* __restrict__ bm,
                                                         int64_t Wp, int64_t F, int64_t n_tiles,
                                                         int64_t n_blocks,
                                                         uint32_t* __restrict__ out) {
  __shared__ uint2 lut[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x)
    lut[i] = make_uint2(nib((uint32_t)i & 0xFu), nib((uint32_t)i >> 4));
  __syncthreads();
  // XCD-aware bijective remap (cdna_hip_programming.md §5): consecutive logical tiles go to
  // the same XCD (blockIdx % 8 labels an XCD group).
  const int64_t orig = blockIdx.x;
  const int64_t q = n_blocks / 8, rr = n_blocks % 8, xcd = orig % 8;
  int64_t idx = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  int64_t ti = 0;
  while (idx >= n_tiles - ti) { idx -= n_tiles - ti; ++ti; }
  const int64_t tj = ti + idx;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  const int64_t a0 = ti * kTile + wr * 64 + r, a1 = a0 + 32;
  const int64_t b0 = tj * kTile + wc * 64 + r, b1 = b0 + 32;
  const bool va0 = a0 < F, va1 = a1 < F, vb0 = b0 < F, vb1 = b1 < F;
  const ulonglong2* pa0 = reinterpret_cast<const ulonglong2*>(bm + (va0 ? a0 : 0) * Wp);
  const ulonglong2* pa1 = reinterpret_cast<const ulonglong2*>(bm + (va1 ? a1 : 0) * Wp);
  const ulonglong2* pb0 = reinterpret_cast<const ulonglong2*>(bm + (vb0 ? b0 : 0) * Wp);
  const ulonglong2* pb1 = reinterpret_cast<const ulonglong2*>(bm + (vb1 ? b1 : 0) * Wp);

  v16i acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
  const int shift = 16 * h;
  // partial Gram tiles of the split-K blocks are combined with integer atomics, so the result is
  // exact and order-independent
  // split-K by interleaved 16-word stripes: block y takes stripes y, y + ks, y + 2ks, ...  All
  // blocks then sweep the transaction axis together, so the rows' words in use at any moment lie
  // in a narrow window (one translation page per row).  Contiguous K slices per block touched
  // ~ks pages per row at once: at 100M transactions the UTCL1 missed 73 % of translations
  // (TCP_UTCL1_TRANSLATION_MISS 7.2e9 vs HIT 2.6e9; 0 % at 10M) and the gram ran at 14 % of the
  // i8 peak.  16 words = one 128-byte line per row per stripe.
  const int64_t ks = gridDim.y, y = blockIdx.y;
  const int64_t n_stripes = (Wp + kStripe - 1) / kStripe;
  const int64_t my_stripes = y < n_stripes ? (n_stripes - y + ks - 1) / ks : 0;
  const int64_t n_iter = my_stripes * (kStripe / 4);  // 4-word chunks
  const int64_t W2 = Wp >> 1;                        // row length in 16-byte units
  auto chunk_w2 = [&](int64_t it) {                  // first 16-byte unit of chunk `it`
    return ((it / (kStripe / 4)) * ks + y) * (kStripe / 2) + (it % (kStripe / 4)) * 2;
  };
  // software-pipelined: the next 4-word chunk's row loads are issued before this chunk's 32
  // MFMAs, so one chunk of HBM/L2 latency hides behind ~1000 matrix-core cycles per wave
  auto load = [&](int64_t w2, ulonglong2 (&A0)[2], ulonglong2 (&A1)[2], ulonglong2 (&B0)[2],
                  ulonglong2 (&B1)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool in = w2 + u < W2;
      A0[u] = va0 && in ? pa0[w2 + u] : make_ulonglong2(0, 0);
      A1[u] = va1 && in ? pa1[w2 + u] : make_ulonglong2(0, 0);
      B0[u] = vb0 && in ? pb0[w2 + u] : make_ulonglong2(0, 0);
      B1[u] = vb1 && in ? pb1[w2 + u] : make_ulonglong2(0, 0);
    }
  };
  ulonglong2 nA0[2], nA1[2], nB0[2], nB1[2];
  if (n_iter > 0) load(chunk_w2(0), nA0, nA1, nB0, nB1);
  for (int64_t it = 0; it < n_iter; ++it) {
    ulonglong2 A0[2], A1[2], B0[2], B1[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      A0[u] = nA0[u];
      A1[u] = nA1[u];
      B0[u] = nB0[u];
      B1[u] = nB1[u];
    }
    if (it + 1 < n_iter) load(chunk_w2(it + 1), nA0, nA1, nB0, nB1);
#pragma unroll
    for (int wd = 0; wd < 4; ++wd) {
      const unsigned long long xa0 = (wd & 1) ? A0[wd >> 1].y : A0[wd >> 1].x;
      const unsigned long long xa1 = (wd & 1) ? A1[wd >> 1].y : A1[wd >> 1].x;
      const unsigned long long xb0 = (wd & 1) ? B0[wd >> 1].y : B0[wd >> 1].x;
      const unsigned long long xb1 = (wd & 1) ? B1[wd >> 1].y : B1[wd >> 1].x;
#pragma unroll
      for (int half = 0; half < 2; ++half) {  // 32 transactions per MFMA K-step
        const int sh = 32 * half + shift;
        const v4i fa0 = unpack16((uint32_t)(xa0 >> sh) & 0xFFFFu, lut);
        const v4i fa1 = unpack16((uint32_t)(xa1 >> sh) & 0xFFFFu, lut);
        const v4i fb0 = unpack16((uint32_t)(xb0 >> sh) & 0xFFFFu, lut);
        const v4i fb1 = unpack16((uint32_t)(xb1 >> sh) & 0xFFFFu, lut);
        acc00 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa0, fb0, acc00, 0, 0, 0);
        acc01 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa0, fb1, acc01, 0, 0, 0);
        acc10 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa1, fb0, acc10, 0, 0, 0);
        acc11 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa1, fb1, acc11, 0, 0, 0);
      }
    }
  }
  // epilogue: row = (reg&3) + 8*(reg>>2) + 4h (within the 32-row MFMA tile), col = lane&31
  const int64_t rowb0 = ti * kTile + wr * 64, colb0 = tj * kTile + wc * 64;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    const int64_t rA = rowb0 + row, rB = rowb0 + 32 + row;
    const int64_t cA = colb0 + r, cB = colb0 + 32 + r;
    if (gridDim.y == 1) {
      if (rA < F) {
        if (cA < F && cA > rA) out[rA * F + cA] = (uint32_t)acc00[reg];
        if (cB < F && cB > rA) out[rA * F + cB] = (uint32_t)acc01[reg];
      }
      if (rB < F) {
        if (cA < F && cA > rB) out[rB * F + cA] = (uint32_t)acc10[reg];
        if (cB < F && cB > rB) out[rB * F + cB] = (uint32_t)acc11[reg];
      }
    } else {
      if (rA < F) {
        if (cA < F && cA > rA && acc00[reg]) atomicAdd(&out[rA * F + cA], (uint32_t)acc00[reg]);
        if (cB < F && cB > rA && acc01[reg]) atomicAdd(&out[rA * F + cB], (uint32_t)acc01[reg]);
      }
      if (rB < F) {
        if (cA < F && cA > rB && acc10[reg]) atomicAdd(&out[rB * F + cA], (uint32_t)acc10[reg]);
        if (cB < F && cB > rB && acc11[reg]) atomicAdd(&out[rB * F + cB], (uint32_t)acc11[reg]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// LDS-staged variant (the default; KMLS_GRAM_LDS=0 selects the direct kernel above): same MFMA
// tiling, split-K stripes and epilogue as k_pair_gram_mfma, but the operand words reach the
// waves through LDS.  In the direct kernel every 16-byte load instruction touches 32 rows = 32
// cache lines and uses 16 B of each; here a block stages one 16-word stripe of its 256 rows (128 A + 128 B) with coalesced loads
// (8 lanes per 128-byte line, every line loaded once per block instead of once per wave) into a
// double-buffered LDS slab, and the next stripe's loads are in flight in registers while the
// current stripe's 128 MFMAs per wave run.  Rows are padded to 144 B so the ds_read_b128 lane
// groups of the MFMA fragment reads (16 rows at one column) hit distinct banks.
constexpr int kStageRowB = 144;                 // bytes per staged row (128 + 16 pad)
constexpr int kStageB = 2 * kTile * kStageRowB;  // one stripe of A and B rows

// ---------------------------------------------------------------------------------------------
// FP4 variant: the 0/1 operands are exact in OCP e2m1 (1.0 = nibble 0x2), and the block-scaled
// v_mfma_scale_f32_32x32x64_f8f6f4 with FP4 operands runs at twice the i8 rate (4x bf16 per clock,
// MI355X_MICROARCH.md matrix-core table) with K = 64 transactions = one bitmap word per MFMA.
// Lane l (r = l&31, h = l>>5) supplies the 32 elements of word half h of its row (A: row r of the
// tile, B: column r); whatever order the hardware assigns to elements inside a fragment, A and B
// are expanded identically, so every product pairs the same transaction.  Bits are expanded
// through a byte → 8-nibble LDS table (one ds_read_b32 per 8 transactions, half the bytes of the
// i8 expansion).  The f32 accumulators hold integers exactly while a block's K slice stays below
// 2^24 transactions (enforced by the split-K below); the epilogue converts them back to u32.
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ v8i unpack32_fp4(uint32_t bits, const uint32_t* __restrict__ lut) {
  v8i r;
  r[0] = (int)lut[bits & 0xFFu];
  r[1] = (int)lut[(bits >> 8) & 0xFFu];
  r[2] = (int)lut[(bits >> 16) & 0xFFu];
  r[3] = (int)lut[bits >> 24];
  r[4] = 0;
  r[5] = 0;
  r[6] = 0;
  r[7] = 0;
  return r;
}

template <bool FP4>
__global__ __launch_bounds__(256, 2) void k_pair_gram_lds(const unsigned long long* __restrict__ bm,
                                                          int64_t Wp, int64_t F, int64_t n_tiles,
                                                          int64_t n_blocks, int scale,
                                                          uint32_t* __restrict__ out) {
  __shared__ uint2 lut[256];     // i8: byte -> 8 bytes
  __shared__ uint32_t lut4[256];  // FP4: byte -> 8 e2m1 nibbles (1.0 = 0x2)
  __shared__ __attribute__((aligned(16))) unsigned char stage[2][kStageB];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    if constexpr (FP4) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 8; ++b) v |= ((uint32_t)(i >> b) & 1u) << (4 * b + 1);
      lut4[i] = v;
    } else {
      lut[i] = make_uint2(nib((uint32_t)i & 0xFu), nib((uint32_t)i >> 4));
    }
  }
  const int64_t orig = blockIdx.x;
  const int64_t q = n_blocks / 8, rr = n_blocks % 8, xcd = orig % 8;
  int64_t idx = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  int64_t ti = 0;
  while (idx >= n_tiles - ti) { idx -= n_tiles - ti; ++ti; }
  const int64_t tj = ti + idx;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int r = lane & 31, h = lane >> 5;

  // staging role: thread t copies 16-byte segment (t & 7) of local rows (t >> 3) + 32 k,
  // k = 0..7 (local rows 0..127 = A tile rows, 128..255 = B tile rows)
  const int seg = tid & 7, lrow0 = tid >> 3;
  const int64_t W2 = Wp >> 1;  // row length in 16-byte units
  const ulonglong2* src[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int lr = lrow0 + 32 * k;
    const int64_t grow = lr < kTile ? ti * kTile + lr : tj * kTile + (lr - kTile);
    src[k] = grow < F ? reinterpret_cast<const ulonglong2*>(bm + grow * Wp) + seg : nullptr;
  }
  const int64_t ks = gridDim.y, y = blockIdx.y;
  const int64_t n_stripes = (Wp + kStripe - 1) / kStripe;
  const int64_t my_stripes = y < n_stripes ? (n_stripes - y + ks - 1) / ks : 0;
  auto gload = [&](int64_t it, ulonglong2 (&R)[8]) {
    const int64_t u = (it * ks + y) * (kStripe / 2) + seg;  // 16-byte unit of this thread
    const bool in = u < W2;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      R[k] = (src[k] && in) ? src[k][u - seg] : make_ulonglong2(0, 0);
  };
  auto swrite = [&](int buf, const ulonglong2 (&R)[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      *reinterpret_cast<ulonglong2*>(&stage[buf][(lrow0 + 32 * k) * kStageRowB + seg * 16]) = R[k];
  };

  using Acc = typename std::conditional<FP4, v16f, v16i>::type;
  Acc acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
  const int shift = 16 * h;
  const int la0 = wr * 64 + r, la1 = la0 + 32;
  const int lb0 = kTile + wc * 64 + r, lb1 = lb0 + 32;
  ulonglong2 R[8];
  if (my_stripes > 0) gload(0, R);
  for (int64_t it = 0; it < my_stripes; ++it) {
    const int buf = (int)(it & 1);
    swrite(buf, R);
    __syncthreads();  // stripe `it` visible; buffer buf^1 (stripe it-1) no longer read
    if (it + 1 < my_stripes) gload(it + 1, R);
    const unsigned char* sb = stage[buf];
    const ulonglong2* pa0 = reinterpret_cast<const ulonglong2*>(sb + la0 * kStageRowB);
    const ulonglong2* pa1 = reinterpret_cast<const ulonglong2*>(sb + la1 * kStageRowB);
    const ulonglong2* pb0 = reinterpret_cast<const ulonglong2*>(sb + lb0 * kStageRowB);
    const ulonglong2* pb1 = reinterpret_cast<const ulonglong2*>(sb + lb1 * kStageRowB);
#pragma unroll 2
    for (int c = 0; c < (int)(kStripe / 2); c += 2) {  // 4-word chunks
      ulonglong2 A0[2], A1[2], B0[2], B1[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        A0[u] = pa0[c + u];
        A1[u] = pa1[c + u];
        B0[u] = pb0[c + u];
        B1[u] = pb1[c + u];
      }
#pragma unroll
      for (int wd = 0; wd < 4; ++wd) {
        const unsigned long long xa0 = (wd & 1) ? A0[wd >> 1].y : A0[wd >> 1].x;
        const unsigned long long xa1 = (wd & 1) ? A1[wd >> 1].y : A1[wd >> 1].x;
        const unsigned long long xb0 = (wd & 1) ? B0[wd >> 1].y : B0[wd >> 1].x;
        const unsigned long long xb1 = (wd & 1) ? B1[wd >> 1].y : B1[wd >> 1].x;
        if constexpr (FP4) {  // one K=64 block-scaled MFMA per word: lane half h = word half h
          const int sh4 = 32 * h;
          const v8i fa0 = unpack32_fp4((uint32_t)(xa0 >> sh4), lut4);
          const v8i fa1 = unpack32_fp4((uint32_t)(xa1 >> sh4), lut4);
          const v8i fb0 = unpack32_fp4((uint32_t)(xb0 >> sh4), lut4);
          const v8i fb1 = unpack32_fp4((uint32_t)(xb1 >> sh4), lut4);
          acc00 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa0, fb0, acc00, 4, 4, 0, scale, 0, scale);
          acc01 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa0, fb1, acc01, 4, 4, 0, scale, 0, scale);
          acc10 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa1, fb0, acc10, 4, 4, 0, scale, 0, scale);
          acc11 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa1, fb1, acc11, 4, 4, 0, scale, 0, scale);
        } else {
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int sh = 32 * half + shift;
            const v4i fa0 = unpack16((uint32_t)(xa0 >> sh) & 0xFFFFu, lut);
            const v4i fa1 = unpack16((uint32_t)(xa1 >> sh) & 0xFFFFu, lut);
            const v4i fb0 = unpack16((uint32_t)(xb0 >> sh) & 0xFFFFu, lut);
            const v4i fb1 = unpack16((uint32_t)(xb1 >> sh) & 0xFFFFu, lut);
            acc00 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa0, fb0, acc00, 0, 0, 0);
            acc01 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa0, fb1, acc01, 0, 0, 0);
            acc10 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa1, fb0, acc10, 0, 0, 0);
            acc11 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa1, fb1, acc11, 0, 0, 0);
          }
        }
      }
    }
  }
  const int64_t rowb0 = ti * kTile + wr * 64, colb0 = tj * kTile + wc * 64;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    const int64_t rA = rowb0 + row, rB = rowb0 + 32 + row;
    const int64_t cA = colb0 + r, cB = colb0 + 32 + r;
    if (gridDim.y == 1) {
      if (rA < F) {
        if (cA < F && cA > rA) out[rA * F + cA] = (uint32_t)acc00[reg];
        if (cB < F && cB > rA) out[rA * F + cB] = (uint32_t)acc01[reg];
      }
      if (rB < F) {
        if (cA < F && cA > rB) out[rB * F + cA] = (uint32_t)acc10[reg];
        if (cB < F && cB > rB) out[rB * F + cB] = (uint32_t)acc11[reg];
      }
    } else {
      if (rA < F) {
        if (cA < F && cA > rA && acc00[reg]) atomicAdd(&out[rA * F + cA], (uint32_t)acc00[reg]);
        if (cB < F && cB > rA && acc01[reg]) atomicAdd(&out[rA * F + cB], (uint32_t)acc01[reg]);
      }
      if (rB < F) {
        if (cA < F && cA > rB && acc10[reg]) atomicAdd(&out[rB * F + cA], (uint32_t)acc10[reg]);
        if (cB < F && cB > rB && acc11[reg]) atomicAdd(&out[rB * F + cB], (uint32_t)acc11[reg]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Wide-tile variant (KMLS_GRAM_TILE=256): each wave owns a 128x128 output block = 4x4 MFMA tiles
// (16 accumulators, 256 AGPRs, one wave per SIMD), so every unpacked fragment feeds 4 MFMAs
// instead of 2.  In the 128-tile kernel the LUT expansion (one fragment per MFMA) kept the LDS
// pipe as busy as the matrix cores (r2_large_pmc.md: 63 % MFMA busy, 0.4 conflict cycles per LDS
// instruction); here it is half of that, and the 256-row block tiles also halve the bitmap words
// read per output (each staged row feeds 256 outputs).  Stripes are 8 words (512 transactions)
// so a thread stages 8 x 16 B per stripe; rows are padded to 80 B in LDS.
constexpr int kWTile = 256;
constexpr int64_t kWStripe = 8;
constexpr int kWRowB = 80;                        // bytes per staged row (64 + 16 pad)
constexpr int kWStageB = 2 * kWTile * kWRowB;     // one stripe of A and B rows (40 KB)

// MODE 0: i8 operands (LUT unpack), 1: FP4 operands (LUT unpack), 2: FP4 masked nibbles (below)
template <int MODE>
__global__ __launch_bounds__(256, 1) void k_pair_gram_wide(const unsigned long long* __restrict__ bm,
                                                           int64_t Wp, int64_t F, int64_t n_tiles,
                                                           int64_t n_blocks, int scale,
                                                           uint32_t* __restrict__ out,
                                                           int xcd_2d) {
  constexpr bool FP4 = MODE != 0;
  __shared__ uint2 lut[256];
  __shared__ uint32_t lut4[256];
  __shared__ __attribute__((aligned(16))) unsigned char stage[2][kWStageB];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    if constexpr (FP4) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 8; ++b) v |= ((uint32_t)(i >> b) & 1u) << (4 * b + 1);
      lut4[i] = v;
    } else {
      lut[i] = make_uint2(nib((uint32_t)i & 0xFu), nib((uint32_t)i >> 4));
    }
  }
  int64_t idx, y;
  if (xcd_2d) {
    // XCD-aware over the whole (tile pair, K slice) grid: the hardware deals linear workgroup
    // ids round-robin over the 8 XCDs, so remap them such that the bw tile-pair blocks of one
    // K slice (which stage the same stripes of the same row tiles) share an XCD and its L2
    const int64_t n = (int64_t)gridDim.x * gridDim.y;
    const int64_t h = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    const int64_t q2 = n / 8, r2 = n % 8, x8 = h % 8;
    const int64_t li = (x8 < r2 ? x8 * (q2 + 1) : r2 * (q2 + 1) + (x8 - r2) * q2) + h / 8;
    y = li / gridDim.x;
    idx = li % gridDim.x;
  } else {
    const int64_t orig = blockIdx.x;
    const int64_t q = n_blocks / 8, rr = n_blocks % 8, xcd = orig % 8;
    idx = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
    y = blockIdx.y;
  }
  int64_t ti = 0;
  while (idx >= n_tiles - ti) { idx -= n_tiles - ti; ++ti; }
  const int64_t tj = ti + idx;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int r = lane & 31, h = lane >> 5;

  // staging role: thread t copies 16-byte segment (t & 3) of local rows (t >> 2) + 64 k, k = 0..7
  // (local rows 0..255 = A tile rows, 256..511 = B tile rows)
  const int seg = tid & 3, lrow0 = tid >> 2;
  const int64_t W2 = Wp >> 1;
  const ulonglong2* src[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int lr = lrow0 + 64 * k;
    const int64_t grow = lr < kWTile ? ti * kWTile + lr : tj * kWTile + (lr - kWTile);
    src[k] = grow < F ? reinterpret_cast<const ulonglong2*>(bm + grow * Wp) : nullptr;
  }
  const int64_t ks = gridDim.y;
  const int64_t n_stripes = (Wp + kWStripe - 1) / kWStripe;
  const int64_t my_stripes = y < n_stripes ? (n_stripes - y + ks - 1) / ks : 0;
  auto gload = [&](int64_t it, ulonglong2 (&R)[8]) {
    const int64_t u = (it * ks + y) * (kWStripe / 2) + seg;
    const bool in = u < W2;
#pragma unroll
    for (int k = 0; k < 8; ++k) R[k] = (src[k] && in) ? src[k][u] : make_ulonglong2(0, 0);
  };
  auto swrite = [&](int buf, const ulonglong2 (&R)[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      *reinterpret_cast<ulonglong2*>(&stage[buf][(lrow0 + 64 * k) * kWRowB + seg * 16]) = R[k];
  };

  using Acc = typename std::conditional<FP4, v16f, v16i>::type;
  Acc acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = Acc{};
  const int la = wr * 128 + r;           // + 32 m: A fragment rows
  const int lb = kWTile + wc * 128 + r;  // + 32 n: B fragment columns
  ulonglong2 R[8];
  if (my_stripes > 0) gload(0, R);
  for (int64_t it = 0; it < my_stripes; ++it) {
    const int buf = (int)(it & 1);
    swrite(buf, R);
    __syncthreads();  // stripe `it` visible; buffer buf^1 (stripe it-1) no longer read
    if (it + 1 < my_stripes) gload(it + 1, R);
    const unsigned char* sb = stage[buf];
    if constexpr (MODE == 2) {
      // Masked nibbles, no unpack: a lane's 16 raw bytes ARE 32 FP4 elements (nibble e = bits
      // 4e..4e+3).  Masking every nibble to one bit position j leaves element value bit_j * v_j
      // (e2m1 0b0001 = 0.5, 0b0010 = 1.0, 0b0100 = 2.0; bit 3 is the sign bit, so it is shifted
      // down to bit 2 first), and the block scale s_j = 1 / v_j (e8m0 128 / 127 / 126) makes every
      // coinciding pair contribute exactly 1.0.  Four MFMAs (j = 0..3) cover the 256 transactions
      // of a 4-word chunk: lane half h holds words 2h, 2h+1.  Operand preparation is one AND per
      // VGPR (two for j = 3) and one ds_read_b128 per fragment per 4 words, instead of four LDS
      // table reads per fragment per word: the LDS pipe leaves the matrix cores' way.
#pragma unroll
      for (int c = 0; c < (int)(kWStripe / 4); ++c) {  // 4-word chunks
        v4i A[4], B[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          A[m] = *reinterpret_cast<const v4i*>(sb + (la + 32 * m) * kWRowB + c * 32 + h * 16);
          B[m] = *reinterpret_cast<const v4i*>(sb + (lb + 32 * m) * kWRowB + c * 32 + h * 16);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int msk = j == 0 ? 0x11111111 : j == 1 ? 0x22222222 : 0x44444444;
          const int sc = j == 0 ? 128 : j == 1 ? 127 : 126;
          v8i fa[4], fb[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) {
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              fa[m][d] = (j == 3 ? (int)((uint32_t)A[m][d] >> 1) : A[m][d]) & msk;
              fb[m][d] = (j == 3 ? (int)((uint32_t)B[m][d] >> 1) : B[m][d]) & msk;
              fa[m][d + 4] = 0;
              fb[m][d + 4] = 0;
            }
          }
#pragma unroll
          for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int m = 0; m < 4; ++m)
              acc[m][n] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[m], fb[n], acc[m][n], 4, 4,
                                                                          0, sc, 0, sc);
        }
      }
    } else if constexpr (FP4) {
      // software-pipelined over the stripe's 8 words: word s+1's fragments are unpacked (LDS
      // table reads) before word s's 16 MFMAs issue, so with one wave per SIMD the table latency
      // hides behind ~512 matrix-core cycles instead of stalling them
      const int sh4 = 32 * h;
      ulonglong2 A[4], B[4];
      v8i fa[2][4], fb[2][4];
      auto rows = [&](int c) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          A[m] = *reinterpret_cast<const ulonglong2*>(sb + (la + 32 * m) * kWRowB + c * 16);
          B[m] = *reinterpret_cast<const ulonglong2*>(sb + (lb + 32 * m) * kWRowB + c * 16);
        }
      };
      auto unpack = [&](int wd, v8i (&xa)[4], v8i (&xb)[4]) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          xa[m] = unpack32_fp4((uint32_t)((wd ? A[m].y : A[m].x) >> sh4), lut4);
          xb[m] = unpack32_fp4((uint32_t)((wd ? B[m].y : B[m].x) >> sh4), lut4);
        }
      };
      rows(0);
      unpack(0, fa[0], fb[0]);
#pragma unroll
      for (int w = 0; w < (int)kWStripe; ++w) {
        const int cur = w & 1;
        if (w + 1 < (int)kWStripe) {
          if (((w + 1) & 1) == 0) rows((w + 1) >> 1);
          unpack((w + 1) & 1, fa[cur ^ 1], fb[cur ^ 1]);
        }
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int m = 0; m < 4; ++m)
            acc[m][n] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[cur][m], fb[cur][n], acc[m][n],
                                                                        4, 4, 0, scale, 0, scale);
      }
    } else {
#pragma unroll 1
      for (int c = 0; c < (int)(kWStripe / 2); ++c) {  // 2-word chunks
        ulonglong2 A[4], B[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          A[m] = *reinterpret_cast<const ulonglong2*>(sb + (la + 32 * m) * kWRowB + c * 16);
          B[m] = *reinterpret_cast<const ulonglong2*>(sb + (lb + 32 * m) * kWRowB + c * 16);
        }
        for (int wd = 0; wd < 2; ++wd) {
#pragma unroll 1
          for (int half = 0; half < 2; ++half) {
            const int sh = 32 * half + 16 * h;
            v4i fa[4];
#pragma unroll
            for (int m = 0; m < 4; ++m)
              fa[m] = unpack16((uint32_t)((wd ? A[m].y : A[m].x) >> sh) & 0xFFFFu, lut);
#pragma unroll
            for (int n = 0; n < 4; ++n) {
              const v4i fb = unpack16((uint32_t)((wd ? B[n].y : B[n].x) >> sh) & 0xFFFFu, lut);
#pragma unroll
              for (int m = 0; m < 4; ++m)
                acc[m][n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[m], fb, acc[m][n], 0, 0, 0);
            }
          }
        }
      }
    }
  }
  // epilogue: row = (reg&3) + 8*(reg>>2) + 4h within a 32x32 MFMA tile, col = lane&31
  const int64_t rowb = ti * kWTile + wr * 128, colb = tj * kWTile + wc * 128;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int64_t rw = rowb + 32 * m + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const int64_t cl = colb + 32 * n + r;
        const uint32_t v = (uint32_t)acc[m][n][reg];
        if (rw < F && cl < F && cl > rw) {
          if (gridDim.y == 1) out[rw * F + cl] = v;
          else if (v) atomicAdd(&out[rw * F + cl], v);
        }
      }
    }
  }
}

// (A 16-word-stripe variant of MODE 2, half the block barriers per transaction, measured no
// faster: 100M gram 14.18 vs 14.24 ms, config-5 10M gram 402 vs 385 ms; removed.)
// Masked-nibble FP4 with two waves per SIMD (KMLS_GRAM_FP4=mask8): 512-thread blocks of 8 waves
// (2 row x 4 column groups), each wave a 128x64 output block = 4x2 MFMA tiles (8 accumulators,
// 128 AGPRs), so each SIMD holds two waves and one issues while the other waits on an operand or
// the matrix pipe.  Same 256-row block tiles, stripes and LDS slab as k_pair_gram_wide; a fragment
// now feeds 2 or 4 MFMAs instead of 4.
__global__ __launch_bounds__(512, 1) void k_pair_gram_mask8(const unsigned long long* __restrict__ bm,
                                                            int64_t Wp, int64_t F, int64_t n_tiles,
                                                            int64_t n_blocks,
                                                            uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) unsigned char stage[2][kWStageB];
  const int64_t orig = blockIdx.x;
  const int64_t q = n_blocks / 8, rr = n_blocks % 8, xcd = orig % 8;
  int64_t idx = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  int64_t ti = 0;
  while (idx >= n_tiles - ti) { idx -= n_tiles - ti; ++ti; }
  const int64_t tj = ti + idx;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int r = lane & 31, h = lane >> 5;
  // staging: thread t copies 16-byte segment (t & 3) of local rows (t >> 2) + 128 k, k = 0..3
  const int seg = tid & 3, lrow0 = tid >> 2;
  const int64_t W2 = Wp >> 1;
  const ulonglong2* src[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int lr = lrow0 + 128 * k;
    const int64_t grow = lr < kWTile ? ti * kWTile + lr : tj * kWTile + (lr - kWTile);
    src[k] = grow < F ? reinterpret_cast<const ulonglong2*>(bm + grow * Wp) : nullptr;
  }
  const int64_t ks = gridDim.y, y = blockIdx.y;
  const int64_t n_stripes = (Wp + kWStripe - 1) / kWStripe;
  const int64_t my_stripes = y < n_stripes ? (n_stripes - y + ks - 1) / ks : 0;
  auto gload = [&](int64_t it, ulonglong2 (&R)[4]) {
    const int64_t u = (it * ks + y) * (kWStripe / 2) + seg;
    const bool in = u < W2;
#pragma unroll
    for (int k = 0; k < 4; ++k) R[k] = (src[k] && in) ? src[k][u] : make_ulonglong2(0, 0);
  };
  auto swrite = [&](int buf, const ulonglong2 (&R)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      *reinterpret_cast<ulonglong2*>(&stage[buf][(lrow0 + 128 * k) * kWRowB + seg * 16]) = R[k];
  };
  v16f acc[4][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[m][n] = v16f{};
  const int la = wr * 128 + r;          // + 32 m
  const int lb = kWTile + wc * 64 + r;  // + 32 n
  ulonglong2 R[4];
  if (my_stripes > 0) gload(0, R);
  for (int64_t it = 0; it < my_stripes; ++it) {
    const int buf = (int)(it & 1);
    swrite(buf, R);
    __syncthreads();
    if (it + 1 < my_stripes) gload(it + 1, R);
    const unsigned char* sb = stage[buf];
#pragma unroll
    for (int c = 0; c < (int)(kWStripe / 4); ++c) {
      v4i A[4], B[2];
#pragma unroll
      for (int m = 0; m < 4; ++m)
        A[m] = *reinterpret_cast<const v4i*>(sb + (la + 32 * m) * kWRowB + c * 32 + h * 16);
#pragma unroll
      for (int n = 0; n < 2; ++n)
        B[n] = *reinterpret_cast<const v4i*>(sb + (lb + 32 * n) * kWRowB + c * 32 + h * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int msk = j == 0 ? 0x11111111 : j == 1 ? 0x22222222 : 0x44444444;
        const int sc = j == 0 ? 128 : j == 1 ? 127 : 126;
        v8i fa[4], fb[2];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            fa[m][d] = (j == 3 ? (int)((uint32_t)A[m][d] >> 1) : A[m][d]) & msk;
            fa[m][d + 4] = 0;
          }
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            fb[n][d] = (j == 3 ? (int)((uint32_t)B[n][d] >> 1) : B[n][d]) & msk;
            fb[n][d + 4] = 0;
          }
        }
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int m = 0; m < 4; ++m)
            acc[m][n] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[m], fb[n], acc[m][n], 4, 4, 0,
                                                                        sc, 0, sc);
      }
    }
  }
  const int64_t rowb = ti * kWTile + wr * 128, colb = tj * kWTile + wc * 64;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int64_t rw = rowb + 32 * m + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const int64_t cl = colb + 32 * n + r;
        const uint32_t v = (uint32_t)acc[m][n][reg];
        if (rw < F && cl < F && cl > rw) {
          if (gridDim.y == 1) out[rw * F + cl] = v;
          else if (v) atomicAdd(&out[rw * F + cl], v);
        }
      }
}

__global__ __launch_bounds__(256) void k_pair_gram_fp4(const unsigned long long* __restrict__ bm,
                                                        int64_t Wp, int64_t F, int64_t n_tiles,
                                                        int64_t n_blocks, int scale,
                                                        uint32_t* __restrict__ out) {
  __shared__ uint32_t lut[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) v |= ((uint32_t)(i >> b) & 1u) << (4 * b + 1);  // 1 → 0x2 (1.0)
    lut[i] = v;
  }
  __syncthreads();
  const int64_t orig = blockIdx.x;  // XCD-aware remap, as in k_pair_gram_mfma
  const int64_t q = n_blocks / 8, rr = n_blocks % 8, xcd = orig % 8;
  int64_t idx = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  int64_t ti = 0;
  while (idx >= n_tiles - ti) { idx -= n_tiles - ti; ++ti; }
  const int64_t tj = ti + idx;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  const int64_t a0 = ti * kTile + wr * 64 + r, a1 = a0 + 32;
  const int64_t b0 = tj * kTile + wc * 64 + r, b1 = b0 + 32;
  const bool va0 = a0 < F, va1 = a1 < F, vb0 = b0 < F, vb1 = b1 < F;
  const ulonglong2* pa0 = reinterpret_cast<const ulonglong2*>(bm + (va0 ? a0 : 0) * Wp);
  const ulonglong2* pa1 = reinterpret_cast<const ulonglong2*>(bm + (va1 ? a1 : 0) * Wp);
  const ulonglong2* pb0 = reinterpret_cast<const ulonglong2*>(bm + (vb0 ? b0 : 0) * Wp);
  const ulonglong2* pb1 = reinterpret_cast<const ulonglong2*>(bm + (vb1 ? b1 : 0) * Wp);

  v16f acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
  const int shift = 32 * h;
  // split-K by interleaved 16-word stripes: block y takes stripes y, y + ks, y + 2ks, ...  All
  // blocks then sweep the transaction axis together, so the rows' words in use at any moment lie
  // in a narrow window (one translation page per row).  Contiguous K slices per block touched
  // ~ks pages per row at once: at 100M transactions the UTCL1 missed 73 % of translations
  // (TCP_UTCL1_TRANSLATION_MISS 7.2e9 vs HIT 2.6e9; 0 % at 10M) and the gram ran at 14 % of the
  // i8 peak.  16 words = one 128-byte line per row per stripe.
  const int64_t ks = gridDim.y, y = blockIdx.y;
  const int64_t n_stripes = (Wp + kStripe - 1) / kStripe;
  const int64_t my_stripes = y < n_stripes ? (n_stripes - y + ks - 1) / ks : 0;
  const int64_t n_iter = my_stripes * (kStripe / 4);  // 4-word chunks
  const int64_t W2 = Wp >> 1;                        // row length in 16-byte units
  auto chunk_w2 = [&](int64_t it) {                  // first 16-byte unit of chunk `it`
    return ((it / (kStripe / 4)) * ks + y) * (kStripe / 2) + (it % (kStripe / 4)) * 2;
  };
  auto load = [&](int64_t w2, ulonglong2 (&A0)[2], ulonglong2 (&A1)[2], ulonglong2 (&B0)[2],
                  ulonglong2 (&B1)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool in = w2 + u < W2;
      A0[u] = va0 && in ? pa0[w2 + u] : make_ulonglong2(0, 0);
      A1[u] = va1 && in ? pa1[w2 + u] : make_ulonglong2(0, 0);
      B0[u] = vb0 && in ? pb0[w2 + u] : make_ulonglong2(0, 0);
      B1[u] = vb1 && in ? pb1[w2 + u] : make_ulonglong2(0, 0);
    }
  };
  ulonglong2 nA0[2], nA1[2], nB0[2], nB1[2];
  if (n_iter > 0) load(chunk_w2(0), nA0, nA1, nB0, nB1);
  for (int64_t it = 0; it < n_iter; ++it) {
    ulonglong2 A0[2], A1[2], B0[2], B1[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      A0[u] = nA0[u];
      A1[u] = nA1[u];
      B0[u] = nB0[u];
      B1[u] = nB1[u];
    }
    if (it + 1 < n_iter) load(chunk_w2(it + 1), nA0, nA1, nB0, nB1);
#pragma unroll
    for (int wd = 0; wd < 4; ++wd) {  // one 64-transaction word per MFMA K-step
      const unsigned long long xa0 = (wd & 1) ? A0[wd >> 1].y : A0[wd >> 1].x;
      const unsigned long long xa1 = (wd & 1) ? A1[wd >> 1].y : A1[wd >> 1].x;
      const unsigned long long xb0 = (wd & 1) ? B0[wd >> 1].y : B0[wd >> 1].x;
      const unsigned long long xb1 = (wd & 1) ? B1[wd >> 1].y : B1[wd >> 1].x;
      const v8i fa0 = unpack32_fp4((uint32_t)(xa0 >> shift), lut);
      const v8i fa1 = unpack32_fp4((uint32_t)(xa1 >> shift), lut);
      const v8i fb0 = unpack32_fp4((uint32_t)(xb0 >> shift), lut);
      const v8i fb1 = unpack32_fp4((uint32_t)(xb1 >> shift), lut);
      acc00 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa0, fb0, acc00, 4, 4, 0, scale, 0, scale);
      acc01 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa0, fb1, acc01, 4, 4, 0, scale, 0, scale);
      acc10 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa1, fb0, acc10, 4, 4, 0, scale, 0, scale);
      acc11 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa1, fb1, acc11, 4, 4, 0, scale, 0, scale);
    }
  }
  const int64_t rowb0 = ti * kTile + wr * 64, colb0 = tj * kTile + wc * 64;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    const int64_t rA = rowb0 + row, rB = rowb0 + 32 + row;
    const int64_t cA = colb0 + r, cB = colb0 + 32 + r;
    const uint32_t v00 = (uint32_t)acc00[reg], v01 = (uint32_t)acc01[reg];
    const uint32_t v10 = (uint32_t)acc10[reg], v11 = (uint32_t)acc11[reg];
    if (gridDim.y == 1) {
      if (rA < F) {
        if (cA < F && cA > rA) out[rA * F + cA] = v00;
        if (cB < F && cB > rA) out[rA * F + cB] = v01;
      }
      if (rB < F) {
        if (cA < F && cA > rB) out[rB * F + cA] = v10;
        if (cB < F && cB > rB) out[rB * F + cB] = v11;
      }
    } else {
      if (rA < F) {
        if (cA < F && cA > rA && v00) atomicAdd(&out[rA * F + cA], v00);
        if (cB < F && cB > rA && v01) atomicAdd(&out[rA * F + cB], v01);
      }
      if (rB < F) {
        if (cA < F && cA > rB && v10) atomicAdd(&out[rB * F + cA], v10);
        if (cB < F && cB > rB && v11) atomicAdd(&out[rB * F + cB], v11);
      }
    }
  }
}

}  // namespace

// Operand format of the MFMA gram (KMLS_GRAM_FP4):
//   unset / "mask": masked-nibble FP4 operands in the wide-tile kernel (the default: 100M x 754
//                   items 23.1 -> 14.3 ms, config-5 width 679 -> 387 ms; profiles/r2_gram_wide.md)
//   "0": i8 operands (LUT unpack) — the 128-tile LDS-staged kernel, or the wide one with
//        KMLS_GRAM_TILE=256, or the direct-load one with KMLS_GRAM_LDS=0
//   "1": FP4 operands through the LUT unpack (128-tile LDS-staged, or wide with KMLS_GRAM_TILE=256)
//   "direct": FP4 LUT operands, direct (unstaged) loads
// KMLS_GRAM_FP4_SCALE overrides the e8m0 scale byte of the LUT FP4 paths (127 = 1.0).
static int gram_fp4() {
  const char* e = std::getenv("KMLS_GRAM_FP4");
  if (!e || !e[0] || std::string(e) == "mask") return 3;
  if (std::string(e) == "mask8") return 4;  // masked nibbles, 8 waves (2 per SIMD), A/B
  if (e[0] == '1') return 1;
  return std::string(e) == "direct" ? 2 : 0;
}
// default: the LDS-staged variant (coalesced stripe loads; 100M x 754 items: 101 -> 23 ms);
// KMLS_GRAM_LDS=0 selects the direct-load kernel (A/B)
static bool gram_lds() {
  const char* e = std::getenv("KMLS_GRAM_LDS");
  return !(e && e[0] == '0');
}
// KMLS_GRAM_TILE=256: the wide-tile LDS-staged kernel (4x4 MFMA tiles per wave)
static bool gram_wide() {
  const char* e = std::getenv("KMLS_GRAM_TILE");
  return e && std::string(e) == "256";
}

void pair_gram_mfma_i8(const uint64_t* bm, int64_t Wp, int64_t F, uint32_t* out, hipStream_t s) {
  if (F < 2) return;
  if (Wp % 4 != 0) throw std::runtime_error("kmls: pair_gram_mfma_i8 needs Wp % 4 == 0");
  const int64_t nt = (F + kTile - 1) / kTile;
  const int64_t blocks = nt * (nt + 1) / 2;
  // split K so that the grid fills the resident block slots in ONE round (a 1.3-round grid left
  // a third of the chip idle in the second round), slices >= 1024 words
  static const int64_t slots = [] {
    int dev = 0, per_cu = 1;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return (int64_t)1024;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pair_gram_mfma, 256, 0) != hipSuccess)
      per_cu = 2;
    return (int64_t)std::max(1, per_cu) * std::max(1, p.multiProcessorCount);
  }();
  int64_t ks = std::max<int64_t>(1, std::min<int64_t>(slots / blocks, Wp / 1024));
  const char* se = std::getenv("KMLS_GRAM_FP4_SCALE");
  const int scale = se ? std::atoi(se) : 127;
  const int fp4 = gram_fp4();
  if (fp4 == 2) {
    // exact f32 accumulation: every block's stripes hold < 2^24 transactions (<= 2^17 words
    // at this split, with margin for the rounding of stripes)
    ks = std::max<int64_t>(ks, (Wp + (1 << 17) - 1) >> 17);
    hipLaunchKernelGGL(k_pair_gram_fp4, dim3((unsigned)blocks, (unsigned)ks), dim3(256), 0, s,
                       (const unsigned long long*)bm, Wp, F, nt, blocks, scale, out);
  } else if (gram_wide() || fp4 >= 3) {
    const int64_t ntw = (F + kWTile - 1) / kWTile;
    const int64_t bw = ntw * (ntw + 1) / 2;
    static const int64_t slots_w = [] {
      int dev = 0;
      hipDeviceProp_t p;
      if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return (int64_t)256;
      return (int64_t)std::max(1, p.multiProcessorCount);  // one 4-wave block per CU (256 AGPRs)
    }();
    const int64_t n_stripes = (Wp + kWStripe - 1) / kWStripe;
    // XCD-aware remap over the whole 2-D grid: L2 hit rate 31 % -> 84 % at 10M x 754 items
    // (TCC_HIT/MISS), time unchanged (14.32 vs 14.34 ms at 100M: the kernel is matrix-core
    // bound), so the fabric carries a quarter of the traffic; KMLS_GRAM_XCD=1d: per-row remap
    const char* xe = std::getenv("KMLS_GRAM_XCD");
    const int xcd2 = (xe && std::string(xe) == "1d") ? 0 : 1;
    int64_t ksw = std::max<int64_t>(1, std::min<int64_t>(slots_w / bw, Wp / 256));
    // FP4: a block's f32 accumulators stay exact while its stripes (512 transactions each)
    // number < 2^15
    if (fp4 == 1 || fp4 >= 3) ksw = std::max<int64_t>(ksw, (n_stripes + 32767) / 32768 + 1);
    if (fp4 == 4)
      hipLaunchKernelGGL(k_pair_gram_mask8, dim3((unsigned)bw, (unsigned)ksw), dim3(512), 0, s,
                         (const unsigned long long*)bm, Wp, F, ntw, bw, out);
    else if (fp4 == 3)
      hipLaunchKernelGGL(k_pair_gram_wide<2>, dim3((unsigned)bw, (unsigned)ksw), dim3(256), 0, s,
                         (const unsigned long long*)bm, Wp, F, ntw, bw, scale, out, xcd2);
    else if (fp4 == 1)
      hipLaunchKernelGGL(k_pair_gram_wide<1>, dim3((unsigned)bw, (unsigned)ksw), dim3(256), 0, s,
                         (const unsigned long long*)bm, Wp, F, ntw, bw, scale, out, xcd2);
    else
      hipLaunchKernelGGL(k_pair_gram_wide<0>, dim3((unsigned)bw, (unsigned)ksw), dim3(256), 0, s,
                         (const unsigned long long*)bm, Wp, F, ntw, bw, scale, out, xcd2);
  } else if (gram_lds() || fp4 == 1) {
    static const int64_t slots_lds = [] {
      int dev = 0, per_cu = 1;
      hipDeviceProp_t p;
      if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return (int64_t)512;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pair_gram_lds<false>, 256, 0) != hipSuccess)
        per_cu = 2;
      return (int64_t)std::max(1, per_cu) * std::max(1, p.multiProcessorCount);
    }();
    int64_t ks_lds = std::max<int64_t>(1, std::min<int64_t>(slots_lds / blocks, Wp / 256));
    if (fp4 == 1) {
      // f32 accumulators are exact below 2^24: a block's interleaved stripes (16 words = 1024
      // transactions each) must number < 2^14
      ks_lds = std::max<int64_t>(ks_lds, ((Wp + kStripe - 1) / kStripe + 16383) / 16384 + 1);
      hipLaunchKernelGGL(k_pair_gram_lds<true>, dim3((unsigned)blocks, (unsigned)ks_lds), dim3(256),
                         0, s, (const unsigned long long*)bm, Wp, F, nt, blocks, scale, out);
    } else {
      hipLaunchKernelGGL(k_pair_gram_lds<false>, dim3((unsigned)blocks, (unsigned)ks_lds), dim3(256),
                         0, s, (const unsigned long long*)bm, Wp, F, nt, blocks, scale, out);
    }
  } else {
    hipLaunchKernelGGL(k_pair_gram_mfma, dim3((unsigned)blocks, (unsigned)ks), dim3(256), 0, s,
                       (const unsigned long long*)bm, Wp, F, nt, blocks, out);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e));
}

}  // namespace kern
}  // namespace kmls
