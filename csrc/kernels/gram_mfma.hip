// Level-2 co-occurrence GEMM on the matrix cores: G = A·Aᵀ over the transaction axis, with A
// the 0/1 one-hot matrix of frequent items stored as packed tid-bitmaps (SURVEY §2.C O8,
// BASELINE north star "MFMA one-hot x one-hot co-occurrence GEMM for the first pass").
//
// Operands: block-scaled FP4 (v_mfma_scale_f32_32x32x64_f8f6f4, twice the i8 rate on gfx950)
// fed straight from the packed bits.  A lane's 16 raw bytes ARE 32 e2m1 elements (nibble e =
// bits 4e..4e+3); masking every nibble to one bit position j leaves element value bit_j * v_j and
// the block scale 1 / v_j makes every coinciding pair contribute exactly 1.0, so four MFMAs cover
// a 4-word chunk with one AND per VGPR and no unpack: HBM/L2 traffic stays at 1 bit per (item,
// transaction) and the LDS pipe stays out of the matrix cores' way.  The f32 accumulators hold
// integers exactly while a block's K slice stays below 2^24 transactions (split-K below).
//
// Tiling: 256-thread block = 4 waves (2x2) -> 256x256 output tile; each wave 128x128 = 4x4 MFMA
// tiles (16 accumulators, 256 AGPRs, one wave per SIMD), so every operand fragment feeds 4 MFMAs.
// The block stages 8-word stripes of its 512 rows through a double-buffered LDS slab (coalesced
// 16-byte loads, rows padded to 80 B), the next stripe's loads in flight while the current
// stripe's MFMAs run.  Only upper-triangular tile pairs are launched (G is symmetric).
//
// Measured alternatives, removed (profiles/r2_*): i8 operands through an LDS byte table (128 and
// 256 tiles, direct or LDS-staged loads), FP4 through the table, 8-wave masked blocks, 16-word
// stripes -- the masked 256-tile kernel beat each (100M x 754 items 23.1 -> 14.3 ms, config-5
// 10M x 14.8k 679 -> 387 ms).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "kernels.hpp"

namespace kmls {
namespace kern {

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kWTile = 256;
constexpr int64_t kWStripe = 8;
constexpr int kWRowB = 80;                        // bytes per staged row (64 + 16 pad)
constexpr int kWStageB = 2 * kWTile * kWRowB;     // one stripe of A and B rows (40 KB)

__global__ __launch_bounds__(256, 1) void k_pair_gram_fp4mask(const unsigned long long* __restrict__ bm,
                                                              int64_t Wp, int64_t F,
                                                              int64_t n_tiles,
                                                              uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) unsigned char stage[2][kWStageB];
  // XCD-aware over the whole (tile pair, K slice) grid: the hardware deals linear workgroup ids
  // round-robin over the 8 XCDs, so remap them such that the tile-pair blocks of one K slice
  // (which stage the same stripes of the same row tiles) share an XCD and its L2 (TCC hit rate
  // 31 -> 84 % at 10M x 754 items; the kernel is matrix-core bound, so the time is unchanged
  // but the fabric carries a quarter of the traffic)
  int64_t idx, y;
  {
    const int64_t n = (int64_t)gridDim.x * gridDim.y;
    const int64_t h = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    const int64_t q2 = n / 8, r2 = n % 8, x8 = h % 8;
    const int64_t li = (x8 < r2 ? x8 * (q2 + 1) : r2 * (q2 + 1) + (x8 - r2) * q2) + h / 8;
    y = li / gridDim.x;
    idx = li % gridDim.x;
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

  v16f acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = v16f{};
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


}  // namespace

void pair_gram_mfma(const uint64_t* bm, int64_t Wp, int64_t F, uint32_t* out, hipStream_t s) {
  if (F < 2) return;
  if (Wp % 4 != 0) throw std::runtime_error("kmls: pair_gram_mfma needs Wp % 4 == 0");
  const int64_t ntw = (F + kWTile - 1) / kWTile;
  const int64_t bw = ntw * (ntw + 1) / 2;
  static const int64_t slots = [] {
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return (int64_t)256;
    return (int64_t)std::max(1, p.multiProcessorCount);  // one 4-wave block per CU (256 AGPRs)
  }();
  const int64_t n_stripes = (Wp + kWStripe - 1) / kWStripe;
  // split K so the grid fills the CUs in one round (slices >= 256 words); a block's f32
  // accumulators stay exact while its stripes (512 transactions each) number < 2^15
  int64_t ks = std::max<int64_t>(1, std::min<int64_t>(slots / bw, Wp / 256));
  ks = std::max<int64_t>(ks, (n_stripes + 32767) / 32768 + 1);
  hipLaunchKernelGGL(k_pair_gram_fp4mask, dim3((unsigned)bw, (unsigned)ks), dim3(256), 0, s,
                     (const unsigned long long*)bm, Wp, F, ntw, out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e));
}

}  // namespace kern
}  // namespace kmls
