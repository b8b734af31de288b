// Host driver of the count-only deep miner (kernels/deep.hip): full FP-Growth output size and
// content digest at supports whose itemsets cannot be materialised (BASELINE config 2: ds1 at
// 0.01-0.02, 1e9-1e10 itemsets; the reference mines all sizes, machine-learning/main.py:272, and
// sweeps min_support downwards, main.py:450-473).
//
// Call sequence (one rank = one GPU; every rank runs the same prologue on the full data):
//   supports -> selection -> bitmaps [F][Wp] -> transposed root block ->
//   level-2 classes (the popcount gram read by a count pass, a device prefix scan, a fill pass
//   over the surviving groups only) -> every level-3 task's cost probed on the device, the tasks
//   cost-ordered and dealt to the ranks in a snake (deep_order.hip) -> one stealing launch of
//   k_deep_count over this rank's share (idle waves take open classes from busy ones) ->
//   per-size counts + digest, all-reduced over the ranks.  Emit mode writes a node arena instead,
//   compacted into a parent-first trie on the device (deep_trie.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "deep_run.hpp"
#include "kmls/digest.hpp"
#include "kmls/gpu.hpp"

#define KMLS_HIP(expr)                                                                  \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +      \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__));     \
  } while (0)

namespace kmls {
namespace gpu {

DeepResult GpuMiner::mine_deep(double min_support, int max_len, int rank, int world, Comm* comm,
                               const DeepOpts& opt) {
  drain_prefetch();
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  KMLS_CHECK(world >= 1 && rank >= 0 && rank < world, "mine_deep: bad rank/world");
  KMLS_CHECK(comm == nullptr || comm->world() == world, "mine_deep: comm world differs");
  const int W_real = (int)((n_tx_ + 63) / 64);
  KMLS_CHECK(W_real <= kern::deep_max_words(),
             "mine_deep: transactions longer than 4096 (use the level-wise tx-DP miner)");
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms_since = [&](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(now() - t).count();
  };
  DeepResult res;
  const auto t0 = now();

  // ---- prologue: supports, selection, bitmaps ----
  const size_t mark = arena_->mark();
  uint32_t* d_cnt = (uint32_t*)arena_->push((size_t)std::max<int64_t>(n_items_, 1) * 4);
  item_support((uintptr_t)d_cnt);
  std::vector<uint32_t> cnt((size_t)n_items_);
  KMLS_HIP(hipMemcpyAsync(cnt.data(), d_cnt, cnt.size() * 4, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  arena_->pop_to(mark);
  const int64_t F = select(cnt.data(), n_tx_, min_support);
  const int64_t Wp = words_local();
  const size_t need_bm = (size_t)std::max<int64_t>(F, 1) * Wp * 8;
  if (need_bm > own_bm_bytes_) {
    if (d_own_bm_) KMLS_HIP(hipFree(d_own_bm_));
    KMLS_HIP(hipMalloc((void**)&d_own_bm_, need_bm));
    own_bm_bytes_ = need_bm;
  }
  if (F) encode_bitmaps_fresh(d_own_bm_, F, Wp);
  const uint32_t minsup = fi_.minsup2;
  res.n_frequent_items = F;
  std::vector<uint64_t> per(64, 0);
  uint64_t dsum = 0, dxor = 0;
  if (rank == 0) {  // level 1 (every rank holds it; rank 0 counts it)
    per[1] = (uint64_t)F;
    for (int64_t r = 0; r < F; ++r) {
      const DigestTerms t = digest_terms(item_mix((uint64_t)fi_.ids[(size_t)r]), fi_.counts[(size_t)r]);
      dsum += t.sum;
      dxor ^= t.xr;
    }
  }
  if (!deep_) deep_.reset(new DeepBufs());
  deep_->device = device_;
  DeepInput in;
  in.bm = d_own_bm_;
  in.Wp = Wp;
  in.F = F;
  in.W_real = W_real;
  in.d_ids = d_ids_;
  in.counts = fi_.counts.data();
  in.minsup = minsup;
  in.max_len = max_len;
  in.n_cus = n_cus_;
  in.stream = s;
  res.ms_prologue = ms_since(t0);
  DeepLocal loc;
  for (int attempt = 0;; ++attempt) {
    try {
      loc = deep_run(*deep_, in, rank, world, opt);
      break;
    } catch (const ArenaOverflow& ex) {  // emit: the arena is regrown from the count and rerun
      if (attempt >= 2) throw;
    }
  }
  DeepBufs& b = *deep_;
  for (int d = 2; d < 64; ++d) per[(size_t)d] += loc.per_depth[(size_t)d];
  dsum += loc.dsum;
  dxor ^= loc.dxor;
  uint64_t cands = loc.candidates;
  res.chunks = (int64_t)loc.chunks;
  res.level2_tasks = loc.level2_tasks;
  res.round_tasks = loc.round_tasks;
  res.spilled_tasks = loc.spilled_tasks;
  res.handoffs = loc.handoffs;
  res.round_ms = loc.round_ms;
  res.ms_root = loc.ms_root;
  res.ms_rounds = loc.ms_rounds;
  res.ms_assign = loc.ms_assign;
  res.ms_presplit = loc.ms_presplit;
  res.arena_nodes = loc.arena_nodes;
  res.arena_cap = deep_->arena_cap;
  res.presplit_in = loc.presplit_in;
  res.presplit_out = loc.presplit_out;
  res.trace = std::move(loc.trace);
  res.task_ticks = std::move(loc.task_ticks);
  res.task_ids = std::move(loc.task_ids);
  res.task_cost = std::move(loc.task_cost);
  res.clock_khz = loc.clock_khz;
  res.t_drain = loc.t_drain;
  res.trace_bucket = loc.trace_bucket;
  if (b.xor_cap < world) {
    if (b.d_xor) KMLS_HIP(hipFree(b.d_xor));
    KMLS_HIP(hipMalloc((void**)&b.d_xor, (size_t)world * 8));
    b.xor_cap = world;
  }

  // ---- combine over ranks (RCCL or the host communicator, stream-ordered) ----
  const auto t3 = now();
  if (comm && world > 1) {
    std::vector<uint64_t> red(66);
    std::copy(per.begin(), per.end(), red.begin());
    red[64] = dsum;
    red[65] = cands;
    KMLS_HIP(hipMemcpyAsync(b.d_red, red.data(), 66 * 8, hipMemcpyHostToDevice, s));
    KMLS_HIP(hipMemcpyAsync(b.d_xor + rank, &dxor, 8, hipMemcpyHostToDevice, s));
    comm->all_reduce(b.d_red, b.d_red, 66, CommDtype::U64, false, s);
    comm->all_gather(b.d_xor + rank, b.d_xor, 1, CommDtype::U64, s);
    std::vector<uint64_t> xs((size_t)world);
    KMLS_HIP(hipMemcpyAsync(red.data(), b.d_red, 66 * 8, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipMemcpyAsync(xs.data(), b.d_xor, (size_t)world * 8, hipMemcpyDeviceToHost, s));
    comm->wait_stream(s);
    std::copy(red.begin(), red.begin() + 64, per.begin());
    dsum = red[64];
    cands = red[65];
    dxor = 0;
    for (uint64_t x : xs) dxor ^= x;
  }
  res.ms_combine = ms_since(t3);
  res.per_level.assign(per.begin(), per.end());
  while (res.per_level.size() > 2 && res.per_level.back() == 0) res.per_level.pop_back();
  res.n_itemsets = 0;
  for (size_t d = 1; d < res.per_level.size(); ++d) res.n_itemsets += (int64_t)res.per_level[d];
  res.max_depth = 0;
  for (size_t d = 1; d < res.per_level.size(); ++d)
    if (res.per_level[d]) res.max_depth = (int)d;
  res.digest_sum = dsum;
  res.digest_xor = dxor;
  res.candidates = (int64_t)cands;
  res.ms_total = ms_since(t0);
  return res;
}

GpuMiner::ArenaDigest GpuMiner::deep_arena_digest(int min_depth) {
  KMLS_CHECK(deep_ && deep_->arena_used > 0, "deep_arena_digest: no emit-mode mine_deep yet");
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  DeepBufs& b = *deep_;
  const int64_t n = std::min(b.arena_used, b.arena_cap);
  uint64_t* hash = nullptr;
  unsigned long long* out = nullptr;
  KMLS_HIP(hipMalloc((void**)&hash, (size_t)n * 8));
  KMLS_HIP(hipMalloc((void**)&out, 66 * 8));
  ArenaDigest r;
  try {
    KMLS_HIP(hipMemsetAsync(out, 0, 66 * 8, s));
    kern::deep_arena_digest(b.n_parent, b.n_item, b.n_count, b.n_depth, n, d_ids_, b.max_depth,
                            std::max(min_depth, 1), hash, out, s);
    std::vector<unsigned long long> h(66);
    KMLS_HIP(hipMemcpyAsync(h.data(), out, 66 * 8, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipStreamSynchronize(s));
    r.per_depth.assign(64, 0);
    for (int d = 1; d < 62; ++d) r.per_depth[(size_t)d] = h[(size_t)(2 + d)];
    r.sum = h[0];
    r.xr = h[1];
    for (int d = 1; d < 62; ++d) r.n += r.per_depth[(size_t)d];
  } catch (...) {
    (void)hipFree(hash);
    (void)hipFree(out);
    throw;
  }
  (void)hipFree(hash);
  (void)hipFree(out);
  return r;
}

void GpuMiner::deep_arena_download(int64_t n, int64_t* parent, int32_t* item, uint32_t* count,
                                   uint8_t* depth) {
  KMLS_CHECK(deep_ && n <= std::min(deep_->arena_used, deep_->arena_cap),
             "deep_arena_download: n past the arena");
  KMLS_HIP(hipSetDevice(device_));
  DeepBufs& b = *deep_;
  std::vector<uint32_t> p((size_t)n), it((size_t)n);
  KMLS_HIP(hipMemcpy(p.data(), b.n_parent, (size_t)n * 4, hipMemcpyDeviceToHost));
  KMLS_HIP(hipMemcpy(it.data(), b.n_item, (size_t)n * 4, hipMemcpyDeviceToHost));
  KMLS_HIP(hipMemcpy(count, b.n_count, (size_t)n * 4, hipMemcpyDeviceToHost));
  KMLS_HIP(hipMemcpy(depth, b.n_depth, (size_t)n, hipMemcpyDeviceToHost));
  for (int64_t v = 0; v < n; ++v) {
    parent[v] = p[(size_t)v] == 0xffffffffu ? -1 : (int64_t)p[(size_t)v];
    item[v] = depth[v] ? fi_.ids[(size_t)it[(size_t)v]] : -1;
  }
}

int64_t GpuMiner::deep_arena_trie(int min_depth, int64_t base, bool* item16) {
  KMLS_CHECK(deep_ && deep_->arena_used > 0 && deep_->arena_used <= deep_->arena_cap,
             "deep_arena_trie: no emit-mode mine_deep yet");
  KMLS_CHECK(n_tx_ < 65536, "deep_arena_trie: supports must fit 16 bits");
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  DeepBufs& b = *deep_;
  const int64_t n = b.arena_used;
  const int nd = std::min(b.max_depth + 1, 64);
  auto dgrow = [&](auto*& p, size_t bytes) {
    if (p) KMLS_HIP(hipFree(p));
    p = nullptr;
    KMLS_HIP(hipMalloc((void**)&p, std::max<size_t>(bytes, 256)));
  };
  if (b.t_ids_cap < n) {
    dgrow(b.t_new_id, (size_t)n * 4);
    b.t_ids_cap = n;
  }
  const size_t tb = kern::deep_trie_scratch_bytes(n, nd);
  if (b.t_tmp_bytes < tb) {
    dgrow(b.t_tmp, tb);
    b.t_tmp_bytes = tb;
  }
  const int64_t m = kern::deep_trie_layout(b.n_depth, n, std::max(min_depth, 1), nd, b.t_new_id,
                                           b.t_tmp, b.t_tmp_bytes, s);
  KMLS_CHECK(base >= 0 && base + m < ((int64_t)1 << 31),
             "deep_arena_trie: 2^31 trie nodes (i32 parent ids)");
  if (b.tr_cap < m) {
    dgrow(b.t_parent, (size_t)m * 4);
    dgrow(b.t_item, (size_t)m * 4);
    dgrow(b.t_count, (size_t)m * 2);
    dgrow(b.t_depth, (size_t)m);
    b.tr_cap = m;
  }
  b.t_item16 = n_items_ <= 65536;
  kern::deep_trie_scatter(b.n_parent, b.n_item, b.n_count, b.n_depth, n, b.t_new_id, d_ids_, base,
                          b.t_parent, b.t_item, b.t_item16, b.t_count, b.t_depth, s);
  b.t_n = m;
  if (item16) *item16 = b.t_item16;
  return m;
}

void GpuMiner::deep_trie_download(int32_t* parent, void* item, uint16_t* count, uint8_t* depth) {
  KMLS_CHECK(deep_ && deep_->t_n >= 0, "deep_trie_download: deep_arena_trie first");
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  DeepBufs& b = *deep_;
  const size_t m = (size_t)b.t_n;
  KMLS_HIP(hipMemcpyAsync(parent, b.t_parent, m * 4, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipMemcpyAsync(item, b.t_item, m * (b.t_item16 ? 2 : 4), hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipMemcpyAsync(count, b.t_count, m * 2, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipMemcpyAsync(depth, b.t_depth, m, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
}

}  // namespace gpu
}  // namespace kmls
