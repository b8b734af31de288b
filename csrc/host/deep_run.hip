// Device orchestration of the count-only deep miner (see deep_run.hpp and kernels/deep.hip).
#include "deep_run.hpp"
#include "kmls/hooks.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#define KMLS_HIP(expr)                                                                  \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +      \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__));     \
  } while (0)

namespace kmls {
namespace gpu {

DeepBufs::~DeepBufs() {
  (void)hipSetDevice(device);
  for (void* p : {(void*)stacks, (void*)stacks0, (void*)fstacks, (void*)q[0], (void*)q[1], (void*)ready, (void*)req, (void*)inbox, (void*)inbox_state, (void*)d_key, (void*)heap[0],
                  (void*)heap[1], (void*)root, (void*)ctl, (void*)d_red, (void*)d_xor,
                  (void*)d_m, (void*)d_off, (void*)d_toff, (void*)d_cost, (void*)d_order,
                  (void*)d_trace, (void*)d_ticks, (void*)n_parent, (void*)n_item,
                  (void*)n_count, (void*)n_depth, (void*)d_node_off, (void*)d_split_q,
                  (void*)d_split_heap, (void*)d_ocost, (void*)d_otmp, (void*)t_new_id,
                  (void*)t_tmp, (void*)t_parent, (void*)t_item, (void*)t_count, (void*)t_depth,
                  (void*)d_part, (void*)d_wt, (void*)d_gram})
    if (p) (void)hipFree(p);
  if (h_ctl) (void)hipHostFree(h_ctl);
  if (h_tot) (void)hipHostFree(h_tot);
}

void DeepBufsDeleter::operator()(DeepBufs* p) const { delete p; }

namespace {

size_t env_bytes_mb(const char* name, size_t dflt_mb) {
  if (const char* e = std::getenv(name)) {
    const double v = std::atof(e);
    if (v > 0) return (size_t)(v * (double)(1ull << 20));
  }
  return dflt_mb << 20;
}

template <typename T>
void grow(T*& p, int64_t& cap_elems, int64_t need) {
  if (cap_elems >= need && p) return;
  if (p) KMLS_HIP(hipFree(p));
  p = nullptr;
  KMLS_HIP(hipMalloc((void**)&p, (size_t)std::max<int64_t>(need, 1) * sizeof(T)));
  cap_elems = need;
}

}  // namespace

DeepLocal deep_run(DeepBufs& b, const DeepInput& in, int rank, int world, const DeepOpts& opt) {
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms_since = [&](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(now() - t).count();
  };
  hipStream_t s = in.stream;
  const int64_t F = in.F;
  const int W = kern::deep_row_words(in.W_real);
  const int64_t Fpad = (F + 15) / 16 * 16;
  const int E = opt.emit ? 1 : 0;  // emit mode: blocks carry a node-word row
  DeepLocal res;

  // width tier of every root class: its rows are projected onto tid(item), |tid(item)| = support
  std::vector<int> wt((size_t)F, W);
  int widest = 1;
  for (int64_t i = 0; i < F; ++i) {
    const int64_t words = ((int64_t)in.counts[(size_t)i] + 63) / 64;
    wt[(size_t)i] = std::min(W, kern::deep_tier((int)std::max<int64_t>(words, 1)));
    widest = std::max(widest, wt[(size_t)i]);
  }
  const int maxt = kern::deep_count_maxt(widest);
  res.maxt = maxt;

  // ---- buffers (kept across calls) ----
  const auto t0 = now();
  // one 4-wave block per SIMD slot of the kernel instance (blocks_per_cu picks the instance)
  const int blocks_per_cu = kern::deep_count_wps(maxt, opt.blocks_per_cu, E != 0);
  const int grid = std::max(1, in.n_cus * blocks_per_cu);
  const int64_t waves = (int64_t)grid * kern::deep_waves_per_block();
  // Per-wave strides that are NOT powers of two: every wave works near the bottom of its own
  // stack, so 4 MiB-aligned stacks (and 128 KiB-aligned frame stacks) put the hot lines of all
  // 512 waves of an XCD into the same L2 sets (index bits 7-17), a few hundred of its 2048.
  // An odd number of 128-byte lines past the power of two spreads wave g's base over every set
  // (g x odd mod 2048 has full period).
  const size_t stack_need = std::max<size_t>(
      opt.stack_mb > 0 ? (size_t)opt.stack_mb << 20 : env_bytes_mb("KMLS_DEEP_STACK_MB", 4),
      4 * kern::deep_row_block_bytes(W, F, E)) + 69 * 128;
  const int fcap = std::max(4096, kern::deep_min_fcap()) + 36;  // 4132 x 32 B = 1033 lines
  // the dense first stack segment (off by default; KMLS_TEST_HOOKS deep_seg0_kb=<KB> turns it on), its stride skewed
  // off a power of two like the others
  const long long seg0_kb = test_hook("deep_seg0_kb", 0);  // (measured: 256 KB segments 29.4-30.2 ms vs 28.9-29.4 without, profiles/r6i_*)
  const size_t seg0 = seg0_kb > 0 ? ((size_t)seg0_kb << 10) + 69 * 128 : 0;
  if (b.waves < waves || b.stack_bytes < stack_need || b.fcap < fcap || b.seg0 != seg0) {
    if (b.stacks) KMLS_HIP(hipFree(b.stacks));
    if (b.stacks0) KMLS_HIP(hipFree(b.stacks0));
    if (b.fstacks) KMLS_HIP(hipFree(b.fstacks));
    b.stacks = nullptr;
    b.stacks0 = nullptr;
    b.fstacks = nullptr;
    KMLS_HIP(hipMalloc((void**)&b.stacks, (size_t)waves * stack_need));
    if (seg0) KMLS_HIP(hipMalloc((void**)&b.stacks0, (size_t)waves * seg0));
    KMLS_HIP(hipMalloc((void**)&b.fstacks, (size_t)waves * fcap * sizeof(kern::DeepFrame)));
    b.waves = waves;
    b.stack_bytes = stack_need;
    b.seg0 = seg0;
    b.fcap = fcap;
  }
  const int64_t q_cap = (int64_t)(env_bytes_mb("KMLS_DEEP_QUEUE_MB", 512) / sizeof(kern::DeepFrame));
  if (b.q_cap < q_cap) {
    for (auto& q : b.q) {
      if (q) KMLS_HIP(hipFree(q));
      q = nullptr;
      KMLS_HIP(hipMalloc((void**)&q, (size_t)q_cap * sizeof(kern::DeepFrame)));
    }
    if (b.ready) KMLS_HIP(hipFree(b.ready));
    KMLS_HIP(hipMalloc((void**)&b.ready, (size_t)q_cap * sizeof(unsigned)));
    KMLS_HIP(hipMemsetAsync(b.ready, 0, (size_t)q_cap * sizeof(unsigned), s));
    b.epoch = 0;
    b.q_cap = q_cap;
  }
  const size_t heap_cap = env_bytes_mb("KMLS_DEEP_HEAP_MB", 4096);
  if (b.heap_cap < heap_cap) {
    for (auto& h : b.heap) {
      if (h) KMLS_HIP(hipFree(h));
      h = nullptr;
      KMLS_HIP(hipMalloc((void**)&h, heap_cap));
    }
    b.heap_cap = heap_cap;
  }
  if (!b.ctl) {
    KMLS_HIP(hipMalloc((void**)&b.ctl, sizeof(kern::DeepCtl)));
    KMLS_HIP(hipHostMalloc((void**)&b.h_ctl, sizeof(kern::DeepCtl)));
    KMLS_HIP(hipHostMalloc((void**)&b.h_tot, 4 * sizeof(int64_t)));
    KMLS_HIP(hipMalloc((void**)&b.d_red, 66 * 8));
  }
  if (b.f_cap < F + 1) {
    int64_t c1 = b.f_cap, c2 = b.f_cap, c3 = b.f_cap, c4 = b.f_cap, c5 = b.f_cap;
    grow(b.d_m, c1, F + 1);
    grow(b.d_off, c2, F + 1);
    grow(b.d_toff, c3, F + 1);
    grow(b.d_node_off, c4, F + 1);
    grow(b.d_wt, c5, F + 1);
    b.node_off_cap = c4;
    b.f_cap = F + 1;
  }
  {
    const int64_t np = F * kern::deep_root_chunks(F);
    int64_t c = b.part_cap;
    grow(b.d_part, c, np);
    b.part_cap = c;
  }
  KMLS_HIP(hipMemsetAsync(b.ctl, 0, sizeof(kern::DeepCtl), s));
  res.ms_alloc = ms_since(t0);

  // ---- level 2: root classes (deterministic on every rank) ----
  const auto t1 = now();
  int64_t n_tasks = 0;
  int64_t n_heavy = 0;  // assign = 1: the queue's prefix of tasks with cost >= presplit_cost
  std::vector<int64_t> split_q, split_heap;  // pre-split layout of the heavy prefix (host)
  std::vector<int32_t> m;                     // (pre-split only) class sizes and offsets
  std::vector<int64_t> off, toff;
  int64_t split_tasks = 0, split_bytes = 0;
  if (F >= 2 && in.max_len != 1) {
    const size_t root_blk = (size_t)(W + 1) * (size_t)Fpad * 8;
    auto ensure_root = [&](size_t bytes, size_t keep) {  // keep: leading bytes to preserve
      if (b.root_bytes >= bytes) return;
      const size_t nb = std::max(bytes, b.root_bytes * 2);
      char* p = nullptr;
      KMLS_HIP(hipMalloc((void**)&p, nb));
      if (b.root && keep) KMLS_HIP(hipMemcpyAsync(p, b.root, keep, hipMemcpyDeviceToDevice, s));
      KMLS_HIP(hipStreamSynchronize(s));
      if (b.root) KMLS_HIP(hipFree(b.root));
      b.root = p;
      b.root_bytes = nb;
    };
    ensure_root(root_blk, 0);
    kern::deep_transpose(in.bm, in.Wp, F, W, in.W_real, in.d_ids, (uint64_t*)b.root, Fpad, s);
    // level-2 classes laid out on the device: chunk counts -> class sizes, block / task / node
    // offsets (prefix sums); one readback of the three totals (T is needed for the task order)
    KMLS_HIP(hipMemcpyAsync(b.d_wt, wt.data(), (size_t)F * 4, hipMemcpyHostToDevice, s));
    // the level-2 supports through the LDS-tiled popcount bit-GEMM (each row read once per tile)
    // instead of one AND + popcount per candidate pair in the class kernel (k_deep_root at
    // 140 + 277 us for F = 2032, gpurun_out/r5d_prof)
    {
      int64_t c = b.gram_cap;
      grow(b.d_gram, c, F * F);
      b.gram_cap = c;
      if (kern::pair_gram_dev_needs_zero(in.Wp, F))
        KMLS_HIP(hipMemsetAsync(b.d_gram, 0, (size_t)F * F * 4, s));
      kern::pair_gram_popcount(in.bm, in.Wp, F, b.d_gram, s);
    }
    kern::deep_root((const uint64_t*)b.root, Fpad, F, W, in.minsup, nullptr, b.d_part, nullptr,
                    nullptr, nullptr, false, s, nullptr, b.d_gram);
    kern::deep_root_scan(b.d_part, F, b.d_wt, E, (int64_t)root_blk, b.d_m, b.d_off, b.d_toff,
                         b.d_node_off, s);
    KMLS_HIP(hipMemcpyAsync(&b.h_tot[0], b.d_off + F, 8, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipMemcpyAsync(&b.h_tot[1], b.d_toff + F, 8, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipMemcpyAsync(&b.h_tot[2], b.d_node_off + F, 8, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipStreamSynchronize(s));
    const int64_t blk_end = b.h_tot[0], T = b.h_tot[1], pairs = b.h_tot[2];
    if (pairs < 0 || pairs > F * (F - 1) / 2 || T < 0 || blk_end < (int64_t)root_blk)
      throw std::runtime_error("deep_run: bad level-2 layout");
    if (rank == 0) res.per_depth[2] = (uint64_t)pairs;
    const bool deeper = in.max_len == 0 || in.max_len >= 3;
    ensure_root((size_t)blk_end, root_blk);
    kern::DeepNodes nodes{};
    if (E) {
      // the arena: level-1 nodes (ids = ranks), level-2 nodes (F + node_off[i] + slot), then
      // per-wave chunks from node_top; sizes reset to 0 (unused ids) over what the last call used
      // first guess: the two root levels x 8 and two node chunks per wave; a call that overflows
      // learns the exact need (node_top) and reruns.  The arena is regrown only when the last
      // call's ids come within 3 % of it, then to 10 % past them: node_top varies a little from
      // call to call (partly used per-wave chunks), and regrowing on every such wobble re-allocates
      // ~20 GB inside a timed step (164 vs 46 ms in one bench run)
      const int64_t guess = (F + pairs) * 8 + waves * 2 * kern::deep_node_chunk();
      const int64_t need = std::max<int64_t>({guess, b.arena_cap, (int64_t)(b.arena_used * 1.1)});
      if (need >= ((int64_t)1 << 32))
        throw std::runtime_error("deep_run: emit needs more than 2^32 trie nodes (u32 parent "
                                 "ids); use the count-only miner at this support");
      if (b.arena_cap < std::max<int64_t>(guess, (int64_t)(b.arena_used * 1.03))) {
        for (void* p : {(void*)b.n_parent, (void*)b.n_item, (void*)b.n_count, (void*)b.n_depth})
          if (p) KMLS_HIP(hipFree(p));
        KMLS_HIP(hipMalloc((void**)&b.n_parent, (size_t)need * 4));
        KMLS_HIP(hipMalloc((void**)&b.n_item, (size_t)need * 4));
        KMLS_HIP(hipMalloc((void**)&b.n_count, (size_t)need * 4));
        KMLS_HIP(hipMalloc((void**)&b.n_depth, (size_t)need));
        KMLS_HIP(hipMemsetAsync(b.n_depth, 0, (size_t)need, s));
        b.arena_cap = need;
        b.arena_used = 0;
      } else if (b.arena_used > 0) {
        KMLS_HIP(hipMemsetAsync(b.n_depth, 0, (size_t)std::min(b.arena_used, b.arena_cap), s));
      }
      std::vector<uint32_t> l1p((size_t)F, 0xffffffffu), l1i((size_t)F);
      std::vector<uint8_t> l1d((size_t)F, 1);
      for (int64_t i = 0; i < F; ++i) l1i[(size_t)i] = (uint32_t)i;
      KMLS_HIP(hipMemcpyAsync(b.n_parent, l1p.data(), (size_t)F * 4, hipMemcpyHostToDevice, s));
      KMLS_HIP(hipMemcpyAsync(b.n_item, l1i.data(), (size_t)F * 4, hipMemcpyHostToDevice, s));
      KMLS_HIP(hipMemcpyAsync(b.n_count, in.counts, (size_t)F * 4, hipMemcpyHostToDevice, s));
      KMLS_HIP(hipMemcpyAsync(b.n_depth, l1d.data(), (size_t)F, hipMemcpyHostToDevice, s));
      b.h_ctl->node_top = (unsigned long long)(F + pairs);
      KMLS_HIP(hipMemcpyAsync(&b.ctl->node_top, &b.h_ctl->node_top, 8, hipMemcpyHostToDevice, s));
      KMLS_HIP(hipStreamSynchronize(s));  // the pageable staging vectors die at scope end
      nodes = kern::DeepNodes{b.n_parent, b.n_item, b.n_count, b.n_depth, b.d_node_off};
    }
    kern::deep_root((const uint64_t*)b.root, Fpad, F, W, in.minsup, b.d_m, b.d_part, b.d_off,
                    b.root, rank == 0 ? b.ctl : nullptr, true, s, E ? &nodes : nullptr, b.d_gram);
    const int64_t* d_order = nullptr;
    if (deeper && T > 0 && (opt.assign == 1 || opt.trace)) {
      // every task's class size (its level-3 survivors) on the device; tasks ordered largest
      // first (device radix sort, stable in t) and dealt over the ranks in snake order, so every
      // rank gets an equal share of each size class and starts its queue with its largest tasks
      // (the long subtrees begin first instead of last: a shorter tail)
      const auto ta = now();
      int64_t c1 = b.t_cap, c2 = b.t_cap, c3 = b.t_cap;
      grow(b.d_cost, c1, T);
      grow(b.d_order, c2, T);
      grow(b.d_ocost, c3, T);
      b.t_cap = std::min({c1, c2, c3});
      // the deal's sort key (test hook deep_cost_key): 0 the class size (cost), 1 the class's
      // support mass (default: per-rank itemset shares 0.88-1.16 of the mean on 8 ranks, against
      // 0.77-1.18 by class size; profiles/r6s_*), 2 its square; a rank split only (one GPU takes
      // every task anyway)
      const int key_mode =
          world > 1 ? (opt.deal_key >= 0 ? opt.deal_key : (int)test_hook("deep_cost_key", 1)) : 0;
      if (key_mode) {
        int64_t c4 = b.key_cap;
        grow(b.d_key, c4, T);
        b.key_cap = c4;
      }
      kern::deep_task_cost(b.d_off, b.d_m, b.d_toff, F, b.root, in.minsup, b.d_cost, s, E,
                           key_mode ? b.d_key : nullptr, key_mode);
      std::vector<int64_t> mine;
      std::vector<uint32_t> cost;  // cost[q] of the rank's q-th task (host copies: pre-split, trace)
      if (opt.assign == 1) {
        // sorted and dealt on the device (deep_order.hip): no copy of the costs, no sync here
        if (b.otmp_bytes < kern::deep_task_order_bytes(T)) {
          if (b.d_otmp) KMLS_HIP(hipFree(b.d_otmp));
          b.otmp_bytes = kern::deep_task_order_bytes(T);
          KMLS_HIP(hipMalloc((void**)&b.d_otmp, b.otmp_bytes));
        }
        n_tasks = kern::deep_task_order(b.d_cost, T, rank, world, b.d_otmp, b.otmp_bytes,
                                        b.d_order, b.d_ocost, s, key_mode ? b.d_key : nullptr);
        if (n_tasks > b.q_cap) throw std::runtime_error("deep_run: level-3 task list exceeds the queue");
        const bool deeper4 = in.max_len == 0 || in.max_len >= 4;  // the split classes expand
        const bool presplit = opt.presplit_cost > 0 && opt.presplit_budget > 0 && opt.steal &&
                              deeper4 && world > 1;
        if (presplit || opt.trace) {
          mine.resize((size_t)n_tasks);
          cost.resize((size_t)n_tasks);
          KMLS_HIP(hipMemcpyAsync(mine.data(), b.d_order, (size_t)n_tasks * 8, hipMemcpyDeviceToHost, s));
          KMLS_HIP(hipMemcpyAsync(cost.data(), b.d_ocost, (size_t)n_tasks * 4, hipMemcpyDeviceToHost, s));
          if (presplit) {  // the heavy tasks' class layout (host pre-split plan below)
            m.resize((size_t)F);
            off.resize((size_t)F + 1);
            toff.resize((size_t)F + 1);
            KMLS_HIP(hipMemcpyAsync(m.data(), b.d_m, (size_t)F * 4, hipMemcpyDeviceToHost, s));
            KMLS_HIP(hipMemcpyAsync(off.data(), b.d_off, (size_t)(F + 1) * 8, hipMemcpyDeviceToHost, s));
            KMLS_HIP(hipMemcpyAsync(toff.data(), b.d_toff, (size_t)(F + 1) * 8, hipMemcpyDeviceToHost, s));
          }
          KMLS_HIP(hipStreamSynchronize(s));
        }
        // (a rank split only: on one GPU the extra launch costs more than the shorter tail gains,
        // profiles/r4i_*)
        if (presplit)
          while (n_heavy < n_tasks && cost[(size_t)n_heavy] >= std::max(opt.presplit_cost, 2u) &&
                 cost[(size_t)n_heavy] > opt.split_min)
            ++n_heavy;
      } else {
        std::vector<uint32_t> all((size_t)T);
        KMLS_HIP(hipMemcpyAsync(all.data(), b.d_cost, (size_t)T * 4, hipMemcpyDeviceToHost, s));
        KMLS_HIP(hipStreamSynchronize(s));
        for (int64_t t = rank; t < T; t += world) {
          mine.push_back(t);
          cost.push_back(all[(size_t)t]);
        }
        n_tasks = (int64_t)mine.size();
        if (n_tasks > b.q_cap) throw std::runtime_error("deep_run: level-3 task list exceeds the queue");
        KMLS_HIP(hipMemcpyAsync(b.d_order, mine.data(), (size_t)n_tasks * 8, hipMemcpyHostToDevice, s));
      }
      if (n_heavy > 0) {
        // every heavy task (i, k) becomes its class of c = cost members after one row step,
        // spilled as c - 1 single-member tasks over one heap copy of at most the root class
        // width: exact queue slots and heap offsets, no shared counter in the launch
        std::vector<int32_t> root_of((size_t)T);
        for (int64_t i = 0; i < F; ++i)
          for (int64_t t = toff[(size_t)i]; t < toff[(size_t)i + 1]; ++t) root_of[(size_t)t] = (int32_t)i;
        split_q.resize((size_t)n_heavy);
        split_heap.resize((size_t)n_heavy);
        for (int64_t q = 0; q < n_heavy; ++q) {
          const int64_t t = mine[(size_t)q];
          const int64_t i = root_of[(size_t)t];
          const int64_t c = cost[(size_t)q];
          const int64_t pad_i = (m[(size_t)i] + 15) / 16 * 16;
          const int64_t wt_i = (off[(size_t)i + 1] - off[(size_t)i]) / (8 * pad_i) - 1 - E;
          split_q[(size_t)q] = split_tasks;
          split_heap[(size_t)q] = split_bytes;
          split_tasks += c - 1;
          split_bytes += (wt_i + 1 + E) * ((c + 15) / 16 * 16) * 8;
        }
      }
      d_order = b.d_order;
      if (opt.trace) {
        res.task_ids = mine;
        res.task_cost = cost;
      }
      if (opt.assign != 1) KMLS_HIP(hipStreamSynchronize(s));  // `mine` dies at scope end
      res.ms_assign = ms_since(ta);
    } else {
      n_tasks = deeper ? (T - rank + world - 1) / world : 0;
      if (n_tasks > b.q_cap) throw std::runtime_error("deep_run: level-3 task list exceeds the queue");
    }
    if (n_tasks > 0)
      kern::deep_root_tasks(b.d_off, b.d_m, b.d_toff, F, b.root, (const uint64_t*)b.root, Fpad, W,
                            rank, world, d_order, n_tasks, b.q[0], s, E);
    KMLS_HIP(hipStreamSynchronize(s));  // pageable off/toff die at scope end
    res.level2_tasks = T;
  }
  res.ms_root = ms_since(t1);

  // ---- rounds ----
  const auto t2 = now();
  kern::DeepArgs a{};
  a.stacks = b.stacks;
  a.stack_bytes = b.stack_bytes;
  a.stacks0 = b.stacks0;
  a.seg0 = b.seg0;
  a.fstacks = b.fstacks;
  a.fcap = b.fcap;
  a.ctl = b.ctl;
  a.W = W;  // root width; every frame carries its own block width
  a.minsup = in.minsup;
  a.max_len = in.max_len;
  a.split_min = opt.split_min;
  // hand-offs split classes of >= 32 first members, keeping 5/16 of them (1 GPU: 29.3-29.9 ms
  // against 30.0-31.1 unsplit; 8 ranks: 8.1-8.3 vs 7.9-8.2 unsplit, 8.5-9.1 at >= 8 members)
  a.split_firsts = (unsigned)std::max<long long>(2, test_hook("deep_split_firsts", 32));
  a.split_keep16 = (unsigned)std::min<long long>(15, test_hook("deep_split_keep16", 5));
  a.ask_mask = (unsigned)test_hook("deep_ask_mask", 7);
  // a waiting wave asks 4 victims at once (the first donor fills its inbox): 1 GPU rounds
  // 27.8-27.9 vs 28.3-29.1 ms with one, 8 ranks 7.3-7.4 vs 7.6-8.0 ms (profiles/r6s_*)
  a.ask_fanout = (unsigned)std::max<long long>(1, std::min<long long>(64, test_hook("deep_ask_fanout", 4)));
  a.sleep_n = (unsigned)test_hook("deep_sleep_n", 1u << 30);
  a.out_cap = b.q_cap;
  a.heap_cap = b.heap_cap;
  a.trace = nullptr;
  a.task_ticks = nullptr;
  a.node_parent = E ? b.n_parent : nullptr;
  a.node_item = E ? b.n_item : nullptr;
  a.node_count = E ? b.n_count : nullptr;
  a.node_depth = E ? b.n_depth : nullptr;
  a.node_cap = E ? (unsigned long long)b.arena_cap : 0ull;
  a.split_q = nullptr;
  a.split_heap = nullptr;
  if (opt.trace && opt.steal && n_tasks > 0) {
    int64_t c1 = b.trace_cap, c2 = b.ticks_cap;
    grow(b.d_trace, c1, waves * kern::kDeepTraceWords);
    grow(b.d_ticks, c2, n_tasks);
    b.trace_cap = c1;
    b.ticks_cap = c2;
    KMLS_HIP(hipMemsetAsync(b.d_ticks, 0, (size_t)n_tasks * 8, s));
    KMLS_HIP(hipMemsetAsync(b.d_trace, 0, (size_t)waves * kern::kDeepTraceWords * 8, s));
    a.trace = b.d_trace;
    a.task_ticks = b.d_ticks;
    int khz = 0;
    KMLS_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, b.device));
    // 200 us buckets for a rank split, 1 ms for a whole problem
    a.trace_bucket = (unsigned long long)std::max(1, khz) * (world > 1 ? 1ull : 5ull) / 5ull;
  }
  {
    int khz = 0;
    KMLS_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, b.device));
    res.clock_khz = (double)khz;
    double secs = 120.0;
    if (const char* e = std::getenv("KMLS_DEEP_ROUND_TIMEOUT_S")) secs = std::max(1.0, std::atof(e));
    a.timeout_ticks = (unsigned long long)(secs * 1000.0 * (double)std::max(khz, 1));
  }
  kern::DeepFrame* steal_q = b.q[0];
  char* steal_heap = b.heap[0];
  int64_t steal_n = n_tasks;
  if (opt.steal && n_heavy > 0) {
    // pre-split: the heavy prefix runs one row step each without stealing and spills its class
    // at the host's offsets into q[1] / heap[0]; the light tasks are appended behind them and
    // the stealing launch takes q[1] (its own spills go to heap[1])
    const auto tp = now();
    const int64_t n_light = n_tasks - n_heavy;
    if (split_tasks + n_light > b.q_cap || (size_t)split_bytes > b.heap_cap)
      throw std::runtime_error("deep_run: pre-split tasks exceed the queue / heap; raise "
                               "KMLS_DEEP_QUEUE_MB / KMLS_DEEP_HEAP_MB");
    int64_t c1 = b.split_cap, c2 = b.split_cap;
    grow(b.d_split_q, c1, n_heavy);
    grow(b.d_split_heap, c2, n_heavy);
    b.split_cap = std::max(c1, c2);
    KMLS_HIP(hipMemcpyAsync(b.d_split_q, split_q.data(), (size_t)n_heavy * 8, hipMemcpyHostToDevice, s));
    KMLS_HIP(hipMemcpyAsync(b.d_split_heap, split_heap.data(), (size_t)n_heavy * 8,
                            hipMemcpyHostToDevice, s));
    KMLS_HIP(hipMemsetAsync(b.ctl, 0, 3 * sizeof(unsigned long long), s));  // ticket, n_out, heap
    kern::DeepArgs p = a;
    p.in = b.q[0];
    p.n_in = n_heavy;
    p.out = b.q[1];
    p.heap = b.heap[0];
    p.budget = 1;
    p.steal = 0;
    p.trace = nullptr;
    p.task_ticks = nullptr;
    p.split_q = (const long long*)b.d_split_q;
    p.split_heap = (const unsigned long long*)b.d_split_heap;
    kern::deep_count(p, maxt, blocks_per_cu,
                     (int)std::min<int64_t>(grid, (n_heavy + kern::deep_waves_per_block() - 1) /
                                                      kern::deep_waves_per_block()), s);
    if (n_light)
      KMLS_HIP(hipMemcpyAsync(b.q[1] + split_tasks, b.q[0] + n_heavy,
                              (size_t)n_light * sizeof(kern::DeepFrame), hipMemcpyDeviceToDevice, s));
    KMLS_HIP(hipMemcpyAsync(b.h_ctl, b.ctl, sizeof(kern::DeepCtl), hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipStreamSynchronize(s));  // (also: split_q / split_heap die at scope end)
    if (b.h_ctl->error)
      throw std::runtime_error("deep_run: the pre-split launch failed (error " +
                               std::to_string(b.h_ctl->error) + ")");
    steal_q = b.q[1];
    steal_heap = b.heap[1];
    steal_n = split_tasks + n_light;
    a.task_ticks = nullptr;  // the queue no longer holds the level-3 tasks in order
    res.presplit_in = n_heavy;
    res.presplit_out = split_tasks;
    res.round_tasks.push_back(n_heavy);
    res.round_ms.push_back(ms_since(tp));
    res.ms_presplit = ms_since(tp);
  }
  if (opt.steal && steal_n > 0) {
    // one launch: spilled tasks are queued behind the level-3 tasks and taken by waiting waves
    const auto tr = now();
    KMLS_HIP(hipMemsetAsync(b.ctl, 0, 5 * sizeof(unsigned long long), s));
    if (b.req_cap < waves) {
      for (void* p : {(void*)b.req, (void*)b.inbox, (void*)b.inbox_state})
        if (p) KMLS_HIP(hipFree(p));
      KMLS_HIP(hipMalloc((void**)&b.req, (size_t)waves * 8));
      KMLS_HIP(hipMalloc((void**)&b.inbox, (size_t)waves * sizeof(kern::DeepFrame)));
      KMLS_HIP(hipMalloc((void**)&b.inbox_state, (size_t)waves * 4));
      KMLS_HIP(hipMemsetAsync(b.req, 0, (size_t)waves * 8, s));
      KMLS_HIP(hipMemsetAsync(b.inbox_state, 0, (size_t)waves * 4, s));
      b.req_cap = waves;
    }
    b.h_ctl->pending = (unsigned long long)steal_n;
    KMLS_HIP(hipMemcpyAsync(&b.ctl->pending, &b.h_ctl->pending, 8, hipMemcpyHostToDevice, s));
    if (++b.epoch >= (1u << 30)) {  // 2^30 launches: restart the stamps
      KMLS_HIP(hipMemsetAsync(b.ready, 0, (size_t)b.q_cap * sizeof(unsigned), s));
      KMLS_HIP(hipMemsetAsync(b.req, 0, (size_t)b.req_cap * 8, s));
      KMLS_HIP(hipMemsetAsync(b.inbox_state, 0, (size_t)b.req_cap * 4, s));
      b.epoch = 1;
    }
    a.in = steal_q;
    a.n_in = steal_n;
    a.out = steal_q;
    a.heap = steal_heap;
    a.budget = std::max<unsigned long long>(opt.budget, 1);
    a.ready = b.ready;
    a.epoch = b.epoch;
    a.steal = 1;
    a.steal_eager = opt.steal_idle == 0 ? 1 : opt.steal_idle == 2 ? 2 : 0;
    a.req = b.req;
    a.inbox = b.inbox;
    a.inbox_state = b.inbox_state;
    a.nwaves = waves;
    kern::deep_count(a, maxt, blocks_per_cu, grid, s);
    KMLS_HIP(hipMemcpyAsync(b.h_ctl, b.ctl, sizeof(kern::DeepCtl), hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipStreamSynchronize(s));
    if (b.h_ctl->error & 4)
      throw std::runtime_error("deep_run: the launch ran past KMLS_DEEP_ROUND_TIMEOUT_S and gave up");
    if (b.h_ctl->error)
      throw std::runtime_error(std::string("deep_run: launch failed (") +
                               ((b.h_ctl->error & 8) ? "bad block width" :
                                (b.h_ctl->error & 1) ? "task queue overflow" : "spill heap overflow") +
                               "); raise KMLS_DEEP_QUEUE_MB / KMLS_DEEP_HEAP_MB");
    res.round_tasks.push_back(steal_n);
    res.round_ms.push_back(ms_since(tr));
    res.spilled_tasks = (int64_t)b.h_ctl->n_out;
    res.handoffs = (int64_t)b.h_ctl->handoffs;
    if (a.trace) {
      res.t_drain = b.h_ctl->t_drain;
      res.trace_bucket = a.trace_bucket;
      res.trace.resize((size_t)waves * kern::kDeepTraceWords);
      res.task_ticks.resize(a.task_ticks ? (size_t)n_tasks : 0);
      KMLS_HIP(hipMemcpy(res.trace.data(), b.d_trace, res.trace.size() * 8, hipMemcpyDeviceToHost));
      if (!res.task_ticks.empty())
        KMLS_HIP(hipMemcpy(res.task_ticks.data(), b.d_ticks, res.task_ticks.size() * 8,
                           hipMemcpyDeviceToHost));
    }
    n_tasks = 0;  // the rounds below have nothing left
  }
  int cur = 0;
  int64_t n_in = n_tasks;
  for (int round = 0; n_in > 0; ++round) {
    if (round >= 4096) throw std::runtime_error("deep_run: no progress after 4096 rounds");
    const auto tr = now();
    KMLS_HIP(hipMemsetAsync(b.ctl, 0, 3 * sizeof(unsigned long long), s));  // ticket, n_out, heap
    a.in = b.q[cur];
    a.n_in = n_in;
    a.out = b.q[cur ^ 1];
    a.heap = b.heap[round & 1];
    a.budget = round == 0 ? opt.budget0 : opt.budget;
    kern::deep_count(a, maxt, blocks_per_cu, (int)std::min<int64_t>(grid, (n_in + kern::deep_waves_per_block() - 1) /
                                                         kern::deep_waves_per_block()), s);
    KMLS_HIP(hipMemcpyAsync(b.h_ctl, b.ctl, sizeof(kern::DeepCtl), hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipStreamSynchronize(s));
    if (b.h_ctl->error & 4)
      throw std::runtime_error("deep_run: round " + std::to_string(round) +
                               " ran past KMLS_DEEP_ROUND_TIMEOUT_S and gave up");
    if (b.h_ctl->error)
      throw std::runtime_error("deep_run: round " + std::to_string(round) + " failed (" +
                               ((b.h_ctl->error & 8) ? "bad block width" :
                                (b.h_ctl->error & 1) ? "task queue overflow" : "spill heap overflow") +
                               "); raise KMLS_DEEP_QUEUE_MB / KMLS_DEEP_HEAP_MB");
    res.round_tasks.push_back(n_in);
    res.round_ms.push_back(ms_since(tr));
    n_in = (int64_t)b.h_ctl->n_out;
    res.spilled_tasks += n_in;
    cur ^= 1;
  }
  KMLS_HIP(hipMemcpyAsync(b.h_ctl, b.ctl, sizeof(kern::DeepCtl), hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  res.ms_rounds = ms_since(t2);
  for (int d = 3; d < 64; ++d) res.per_depth[(size_t)d] += b.h_ctl->per_depth[d];
  if (E) {
    const int64_t used = (int64_t)b.h_ctl->node_top;
    b.arena_used = used;  // (past the capacity after an overflow: the next call's size)
    b.max_depth = 2;
    for (int d = 3; d < 64; ++d)
      if (b.h_ctl->per_depth[d]) b.max_depth = d;
    if (used > b.arena_cap) throw ArenaOverflow(used);
    res.arena_nodes = used;
  }
  res.dsum = b.h_ctl->digest_sum;  // level-2 terms (rank 0) + the rounds
  res.dxor = b.h_ctl->digest_xor;
  res.candidates = b.h_ctl->candidates;
  res.chunks = b.h_ctl->chunks;
  return res;
}

}  // namespace gpu
}  // namespace kmls
