// Device orchestration of the count-only deep miner (deep_run.hip): level-2 classes, the rank's
// level-3 tasks, and the spill rounds of k_deep_count.  Free of GpuMiner so the CPU wave
// emulator (csrc/emu, tests only) can drive the same code over host memory.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <vector>

#include "../kernels/kernels.hpp"
#include "kmls/gpu.hpp"

namespace kmls {
namespace gpu {

// device buffers of the deep miner, kept across calls (allocation maps HBM eagerly)
struct DeepBufs {
  int device = 0;
  char* stacks = nullptr;
  size_t stack_bytes = 0;  // per wave
  char* stacks0 = nullptr;  // per wave: the dense first segment of its stack (kern::DeepArgs)
  size_t seg0 = 0;
  int64_t waves = 0;
  kern::DeepFrame* fstacks = nullptr;
  int fcap = 0;
  kern::DeepFrame* q[2] = {nullptr, nullptr};
  int64_t q_cap = 0;
  unsigned* ready = nullptr;  // [q_cap] steal-mode publish flags (zeroed once at allocation)
  unsigned long long* req = nullptr;  // [req_cap] steal-mode mailboxes (one per wave)
  kern::DeepFrame* inbox = nullptr;   // [req_cap] direct hand-offs
  unsigned* inbox_state = nullptr;    // [req_cap]
  int64_t req_cap = 0;
  unsigned epoch = 0;         // steal-mode launch stamp of the flags

  char* heap[2] = {nullptr, nullptr};
  size_t heap_cap = 0;
  char* root = nullptr;  // root block + level-2 blocks
  size_t root_bytes = 0;
  int32_t* d_m = nullptr;  // [F] level-2 class sizes
  int32_t* d_part = nullptr;  // [F][deep_root_chunks(F)] level-2 chunk counts / bases
  int64_t part_cap = 0;
  int32_t* d_wt = nullptr;    // [F] projected width tier of each root class
  uint32_t* d_gram = nullptr; // [F][F] level-2 pair gram (upper triangle)
  int64_t gram_cap = 0;
  int64_t* h_tot = nullptr;   // pinned [4]: layout totals read back once per call
  int64_t* d_off = nullptr;  // [F + 1] block byte offsets
  int64_t* d_toff = nullptr;  // [F + 1] task offsets
  int64_t f_cap = 0;
  uint32_t* d_cost = nullptr;   // [T] level-3 task costs (assign = 1)
  uint32_t* d_key = nullptr;    // [key_cap] the deal's sort key (test hook deep_cost_key)
  int64_t key_cap = 0;
  int64_t* d_order = nullptr;   // [T] this rank's task ids in queue order
  uint32_t* d_ocost = nullptr;  // [T] their costs
  int64_t t_cap = 0;
  char* d_otmp = nullptr;       // kern::deep_task_order scratch
  size_t otmp_bytes = 0;
  // emit mode: the node arena (SoA, arena_cap ids) and the level-2 node bases
  unsigned* n_parent = nullptr;
  unsigned* n_item = nullptr;
  unsigned* n_count = nullptr;
  unsigned char* n_depth = nullptr;
  int64_t arena_cap = 0, arena_used = 0;
  int max_depth = 0;
  int64_t* d_node_off = nullptr;
  // the arena as a dense trie (GpuMiner::deep_arena_trie): new ids, scratch, narrow outputs
  uint32_t* t_new_id = nullptr;
  char* t_tmp = nullptr;
  size_t t_tmp_bytes = 0;
  int32_t* t_parent = nullptr;
  int32_t* t_item = nullptr;     // u16 or i32 items
  uint16_t* t_count = nullptr;
  unsigned char* t_depth = nullptr;
  int64_t tr_cap = 0, t_ids_cap = 0;
  int64_t t_n = 0;               // nodes of the last layout
  bool t_item16 = true;
  int64_t* d_split_q = nullptr;   // pre-split layout: queue slot and heap offset per heavy task
  int64_t* d_split_heap = nullptr;
  int64_t split_cap = 0;
  int64_t node_off_cap = 0;
  unsigned long long* d_trace = nullptr;  // [waves * kDeepTraceWords] (opts.trace)
  unsigned long long* d_ticks = nullptr;  // [T] (opts.trace)
  int64_t trace_cap = 0, ticks_cap = 0;
  kern::DeepCtl* ctl = nullptr;
  kern::DeepCtl* h_ctl = nullptr;  // pinned readback
  uint64_t* d_red = nullptr;       // [66]: per_depth[64], digest_sum, candidates (all-reduce)
  uint64_t* d_xor = nullptr;       // [world] (all-gather)
  int xor_cap = 0;
  ~DeepBufs();
};

struct DeepInput {
  const uint64_t* bm = nullptr;   // device [F][Wp] frequent-item bitmaps (rank order)
  int64_t Wp = 0, F = 0;
  int W_real = 0;                 // ceil(T / 64)
  const int32_t* d_ids = nullptr; // device [F] rank -> original item id
  const uint32_t* counts = nullptr;  // host [F] supports (root class i's tid projection width)
  uint32_t minsup = 0;            // count threshold for |S| >= 2
  int max_len = 0;
  int n_cus = 256;
  hipStream_t stream = nullptr;
};

// This rank's share: counts of sizes >= 2 (size 2 on rank 0 only), digest terms, stats.
struct DeepLocal {
  std::vector<uint64_t> per_depth = std::vector<uint64_t>(64, 0);
  uint64_t dsum = 0, dxor = 0, candidates = 0, chunks = 0;
  int64_t level2_tasks = 0;
  int maxt = 0;  // widest block tier of the count kernel instance
  std::vector<int64_t> round_tasks;
  int64_t spilled_tasks = 0;  // tasks spilled inside the launch(es)
  int64_t handoffs = 0;       // classes handed straight to a requesting wave (steal mode)
  std::vector<double> round_ms;
  double ms_alloc = 0, ms_root = 0, ms_rounds = 0, ms_assign = 0, ms_presplit = 0;
  int64_t presplit_in = 0, presplit_out = 0;
  int64_t arena_nodes = 0;  // emit: node ids used, holes included
  std::vector<uint64_t> trace, task_ticks;  // opts.trace
  std::vector<int64_t> task_ids;
  std::vector<uint32_t> task_cost;
  double clock_khz = 0;
  uint64_t t_drain = 0, trace_bucket = 0;  // (trace) queue drained at; bucket width (ticks)
};

// emit mode: the arena was too small (node_top counts on past its end); `needed` ids
struct ArenaOverflow : std::runtime_error {
  int64_t needed;
  explicit ArenaOverflow(int64_t n)
      : std::runtime_error("deep_run: node arena overflow"), needed(n) {}
};
DeepLocal deep_run(DeepBufs& b, const DeepInput& in, int rank, int world, const DeepOpts& opt);

}  // namespace gpu
}  // namespace kmls
