// HIP (gfx950) runtime API of kmls: the GPU FP-Growth miner and the HBM-resident rule index.
//
// Host code talks to the device only through this header; kernels live in csrc/kernels/*.hip.
#pragma once

#include <cstdint>
#include <memory>
#include <atomic>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "kmls/comm_host.hpp"
#include "kmls/common.hpp"
#include "kmls/host.hpp"

namespace pybind11 { class module_; }

namespace kmls {

void register_gpu_bindings(pybind11::module_& m);
void register_front_bindings(pybind11::module_& m);  // bindings_front.cpp

namespace gpu {

bool available();
int device_count();
std::string device_name(int dev);

// Thrown by DeviceArena::push when the arena is full (callers with a growable arena retry).
struct ArenaExhausted : std::runtime_error {
  size_t needed, cap;
  ArenaExhausted(size_t n, size_t c)
      : std::runtime_error("kmls: device arena exhausted (" + std::to_string(n) + " > " +
                           std::to_string(c) + " bytes); raise KMLS_ARENA_GB"),
        needed(n), cap(c) {}
};

// Bump/stack allocator over one big hipMalloc (DFS-of-batches needs strictly LIFO buffers).
class DeviceArena {
 public:
  explicit DeviceArena(size_t bytes);
  ~DeviceArena();
  void* push(size_t bytes);   // 256-byte aligned
  size_t mark() const { return top_; }
  void pop_to(size_t mark) { top_ = mark; }
  size_t capacity() const { return cap_; }
  size_t high_water() const { return hw_; }
  size_t used() const { return top_; }
 private:
  char* base_ = nullptr;
  size_t cap_ = 0, top_ = 0, hw_ = 0;
};

struct Phase {
  std::string name;
  double ms;
};

// Recycling pool of pinned host buffers (hipHostMalloc): results are handed to Python as numpy
// arrays that alias a buffer; the buffer returns to the pool when the last array dies, so the
// steady-state download costs no allocation and runs at pinned-DMA speed.
class PinnedPool : public std::enable_shared_from_this<PinnedPool> {
 public:
  ~PinnedPool();
  std::shared_ptr<void> get(size_t bytes);
 private:
  struct Buf { void* p; size_t bytes; bool busy; };
  std::vector<Buf> bufs_;
  void* mu_ = nullptr;  // std::mutex (kept out of the header)
  friend std::shared_ptr<PinnedPool> make_pinned_pool();
};
std::shared_ptr<PinnedPool> make_pinned_pool();

struct GpuMineResult {
  ItemsetTrie trie;           // host vectors (unused when the pinned arrays below are set)
  int64_t n_nodes = 0;
  std::shared_ptr<void> h_parent, h_item, h_count, h_depth;  // pinned, n_nodes entries
  int par_w = 8, item_w = 4, cnt_w = 4;  // element bytes of h_parent / h_item / h_count
  MineStats stats;
  std::vector<Phase> phases;  // hipEvent-timed phases
  int64_t arena_high_water = 0;
  std::string levels_path = "none";  // "fused" | "chunked" | "persistent" | "none"
  std::string level2_method = "gram";  // "gram" (bit-GEMM) | "cooc" (horizontal pair count)
  int64_t cooc_pairs = -1;             // sum_t k_t(k_t-1)/2 of the shard when it was measured
  // horizontal levels: filtered transactions / items, itemsets and containing-hit totals per size
  int64_t hl_tx_kept = -1, hl_nnz_kept = -1;
  std::vector<int64_t> hl_per_level, hl_hits;
  std::string level2_comm = "none";    // tx-DP: how the shard grams were combined
  // rule map (cfg.rule_index): CSR by item id, rows sorted by (count desc, tie key asc); pinned
  int64_t idx_nnz = -1;  // -1: not built
  int64_t n_items_idx = 0;  // row_ptr has n_items_idx entries (n_items + 1)
  std::shared_ptr<void> h_idx_row_ptr, h_idx_cons, h_idx_cnt;
};

// Native RCCL communicator (comm_rccl.cpp) over the librccl torch already loaded.
enum class CommDtype { U32, I64, U64, F64 };
size_t comm_dtype_bytes(CommDtype t);
std::string comm_unique_id();  // 128 opaque bytes, broadcast by the caller (torch.distributed)
class Comm {
 public:
  // backend "rccl" (uid from comm_unique_id) or "host" (uid from host_comm_unique_id)
  Comm(int rank, int world, const std::string& uid, int device, const std::string& backend = "rccl");
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;
  int rank() const { return rank_; }
  int world() const { return world_; }
  const std::string& backend() const { return backend_; }
  // stream-ordered collectives on `stream` (a hipStream_t); in place when send == recv
  void all_reduce(const void* send, void* recv, size_t count, CommDtype t, bool max_op,
                  void* stream);
  void all_gather(const void* send, void* recv, size_t count, CommDtype t, void* stream);
  // send = world blocks of recv_count elements; recv = the reduction of every rank's block
  // `rank` (row-block ownership of a matrix summed over transaction shards)
  void reduce_scatter(const void* send, void* recv, size_t recv_count, CommDtype t, bool max_op,
                      void* stream);
  // send = world blocks of `count` elements; recv block r = rank r's block `rank`
  void all_to_all(const void* send, void* recv, size_t count, CommDtype t, void* stream);
  // collective point-to-point: every rank sends to send_peer and receives from recv_peer
  // (equal sizes within a call: ring shifts of the context-parallel pass)
  void sendrecv(const void* send, int send_peer, void* recv, int recv_peer, size_t count,
                CommDtype t, void* stream);
  // bounded host wait for `stream` (KMLS_COMM_TIMEOUT_S): aborts the communicator and throws
  // when a collective never completes (a peer died)
  void wait_stream(void* stream);
  void abort();

 private:
  void progress(const char* what);
  void* stage(size_t bytes);
  int rank_ = 0, world_ = 1;
  bool direct_ = false;  // one rank, no communicator: collectives are local copies
  double timeout_s_ = 300.0;
  std::string backend_;
  void* comm_ = nullptr;
  std::unique_ptr<ShmComm> host_;
  void* staging_ = nullptr;  // pinned (host backend)
  size_t staging_bytes_ = 0;
};

struct OutBufs;  // persistent device trie buffers + download stream (miner_gpu.hip)
struct DeepBufs;  // count-only deep miner buffers (deep_gpu.hip)
struct DeepBufsDeleter {
  void operator()(DeepBufs* p) const;
};

// Count-only deep mining (deep_gpu.hip, kernels/deep.hip): per-size itemset counts and the
// content digest (kmls/digest.hpp; equal to trie_digest of the full trie) without a trie.
struct DeepOpts {
  // (defaults: the best of the r3e sweep at ds1 @0.02, profiles/r3_deep_sweep_projected.log)
  unsigned long long budget0 = 1024;  // rounds: 64-lane passes a first-round task may take
  unsigned long long budget = 16;     // steal: passes between mailbox checks (r3s sweep with
                                      // direct hand-offs: 8 / 16 / 64 / 256 -> 42.7 / 42.7 / 44.3
                                      // / 51.6 ms at ds1 @0.02, 8-rank split 9.4 / 9.6 / 11.2 /
                                      // 23.4 ms; r4i: 8 beat 16 by 1-3 %; with splitting
                                      // hand-offs (r7e/r7f) 2 / 4 / 8 / 16 / 32 / 64 -> 8-rank
                                      // 8.9-9.1 / 8.1-8.3 / 7.6-8.3 / 7.5-7.8 / 8.3 / 9.7-9.9 ms,
                                      // 1 GPU 28.3 at 16 vs 28.3-29.0 at 8);
                                      // rounds: later-round budget (1024 there)
  unsigned split_min = 8;             // spilled frames above this many members split per member
  int blocks_per_cu = 0;              // 0 = the kernel instance's occupancy (deep_waves_per_simd)
  int stack_mb = 0;                   // per-wave stack (0: KMLS_DEEP_STACK_MB or 4)
  bool steal = true;                  // one launch, spills taken by waiting waves (budget =
                                      // passes between checks for a waiting wave); false =
                                      // spill rounds (budget0/budget = per-task step budgets)
  unsigned steal_idle = 1;            // steal: 1 = hand over when a waiting wave asks; tests:
                                      // 0 = to the queue at every check, 2 = to the partner wave
  int assign = 1;                     // level-3 tasks: 1 = ordered by their measured class size
                                      // (largest first) and dealt over the ranks in snake order;
                                      // 0 = task t to rank t % world in index order
  bool trace = false;                 // per-wave / per-task timing of the launch (DeepResult)
  int deal_key = -1;                  // the snake deal's sort key at world > 1: 0 the class size,
                                      // 1 the class's support mass, -1 the default (1; test hook
                                      // deep_cost_key).  A partition recorded under one key (the
                                      // config-2 virtual ranks, profiles/config2_full) needs it.
  // pre-split (assign = 1, rank splits only): the rank's level-3 tasks whose class has >=
  // presplit_cost members
  // first run `presplit_budget` passes in a non-stealing launch that spills their open classes
  // as one task per member; the stealing launch then starts from those finer tasks (0 = off)
  unsigned presplit_cost = 16;
  unsigned long long presplit_budget = 1;
  // materialise: every frequent itemset becomes a node of an HBM trie arena (parent node id,
  // item rank, support, size), kept on the device after the call (GpuMiner::deep_arena_*)
  bool emit = false;
};
struct DeepResult {
  std::vector<uint64_t> per_level;  // [d] = frequent itemsets of size d (index 0 unused)
  int64_t n_itemsets = 0, n_frequent_items = 0, candidates = 0, chunks = 0, level2_tasks = 0;
  int max_depth = 0;
  uint64_t digest_sum = 0, digest_xor = 0;
  std::vector<int64_t> round_tasks;
  int64_t spilled_tasks = 0;
  int64_t handoffs = 0;
  std::vector<double> round_ms;
  double ms_prologue = 0, ms_root = 0, ms_rounds = 0, ms_combine = 0, ms_total = 0;
  double ms_assign = 0;               // task costs + ordering (inside ms_root)
  int64_t presplit_in = 0, presplit_out = 0;  // heavy tasks pre-split, tasks they became
  double ms_presplit = 0;
  int64_t arena_nodes = 0;            // emit: node ids used (holes included), arena capacity
  int64_t arena_cap = 0;
  // opts.trace: per wave kern::kDeepTraceWords words; per queued task (queue order) its id,
  // its class-size cost and the ticks its dequeuing wave spent on it; the clock rate
  std::vector<uint64_t> trace, task_ticks;
  std::vector<int64_t> task_ids;
  std::vector<uint32_t> task_cost;
  double clock_khz = 0;
  uint64_t t_drain = 0, trace_bucket = 0;  // (trace) queue drained at; busy bucket width (ticks)
};
struct GraphCache;  // captured launch sequence of the resident path (miner_gpu.hip)
struct Prefetch;    // a resident call launched ahead of its mine() (miner_gpu.hip)
}  // namespace gpu
namespace kern { struct FCtl; }
namespace gpu {

// Resident-data GPU miner.  Typical use: load() once (CSR → HBM), mine() many times.
// Multi-GPU: every rank calls the same sequence; collectives are done by the Python layer
// (torch.distributed / RCCL) on the buffers exposed through the *_dev accessors.
class GpuMiner {
 public:
  GpuMiner(int device, size_t arena_bytes, uintptr_t stream);
  ~GpuMiner();

  // Transaction CSR (rows duplicate-free) → HBM.  tx ids are local to this shard.
  void load_csr(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx, int64_t n_items);
  int64_t n_tx() const { return n_tx_; }
  int64_t n_items() const { return n_items_; }

  // Phase A: per-item supports of the resident shard into `counts_dev` (uint32[n_items]).
  void item_support(uintptr_t counts_dev);
  // Phase B: frequent-item selection from GLOBAL supports (host array) + global T.
  // Returns F.  `owned` (optional, size F): which top-level classes this rank mines.
  int64_t select(const uint32_t* global_counts, int64_t global_n_tx, double min_support);
  int64_t select_device(const uint32_t* d_counts, int64_t global_n_tx, double min_support,
                        Comm* comm = nullptr);
  // Item-sharded rounds (parallel/item_shard.py): make the frequent items at positions keep[]
  // (ascending, into the last select()'s order) the current set, for mine_bitmaps only — the
  // encode tables keep the full selection, and the next select() starts over.  Host work is O(n)
  // against select()'s O(n_items) table rebuild.
  void use_frequent_subset(const int64_t* keep, int64_t n);
  // a use_frequent_subset() set is current: d_rank_of_ / d_fmask_ / the encode tables still
  // describe the full selection, so the CSR-driven methods (cooc_*, pair_counts_csr,
  // rule_map_from_gram) would index past an F-row gram; they refuse while this holds
  bool subset_active() const { return fi_.ids.size() != sel_ids_.size(); }
  // Phase C: tid-bitmaps of frequent items for the resident shard, into an external buffer
  // (uint64[F][Wp]) at word offset `word_off` of rows of stride `Wp_total` words.
  int64_t words_local() const;  // padded words for the local shard
  bool encode_bitmaps(uintptr_t bm_dev, int64_t Wp_total, int64_t word_off);  // true: tiled
  void encode_bitmaps_fresh(uint64_t* bm, int64_t F, int64_t Wp);  // stale buffer ok
  // Phase D: full mining over replicated bitmaps (uint64[F][Wp_total]) covering `n_tx_total`.
  //   owned_mask: optional uint8[F] (top-level classes to expand; level-1 nodes always emitted
  //   by rank 0 only when emit_level1).
  GpuMineResult mine_bitmaps(uintptr_t bm_dev, int64_t Wp_total, const MineConfig& cfg,
                             const uint8_t* owned_mask, bool emit_level1, bool download);
  // Convenience single-GPU path: A + B + C + D.
  // prefetch: after launching this call, launch the next identical call (steady-state graph
  // replay only) before waiting, so its GPU work overlaps this call's host-side completion; the
  // next mine() with the same configuration adopts it.  At most one call is in flight ahead.
  GpuMineResult mine(const MineConfig& cfg, bool download, bool prefetch = false);
  // Replicated-data multi-GPU step (small datasets): every rank holds the full CSR, runs the
  // device-resident prologue, and expands only the root classes the device-side snake
  // partition assigns to `rank` — no collective inside; the caller all-reduces the count.
  bool resident_ok(const MineConfig& cfg) const;
  GpuMineResult mine_partition(const MineConfig& cfg, bool download, int rank, int world,
                               bool prefetch = false);
  // Transaction-data-parallel mining (large T): this rank holds a transaction shard; supports
  // are counted in `support_tiles` tiles whose all-reduces overlap the next tile's histogram
  // (comm stream); bitmaps stay shard-local ([F][Ws] words), and every level's candidate
  // counts are all-reduced in the loop, so all ranks build the identical global trie without
  // ever replicating bitmaps.  comm == nullptr behaves as world size 1.
  GpuMineResult mine_txdp(Comm* comm, int64_t global_n_tx, const MineConfig& cfg, bool download,
                          int support_tiles);
  // Item-sharded mining of sparse long shards without bitmaps (miner_gpu.hip): this rank's
  // sub-trie (level 1 + the subtrees of ranks r with r % world == rank); *declined when the
  // horizontal plan does not apply (nothing mined: the caller takes the bitmap protocol)
  GpuMineResult mine_shard(Comm* comm, int64_t global_n_tx, const MineConfig& cfg, bool download,
                           int support_tiles, bool* declined);
  // Count-only full mining (short transactions, T <= 4096): every rank holds the full CSR and
  // builds the level-2 classes; rank r mines level-3 tasks t with t % world == r; counts and
  // digests are combined through `comm` (nullptr: world must be 1, or the caller combines).
  DeepResult mine_deep(double min_support, int max_len, int rank, int world, Comm* comm,
                       const DeepOpts& opts);
  // The trie arena of the last mine_deep(emit) call: its content digest ([min_depth, ...] sizes,
  // set hashes rebuilt size by size on the device; equal to the count-only digest of the same
  // share) and, for small results, the arena itself (ids [0, n): parent node id or -1, original
  // item id, support, size; size 0 = an unused id)
  struct ArenaDigest {
    uint64_t sum = 0, xr = 0, n = 0;
    std::vector<uint64_t> per_depth;
  };
  ArenaDigest deep_arena_digest(int min_depth);
  void deep_arena_download(int64_t n, int64_t* parent, int32_t* item, uint32_t* count,
                           uint8_t* depth);
  // The arena of the last mine_deep(emit) as a dense trie whose parents come first (the product
  // output: kern::deep_trie_*), built on the device.  Nodes of size >= min_depth (a rank > 0 of
  // a split: 3, its share); their parents are new ids + `base` when exported, else their arena
  // id (levels 1-2: the same on every rank, and their ids in rank 0's export).  Returns the node
  // count; deep_trie_download copies the narrow arrays (parent i32, item u16 when item16 else
  // i32, support u16, size u8) to host memory.
  int64_t deep_arena_trie(int min_depth, int64_t base, bool* item16);
  void deep_trie_download(int32_t* parent, void* item, uint16_t* count, uint8_t* depth);

  // Frequent items of the last select(): ids (ascending support) and counts.
  const FrequentItems& frequent() const { return fi_; }
  // Pair supports (level-2) between frequent items as a dense upper-triangular matrix
  // count[F][F] (row-major, only i<j valid) via the bit-GEMM kernels. Used by the rule-map
  // fast path and by the multi-GPU pair all-reduce.
  void pair_counts(uintptr_t bm_dev, int64_t Wp_total, uintptr_t out_dev, bool use_mfma);
  // The same gram of the RESIDENT CSR shard counted horizontally (kern::cooc_count: every
  // co-occurring frequent pair once, no bitmaps), out[F][ld] zeroed here.  Sparse data (the
  // large BASELINE shapes) pays sum_t k_t^2/2 atomics instead of F^2 T/2 bit-ANDs.  False (out
  // untouched) when a transaction holds more than kern::cooc_max_k() frequent items.
  struct CoocStats {
    uint64_t pairs = 0;  // sum_t k_t (k_t - 1) / 2
    uint64_t max_k = 0;
  };
  CoocStats cooc_stats();
  bool pair_counts_csr(uintptr_t out_dev, int64_t ld);
  // after a pair_counts_csr on the stream: synchronises and throws if the count kernel met a
  // transaction with more frequent items than its entry buffer (pairs would be missing) or a
  // row holding one frequent item twice (load_csr's duplicate-free precondition broken)
  void cooc_check();
  // level-2 cost model: the horizontal count is predicted cheaper than the bit-GEMM over Wp words
  static bool cooc_cheaper(int64_t F, int64_t Wp, int64_t nnz, const CoocStats& st);
  // the model applied to this shard and the last select() (one stats pass; false below 64k tx)
  bool cooc_preferred();
  // the same decision from the supports alone (mean frequent items per transaction from the
  // selected counts; no CSR pass), and the count without the stats pass: 1 = done, 0 = a
  // transaction held more frequent items than the entry buffer (out is invalid: use the
  // bit-GEMM); synchronises; throws on a duplicated item.  Config 5 drops its 17 ms stats pass.
  bool cooc_likely();
  bool pair_counts_csr_direct(uintptr_t out_dev, int64_t ld);
  // Rule map (O10 pairs_to_csr) from a pair-count matrix already on the device (upper triangle,
  // rank order of the last select(), row stride ld): CSR by item id, rows by (count desc, tie
  // key asc).  For callers that own the gram (the large-shape pairs pipeline); the resident
  // mining call builds the same map inside its own launch sequence (MineConfig::rule_index).
  struct RuleMap {
    int64_t nnz = 0;
    unsigned status = 0;  // 1 entry overflow, 2 row longer than the device sort
    std::vector<int64_t> row_ptr;
    std::vector<int32_t> cons;
    std::vector<uint32_t> cnt;
  };
  RuleMap rule_map_from_gram(uintptr_t gram_dev, int64_t ld, uint32_t minsup);
  // Multi-GPU rule map (one rank's share): gram_mirror fills the lower triangle of an
  // upper-triangular gram; rule_map_rows builds the CSR of the row block [r0, r0 + nrows) x F of
  // a FULL symmetric gram (row_ptr by local row, cons = item ids, rows ordered as the single-GPU
  // map: count desc, tie key asc).
  void gram_mirror(uintptr_t gram_dev, int64_t ld, int64_t F);
  RuleMap rule_map_rows(uintptr_t rows_dev, int64_t ld, int64_t r0, int64_t nrows, uint32_t minsup);
  // Item-sharded mining (parallel/item_shard.py), on this miner's stream: union mask of rows,
  // per-word popcounts, and rows compressed onto a mask (see kern::compact_rows).
  void rows_union(uintptr_t rows, int64_t Wp, uintptr_t idx, int n, int64_t W, uintptr_t mask);
  void word_popc(uintptr_t mask, int64_t W, uintptr_t cnt);
  void compact_rows(uintptr_t rows, int64_t R, int64_t Wp_in, uintptr_t mask, uintptr_t nzw,
                    uintptr_t off, int64_t n_nz, uintptr_t out, int64_t Wp_out);
  // Context-parallel pair rows (parallel/pairs.py "ring"), native: X = this rank's [F][Ws]
  // transaction-shard bitmaps; rank r keeps its owned rows [r0, r1) of the pair-support matrix
  // (row_block) while the shards rotate around the ring through comm.sendrecv on a side stream,
  // block k counted on the miner's stream while block k+1 travels.  out[r1 - r0][ldo] (zeroed
  // here) = the owned rows summed over every shard.  Two shard copies of arena scratch.
  void ring_pair_rows(Comm* comm, uintptr_t X, int64_t F, int64_t Ws, uintptr_t out, int64_t ldo);
  // C[Fa][ldc] += popcount(A_i & B_j) over Wp words (ring-pass pair counting)
  void bitgemm_rect(uintptr_t A, int64_t Fa, uintptr_t B, int64_t Fb, int64_t Wp, uintptr_t C,
                    int64_t ldc);

  // Tie key of the rule-map rows (e.g. the rank of each item's name, so equal scores order by
  // consequent name as serve/index.py does); must be a permutation of [0, n_items).  Unset:
  // item id order.
  void set_tie_rank(const int32_t* tie, int64_t n);

  uintptr_t stream() const { return (uintptr_t)stream_; }
  void synchronize();
  size_t arena_capacity() const;

 private:
  int device_;
  void* stream_ = nullptr;
  bool own_stream_ = false;
  std::unique_ptr<DeviceArena> arena_;
  int64_t n_tx_ = 0, n_items_ = 0, nnz_ = 0;
  int64_t* d_tx_ptr_ = nullptr;
  int32_t* d_items_ = nullptr;
  FrequentItems fi_;
  std::vector<int32_t> sel_ids_;    // the last select()'s ids / counts (use_frequent_subset)
  std::vector<uint32_t> sel_counts_;
  int64_t global_n_tx_ = 0;
  int32_t* d_rank_of_ = nullptr;
  uint32_t* d_fmask_ = nullptr;  // frequent-item bit mask (large vocabularies, select())
  unsigned long long* d_fgroup_ = nullptr;  // encode tables (kern::frequent_groups)
  int32_t* d_c2r_ = nullptr;
  void build_encode_tables(int64_t F);  // syncs the stream
  void ensure_select_bufs();
  int64_t sel_cap_ = 0;           // vocabulary size the selection tables above are allocated for
  bool encode_tables_ = false;    // d_fgroup_ / d_c2r_ hold the current selection's tables
  int32_t* d_ids_ = nullptr;
  uint64_t* d_own_bm_ = nullptr;  // single-GPU bitmap buffer
  size_t own_bm_bytes_ = 0;
  std::shared_ptr<PinnedPool> pinned_;
  int64_t* h_scalar_ = nullptr;   // pinned readback scratch (allocated once: hipHostFree syncs)
  kern::FCtl* call_params_ = nullptr;  // pinned per-call control blocks [2] (read by the init kernel)
  unsigned int* d_call_seq_ = nullptr;  // device call counter: the init kernel reads slot seq & 1
  uint64_t call_seq_ = 0;               // host mirror (init launches enqueued)
  std::unique_ptr<Prefetch> pre_;       // a launched-ahead steady-state call (mine(prefetch))
  void drain_prefetch();
  uint64_t* d_pair_ = nullptr;    // device [survivors, next-level candidates]
  int n_cus_ = 256;
  bool mine_resident(const MineConfig& cfg, bool download, GpuMineResult& res, int part_rank,
                     int part_world, bool prefetch = false);
  // default-sized arenas start at 8 GiB and grow (x4, up to arena_max_) when the fused path
  // runs out of room; false if fixed-size, busy or already at the maximum
  bool grow_arena(size_t min_bytes);
  void support_counts(const int32_t* items, int64_t nnz, uint32_t* counts, void* stream);
  void* sup_scratch_ = nullptr;  // partitioned-histogram scratch (grown on demand)
  size_t sup_scratch_bytes_ = 0;
  bool arena_auto_ = false;
  size_t arena_max_ = 0;
  std::string fused_fallback_;
  std::unique_ptr<OutBufs> out_;  // output trie kept allocated across mine() calls
  std::unique_ptr<DeepBufs, DeepBufsDeleter> deep_;  // count-only deep miner buffers
  std::unique_ptr<GraphCache> graph_;  // steady-state hipGraph of mine_resident
  Comm* comm_ = nullptr;          // set during mine_txdp: level counts are all-reduced
  bool gram_csr_ok_ = false;      // mine_bitmaps' bitmaps are this miner's own CSR shard
  // horizontal levels (kern::HLevels, hlevels.hip): sparse long shards skip the bitmap encode;
  // level 2 from the CSR (cooc), levels >= 3 from a filtered CSR
  std::shared_ptr<void> hl_;
  std::shared_ptr<void> prows_;   // kern::PairRows: level-2 pair counts row by row in LDS
  bool pair_rows_ok(int64_t F) const;
  int64_t cooc_pairs_sampled();
  int64_t txdp_select(Comm* comm, int64_t global_n_tx, const MineConfig& cfg, int support_tiles);
  Comm* shard_comm_ = nullptr;    // mine_shard: the CSR all-gather's communicator
  int64_t hl_pairs_est_ = -1;
  bool prows_fresh_ = false;      // the last pair_counts_csr used the row count (its CSR is valid)
  bool pair_rows_count(uint32_t* gram, int64_t ld);
  bool hl_plan_ = false;          // the current mine_bitmaps call runs without bitmaps
  // need_rows: the plan also requires the row form of the pair count (item sharding: the
  // scattered-atomic fallback counts only this rank's CSR and nothing would reduce it)
  bool hlevels_plan(const MineConfig& cfg, int64_t F, int64_t Wp, Comm* comm,
                    bool need_rows = false);
  std::string hl_stats_;          // last horizontal run (JSON-ish summary for the phases)
  void txdp_gram_combine(uint32_t* gram, int64_t F, int64_t per, uint32_t minsup);
  unsigned long long* d_cooc_ = nullptr;  // [3]: cooc stats (pairs, max k) + error flag
  uint64_t sel_gen_ = 0;          // bumped by load_csr / select*: invalidates cached cooc stats
  uint64_t cooc_gen_ = ~0ull;
  CoocStats cooc_cache_;
  std::vector<int64_t> tile_tx_;  // 65 evenly spaced transaction boundaries of the shard
  std::vector<int64_t> tile_nnz_; // and their item offsets
  int64_t last_nodes_ = 0;        // size of the previous trie (pinned download sizing)
  int64_t fused_need_ = 0;        // trie nodes a fused call ran out of (output sizing hint)
  int32_t* d_tie_ = nullptr;      // rule-map tie key (item id -> rank) and its inverse
  int32_t* d_inv_tie_ = nullptr;
  int64_t idx_cap_ = 1 << 20;     // rule-map entry capacity (grown after an overflow)
  void* comm_s_ = nullptr;        // tx-DP: support-tile all-reduce stream (created once)
  std::vector<void*> tile_ev_;    // tx-DP: support-tile events (created once)
  void* idx_s_ = nullptr;         // rule-map side stream (a forked branch of the captured graph)
  void* idx_ev_[2] = {nullptr, nullptr};  // fork / join
  size_t idx_scan_bytes_ = 0;
  bool big_lds_ = false;
};

// Association rules on the GPU (rules_gpu.hip / kernels/rules.hip): same output and order as
// association_rules_cpu.  kernel_ms (optional) = hash build + both rule passes.
RuleSet association_rules_gpu(int device, const int64_t* parent, const int32_t* item,
                              const uint32_t* count, const uint8_t* depth, int64_t n, int64_t n_tx,
                              RuleMetric metric, double min_threshold, int max_antecedent,
                              double* kernel_ms);

// Transaction builder on the GPU (kernels/groupby.hip): same CSR as group_to_csr(dedup,
// sort_rows=true).
CSR group_to_csr_gpu(int device, const int32_t* keys, const int32_t* vals, int64_t n,
                     int32_t n_keys, bool dedup);

// HBM-resident rule index + batched matcher kernel (serve_match_topk).
class GpuRuleIndex {
 public:
  GpuRuleIndex(int device, const RuleIndex& host, uintptr_t stream);
  ~GpuRuleIndex();
  // q_ptr: int64[B+1], seeds: int32[nnz] (host).  Output host arrays ids[B*k], n[B]
  // with n = -1 when no seed is a key.  Exact reference ordering (score desc, then
  // first-insertion order).
  void query_batch(const int64_t* q_ptr, int64_t B, const int32_t* seeds, int k, int32_t* out_ids,
                   int32_t* out_n);
  // The same answers through the device's persistent serving kernel (GpuServeLoop): no launch
  // and no stream synchronisation per batch.  Only queries with <= kServeMaxSeeds seeds whose
  // merged rows fit the wave matcher (<= kServeWaveMerge entries) are answered there; others get
  // out_n = -2 (the caller answers them).  False: the loop is paused (an index is being built
  // or freed) or failed — nothing was answered.
  bool query_loop(const int64_t* q_ptr, int64_t B, const int32_t* seeds, int k,
                  int32_t* out_ids, int32_t* out_n);
  // merged entries of one query (sum of its key seeds' row lengths; the router's size)
  int64_t merged_size(const int32_t* seeds, int64_t n) const;
  int64_t nnz() const { return nnz_; }
  int64_t n_items() const { return n_items_; }
  int max_row() const { return max_row_; }

 private:
  int device_;
  void* stream_ = nullptr;
  bool own_stream_ = false;
  int64_t n_items_ = 0, nnz_ = 0;
  int max_row_ = 0;
  int64_t* d_row_ptr_ = nullptr;
  int32_t* d_cons_ = nullptr;
  uint32_t* d_score_ = nullptr;  // dense rank of the score (exact order key), see serve.hip
  bool narrow_ = false;          // score ranks < 2^23: the matcher's 32-bit order keys
  uint8_t* d_is_key_ = nullptr;
  int32_t* d_id_cons_ = nullptr;  // per row: consequents sorted by id (long-merge kernel)
  int32_t* d_id_pos_ = nullptr;   // ... and their index in the score-ordered row
  std::vector<int64_t> h_row_ptr_;  // host copies: per-query merge size decides the kernel
  std::vector<uint8_t> h_is_key_;
  // mapped pinned staging (queries in, results out; grown on demand)
  int32_t* h_pinned_ = nullptr;
  int64_t cap_pinned_ = 0;
};

// The device's persistent serving kernel: one 256-thread workgroup that polls a request word
// in mapped, coherent host memory, answers the batch with the wave matcher (4 queries at a
// time), publishes the results and a done word, and polls again — a round trip is two PCIe
// crossings instead of a kernel launch plus a stream synchronisation (~14.5 us per batch).  It
// exits after idle_ms without a request, after life_ms in all, or when stopped; the next
// request relaunches it.  While any index of the device is being built or freed the loops are
// paused (allocation calls must not wait behind a running kernel) and refuse requests.
struct ServeLoopStats {
  uint64_t requests = 0, queries = 0, launches = 0, refused = 0;
  double last_us = 0, sum_us = 0;
  double kernel_us = 0;  // sum over requests of the kernel's own time (request seen -> done)
  double stage_us = 0, compute_us = 0;  // ... of which: staging the request, answering it
  double phase_us[4] = {0, 0, 0, 0};  // first query: table init + seeds, row loads, inserts, top-k
};
class GpuServeLoop {
 public:
  static GpuServeLoop& for_device(int device);
  // one batch; false when paused / failed / every slot busy (nothing answered: the caller uses
  // the C++ matcher).  Thread-safe: callers on different threads use different request slots
  // and are answered concurrently.
  bool run(const int64_t* d_row_ptr, const int32_t* d_cons, const uint32_t* d_score,
           const uint8_t* d_is_key, int64_t n_items, const int64_t* q_ptr, int64_t B,
           const int32_t* seeds, int k, int32_t* out_ids, int32_t* out_n, bool narrow = false);
  void pause();   // stop the kernel, wait for it to exit; run() refuses until resume()
  void resume();
  ServeLoopStats stats();
  ~GpuServeLoop();

 private:
  explicit GpuServeLoop(int device);
  bool run_one(int slot, const int64_t* d_row_ptr, const int32_t* d_cons,
               const uint32_t* d_score, const uint8_t* d_is_key, int64_t n_items,
               const int64_t* q_ptr, int64_t B, const int32_t* seeds, int k, int32_t* out_ids,
               int32_t* out_n, bool narrow);
  int claim_slot();
  void release_slot(int slot);
  // under launch_mu_: the generation of a running launch (launching one if none runs); 0 when
  // paused
  unsigned ensure_running_locked();
  bool exited_locked(unsigned gen) const;  // every workgroup of launch `gen` has left
  void stop_and_wait_locked();
  void consume_locked(int slot, unsigned seq);  // no kernel runs: mark a request given up
  int device_;
  int nslots_ = 1;
  void* stream_ = nullptr;
  void* mail_ = nullptr;          // mapped coherent host: kern::ServeMail
  void* ctl_ = nullptr;           // device: kern::ServeLoopCtl
  int32_t* buf_ = nullptr;        // mapped coherent host: each slot's results
  unsigned seq_[16] = {0};        // per slot (owned by the slot's holder)
  std::atomic<uint32_t> free_mask_{0};
  int paused_ = 0;
  bool launched_ = false;
  unsigned gen_ = 0;              // generation of the newest launch
  unsigned long long idle_ticks_ = 0, life_ticks_ = 0;
  double ticks_per_us_ = 100.0;
  ServeLoopStats st_;
  std::mutex launch_mu_, stats_mu_;
};
// pauses every serving loop of `device` for the guard's lifetime (index builds / frees)
struct ServeLoopPause {
  explicit ServeLoopPause(int device);
  ~ServeLoopPause();
  int device;
};

}  // namespace gpu
}  // namespace kmls
