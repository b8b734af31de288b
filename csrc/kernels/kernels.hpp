// Launch wrappers of the CDNA4 kernels (implemented in csrc/kernels/*.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <vector>

namespace kmls {
namespace kern {

// ---- count-only deep mining (deep.hip) ----
struct DeepFrame {  // one class: members P ∪ {x_k}, k in [s0, s0 + m), of a word-major block
  unsigned long long blk;   // device address: W words x pad slots ([w][slot]), then pad item hashes
  unsigned long long hash;  // set hash of the prefix P
  unsigned pad;             // slot stride (multiple of 16)
  unsigned s0;              // first member slot
  unsigned m;               // members
  unsigned meta;            // bits 0-7 |P|, bit 8 single (expand member s0 only), 9-15 block
                            // width (words), 16-31 block index
};
static_assert(sizeof(DeepFrame) == 32, "DeepFrame is read as 8 dwords");
struct DeepCtl {  // per-round control + accumulated results (zeroed once per call)
  unsigned long long next_task;   // dequeue ticket (zeroed per round)
  unsigned long long n_out;       // tasks spilled to the out queue (zeroed per round)
  unsigned long long heap_top;    // bytes of the out heap used (zeroed per round)
  unsigned long long pending;     // steal mode: queued + running tasks (0 = the launch is done)
  unsigned long long handoffs;    // steal mode: classes handed to a requesting wave's inbox
  unsigned long long node_top;    // emit mode: node ids handed out (chunks; keeps counting past
                                  // the arena's capacity, so the host learns the size it needs)
  unsigned long long digest_sum, digest_xor;
  unsigned long long candidates, chunks;
  unsigned long long per_depth[64];
  unsigned error;                 // bit 0 out queue full, bit 1 heap full, bit 2 timeout,
                                  // bit 3 a frame of an uninstantiated width
  unsigned pad_[3];
  unsigned long long t_drain;     // (trace) wall clock when the last queued task was dequeued
};
struct DeepArgs {
  const DeepFrame* in;
  long long n_in;
  DeepFrame* out;
  long long out_cap;
  char* heap;
  unsigned long long heap_cap;
  char* stacks;                   // per wave: stack_bytes of blocks
  unsigned long long stack_bytes;
  char* stacks0;                  // per wave: the first seg0 bytes of its stack, densely packed
  unsigned long long seg0;        // (0: none; see deep.hip WaveStack)
  DeepFrame* fstacks;             // per wave: fcap frames
  int fcap;
  DeepCtl* ctl;
  int W;
  unsigned minsup;
  unsigned long long budget;      // 64-lane passes per task before it spills
  int max_len;                    // 0 = all sizes
  unsigned split_min;             // spilled frames above this many members split per member
  unsigned long long timeout_ticks;  // wall_clock64 ticks a wave may run (then error bit 2)
  // steal mode (one launch, no rounds): out == in, spilled tasks are appended at in[n_in + k]
  // and published by ready[k] = epoch; waves that run out of tasks wait for them, and a busy
  // wave spills its frames when it sees a waiting wave (checked every `budget` passes)
  unsigned* ready;
  unsigned long long* req;        // [nwaves] mailboxes: epoch << 32 | requester + 1
  DeepFrame* inbox;               // [nwaves] direct hand-offs (one frame per wave)
  unsigned* inbox_state;          // [nwaves] epoch << 2 | closed 0 / open 1 / filling 2 / full 3
  long long nwaves;
  unsigned epoch;                 // < 2^30
  int steal;
  unsigned split_firsts;          // a hand-off splits a class of >= this many first members
  unsigned split_keep16;          // ... keeping split_keep16 / 16 of them (0: never split)
  unsigned ask_mask;              // a waiting wave asks a victim every (ask_mask + 1) polls
  unsigned ask_fanout;            // ... and that many victims at once (>= 1)
  unsigned sleep_n;               // poll backoff: s_sleep 2 / 16 / 127 from poll 0 / 4 / 16 on,
                                  // the poll count capped at sleep_n
  int steal_eager;                // tests: 1 = bottom frame to the queue at every check,
                                  // 2 = hand-off to the partner wave (gw ^ 1) whenever it waits
  // optional instrumentation (nullptr = off): per wave [kDeepTraceWords] words (launch start,
  // first task start, last task end, exit, busy ticks, tasks << 32 | inbox receipts) and per
  // initial task the ticks its dequeuing wave spent on it (parts handed away excluded)
  unsigned long long* trace;
  unsigned long long* task_ticks;
  unsigned long long trace_bucket;  // ticks per busy-time bucket of the trace record
  // emit mode (node_parent != nullptr): every frequent itemset of size >= 3 found in the launch
  // becomes a trie node (parent node id, last item's frequency rank, support, size) at an id from
  // a per-wave chunk of ctl->node_top; unused ids keep size 0.  Blocks then carry one more row
  // per slot: (rank << 40) | node id of the member itemset.
  unsigned* node_parent;
  unsigned* node_item;
  unsigned* node_count;
  unsigned char* node_depth;
  unsigned long long node_cap;
  // pre-split launch (non-stealing, budget 1; nullptr otherwise): queued task q spills its one
  // child class at heap byte offset split_heap[q] as tasks out[split_q[q] ...] (host layout)
  const long long* split_q;
  const unsigned long long* split_heap;
};
// trace record per wave: [0] launch start, [1] first task start, [2] last task end, [3] exit,
// [4] busy ticks, [5] tasks << 32 | inbox receipts, [6 ..) busy ticks per time bucket of
// DeepArgs::trace_bucket ticks from the wave's launch start (the last bucket takes the rest)
constexpr int kDeepTraceBuckets = 58;
constexpr int kDeepTraceWords = 6 + kDeepTraceBuckets;
constexpr unsigned long long kDeepNodeMask = (1ull << 40) - 1;  // node id bits of a node word
int deep_max_words();
int deep_tier(int words);     // smallest instantiated block width >= words
int deep_row_words(int W);    // root block width for W-word rows (a tier)
int deep_count_maxt(int widest);    // count kernel instance covering block widths <= widest
int deep_waves_per_simd(int maxt);  // its default occupancy (and blocks per CU)
int deep_count_wps(int maxt, int want, bool emit = false);  // instance occupancy: `want` if instantiated
int deep_waves_per_block();
int deep_min_fcap();
int deep_node_chunk();  // emit mode: node ids a wave takes at a time
size_t deep_row_block_bytes(int W, int64_t m, int extra = 0);  // stack room of a step over m members
                                                               // (extra: emit mode's node row)
void deep_transpose(const uint64_t* bm, int64_t Wp, int64_t F, int W, int W_real,
                    const int32_t* ids, uint64_t* root, int64_t Fpad, hipStream_t s);
// level-2 classes; emit (nodes != nullptr, fill pass): blocks carry the node-word row, and the
// level-2 nodes are written at ids F + node_off[i] + slot
struct DeepNodes {
  unsigned* parent;
  unsigned* item;
  unsigned* count;
  unsigned char* depth;
  const int64_t* node_off;  // [F] level-2 node base of root class i
};
// (chunked: one wave per (class, 256 candidates); part = [F][deep_root_chunks(F)] int32)
// count pass (fill = false): part = per-chunk survivors; deep_root_scan turns them into chunk
// bases and lays the classes out on the device: m[i], off[0..F] (block byte offsets, off[0] =
// root_blk), task_off[0..F], node_off[0..F] (prefix sums, no host round trip); the fill pass
// then writes every block at off[i] (m = the scanned sizes)
int deep_root_chunks(int64_t F);
// gram (optional): the level-2 pair gram (kern::pair_gram_popcount of the root bitmaps, F x F
// upper triangle): the count pass reads it instead of ANDing every candidate pair, and the fill
// pass ANDs only the 64-candidate groups holding a survivor
void deep_root(const uint64_t* root, int64_t Fpad, int64_t F, int W, uint32_t minsup,
               const int32_t* m, int32_t* part, const int64_t* blk_off, char* base, DeepCtl* ctl,
               bool fill, hipStream_t s, const DeepNodes* nodes = nullptr,
               const uint32_t* gram = nullptr);
void deep_root_scan(int32_t* part, int64_t F, const int32_t* wt, int extra, int64_t root_blk,
                    int32_t* m, int64_t* off, int64_t* task_off, int64_t* node_off, hipStream_t s);
// emit-mode verification: digest terms and per-size counts of the node arena (ids [0, n)) for
// sizes >= min_depth, set hashes built size by size (hash = parent's + item_mix(ids[item]));
// out = [sum, xor, per_depth[64]] accumulated; hash = scratch [n] u64
void deep_arena_digest(const unsigned* parent, const unsigned* item, const unsigned* count,
                       const unsigned char* depth, int64_t n, const int32_t* ids, int max_depth,
                       int min_depth, uint64_t* hash, unsigned long long* out, hipStream_t s);
// this rank's level-3 task frames: out[q] = task order[q] (order == nullptr: task q*world+rank),
// q < n; task t = (root i, member k) with t = task_off[i] + k
void deep_root_tasks(const int64_t* blk_off, const int32_t* m, const int64_t* task_off, int64_t F,
                     char* base, const uint64_t* root, int64_t Fpad, int W, int rank, int world,
                     const int64_t* order, int64_t n, DeepFrame* out, hipStream_t s, int extra = 0);
// level-3 survivors of every task (the size of the class the task expands): cost[t]; with key
// != nullptr also the deal's sort key: key_mode 0 the class size, 1 its support mass
// (sum of survivor supports - minsup + 1), 2 its square
void deep_task_cost(const int64_t* blk_off, const int32_t* m, const int64_t* task_off, int64_t F,
                    const char* base, uint32_t minsup, uint32_t* cost, hipStream_t s, int extra = 0,
                    uint32_t* key = nullptr, int key_mode = 0);
void deep_count(const DeepArgs& a, int maxt, int wps, int grid, hipStream_t s);
// (deep_order.hip) tasks by cost, largest first and stable in t, dealt over `world` ranks in
// snake order: order[j] / order_cost[j] = this rank's j-th task and its cost, j < the returned
// count (= deep_task_share); tmp = deep_task_order_bytes(T) bytes of device scratch
int64_t deep_task_share(int64_t T, int rank, int world);
size_t deep_task_order_bytes(int64_t T);
// key (optional): sort by key[t] (32 bits) instead of cost[t]; order_cost still = cost
int64_t deep_task_order(const uint32_t* cost, int64_t T, int rank, int world, void* tmp,
                        size_t tmp_bytes, int64_t* order, uint32_t* order_cost, hipStream_t s,
                        const uint32_t* key = nullptr);
// (deep_trie.hip) emit arena -> dense trie, parents first: new_id[i] for every arena id of size
// in [min_depth, nd) (size-major, arena order inside a size; others kNone), returns the node
// count (synchronises); then the scatter writes the trie at new_id (parent remapped, + base for
// exported parents, arena id kept for parents below min_depth; item rank -> ids[rank])
size_t deep_trie_scratch_bytes(int64_t n, int nd);
int64_t deep_trie_layout(const unsigned char* depth, int64_t n, int min_depth, int nd,
                         uint32_t* new_id, void* tmp, size_t tmp_bytes, hipStream_t s);
void deep_trie_scatter(const unsigned* parent, const unsigned* item, const unsigned* count,
                       const unsigned char* depth, int64_t n, const uint32_t* new_id,
                       const int32_t* ids, int64_t base, int32_t* o_parent, void* o_item,
                       bool item16, uint16_t* o_count, unsigned char* o_depth, hipStream_t s);

// ---- mining (mine.hip) ----
void item_support(const int32_t* items, int64_t nnz, int32_t n_items, uint32_t* counts,
                  hipStream_t s);
// partitioned histogram for large vocabularies (16384 < n_items <= 2M): no per-item global
// atomics; needs support_scratch_bytes() of device scratch (0 → not applicable).  Returns false
// (nothing launched) when it does not apply.
size_t support_scratch_bytes(int64_t nnz, int64_t n_items);
bool item_support_partitioned(const int32_t* items, int64_t nnz, int32_t n_items, uint32_t* counts,
                              void* scratch, size_t scratch_bytes, hipStream_t s);
void encode_bitmap(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx,
                   const int32_t* rank_of, uint64_t* bm, int64_t Wp, int64_t word_off,
                   hipStream_t s, const uint32_t* fmask = nullptr);
// fmask (optional): bit i set iff item i is frequent; tested before the rank_of gather, so the
// (mostly infrequent) items of a million-item vocabulary read a 128 KB L2-resident mask instead
// of a 4 MB table.
// LDS-slab encode for long shards (F <= kEncodeTileMaxF frequent rows, in row bands): writes EVERY word of
// the word columns it covers (zeros included); false (nothing launched) if not applicable
constexpr int64_t kEncodeTileMaxF = 1 << 20;  // row bands past one LDS slab
bool encode_bitmap_tiled(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx,
                         const int32_t* rank_of, uint64_t* bm, int64_t Wp, int64_t word_off,
                         int64_t F, hipStream_t s, const uint32_t* fmask = nullptr,
                         const unsigned long long* fgroup = nullptr, const int32_t* c2r = nullptr);
// fgroup/c2r (frequent_groups; used when F <= kEncodeGroupMaxF): one 8-byte gather per item
// instead of the mask gather followed by the rank gather
constexpr int64_t kEncodeGroupMaxF = 2048;
size_t frequent_groups_temp_bytes(int64_t n_items);
void frequent_groups(const uint32_t* fmask, int64_t n_items, const int32_t* rank_of,
                     unsigned long long* fgroup, int32_t* c2r, void* tmp, size_t tmp_bytes,
                     hipStream_t s);
// frequent items (count >= c1) ranked by (count asc, id asc) on the device: ids / fcounts [F],
// rank_of [n_items] (-1 = infrequent), fmask (optional bit mask), *dF = F
size_t select_large_temp_bytes(int64_t n_items);
void select_large(const uint32_t* cnt, int64_t n_items, uint32_t c1, void* tmp, size_t tmp_bytes,
                  int32_t* ids, uint32_t* fcounts, int32_t* rank_of, uint32_t* fmask,
                  unsigned long long* dF, hipStream_t s);
// dst[i] += src[i]
void add_u32(uint32_t* dst, const uint32_t* src, int64_t n, hipStream_t s);
// exclusive prefix sum over int64[n+1] (in[n] == 0) into out[n+1] (out[n] = total)
size_t scan_temp_bytes(int64_t n);
void exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, void* temp, size_t temp_bytes,
                        hipStream_t s);
// flags (count >= minsup) exclusive scan over n+1 flags → pos[n+1] (pos[n] = survivors)
size_t flag_scan_temp_bytes(int64_t n);
void flag_scan(const uint32_t* cnt, uint32_t minsup, int64_t n, int64_t* pos, void* temp,
               size_t temp_bytes, hipStream_t s);
// candidate support counting, candidates [c0, c1) of a level (cand_off has n_rows+1 entries,
// absolute); writes cnt[c - c0]
void extend_count(const uint64_t* bm, int64_t Wp, const int64_t* cand_off, int64_t n_rows,
                  int64_t c0, int64_t c1, uint32_t* cnt, hipStream_t s);
// extend_count launches so far that split long rows into slices (atomic partial counts)
long long extend_split_launches();
// out2[0] = survivors of chunk, out2[1] = next level's candidate total (one readback)
void child_totals(const int64_t* cand_off, int64_t a0, int64_t a1, int64_t c0, const int64_t* pos,
                  int64_t nc, uint64_t* out2, hipStream_t s);
// materialise the survivors of candidates [c0, c1)
struct LevelOut {
  uint64_t* bm;        // child bitmaps [S][Wp]
  int32_t* rank;       // child last-item Eclat rank
  int64_t* gid;        // child global node id
  int32_t* row_end;    // child class end (child-local index)
  int64_t* len;        // child candidate-row lengths (row_end - s - 1), S+1 entries
  int64_t* out_parent; // global trie arrays (indexed by out_base + s)
  int32_t* out_item;
  uint32_t* out_count;
  uint8_t* out_depth;
  int64_t out_base;
  uint8_t depth;
};
void extend_materialize(const uint64_t* bm, int64_t Wp, const int64_t* cand_off, int64_t n_rows,
                        const int32_t* rank, const int64_t* gid, const int32_t* ids,
                        int64_t c0, int64_t c1, const uint32_t* cnt, uint32_t minsup,
                        const int64_t* pos, const LevelOut& o, hipStream_t s,
                        int64_t n_surv = -1, int64_t* surv_scratch = nullptr);
// n_surv (the survivor count, known on the host) + surv_scratch (n_surv int64): long rows are
// copied by a grid over (survivor, slice) pairs sized by n_surv, not over all candidates
// dense upper-triangular pair counts over a single class of F rows (level 2 bit-GEMM)
void pair_gram_popcount(const uint64_t* bm, int64_t Wp, int64_t F, uint32_t* out, hipStream_t s);
void pair_gram_mfma(const uint64_t* bm, int64_t Wp, int64_t F, uint32_t* out, hipStream_t s);
// Horizontal co-occurrence counting (cooc.hip): level-2 supports of sparse data from the
// transaction CSR.  cooc_stats adds sum_t k_t(k_t-1)/2 to out[0] and max k_t into out[1] (k_t =
// frequent items of transaction t; out zeroed by the caller).  cooc_count adds every co-occurring
// frequent pair into gram[lo * ld + hi] (rank order, upper triangle; gram zeroed by the caller);
// needs max k_t <= cooc_max_k() (err |= 1 otherwise).
int cooc_max_k();
// tx-DP gram combine: the frequent upper entries (count >= minsup) of a reduce-scattered row
// block [nrows][ld] of global rows r0..: counted into cnt[0] (emit == nullptr) or written as
// (row, col, count) u32 triples at slots taken from cnt[0]; gram_scatter writes triples back
// into a zeroed dense gram (zero-count padding triples skipped)
void gram_frequent(const uint32_t* rows, int64_t ld, int64_t r0, int64_t nrows, int64_t F,
                   uint32_t minsup, unsigned long long* cnt, uint32_t* emit, hipStream_t s);
void gram_scatter(const uint32_t* triples, int64_t n, uint32_t* gram, int64_t ld, hipStream_t s);
void cooc_stats(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx, const int32_t* rank_of,
                const uint32_t* fmask, unsigned long long* out, int n_cus, hipStream_t s);
void cooc_count(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx, const int32_t* rank_of,
                const uint32_t* fmask, int64_t F, uint32_t* gram, int64_t ld, unsigned* err,
                int n_cus, hipStream_t s);
// ---- level-2 pair counts row by row in LDS (pairrows.hip) ----
// The sparse (horizontal) path keeps item ranks in 16 bits: ranks 0 .. 65534, 0xFFFF = none
// (devbuf::rank16), pair entries packed as (a << 16 | b)
constexpr int64_t kSparseMaxF = 65535;
struct PrInput {
  const int64_t* tx_ptr;  // this rank's CSR (rebased)
  const int32_t* items;
  int64_t n_tx, n_items;
  const int32_t* ids;     // rank -> item
  int64_t F;
  int n_cus;
  const uint32_t* fmask = nullptr;  // frequent-item bit mask (large vocabularies), or null
  double kept_per_tx = 0.0;  // mean frequent items per transaction (sizes the filter's pools)
};
// Item-sharded counting: the ranks' frequent-rank CSRs are all-gathered (every rank then holds
// every transaction's frequent ranks) and this rank counts only the rows a with a % world == rank
// (the other gram rows stay zero), so every owned row is complete without a gram reduction.
struct PrShard {
  int rank, world;
  // all-gather of `words` u32 per rank from send into recv (world * words), on the stream
  std::function<void(const void* send, void* recv, size_t words)> all_gather;
};
class PairRows {  // grow-only device buffers kept across calls
 public:
  PairRows();
  ~PairRows();
  PairRows(const PairRows&) = delete;
  PairRows& operator=(const PairRows&) = delete;
  // gram[a * ld + b] (ranks a < b) = co-occurrences in the shard; the rest of the F x ld block
  // zero.  False (gram zeroed, nothing counted): a transaction holds > 65535 frequent items.
  // `wait` is the host wait for s (bounded under a communicator).
  bool count(const PrInput& in, uint32_t* gram, int64_t ld, hipStream_t s,
             const std::function<void()>& wait, const struct PrShard* shard = nullptr);
  // the frequent-rank CSR of the last count: rows (off, len) of >= 2 ranks, ascending
  const uint2* txrec() const;
  const uint16_t* fit() const;
  int64_t n_rows() const;
  int64_t nnz() const;
  int64_t pairs() const;  // co-occurring pairs counted (sum k(k-1)/2)
  static size_t lds_bytes(int64_t F);

 private:
  struct Impl;
  Impl* p_;
};

// ---- horizontal levels >= 3 from a filtered CSR (hlevels.hip) ----
struct HlTrieOut {  // device trie arrays (whole arrays; new nodes go to [base, base + n))
  int64_t* parent;
  int32_t* item;
  uint32_t* count;
  uint8_t* depth;
  int64_t base;
  const int32_t* ids;  // rank -> item id (set by HLevels)
};
struct HlInput {
  const int64_t* tx_ptr;   // this rank's CSR (rebased)
  const int32_t* items;
  int64_t n_tx, n_items;
  const int32_t* rank_of;  // item -> frequent rank (-1 otherwise)
  const uint32_t* fmask;   // optional frequent-item bit mask
  const int32_t* ids;      // rank -> item
  const uint32_t* gram;    // level-2 counts, upper triangle, global (all-reduced) counts
  int64_t ld, F;
  uint32_t minsup;
  int max_len;             // 0 = no cap
  int n_cus;
  // optional: the frequent-rank CSR of this shard (PairRows) — re-filtered instead of the items
  const uint2* f_txrec = nullptr;
  const uint16_t* f_fit = nullptr;
  int64_t f_rows = 0;
};
struct HlHooks {
  std::function<HlTrieOut(int64_t n)> reserve;   // room for n more trie nodes (base = first id)
  std::function<void(int64_t n)> commit;         // n nodes written after the last reserve
  std::function<void(uint32_t* cnt, int64_t n)> allreduce;  // tx-DP candidate counts (or empty)
  std::function<void()> wait;                    // host wait for the stream (bounded with comm)
};
struct HlStats {
  int64_t n_tx_kept = 0, nnz_kept = 0, candidates = 0;
  int max_depth = 1;
  std::vector<int64_t> per_level;  // itemsets of size 2, 3, ...
  std::vector<int64_t> hits;       // containing (transaction, itemset) pairs of size 2, 3, ...
};
class HLevels {  // grow-only device buffers kept across calls
 public:
  HLevels();
  ~HLevels();
  HLevels(const HLevels&) = delete;
  HLevels& operator=(const HLevels&) = delete;
  bool run(const HlInput& in, const HlHooks& hooks, hipStream_t s, HlStats& st);

 private:
  struct Impl;
  Impl* p_;
};

// same with F read from the device (grid and row stride sized for F_max)
void pair_gram_popcount_dev(const uint64_t* bm, int64_t Wp, const int64_t* dF, int64_t F_max,
                            uint32_t* out, hipStream_t s);
// false when every i<j<F entry is written directly (no split-K atomics): no zero-fill needed
bool pair_gram_dev_needs_zero(int64_t Wp, int64_t F_max);
// C[i][j] += popcount(A_i & B_j) (rectangular, accumulating; C zeroed by the caller once)
void bitgemm_rect(const uint64_t* A, int64_t Fa, const uint64_t* B, int64_t Fb, int64_t Wp,
                  uint32_t* C, int64_t ldc, hipStream_t s);
// dense Gram (F x F, i<j valid) → per-candidate counts in (a, b) row-major candidate order
void gram_to_cand(const uint32_t* gram, int64_t F, const int64_t* cand_off, int64_t c0, int64_t c1,
                  uint32_t* cnt, hipStream_t s);

// ---- fused host-sync-free levels (levels.hip) ----
struct FLevel {  // device-resident descriptor of one level (rows = itemsets of one size)
  int64_t n_rows;
  const uint64_t* bm;      // [n_rows][Wp]
  const int32_t* rank;     // last item's Eclat rank
  const int64_t* gid;      // trie node id
  const int32_t* prow;     // row in the parent level
  int64_t* cand_off;       // [n_rows + 1] owner-major: row b's candidates pair it with its
                           // earlier siblings (written by the previous level's count)
  int64_t n_cand;
  int64_t* row_end;        // unused (round-1 scan layout)
  int64_t child_base;      // trie id of this level's first child
  unsigned int scan_ticket, count_ticket;
  // row → bitmap row (nullptr: identity).  The short-row count kernel writes each candidate's
  // AND row in place at its candidate index (no compaction pass), so a level's rows point into
  // the candidate-indexed bitmap array of the parent's expansion.
  const int32_t* slot;
  char pad[32];
};
// Pinned host trie written directly by the level kernels (streamed download).  Element widths
// are chosen per call so that only the bytes the data needs cross PCIe: parent 4 B while node
// ids < 2^31, item 2 B while item ids < 2^16, count 2 B while T < 2^16 (the reference's playlist
// datasets: 9 B/itemset instead of 17 B).  A node >= cap sets FCtl::dl_overflow and the host
// falls back to one full-width copy at the end.
struct HostTrie {
  void* parent;
  void* item;
  void* count;
  uint8_t* depth;
  int64_t cap;
  int par_w, item_w, cnt_w;  // bytes: 4|8, 2|4, 2|4
};
// Pinned destinations of the rule-map CSR (pairs.hip; meta == nullptr: no copy-out).
struct PairsHost {   // pinned destinations of the finished CSR (meta == nullptr: no copy-out)
  int64_t* row_ptr;  // [n_items + 1]
  int32_t* cons;     // [cap]
  uint32_t* cnt;     // [cap]
  int64_t cap;
  int64_t* meta;     // [0] = nnz, [1] = status (1 entry overflow, 2 row > sort max, 4 host cap)
};
// Control block of one fused mining call.  Everything that changes from call to call (epoch
// base, pinned host destinations) lives here rather than in kernel arguments, so the launch
// sequence of a call is invariant and can be captured once as a hipGraph and replayed.
struct FCtl {
  char* bump_base;
  unsigned long long bump_cap, bump_top;
  unsigned long long status_cap;   // look-back tiles available
  unsigned long long candidates;   // Σ n_cand over the counted levels
  unsigned int overflow;           // 1 bump, 2 spin, 3/4 capacity → host falls back
  unsigned int dl_overflow;        // pinned host arrays too small → host copies at the end
  unsigned int epoch_base;         // look-back tag of launch i = epoch_base + i (12 bits)
  unsigned int need_out_m;         // overflow 4 on the trie capacity: nodes needed, MiB units
  HostTrie h;                      // streamed download destination (pinned)
  int32_t* host_tab;               // frequent-item tables ids | counts | rank_of (pinned)
  int64_t tab_stride;
  void* rb_dst;                    // descriptor + control-block readback (pinned)
  char pad1[8];
  PairsHost ph;                    // rule-map CSR download destination (pinned)
  char pad2[8];
};
static_assert(sizeof(FCtl) % 16 == 0, "FCtl is read back in 16-byte words");
struct LevelCountArgs {
  int64_t Wp;
  uint32_t minsup;
  const uint32_t* gram;    // root level: dense F x F pair counts (else nullptr)
  int64_t F;
  const int32_t* ids;      // Eclat rank → original item id
  int64_t* out_parent;
  int32_t* out_item;
  uint32_t* out_count;
  uint8_t* out_depth;
  uint8_t child_depth;
  bool download;  // stream the trie to FCtl::h
  unsigned long long* trace;  // per-tile phase timestamps [tile][8] (nullptr: off; diagnostics)
  // deferred download: the launch carries kCopyBlocks extra blocks that copy the PREVIOUS
  // level's nodes (this level's rows, finished by the previous launch) from the device trie to
  // the host trie while the tile blocks run; false = survivors written to the host inline
  bool deferred_dl;
  int copy_blocks;  // copy blocks of the grid when deferred_dl (default kCopyBlocks)
  bool copy_last;   // copy blocks at the end of the grid instead of leading it (A/B)
  bool root;        // level 1: rows = frequent items in descending rank, bitmap rows by rank
  int64_t out_cap;  // device trie capacity (nodes)
  bool leaf;        // last level allowed by max_len: survivors only, no next-level layout
};
// Few copy blocks on purpose: GPU writes to pinned host memory share the L2 -> fabric write path
// with the tiles' HBM stores, and a saturated PCIe link backs that path up (a level-6 trace showed
// tile phase 1 at 42 µs with 64 copy blocks vs 19 µs without concurrent copies).  Headline A/B,
// ms/step by copy blocks per launch: 4: 0.78, 8: 0.68, 12: 0.66, 16: 0.65-0.66, 24: 0.69, 32: 0.70,
// 64: 0.71, 128: 0.71.
constexpr int kCopyBlocks = 16;
// device-resident prologue (single GPU, small vocabularies): selection + root descriptor
// without a host round trip.  select: items with cnt >= c1, ranked by (count asc, id asc)
// (= select_frequent), F → desc[1].n_rows.  root_setup: level-1 trie nodes, root cand_off
// (closed form), iota rank/gid, root children buffers from the bump region.
constexpr int64_t kSelectMaxItems = 16384;
// one launch for the per-call device state of the resident path: zero the support histogram
// and the bitmap buffer, zero the level descriptors and copy the control block from `params`
// (pinned host memory the host fills before the call; read at execution time, so a captured
// graph picks up each call's values).  `params` holds two slots: the kernel reads slot
// (*seq & 1) and increments the device call counter *seq.
void level_prologue_init(uint32_t* cnt, int64_t n_items, uint64_t* bm, int64_t bm_words,
                         FLevel* desc, int n_desc, FCtl* ctl, const FCtl* params,
                         unsigned int* seq, hipStream_t s);
// selection in one launch for small vocabularies (n_items <= kSelectFusedMax): every thread
// ranks its item against all others (no rank accumulator, no memset) and also writes rank_of
// (the third of the frequent-item tables ids | counts | rank_of) straight to FCtl::host_tab
// (nullptr: skip); the root setup writes the other two.
// Falls back to level_select above that size.
constexpr int64_t kSelectFusedMax = 4096;
void level_select_fused(const uint32_t* cnt, int64_t n_items, uint32_t c1, int32_t* ids,
                        uint32_t* fcounts, int32_t* rank_of, FLevel* desc, const FCtl* ctl,
                        hipStream_t s);
void level_select(const uint32_t* cnt, int64_t n_items, uint32_t c1, int32_t* ids,
                  uint32_t* fcounts, int32_t* rank_of, int32_t* rank_acc, FLevel* desc,
                  hipStream_t s);
struct RootSetupArgs {
  const uint64_t* bm;
  int32_t* rank;       // [n_items]
  int64_t* gid;        // [n_items]
  int64_t* cand_off;   // [n_items + 1]
  const int32_t* ids;
  const uint32_t* fcounts;
  int64_t* out_parent;
  int32_t* out_item;
  uint32_t* out_count;
  uint8_t* out_depth;
  int64_t Wp;
  int64_t out_cap;
  const int32_t* prank;  // partition rank of each root class (world > 1), see level_partition
  int world;
  int my_rank;
  bool download;   // level-1 nodes also go straight to FCtl::h (inline download mode)
  bool host_tab;   // frequent-item ids | counts to FCtl::host_tab
  // gram-driven root (level_root_rows → setup → level_root_fill, instead of counting level 1
  // with the look-back kernel): m = frequent pairs per root row; soff/coff [F+1] = the rows'
  // survivor and next-level candidate offsets, filled here.  m == nullptr: counted root.
  const int32_t* m;
  int64_t* soff;
  int64_t* coff;
  bool leaf;       // max_len == 2: level 2 is the last level
  bool interleaved;  // level_rows_interleaved(Wp): the count kernel family of the levels below
  bool dl_level1;    // download requested: with no root count kernel (whose copy blocks carry
                     // level 1 in deferred mode) the setup writes the level-1 nodes itself
};
// true when the levels run the short-row count kernel (64-interleaved candidate-slot rows)
bool level_rows_interleaved(int64_t Wp);
void level_root_setup(FLevel* desc, FCtl* ctl, const RootSetupArgs& a, hipStream_t s);
// frequent pairs per root row (row r = rank F-1-r; rows a rank does not own count 0)
void level_root_rows(const uint32_t* gram, int64_t ld, const FLevel* desc, uint32_t minsup,
                     const int32_t* prank, int world, int my_rank, int64_t F_max, int32_t* m,
                     hipStream_t s);
// level 2 from the gram: one block per root row writes its frequent pairs as level-2 rows
// (trie nodes, AND bitmaps at their own slots, candidate offsets and tile→row entries of level 2)
void level_root_fill(FLevel* desc, FCtl* ctl, const uint32_t* gram, int64_t ld, uint32_t minsup,
                     const RootSetupArgs& a, int32_t* tile_row_nx, int64_t F_max, hipStream_t s);
// rank root classes by estimated cost (n_a^2 + 1 from the gram, desc) for the snake partition;
// with prank == nullptr only the costs are computed (the root setup ranks them)
void level_partition(const uint32_t* gram, int64_t ld, FLevel* desc, uint32_t minsup,
                     int64_t F_max, int64_t* cost, int32_t* prank, hipStream_t s);
int level_grid(int n_cus);
int64_t level_tile();
// trie nodes [lv->child_base, +nx->n_rows) (the last launched level's children) from the device
// trie arrays into FCtl::h (download), plus a readback of rb_bytes (multiple of 16; 0 = none)
// from rb_src to FCtl::rb_dst
void level_copyout(const FLevel* lv, const FLevel* nx, FCtl* ctl, const int64_t* d_parent,
                   const int32_t* d_item, const uint32_t* d_count, const uint8_t* d_depth,
                   bool download, const void* rb_src, size_t rb_bytes, hipStream_t s);
// cand_hint: expected candidate count of the level (the previous call's; -1 unknown) — picks
// the register/latency trade-off of the short-row kernel, never affects results
// count level L (lv = &desc[L], nx = &desc[L+1]; desc[L+2] receives the next buffers).
// tile_row: count tile → first row of level L, written by count(L-1) (nullptr at the root);
// tile_row_nx: the same map for level L+1, written here (double-buffered by the caller).
// status: 2 words per tile.
void level_count(FLevel* lv, FLevel* nx, FCtl* ctl, unsigned long long* status, unsigned epoch,
                 const LevelCountArgs& a, const int32_t* tile_row, int32_t* tile_row_nx, int grid,
                 int64_t cand_hint, hipStream_t s);

// ---- rule map = pair-support CSR (pairs.hip, O10 pairs_to_csr) ----
// Longest row the device sorts (rows are <= F-1 long; longer rows set status bit 2 and the
// host sorts that index instead).
constexpr int64_t kPairsSortMax = 16384;
struct PairsArgs {
  const uint32_t* gram;  // upper triangle (i < j < F valid), row stride ld, Eclat rank order
  int64_t ld;
  const int64_t* dF;     // F on the device (nullptr: F_host)
  int64_t F_host;
  int64_t F_max;         // grid sizing bound on F
  uint32_t minsup;
  const int32_t* ids;      // rank -> item id
  const int32_t* rank_of;  // item id -> rank or -1
  int64_t n_items;
  const int32_t* tie;      // item id -> tie rank (nullptr: the id)
  const int32_t* inv_tie;  // tie rank -> item id (nullptr: identity)
  void* scratch;            // pairs_scratch_bytes(F_max, n_items)
  size_t scratch_bytes;
  unsigned long long* ent;  // [ent_cap] unsorted keys
  int64_t ent_cap;
  // output (device)
  int64_t* row_ptr;        // [n_items + 1], by item id
  int32_t* cons;           // [ent_cap]
  uint32_t* cnt;           // [ent_cap]
  const PairsHost* host;   // device-visible (e.g. &FCtl::ph of the call); nullptr: no copy-out
};
size_t pairs_scratch_bytes(int64_t F_max, int64_t n_items);
void pairs_to_csr(const PairsArgs& a, hipStream_t s);
void pairs_enable_big_lds();  // once per process/device before the first pairs_to_csr
// Multi-GPU rule map: the gram's lower triangle from its upper one (full symmetric rows), then
// the CSR of a row block [r0, r0 + nrows) x F of it (rows by frequent rank, cons = item ids).
void gram_mirror(uint32_t* gram, int64_t ld, int64_t F, hipStream_t s);
// Item-sharded mining (kernels/shard.hip): OR of rows idx[0..n) -> mask[W]; per-word popcount;
// rows [R][Wp_in] compressed onto mask (nzw: the mask's nonzero words, off: their exclusive bit
// offsets) into a ZEROED out [R][Wp_out].
void rows_union(const uint64_t* rows, int64_t Wp, const int32_t* idx, int n, int64_t W,
                uint64_t* mask, hipStream_t s);
void word_popc(const uint64_t* mask, int64_t W, int32_t* cnt, hipStream_t s);
void compact_rows(const uint64_t* rows, int64_t R, int64_t Wp_in, const uint64_t* mask,
                  const int64_t* nzw, const int64_t* off, int64_t n_nz, uint64_t* out,
                  int64_t Wp_out, hipStream_t s);
void rows_count(const uint32_t* rows, int64_t ld, int64_t nrows, int64_t F, int64_t r0,
                uint32_t minsup, uint32_t* len_r, unsigned int* n_long, int32_t* long_rows,
                hipStream_t s);
void rows_fill_sort(const uint32_t* rows, int64_t ld, int64_t nrows, int64_t F, int64_t r0,
                    uint32_t minsup, const int32_t* ids, const int32_t* tie, const int32_t* inv_tie,
                    const uint32_t* len_r, const int64_t* row_ptr, unsigned long long* ent,
                    int64_t ent_cap, int32_t* cons, uint32_t* cnt, unsigned int* status,
                    const unsigned int* n_long, const int32_t* long_rows, bool any_long,
                    hipStream_t s);

// ---- association rules (rules.hip) ----
struct RuleArgs {
  const int64_t* parent;
  const int32_t* item;
  const uint32_t* count;
  const uint8_t* depth;
  int64_t n;
  double T;
  int metric;              // RuleMetric
  double thr;
  int max_ante;
  const unsigned long long* keys;  // (parent+1, item) → node hash
  const int32_t* vals;
  unsigned long long mask;
  int32_t* scratch;        // per-wave global subset tables (k in (12, scratch_bits]) or null
  int scratch_bits;
  unsigned long long* ticket;
  unsigned int* error;     // 1 = subset missing from the trie, 2 = itemset longer than 30
  int pass;                // 0 = count, 1 = write
  int64_t* nrules;         // pass 0: [n+1]
  const int64_t* off;      // pass 1: exclusive scan of nrules
  int64_t* o_itemset;
  int64_t* o_ante;
  int64_t* o_cons;
  double* o_conf;
  double* o_lift;
};
void rules_hash_build(const int64_t* parent, const int32_t* item, int64_t n,
                      unsigned long long* keys, int32_t* vals, unsigned long long mask,
                      hipStream_t s);
int rules_grid(int n_cus);
int rules_waves_per_block();
void rules_pass(const RuleArgs& a, int grid, hipStream_t s);
size_t rules_scan_temp_bytes(int64_t n);
void rules_scan(const int64_t* in, int64_t* out, int64_t n, void* tmp, size_t tb, hipStream_t s);

// ---- transaction builder (groupby.hip) ----
// CSR of vals grouped by keys in [0, n_keys): rows sorted (and duplicate-free when dedup).
// Returns nnz (synchronises the stream).
size_t groupby_csr_temp_bytes(int64_t n, int32_t n_keys);
int64_t groupby_csr(const int32_t* d_keys, const int32_t* d_vals, int64_t n, int32_t n_keys,
                    bool dedup, int64_t* d_ptr, int32_t* d_idx, void* d_tmp, size_t tmp_bytes,
                    hipStream_t s);

// ---- serving (serve.hip) ----
void serve_match_topk(const int64_t* row_ptr, const int32_t* cons, const uint32_t* srank,
                      const uint8_t* is_key, int64_t n_items, const int64_t* q_ptr,
                      const int32_t* seeds, int64_t B, int k, int32_t* out, hipStream_t s,
                      bool narrow = false);
// long-row queries (qlist: indices into the batch, each with <= 256 seeds): one workgroup
// each, threshold-pruned exact merge; id_cons/id_pos = each row's consequents sorted by id and
// their index in the score-ordered row
void serve_topk_big(const int64_t* row_ptr, const int32_t* cons, const uint32_t* srank,
                    const uint8_t* is_key, int64_t n_items, const int32_t* id_cons,
                    const int32_t* id_pos, const int64_t* q_ptr, const int32_t* seeds,
                    const int32_t* qlist, int64_t nq, int k, int32_t* out, hipStream_t s);
constexpr int kServeWaveMerge = 512;  // merged entries the wave kernel takes (its table / 2)
constexpr int kServeLoopStage = 2048;  // int32 words of one loop request staged in LDS
constexpr int kServeLoopOut = 1536;    // int32 words of one loop request's results in LDS
// persistent serving loop (serve.hip k_serve_loop, gpu::GpuServeLoop): mapped coherent host
// memory, every word the two sides poll on a 64-byte line of its own
struct ServeReq {
  const int64_t* row_ptr;
  const int32_t* cons;
  const uint32_t* srank;
  const uint8_t* is_key;
  long long n_items;
  const long long* q_ptr;   // [B + 1] (device view of mapped host memory)
  const int32_t* seeds;
  int32_t* out;             // [B][k + 1]
  long long B;
  long long k;
  long long n_seeds;        // seeds follow q_ptr in the payload: [q_ptr | seeds] contiguous
  long long narrow;         // 1: score ranks < 2^23, 32-bit order keys in the top-k
};
// One request slot of the serving loop: polled by ITS workgroup of the kernel, owned by one host
// thread at a time (a front I/O thread calls the loop directly, no hop to a GPU thread).
struct ServeSlot {
  unsigned long long req;  // host -> device: (inline words << 32) | seq, written after the
                           // descriptor and the inline payload
  unsigned pad0[14];
  unsigned done_seq;    // device -> host, written after the results (the host writes it too,
                        // only while no kernel runs: a request given up is marked consumed)
  unsigned pad1[15];
  unsigned exited_gen;  // device -> host: the launch generation whose workgroup left this slot
  unsigned pad2[15];
  // device wall clock (instrumentation): request seen, descriptor + payload staged, answers in
  // LDS, done word written
  unsigned long long t_seen, t_staged, t_computed, t_done;
  unsigned long long t_phase[6];  // the first query's matcher phases (wall clock)
  unsigned pad3[12];
  // [descriptor | q_ptr (B + 1 int64) | seeds]: read by the kernel in ONE round of parallel
  // system-scope loads (the inline word count travels in `req`)
  ServeReq req_desc;
  int32_t payload[kServeLoopStage];
};
constexpr int kServeLoopSlots = 8;  // request slots = polling workgroups of one launch
struct ServeMail {
  unsigned stop;  // host -> device: every workgroup exits
  unsigned pad0[31];
  ServeSlot slot[kServeLoopSlots];
};
// device-memory coordination of one launch's workgroups (agent-scope atomics): the newest
// request's clock (idle exit is decided once, by workgroup 0, for all) and the quit word
struct ServeLoopCtl {
  unsigned long long last_activity;
  unsigned quit;  // == the launch's generation: every workgroup of that launch leaves
  unsigned pad;
};
void serve_loop_launch(ServeMail* mail, ServeLoopCtl* ctl, unsigned gen, int nslots,
                       unsigned long long idle_ticks, unsigned long long life_ticks,
                       hipStream_t s);
constexpr int kServeMaxSeeds = 256;

}  // namespace kern
}  // namespace kmls
