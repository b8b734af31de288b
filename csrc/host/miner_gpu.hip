// Host driver of the GPU FP-Growth miner (HIP runtime; kernels in csrc/kernels/mine.hip).
//
// Search order is "DFS over batches": each level of the equivalence-class tree is expanded in
// candidate chunks (BFS-wide inside a chunk, so a launch has millions of teams to fill 256
// CUs), and each chunk's survivors are recursed into before the next chunk, so HBM use is
// bounded by one chunk per depth (LIFO device arena) instead of a whole level.
// Replaces mlxtend's recursive conditional-FP-tree generator (machine-learning/main.py:272,
// SURVEY §3.1 "HOT LOOP 3").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../kernels/kernels.hpp"
#include "kmls/gpu.hpp"
#include "kmls/hooks.hpp"
#include "kmls/trace.hpp"

#define KMLS_HIP(expr)                                                                  \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +      \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__));     \
  } while (0)

namespace kmls {
namespace gpu {

bool available() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return n > 0;
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

std::string device_name(int dev) {
  hipDeviceProp_t p;
  KMLS_HIP(hipGetDeviceProperties(&p, dev));
  return std::string(p.name) + " (" + p.gcnArchName + ")";
}

// ------------------------------------------------------------------------------------------
DeviceArena::DeviceArena(size_t bytes) : cap_(bytes) {
  KMLS_HIP(hipMalloc((void**)&base_, bytes));
}
DeviceArena::~DeviceArena() {
  if (base_) (void)hipFree(base_);
}
void* DeviceArena::push(size_t bytes) {
  size_t off = (top_ + 255) & ~(size_t)255;
  if (off + bytes > cap_)
    throw ArenaExhausted(off + bytes, cap_);
  top_ = off + bytes;
  hw_ = std::max(hw_, top_);
  return base_ + off;
}

PinnedPool::~PinnedPool() {
  for (auto& b : bufs_) (void)hipHostFree(b.p);
  delete (std::mutex*)mu_;
}

std::shared_ptr<PinnedPool> make_pinned_pool() {
  auto p = std::shared_ptr<PinnedPool>(new PinnedPool());
  p->mu_ = new std::mutex();
  return p;
}

std::shared_ptr<void> PinnedPool::get(size_t bytes) {
  bytes = std::max<size_t>(bytes, 64);
  std::lock_guard<std::mutex> lk(*(std::mutex*)mu_);
  int best = -1;
  for (int i = 0; i < (int)bufs_.size(); ++i)
    if (!bufs_[i].busy && bufs_[i].bytes >= bytes && (best < 0 || bufs_[i].bytes < bufs_[best].bytes))
      best = i;
  if (best < 0) {
    void* p = nullptr;
    const size_t cap = bytes + (bytes >> 2);
    KMLS_HIP(hipHostMalloc(&p, cap));
    bufs_.push_back({p, cap, false});
    best = (int)bufs_.size() - 1;
  }
  bufs_[best].busy = true;
  void* ptr = bufs_[best].p;
  auto self = shared_from_this();
  return std::shared_ptr<void>(ptr, [self, ptr](void*) {
    std::lock_guard<std::mutex> lk(*(std::mutex*)self->mu_);
    for (auto& b : self->bufs_)
      if (b.p == ptr) b.busy = false;
  });
}

template <typename T>
struct DevVec {  // growable device array (output trie)
  T* p = nullptr;
  int64_t cap = 0;
  void reserve(int64_t n, hipStream_t s) {
    if (n <= cap) return;
    int64_t nc = std::max<int64_t>(n, cap * 2);
    T* q = nullptr;
    KMLS_HIP(hipMalloc((void**)&q, (size_t)nc * sizeof(T)));
    if (p) {
      KMLS_HIP(hipMemcpyAsync(q, p, (size_t)cap * sizeof(T), hipMemcpyDeviceToDevice, s));
      KMLS_HIP(hipStreamSynchronize(s));
      KMLS_HIP(hipFree(p));
    }
    p = q;
    cap = nc;
  }
  ~DevVec() {
    if (p) (void)hipFree(p);
  }
};

// Output trie (parent, item, count, depth) — owned by the GpuMiner so that steady-state mining
// allocates nothing; plus the side stream that streams finished levels to pinned host memory
// while deeper levels are still being mined.
struct OutBufs {
  DevVec<int64_t> parent;
  DevVec<int32_t> item;
  DevVec<uint32_t> count;
  DevVec<uint8_t> depth;
  hipStream_t copy_s = nullptr;
  hipEvent_t ev = nullptr;
  // fused level path (levels.hip): look-back status words (epoch-tagged, zeroed once)
  unsigned long long* status = nullptr;  // [2 * status_cap]: two words per tile (SegAgg)
  int32_t* tile_row = nullptr;   // [2][status_cap] count tile → first row, by level parity
  unsigned long long* trace = nullptr;  // KMLS_LEVEL_TRACE diagnostics ([status_cap][8])
  // tiles per launch: 2^22 x 256 = 1G candidates (KMLS_TEST_HOOKS status_cap=<tiles> shrinks it)
  int64_t status_cap = std::max<long long>(64, test_hook("status_cap", 1ll << 22));
  // look-back tags: tag = epoch_base (per call, in FCtl) + launch index (kernel argument)
  unsigned epoch_base = 0;
  unsigned launch_idx = 0;
  int depth_hint = 6;            // levels enqueued before the first completion check
  std::vector<int64_t> cand_hint;  // candidates per level in the previous call (kernel choice)
  OutBufs() {
    KMLS_HIP(hipStreamCreateWithFlags(&copy_s, hipStreamNonBlocking));
    // device-scope release: a cross-stream fork needs no system-scope L2 writeback
    KMLS_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToDevice));
    KMLS_HIP(hipMalloc((void**)&status, (size_t)status_cap * 2 * sizeof(unsigned long long)));
    KMLS_HIP(hipMemset(status, 0, (size_t)status_cap * 2 * sizeof(unsigned long long)));
    KMLS_HIP(hipMalloc((void**)&tile_row, (size_t)status_cap * 2 * sizeof(int32_t)));
  }
  static constexpr unsigned kLaunchesPerCall = 64;  // level launches per call (<= 61 levels)
  // start a fused call: a fresh 64-tag window (the 12-bit tag wraps after 63 calls: then the
  // status words are zeroed so no stale word can match)
  unsigned begin_call(hipStream_t s) {
    epoch_base += kLaunchesPerCall;
    if (epoch_base + kLaunchesPerCall >= (1u << 12)) {  // 12-bit tags (levels.hip)
      KMLS_HIP(hipMemsetAsync(status, 0, (size_t)status_cap * 2 * sizeof(unsigned long long), s));
      epoch_base = kLaunchesPerCall;
    }
    launch_idx = 0;
    return epoch_base;
  }
  unsigned next_epoch(hipStream_t) {
    if (++launch_idx >= kLaunchesPerCall) throw std::logic_error("kmls: too many level launches");
    return launch_idx;
  }
  ~OutBufs() {
    if (copy_s) (void)hipStreamSynchronize(copy_s);
    if (status) (void)hipFree(status);
    if (tile_row) (void)hipFree(tile_row);
    if (trace) (void)hipFree(trace);
    if (ev) (void)hipEventDestroy(ev);
    if (copy_s) (void)hipStreamDestroy(copy_s);
  }
};

namespace {

struct Level {
  int64_t n = 0;
  const uint64_t* bm = nullptr;
  const int32_t* rank = nullptr;
  const int64_t* gid = nullptr;
  const int32_t* row_end = nullptr;
};

struct Event {
  hipEvent_t e;
  Event() { KMLS_HIP(hipEventCreate(&e)); }
  ~Event() { (void)hipEventDestroy(e); }
};

constexpr int64_t kCandCap = 32ll << 20;  // candidates per chunk

// Host wait for a stream (a hipStreamQuery busy-poll measured no gain on the headline step).
void sync_stream(hipStream_t s) { KMLS_HIP(hipStreamSynchronize(s)); }

// streamed download of the fused levels: each count launch carries copy blocks that move the
// previous level's nodes to the host while its tiles compute (writing survivors to the host
// from the tile blocks themselves made every launch wait for its own PCIe writes: measured
// slower)
bool deferred_dl() { return true; }
size_t fused_bump_cap(size_t bytes);

// long rows use the MFMA gram (the VALU popcount gram only below its crossover)
bool gram_popcount_forced() { return false; }
// deferred-download copy blocks per count launch, at the start of the grid (placing them at
// the end measured no faster)
bool copy_last() { return false; }
int copy_blocks() { return kern::kCopyBlocks; }

struct MineRun {
  hipEvent_t wait_ev = nullptr;  // set: wait for this event instead of the stream (a call was
                                 // launched ahead behind this one)
  bool no_more_batches = false;  // ... and so no further level batch may be enqueued
  hipStream_t s;
  DeviceArena* arena;
  int64_t Wp;
  uint32_t minsup;
  int max_len;
  const int32_t* d_ids;
  const uint32_t* gram = nullptr;  // root-level pair counts (dense F x F) if computed
  int64_t F = 0;
  OutBufs* ob = nullptr;
  DevVec<int64_t>& out_parent;
  DevVec<int32_t>& out_item;
  DevVec<uint32_t>& out_count;
  DevVec<uint8_t>& out_depth;
  int64_t out_size = 0;
  // streamed download: [0, streamed) already queued to the pinned host arrays on ob->copy_s
  bool stream_dl = false;
  int64_t host_cap = 0, streamed = 0;
  kern::HostTrie ht{};  // pinned host arrays + element widths (stream_out needs full widths)
  std::shared_ptr<void> back;  // pinned descriptor + control-block readback (FCtl::rb_dst)
  // hipGraph mode (mine_resident): the first batch of levels is captured (graph_capture; the
  // caller's end_capture instantiates and launches it) or already launched as a replay
  bool graph_capture = false, graph_replay = false;
  int graph_last = 0;                        // replay: last level the graph enqueues
  bool root_from_gram = false;                // level 2 was built by level_root_fill
  std::function<void(int)> end_capture;      // capture: called with the batch's last level

  explicit MineRun(OutBufs* o)
      : ob(o), out_parent(o->parent), out_item(o->item), out_count(o->count), out_depth(o->depth) {}
  int64_t n_candidates = 0;
  int max_depth = 1;
  int64_t* h_scalar = nullptr;  // pinned [2]
  int n_cus = 256;

  uint64_t* d_pair = nullptr;   // device [survivors, next-level candidates]
  Comm* comm = nullptr;         // tx-DP: candidate counts are shard-partial → all-reduce

  void read_pair(int64_t& S, int64_t& next_total) {
    KMLS_HIP(hipMemcpyAsync(h_scalar, d_pair, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    if (comm) comm->wait_stream(s);  // bounded: a dead peer aborts instead of hanging
    else KMLS_HIP(hipStreamSynchronize(s));
    S = h_scalar[0];
    next_total = h_scalar[1];
  }

  // queue the D2H copy of the nodes finished since the last call (ordered after them on s)
  void stream_out() {
    if (!stream_dl || out_size <= streamed) return;
    if (out_size > host_cap) {  // pinned arrays too small: the final download does it all
      stream_dl = false;
      return;
    }
    if (ht.par_w != 8 || ht.item_w != 4 || ht.cnt_w != 4)
      throw std::logic_error("stream_out: compact host trie on a memcpy download path");
    const int64_t a = streamed, n = out_size - streamed;
    KMLS_HIP(hipEventRecord(ob->ev, s));
    KMLS_HIP(hipStreamWaitEvent(ob->copy_s, ob->ev, 0));
    KMLS_HIP(hipMemcpyAsync((int64_t*)ht.parent + a, out_parent.p + a, n * sizeof(int64_t), hipMemcpyDeviceToHost, ob->copy_s));
    KMLS_HIP(hipMemcpyAsync((int32_t*)ht.item + a, out_item.p + a, n * sizeof(int32_t), hipMemcpyDeviceToHost, ob->copy_s));
    KMLS_HIP(hipMemcpyAsync((uint32_t*)ht.count + a, out_count.p + a, n * sizeof(uint32_t), hipMemcpyDeviceToHost, ob->copy_s));
    KMLS_HIP(hipMemcpyAsync(ht.depth + a, out_depth.p + a, n * sizeof(uint8_t), hipMemcpyDeviceToHost, ob->copy_s));
    streamed = out_size;
  }

  void ensure_out(int64_t n) {
    if (n > out_parent.cap || n > out_item.cap || n > out_count.cap || n > out_depth.cap)
      KMLS_HIP(hipStreamSynchronize(ob->copy_s));  // in-flight copies read the old arrays
    out_parent.reserve(n, s);
    out_item.reserve(n, s);
    out_count.reserve(n, s);
    out_depth.reserve(n, s);
  }

  // ---- fused, host-sync-free level expansion (levels.hip) -----------------------------------
  // All levels are enqueued back to back (2 kernels per level, sizes stay on the device); the
  // host synchronises once per batch of levels.  Returns false with nothing committed when a
  // device-side capacity check fails — the caller then runs the chunked path (process()).
  std::shared_ptr<PinnedPool> pinned;
  bool run_fast(const Level& root, const std::vector<int64_t>& root_off, int64_t root_total) {
    constexpr int kMaxLv = 64;
    const int64_t Fr = root.n;
    const size_t mark = arena->mark();
    const int64_t row_bytes = Wp * 8 + 4 + 8 + 4 + 8;  // child bitmap + rank + gid + slot + cand_off
    const size_t root_need = (size_t)(root_total + 1) * (size_t)row_bytes + (size_t)(Fr + 1) * 8 +
                             kMaxLv * sizeof(kern::FLevel) + 4096;
    const size_t free_b = arena->capacity() - arena->used();
    if (root_need + (256ull << 20) > free_b) {
      fallback_reason = "arena too small for the root level";
      return false;
    }
    {
      const int64_t want = std::max<int64_t>(out_size + root_total + 1, fast_hint);
      ensure_out(want);
    }
    const int64_t out_cap = std::min<int64_t>({out_parent.cap, out_item.cap, out_count.cap, out_depth.cap});
    if (out_size + root_total > out_cap) {
      fallback_reason = "output capacity";
      return false;
    }
    kern::FLevel* d_desc = (kern::FLevel*)arena->push(kMaxLv * sizeof(kern::FLevel));
    kern::FCtl* d_ctl = (kern::FCtl*)arena->push(sizeof(kern::FCtl));
    int64_t* d_off = (int64_t*)arena->push((size_t)(Fr + 1) * 8);
    uint64_t* c_bm = (uint64_t*)arena->push((size_t)((std::max<int64_t>(root_total, 1) + 63) & ~63ll) * Wp * 8);
    int32_t* c_rank = (int32_t*)arena->push((size_t)std::max<int64_t>(root_total, 1) * 4);
    int64_t* c_gid = (int64_t*)arena->push((size_t)std::max<int64_t>(root_total, 1) * 8);
    int32_t* c_slot = (int32_t*)arena->push((size_t)std::max<int64_t>(root_total, 1) * 4);
    int64_t* c_co = (int64_t*)arena->push((size_t)(root_total + 1) * 8);
    const size_t rem = arena->capacity() - arena->used();
    const size_t bump_bytes = fused_bump_cap(rem > (320ull << 20) ? rem - (64ull << 20) : 0);
    if (bump_bytes < (16ull << 20)) {
      arena->pop_to(mark);
      fallback_reason = "arena too small for the bump region";
      return false;
    }
    char* bump_base = (char*)arena->push(bump_bytes);
    // host-side descriptors → device (pinned staging, alive until the first sync below)
    const size_t stage_bytes = kMaxLv * sizeof(kern::FLevel) + sizeof(kern::FCtl) + (size_t)(Fr + 1) * 8;
    std::shared_ptr<void> stage = pinned->get(stage_bytes);
    kern::FLevel* h_desc = (kern::FLevel*)stage.get();
    std::memset(h_desc, 0, kMaxLv * sizeof(kern::FLevel));
    kern::FCtl* h_ctl = (kern::FCtl*)(h_desc + kMaxLv);
    std::memset(h_ctl, 0, sizeof(kern::FCtl));
    int64_t* h_off = (int64_t*)(h_ctl + 1);
    std::memcpy(h_off, root_off.data(), (size_t)(Fr + 1) * 8);
    kern::FLevel& r = h_desc[1];
    r.n_rows = Fr;
    r.bm = root.bm;
    r.rank = root.rank;
    r.gid = root.gid;
    r.cand_off = d_off;
    r.n_cand = root_total;
    r.child_base = out_size;
    h_desc[2].bm = c_bm;
    h_desc[2].rank = c_rank;
    h_desc[2].gid = c_gid;
    h_desc[2].slot = c_slot;
    h_desc[2].cand_off = c_co;
    h_ctl->bump_base = bump_base;
    h_ctl->bump_cap = bump_bytes;
    h_ctl->status_cap = (unsigned long long)ob->status_cap;
    h_ctl->epoch_base = ob->begin_call(s);
    h_ctl->h = ht;
    back = pinned->get(kMaxLv * sizeof(kern::FLevel) + sizeof(kern::FCtl));
    h_ctl->rb_dst = back.get();
    KMLS_HIP(hipMemcpyAsync(d_desc, h_desc, stage_bytes - (size_t)(Fr + 1) * 8, hipMemcpyHostToDevice, s));
    KMLS_HIP(hipMemcpyAsync(d_off, h_off, (size_t)(Fr + 1) * 8, hipMemcpyHostToDevice, s));
    if (!levels_loop(d_desc, d_ctl, out_cap)) {
      arena->pop_to(mark);
      return false;
    }
    arena->pop_to(mark);
    return true;
  }

  // The level loop shared by the host- and device-prepared fused paths: count level 1 (root),
  // then scan+count per level, one host sync per batch of levels.  Streamed download: the count
  // kernels write every survivor straight into the pinned host arrays as well (no copy-out
  // kernel, no cross-stream event per level); level-1 nodes are written by the resident
  // prologue's root setup or were queued by stream_out() on the host-prepared path.
  // end of a level batch: the deferred download of level L's children (nodes
  // [desc[L].child_base, + desc[L+1].n_rows)) and the descriptor readback, in one launch
  void finish_batch(kern::FLevel* d_desc, kern::FCtl* d_ctl, int L, bool deferred,
                    size_t back_bytes) {
    kern::level_copyout(&d_desc[L], &d_desc[L + 1], d_ctl, out_parent.p, out_item.p, out_count.p,
                        out_depth.p, deferred, d_desc, back_bytes, s);
  }

  bool levels_loop(kern::FLevel* d_desc, kern::FCtl* d_ctl, int64_t out_cap) {
    constexpr int kMaxLv = 64;
    const int grid = kern::level_grid(n_cus);
    // launch only as many persistent blocks as the previous call's level needed (x2 margin; a
    // bigger level still completes through the ticket counter): dispatching and retiring
    // ~2k idle workgroups is a visible part of a small level's kernel
    auto grid_for_tiles = [&](int64_t tiles_hint) {
      if (tiles_hint < 0) return grid;
      return (int)std::min<int64_t>(grid, std::max<int64_t>(32, 2 * tiles_hint + 16));
    };
    auto hint_at = [](const std::vector<int64_t>& v, int L) {
      return L < (int)v.size() ? v[L] : (int64_t)-1;
    };
    // diagnostics: KMLS_LEVEL_TRACE=<L> records per-tile phase timestamps of level L's count
    // kernel and writes them to KMLS_LEVEL_TRACE_FILE (uint64 [tiles][8]) after the call
    static const int trace_level = [] {
      const char* e = std::getenv("KMLS_LEVEL_TRACE");
      return e ? std::atoi(e) : 0;
    }();
    unsigned long long* d_trace = nullptr;
    if (trace_level > 0) {
      if (!ob->trace) {
        KMLS_HIP(hipMalloc((void**)&ob->trace, (size_t)ob->status_cap * 64));
      }
      KMLS_HIP(hipMemsetAsync(ob->trace, 0, (size_t)ob->status_cap * 64, s));
      d_trace = ob->trace;
    }
    const bool deferred = stream_dl && deferred_dl();
    auto count_level = [&](int L) {
      kern::LevelCountArgs a{Wp, minsup, L == 1 ? gram : nullptr, F, d_ids, out_parent.p,
                             out_item.p, out_count.p, out_depth.p, (uint8_t)(L + 1),
                             stream_dl, L == trace_level ? d_trace : nullptr, deferred,
                             copy_blocks(), copy_last(), L == 1, out_cap,
                             max_len > 0 && L + 1 >= max_len};
      const int64_t hint = hint_at(ob->cand_hint, L);
      const int g = grid_for_tiles(hint < 0 ? -1 : (hint + kern::level_tile() - 1) / kern::level_tile());
      // the count kernels load tile_row[block] speculatively: every block index must be in bounds
      if ((int64_t)g + kern::kCopyBlocks + 64 > ob->status_cap)
        throw std::logic_error("levels_loop: count grid exceeds the tile_row capacity");
      int32_t* tr_cur = ob->tile_row + (size_t)(L & 1) * (size_t)ob->status_cap;
      int32_t* tr_nx = ob->tile_row + (size_t)((L + 1) & 1) * (size_t)ob->status_cap;
      kern::level_count(&d_desc[L], &d_desc[L + 1], d_ctl, ob->status, ob->next_epoch(s), a,
                        L == 1 ? nullptr : tr_cur, tr_nx, g, hint, s);
    };
    // count(L) writes desc[L + 2] (the next level's buffers)
    const int L_allowed = std::min(kMaxLv - 3, max_len ? max_len - 1 : kMaxLv - 3);
    int last = 1;
    int target = std::min(L_allowed, std::max(ob->depth_hint, 2));
    if (graph_replay) {  // the replayed graph already holds count(1) .. count(graph_last)
      last = graph_last;
      target = graph_last;
    } else if (!root_from_gram) {
      count_level(1);
    }
    if (!back) throw std::logic_error("levels_loop: no readback buffer (FCtl::rb_dst)");
    kern::FLevel* b_desc = (kern::FLevel*)back.get();
    kern::FCtl* b_ctl = (kern::FCtl*)(b_desc + kMaxLv);
    bool ok = true;
    for (bool first = true;; first = false) {
     if (!(first && graph_replay)) {
      for (int L = last + 1; L <= target; ++L) {
        count_level(L);
        last = L;
      }
      // d_ctl directly follows d_desc (kMaxLv * 128 bytes, arena alignment 256)
      if ((char*)d_ctl != (char*)(d_desc + kMaxLv))
        throw std::logic_error("levels_loop: control block must follow the descriptors");
      finish_batch(d_desc, d_ctl, last, deferred, kMaxLv * sizeof(kern::FLevel) + sizeof(kern::FCtl));
      if (first && graph_capture) end_capture(last);
     }
      t_presync = std::chrono::steady_clock::now();
      if (wait_ev) KMLS_HIP(hipEventSynchronize(wait_ev));
      else sync_stream(s);
      t_postsync = std::chrono::steady_clock::now();
      if (b_ctl->overflow) {
        ok = false;
        need_nodes = std::max<int64_t>(need_nodes, (int64_t)b_ctl->need_out_m << 20);
        fallback_reason = "device overflow code " + std::to_string(b_ctl->overflow) +
                          " at level " + std::to_string(last) + " (bump " +
                          std::to_string(b_ctl->bump_top >> 20) + "/" +
                          std::to_string(b_ctl->bump_cap >> 20) + " MiB)";
        break;
      }
      if (last < L_allowed && b_desc[last + 1].n_rows >= 2) {
        if (no_more_batches) {
          ok = false;
          fallback_reason = "pipelined call needs more levels than its replayed plan";
          break;
        }
        target = std::min(L_allowed, last + 4);
        continue;
      }
      break;
    }
    KMLS_HIP(hipStreamSynchronize(ob->copy_s));
    if (d_trace && trace_level <= last) {
      const int64_t tiles = (b_desc[trace_level].n_cand + kern::level_tile() - 1) / kern::level_tile();
      std::vector<unsigned long long> h((size_t)tiles * 8);
      KMLS_HIP(hipMemcpy(h.data(), d_trace, h.size() * 8, hipMemcpyDeviceToHost));
      const char* path = std::getenv("KMLS_LEVEL_TRACE_FILE");
      if (FILE* f = std::fopen(path ? path : "level_trace.bin", "wb")) {
        std::fwrite(h.data(), 8, h.size(), f);
        std::fclose(f);
      }
    }
    if (!ok) return false;
    last_desc.assign(b_desc, b_desc + kMaxLv);
    ob->cand_hint.assign((size_t)last + 1, -1);
    for (int L = 1; L <= last; ++L) ob->cand_hint[L] = b_desc[L].n_cand;
    const int64_t new_size = b_desc[last + 1].child_base;
    for (int L = 1; L <= last; ++L)
      if (b_desc[L + 1].n_rows > 0) max_depth = std::max(max_depth, L + 1);
    n_candidates += (int64_t)b_ctl->candidates;
    out_size = new_size;
    if (stream_dl) {  // final full copy when the pinned arrays were too small
      if (b_ctl->dl_overflow || out_size > host_cap) stream_dl = false;
      else streamed = out_size;
    }
    ob->depth_hint = std::max(2, max_depth);
    return true;
  }
  std::vector<kern::FLevel> last_desc;  // host copy of the descriptors after levels_loop
  std::chrono::steady_clock::time_point t_presync, t_postsync;  // host-side profile

  int64_t fast_hint = 0;
  int64_t need_nodes = 0;  // trie nodes a failed fused call needed (overflow 4 on out_cap)
  std::string fallback_reason;

  int64_t read_i64(const int64_t* dptr) {
    KMLS_HIP(hipMemcpyAsync(h_scalar, dptr, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipStreamSynchronize(s));
    return h_scalar[0];
  }

  // Expand every row of level L (itemsets of size `depth`).  `len` (device, L.n+1 entries,
  // len[L.n] == 0) holds each row's candidate count and `total` their sum — both produced by
  // the parent chunk (or the host at the root), so a chunk costs ONE host readback: the
  // survivor count and the child level's candidate total, read together.
  void process(const Level& L, int depth, const int64_t* len, int64_t total) {
    if (L.n < 2 || total == 0 || (max_len && depth >= max_len)) return;
    const size_t mark0 = arena->mark();
    int64_t* cand_off = (int64_t*)arena->push((size_t)(L.n + 1) * sizeof(int64_t));
    const size_t tb = kern::scan_temp_bytes(L.n);
    void* tmp = arena->push(tb);
    kern::exclusive_scan_i64(len, cand_off, L.n, tmp, tb, s);
    struct Chunk { int64_t a0, a1, c0, c1; };
    std::vector<Chunk> chunks;
    if (total <= kCandCap) {
      chunks.push_back({0, L.n, 0, total});
    } else {  // split at row boundaries
      std::vector<int64_t> off((size_t)L.n + 1);
      KMLS_HIP(hipMemcpyAsync(off.data(), cand_off, off.size() * sizeof(int64_t),
                              hipMemcpyDeviceToHost, s));
      KMLS_HIP(hipStreamSynchronize(s));
      int64_t a0 = 0;
      for (int64_t a = 0; a < L.n; ++a) {
        if (off[a + 1] - off[a0] > kCandCap && a > a0) {
          chunks.push_back({a0, a, off[a0], off[a]});
          a0 = a;
        }
      }
      chunks.push_back({a0, L.n, off[a0], off[L.n]});
    }
    for (const Chunk& ch : chunks) {
      const int64_t c0 = ch.c0, c1 = ch.c1, nc = c1 - c0;
      if (nc == 0) continue;
      const size_t mark = arena->mark();
      uint32_t* cnt = (uint32_t*)arena->push((size_t)nc * sizeof(uint32_t));
      if (gram && depth == 1) {
        kern::gram_to_cand(gram, F, cand_off, c0, c1, cnt, s);  // gram already global
      } else {
        kern::extend_count(L.bm, Wp, cand_off, L.n, c0, c1, cnt, s);
        if (comm) comm->all_reduce(cnt, cnt, (size_t)nc, CommDtype::U32, false, s);
      }
      int64_t* pos = (int64_t*)arena->push((size_t)(nc + 1) * sizeof(int64_t));
      const size_t fb = kern::flag_scan_temp_bytes(nc);
      void* ftmp = arena->push(fb);
      kern::flag_scan(cnt, minsup, nc, pos, ftmp, fb, s);
      kern::child_totals(cand_off, ch.a0, ch.a1, c0, pos, nc, d_pair, s);
      n_candidates += nc;
      int64_t S = 0, next_total = 0;
      read_pair(S, next_total);
      if (S == 0) {
        arena->pop_to(mark);
        continue;
      }
      ensure_out(out_size + S);
      Level C;
      C.n = S;
      // children at the max_len depth are leaves: trie nodes only (no bitmaps / class rows)
      const bool leaf = max_len && depth + 1 >= max_len;
      uint64_t* cbm = leaf ? nullptr : (uint64_t*)arena->push((size_t)S * Wp * sizeof(uint64_t));
      int32_t* crank = leaf ? nullptr : (int32_t*)arena->push((size_t)S * sizeof(int32_t));
      int64_t* cgid = leaf ? nullptr : (int64_t*)arena->push((size_t)S * sizeof(int64_t));
      int32_t* cend = leaf ? nullptr : (int32_t*)arena->push((size_t)S * sizeof(int32_t));
      int64_t* clen = leaf ? nullptr : (int64_t*)arena->push((size_t)(S + 1) * sizeof(int64_t));
      if (clen) KMLS_HIP(hipMemsetAsync(clen + S, 0, sizeof(int64_t), s));
      kern::LevelOut o{cbm, crank, cgid, cend, clen, out_parent.p, out_item.p, out_count.p,
                       out_depth.p, out_size, (uint8_t)(depth + 1)};
      int64_t* surv = leaf ? nullptr : (int64_t*)arena->push((size_t)S * sizeof(int64_t));
      kern::extend_materialize(L.bm, Wp, cand_off, L.n, L.rank, L.gid, d_ids, c0, c1, cnt, minsup,
                               pos, o, s, S, surv);
      out_size += S;
      stream_out();
      max_depth = std::max(max_depth, depth + 1);
      if (leaf) {
        arena->pop_to(mark);
        continue;
      }
      C.bm = cbm;
      C.rank = crank;
      C.gid = cgid;
      C.row_end = cend;
      process(C, depth + 1, clen, next_total);
      arena->pop_to(mark);
    }
    arena->pop_to(mark0);
  }
};

size_t fused_bump_cap(size_t bytes) {  // test hook fused_bump_mb: forces the chunked fallback
  const long long mb = test_hook("fused_bump_mb", 0);
  return mb > 0 ? std::min(bytes, (size_t)mb << 20) : bytes;
}

// test hook fused_levels=0: the chunked level path (the fallback of an overflowing fused call)
bool fused_levels_enabled() { return test_hook("fused_levels", 1) != 0; }

size_t default_arena_bytes() {
  size_t free_b = 0, total_b = 0;
  KMLS_HIP(hipMemGetInfo(&free_b, &total_b));
  if (const char* e = std::getenv("KMLS_ARENA_GB")) {
    const double gb = std::atof(e);
    if (gb > 0) return std::min(free_b - (free_b >> 4), (size_t)(gb * (1ull << 30)));
  }
  if (const long long mb = test_hook("arena_init_mb", 0))  // initial size of a growing arena
    return std::min(free_b / 2, (size_t)mb << 20);
  // 8 GiB by default: hipMalloc maps HBM eagerly (~10 ms/GiB), and a job's one-shot mining
  // call should not pay for half of a 288 GB card.  The arena grows on demand (grow_arena) up to
  // half of the free HBM (the other half stays with torch / RCCL buffers).
  return std::min(free_b / 2, (size_t)8 << 30);
}

size_t max_arena_bytes() {
  size_t free_b = 0, total_b = 0;
  KMLS_HIP(hipMemGetInfo(&free_b, &total_b));
  return free_b / 2;
}

float elapsed(const Event& a, const Event& b) {
  float ms = 0.f;
  KMLS_HIP(hipEventElapsedTime(&ms, a.e, b.e));
  return ms;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// The captured launch sequence of the last steady-state resident call (see mine_resident).
// Two executable instances of the captured call: consecutive launches alternate between them,
// so a call launched ahead (prefetch) is never a relaunch of the exec that is still running
// (measured no faster than one instance on the headline, profiles/r2_s15_graph_interleaved.log:
// off).
struct GraphCache {
  std::vector<uint64_t> key;
  hipGraphExec_t exec = nullptr;
  hipGraphExec_t twin = nullptr;
  unsigned flip = 0;
  int last = 0;             // last level the graph enqueues
  unsigned launch_idx = 0;  // look-back launch indices the graph consumes
  void reset(hipGraphExec_t e, std::vector<uint64_t> k, int l, unsigned li,
             hipGraphExec_t t = nullptr) {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (twin) (void)hipGraphExecDestroy(twin);
    exec = e;
    twin = t;
    flip = 0;
    key = std::move(k);
    last = l;
    launch_idx = li;
  }
  hipGraphExec_t next() {  // the instance for the next launch
    const hipGraphExec_t x = (twin && (flip & 1u)) ? twin : exec;
    ++flip;
    return x;
  }
  ~GraphCache() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (twin) (void)hipGraphExecDestroy(twin);
  }
};

static bool graph_twin_enabled() { return false; }

// A steady-state resident call launched ahead (mine(prefetch=true)): its graph replay is on the
// stream behind the call that launched it, writing to its own pinned buffers.  The next
// mine_resident() with the same launch key adopts it instead of launching.
struct Prefetch {
  std::vector<uint64_t> key;
  bool download = false;
  int64_t host_cap = 0;
  int pw = 0, iw = 0, cw = 0;
  std::shared_ptr<void> h_parent, h_item, h_count, h_depth;  // pinned host trie
  std::shared_ptr<void> fstage, back;                          // tables, readback
  std::shared_ptr<void> i_rp, i_cons, i_cnt, i_meta;           // pinned rule-map CSR
  std::chrono::steady_clock::time_point t_launch;
};

GpuMiner::GpuMiner(int device, size_t arena_bytes, uintptr_t stream) : device_(device) {
  KMLS_HIP(hipSetDevice(device));
  if (stream) {
    stream_ = (void*)stream;
  } else {
    hipStream_t s;
    KMLS_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    stream_ = (void*)s;
    own_stream_ = true;
  }
  arena_auto_ = arena_bytes == 0 && !std::getenv("KMLS_ARENA_GB");
  if (arena_auto_) arena_max_ = max_arena_bytes();
  arena_ = std::make_unique<DeviceArena>(arena_bytes ? arena_bytes : default_arena_bytes());
  pinned_ = make_pinned_pool();
  KMLS_HIP(hipHostMalloc((void**)&h_scalar_, 64));
  KMLS_HIP(hipHostMalloc((void**)&call_params_, 2 * sizeof(kern::FCtl)));
  std::memset(call_params_, 0, 2 * sizeof(kern::FCtl));
  KMLS_HIP(hipMalloc((void**)&d_call_seq_, 64));
  KMLS_HIP(hipMemset(d_call_seq_, 0, 64));
  KMLS_HIP(hipMalloc((void**)&d_pair_, 2 * sizeof(uint64_t)));
  hipDeviceProp_t prop;
  KMLS_HIP(hipGetDeviceProperties(&prop, device));
  n_cus_ = std::max(1, prop.multiProcessorCount);
  if (const long long c = test_hook("idx_cap", 0)) idx_cap_ = std::max(16ll, c);
}

GpuMiner::~GpuMiner() {
  (void)hipSetDevice(device_);
  if (stream_) (void)hipStreamSynchronize((hipStream_t)stream_);
  pre_.reset();
  graph_.reset();
  if (d_tx_ptr_) (void)hipFree(d_tx_ptr_);
  if (d_items_) (void)hipFree(d_items_);
  if (d_rank_of_) (void)hipFree(d_rank_of_);
  if (d_cooc_) (void)hipFree(d_cooc_);
  if (d_fmask_) (void)hipFree(d_fmask_);
  if (d_fgroup_) (void)hipFree(d_fgroup_);
  if (d_c2r_) (void)hipFree(d_c2r_);
  if (d_ids_) (void)hipFree(d_ids_);
  if (d_own_bm_) (void)hipFree(d_own_bm_);
  if (h_scalar_) (void)hipHostFree(h_scalar_);
  if (call_params_) (void)hipHostFree(call_params_);
  if (d_call_seq_) (void)hipFree(d_call_seq_);
  if (sup_scratch_) (void)hipFree(sup_scratch_);
  if (d_pair_) (void)hipFree(d_pair_);
  if (d_tie_) (void)hipFree(d_tie_);
  if (d_inv_tie_) (void)hipFree(d_inv_tie_);
  for (void* e : tile_ev_) (void)hipEventDestroy((hipEvent_t)e);
  for (void* e : idx_ev_)
    if (e) (void)hipEventDestroy((hipEvent_t)e);
  if (idx_s_) {
    (void)hipStreamSynchronize((hipStream_t)idx_s_);
    (void)hipStreamDestroy((hipStream_t)idx_s_);
  }
  if (comm_s_) {
    (void)hipStreamSynchronize((hipStream_t)comm_s_);
    (void)hipStreamDestroy((hipStream_t)comm_s_);
  }
  out_.reset();
  arena_.reset();
  if (own_stream_) (void)hipStreamDestroy((hipStream_t)stream_);
}

size_t GpuMiner::arena_capacity() const { return arena_->capacity(); }

// Per-item supports (accumulated into `counts`): the partitioned histogram for large
// vocabularies and inputs (kern::item_support_partitioned, scratch owned by the miner), else the
// LDS/hash kernels.
void GpuMiner::support_counts(const int32_t* items, int64_t nnz, uint32_t* counts, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const size_t need = nnz >= (4ll << 20) ? kern::support_scratch_bytes(nnz, n_items_) : 0;
  if (need) {
    if (need > sup_scratch_bytes_) {
      if (sup_scratch_) KMLS_HIP(hipFree(sup_scratch_));
      sup_scratch_ = nullptr;
      KMLS_HIP(hipMalloc(&sup_scratch_, need));
      sup_scratch_bytes_ = need;
    }
    if (kern::item_support_partitioned(items, nnz, (int32_t)n_items_, counts, sup_scratch_,
                                       sup_scratch_bytes_, s))
      return;
  }
  kern::item_support(items, nnz, (int32_t)n_items_, counts, s);
}

bool GpuMiner::grow_arena(size_t min_bytes) {
  if (!arena_auto_ || arena_->used() != 0) return false;
  const size_t cap = arena_->capacity();
  if (cap >= arena_max_) return false;
  const size_t want = std::min(arena_max_, std::max(min_bytes, cap * 4));
  KMLS_HIP(hipStreamSynchronize((hipStream_t)stream_));
  arena_.reset();
  arena_ = std::make_unique<DeviceArena>(want);
  return true;
}

namespace {
// a fused-path failure that more arena would fix (bump region or arena sizing), not a data limit
bool arena_limited(const std::string& why) {
  return why.empty() || why.find("overflow code 1") != std::string::npos ||
         why.find("arena") != std::string::npos;
}
}  // namespace

void GpuMiner::synchronize() { KMLS_HIP(hipStreamSynchronize((hipStream_t)stream_)); }

void GpuMiner::set_tie_rank(const int32_t* tie, int64_t n) {
  KMLS_CHECK(n == n_items_, "set_tie_rank: size != n_items (load_csr first)");
  std::vector<int32_t> inv((size_t)n, -1);
  for (int64_t i = 0; i < n; ++i) {
    KMLS_CHECK(tie[i] >= 0 && tie[i] < n && inv[(size_t)tie[i]] < 0,
               "set_tie_rank: not a permutation of [0, n_items)");
    inv[(size_t)tie[i]] = (int32_t)i;
  }
  drain_prefetch();
  KMLS_HIP(hipSetDevice(device_));
  KMLS_HIP(hipStreamSynchronize((hipStream_t)stream_));
  if (!d_tie_) {
    KMLS_HIP(hipMalloc((void**)&d_tie_, (size_t)std::max<int64_t>(n, 1) * 4));
    KMLS_HIP(hipMalloc((void**)&d_inv_tie_, (size_t)std::max<int64_t>(n, 1) * 4));
  }
  KMLS_HIP(hipMemcpy(d_tie_, tie, (size_t)n * 4, hipMemcpyHostToDevice));
  KMLS_HIP(hipMemcpy(d_inv_tie_, inv.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  if (graph_) graph_->reset(nullptr, {}, 0, 0);
}

// Wait for a launched-ahead call and drop it (its buffers return to the pinned pool).
void GpuMiner::drain_prefetch() {
  if (!pre_) return;
  KMLS_HIP(hipStreamSynchronize((hipStream_t)stream_));
  pre_.reset();
}

void GpuMiner::load_csr(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx,
                        int64_t n_items) {
  KMLS_HIP(hipSetDevice(device_));
  ++sel_gen_;
  drain_prefetch();
  hipStream_t s = (hipStream_t)stream_;
  if (d_tx_ptr_) KMLS_HIP(hipFree(d_tx_ptr_));
  if (d_items_) KMLS_HIP(hipFree(d_items_));
  d_tx_ptr_ = nullptr;
  d_items_ = nullptr;
  if (d_tie_) KMLS_HIP(hipFree(d_tie_));  // a tie key belongs to one vocabulary: set it again
  if (d_inv_tie_) KMLS_HIP(hipFree(d_inv_tie_));
  d_tie_ = d_inv_tie_ = nullptr;
  if (graph_) graph_->reset(nullptr, {}, 0, 0);
  n_tx_ = n_tx;
  n_items_ = n_items;
  const int64_t base = tx_ptr[0];
  nnz_ = tx_ptr[n_tx] - base;
  std::vector<int64_t> rebased((size_t)n_tx + 1);
  for (int64_t t = 0; t <= n_tx; ++t) rebased[t] = tx_ptr[t] - base;
  tile_tx_.assign(65, 0);
  tile_nnz_.assign(65, 0);
  for (int k = 0; k <= 64; ++k) {
    tile_tx_[k] = n_tx * k / 64;
    tile_nnz_[k] = rebased[tile_tx_[k]];
  }
  for (int64_t p = 0; p < nnz_; ++p) {
    const int32_t it = items[base + p];
    KMLS_CHECK(it >= 0 && it < n_items, "item id out of range in CSR");
  }
  KMLS_HIP(hipMalloc((void**)&d_tx_ptr_, rebased.size() * sizeof(int64_t)));
  // (+16 items of padding: the filter kernels read 16-byte vectors that may run past the end)
  KMLS_HIP(hipMalloc((void**)&d_items_, (size_t)(std::max<int64_t>(nnz_, 4) + 16) * sizeof(int32_t)));
  KMLS_HIP(hipMemcpyAsync(d_tx_ptr_, rebased.data(), rebased.size() * sizeof(int64_t),
                          hipMemcpyHostToDevice, s));
  if (nnz_)
    KMLS_HIP(hipMemcpyAsync(d_items_, items + base, (size_t)nnz_ * sizeof(int32_t),
                            hipMemcpyHostToDevice, s));
  KMLS_HIP(hipStreamSynchronize(s));
}

void GpuMiner::item_support(uintptr_t counts_dev) {
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  KMLS_HIP(hipMemsetAsync((void*)counts_dev, 0, (size_t)n_items_ * sizeof(uint32_t), s));
  support_counts(d_items_, nnz_, (uint32_t*)counts_dev, s);
}

// Device-side selection from device-resident (all-reduced) supports: only the F frequent ids
// and counts cross PCIe (kern::select_large), not the n_items support vector.
// The selection's device tables (rank_of / ids over the whole vocabulary, the frequent bit mask of
// a large one), allocated once per vocabulary size: a reselection (every rule-map step) frees and
// allocates nothing — each hipFree waits for the whole device.
void GpuMiner::ensure_select_bufs() {
  const int64_t I = std::max<int64_t>(n_items_, 1);
  if (sel_cap_ == I) return;
  for (void* p : {(void*)d_rank_of_, (void*)d_ids_, (void*)d_fmask_, (void*)d_fgroup_, (void*)d_c2r_})
    if (p) KMLS_HIP(hipFree(p));
  d_fmask_ = nullptr;
  d_fgroup_ = nullptr;
  d_c2r_ = nullptr;
  KMLS_HIP(hipMalloc((void**)&d_rank_of_, (size_t)I * sizeof(int32_t)));
  KMLS_HIP(hipMalloc((void**)&d_ids_, (size_t)I * sizeof(int32_t)));
  if (n_items_ >= (1 << 16)) KMLS_HIP(hipMalloc((void**)&d_fmask_, (size_t)(I + 31) / 32 * 4));
  sel_cap_ = I;
}

int64_t GpuMiner::select_device(const uint32_t* d_counts, int64_t global_n_tx, double min_support,
                                Comm* comm) {
  hipStream_t s = (hipStream_t)stream_;
  ++sel_gen_;
  global_n_tx_ = global_n_tx;
  const int64_t I = std::max<int64_t>(n_items_, 1);
  ensure_select_bufs();
  const size_t mark = arena_->mark();
  const size_t tb = kern::select_large_temp_bytes(I);
  void* tmp = arena_->push(tb);
  uint32_t* d_fc = (uint32_t*)arena_->push((size_t)I * 4);
  unsigned long long* dF = (unsigned long long*)arena_->push(256);
  const uint32_t c1 = level1_threshold((uint64_t)global_n_tx, min_support);
  kern::select_large(d_counts, n_items_, c1, tmp, tb, d_ids_, d_fc, d_rank_of_, d_fmask_, dF, s);
  KMLS_HIP(hipMemcpyAsync(h_scalar_, dF, 8, hipMemcpyDeviceToHost, s));
  if (comm) comm->wait_stream(s);
  else KMLS_HIP(hipStreamSynchronize(s));
  const int64_t F = h_scalar_[0];
  fi_.ids.assign((size_t)F, 0);
  fi_.counts.assign((size_t)F, 0u);
  if (F) {
    KMLS_HIP(hipMemcpyAsync(fi_.ids.data(), d_ids_, (size_t)F * 4, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipMemcpyAsync(fi_.counts.data(), d_fc, (size_t)F * 4, hipMemcpyDeviceToHost, s));
  }
  // (the encode tables below run on this stream after the copies; one sync at their end)
  fi_.rank_of.clear();  // the device holds it (d_rank_of_); no host reader of a device selection
  fi_.minsup2 = level2_threshold((uint64_t)global_n_tx, min_support);
  build_encode_tables(F);  // syncs the stream: the copies above are complete
  arena_->pop_to(mark);
  sel_ids_ = fi_.ids;
  sel_counts_ = fi_.counts;
  return F;
}

// Encode lookup tables (kern::frequent_groups) for the selection just made; small vocabularies
// or wide frequent sets keep the mask + rank gathers.
void GpuMiner::build_encode_tables(int64_t F) {
  encode_tables_ = false;
  if (!d_fmask_ || F <= 0 || F > kern::kEncodeGroupMaxF) {
    KMLS_HIP(hipStreamSynchronize((hipStream_t)stream_));
    return;
  }
  hipStream_t s = (hipStream_t)stream_;
  const int64_t G = (n_items_ + 31) / 32;
  if (!d_fgroup_) KMLS_HIP(hipMalloc((void**)&d_fgroup_, (size_t)G * 8));  // (freed with d_fmask_)
  if (!d_c2r_) KMLS_HIP(hipMalloc((void**)&d_c2r_, (size_t)kern::kEncodeGroupMaxF * 4));
  encode_tables_ = true;
  const size_t mark = arena_->mark();
  const size_t tb = kern::frequent_groups_temp_bytes(n_items_);
  void* tmp = arena_->push(tb);
  kern::frequent_groups(d_fmask_, n_items_, d_rank_of_, d_fgroup_, d_c2r_, tmp, tb, s);
  KMLS_HIP(hipStreamSynchronize(s));  // the scratch returns to the arena
  arena_->pop_to(mark);
}

int64_t GpuMiner::select(const uint32_t* global_counts, int64_t global_n_tx, double min_support) {
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  ++sel_gen_;
  global_n_tx_ = global_n_tx;
  fi_ = select_frequent(global_counts, n_items_, (uint64_t)global_n_tx, min_support);
  ensure_select_bufs();
  std::vector<uint32_t> mask;
  if (d_fmask_) {  // frequent-item bit mask for the encode gather (kernels.hpp)
    mask.assign((size_t)(n_items_ + 31) / 32, 0u);
    for (int32_t id : fi_.ids) mask[(size_t)id >> 5] |= 1u << (id & 31);
    KMLS_HIP(hipMemcpyAsync(d_fmask_, mask.data(), mask.size() * sizeof(uint32_t),
                            hipMemcpyHostToDevice, s));
  }
  KMLS_HIP(hipMemcpyAsync(d_rank_of_, fi_.rank_of.data(), (size_t)n_items_ * sizeof(int32_t),
                          hipMemcpyHostToDevice, s));
  if (!fi_.ids.empty())
    KMLS_HIP(hipMemcpyAsync(d_ids_, fi_.ids.data(), fi_.ids.size() * sizeof(int32_t),
                            hipMemcpyHostToDevice, s));
  KMLS_HIP(hipStreamSynchronize(s));
  build_encode_tables((int64_t)fi_.ids.size());
  sel_ids_ = fi_.ids;
  sel_counts_ = fi_.counts;
  return (int64_t)fi_.ids.size();
}

void GpuMiner::use_frequent_subset(const int64_t* keep, int64_t n) {
  KMLS_HIP(hipSetDevice(device_));
  const int64_t F = (int64_t)sel_ids_.size();
  KMLS_CHECK(n >= 0 && n <= F, "use_frequent_subset: more positions than frequent items");
  std::vector<int32_t> ids((size_t)n);
  std::vector<uint32_t> cnt((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    KMLS_CHECK(keep[i] >= 0 && keep[i] < F && (i == 0 || keep[i] > keep[i - 1]),
               "use_frequent_subset: positions must be ascending and < F");
    ids[(size_t)i] = sel_ids_[(size_t)keep[i]];
    cnt[(size_t)i] = sel_counts_[(size_t)keep[i]];
  }
  hipStream_t s = (hipStream_t)stream_;
  KMLS_HIP(hipStreamSynchronize(s));  // a queued kernel may still read d_ids_
  fi_.ids.swap(ids);
  fi_.counts.swap(cnt);
  ++sel_gen_;  // cached per-selection state (cooc stats) no longer applies
  if (n) KMLS_HIP(hipMemcpyAsync(d_ids_, fi_.ids.data(), (size_t)n * 4, hipMemcpyHostToDevice, s));
  KMLS_HIP(hipStreamSynchronize(s));
}

int64_t GpuMiner::words_local() const {
  const int64_t w = (n_tx_ + 63) / 64;
  return (w + 3) & ~(int64_t)3;  // 32-byte rows: 16-B team loads and the MFMA 4-word stride
}

bool GpuMiner::encode_bitmaps(uintptr_t bm_dev, int64_t Wp_total, int64_t word_off) {
  KMLS_HIP(hipSetDevice(device_));
  // long shards: LDS-slab encode (test hook encode_tiled=0: the atomic kernel of short shards)
  const bool tiled = test_hook("encode_tiled", 1) != 0;
  const int64_t F = (int64_t)fi_.ids.size();
  // frequent-item mask ahead of the rank gather, and (F <= 2048) the 8-byte group gather (an LDS
  // mask + hash lookup measured slower: 20.5 vs 13.2 ms at 100M x 754 frequent items)
  const uint32_t* fmask = d_fmask_;
  if (tiled && n_tx_ >= (1 << 16) &&
      kern::encode_bitmap_tiled(d_tx_ptr_, d_items_, n_tx_, d_rank_of_, (uint64_t*)bm_dev,
                                Wp_total, word_off, F, (hipStream_t)stream_, fmask,
                                encode_tables_ ? d_fgroup_ : nullptr,
                                encode_tables_ ? d_c2r_ : nullptr))
    return true;
  kern::encode_bitmap(d_tx_ptr_, d_items_, n_tx_, d_rank_of_, (uint64_t*)bm_dev, Wp_total,
                      word_off, (hipStream_t)stream_, fmask);
  return false;
}

// Encode into a bitmap buffer with stale contents.  The LDS-slab encode writes every word of
// the transaction columns (zeros included), so only the row padding past ceil(n_tx/64) words is
// cleared — at 100M transactions a full memset was a 9 GB write ahead of a 9 GB encode.
void GpuMiner::encode_bitmaps_fresh(uint64_t* bm, int64_t F, int64_t Wp) {
  hipStream_t s = (hipStream_t)stream_;
  const bool tiled = test_hook("encode_tiled", 1) != 0 && n_tx_ >= (1 << 16) && F > 0 &&
                     F <= kern::kEncodeTileMaxF;
  const int64_t used = (n_tx_ + 63) / 64;
  if (!tiled) {
    KMLS_HIP(hipMemsetAsync(bm, 0, (size_t)std::max<int64_t>(F, 1) * Wp * 8, s));
  } else if (Wp > used) {
    KMLS_HIP(hipMemset2DAsync(bm + used, (size_t)Wp * 8, 0, (size_t)(Wp - used) * 8, (size_t)F, s));
  }
  if (!encode_bitmaps((uintptr_t)bm, Wp, 0) && tiled) {  // the tiled kernel declined: clear, redo
    KMLS_HIP(hipMemsetAsync(bm, 0, (size_t)std::max<int64_t>(F, 1) * Wp * 8, s));
    encode_bitmaps((uintptr_t)bm, Wp, 0);
  }
}

void GpuMiner::pair_counts(uintptr_t bm_dev, int64_t Wp_total, uintptr_t out_dev, bool use_mfma) {
  KMLS_HIP(hipSetDevice(device_));
  const int64_t F = (int64_t)fi_.ids.size();
  hipStream_t s = (hipStream_t)stream_;
  KMLS_HIP(hipMemsetAsync((void*)out_dev, 0, (size_t)F * F * sizeof(uint32_t), s));
  if (use_mfma)
    kern::pair_gram_mfma((const uint64_t*)bm_dev, Wp_total, F, (uint32_t*)out_dev, s);
  else
    kern::pair_gram_popcount((const uint64_t*)bm_dev, Wp_total, F, (uint32_t*)out_dev, s);
}

GpuMiner::CoocStats GpuMiner::cooc_stats() {
  KMLS_CHECK(!subset_active(), "cooc_stats: a use_frequent_subset() set is active (rank tables "
                               "describe the full selection); select() again first");
  if (cooc_gen_ == sel_gen_) return cooc_cache_;  // same CSR and selection: one pass per step
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  CoocStats st;
  if (!d_cooc_) KMLS_HIP(hipMalloc((void**)&d_cooc_, 4 * sizeof(unsigned long long)));
  KMLS_HIP(hipMemsetAsync(d_cooc_, 0, 4 * sizeof(unsigned long long), s));
  if (n_tx_ > 0 && !fi_.ids.empty())
    kern::cooc_stats(d_tx_ptr_, d_items_, n_tx_, d_rank_of_, d_fmask_, d_cooc_, n_cus_, s);
  unsigned long long h[2] = {0, 0};
  KMLS_HIP(hipMemcpyAsync(h, d_cooc_, sizeof h, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  st.pairs = h[0];
  st.max_k = h[1];
  cooc_cache_ = st;
  cooc_gen_ = sel_gen_;
  return st;
}

// The row form of the horizontal count (kern::PairRows) on long shards: every increment an LDS
// atomic.  KMLS_PAIR_ROWS=0 / test hook pair_rows=0 keeps the scattered-atomic count (cooc.hip).
bool GpuMiner::pair_rows_ok(int64_t F) const {
  static const long long env_dflt = [] {
    const char* e = std::getenv("KMLS_PAIR_ROWS");
    return e ? std::atoll(e) : 1ll;
  }();
  return test_hook("pair_rows", env_dflt) != 0 && F >= 2 && F <= kern::kSparseMaxF &&
         !subset_active();
}

bool GpuMiner::pair_rows_count(uint32_t* gram, int64_t ld) {
  hipStream_t s = (hipStream_t)stream_;
  if (!prows_) prows_ = std::make_shared<kern::PairRows>();
  auto* P = static_cast<kern::PairRows*>(prows_.get());
  const int64_t F = (int64_t)fi_.ids.size();
  kern::PrInput in{d_tx_ptr_, d_items_, n_tx_, n_items_, d_ids_, F, n_cus_, d_fmask_};
  {  // the frequent items' share of the global supports -> mean kept per transaction
    double sum = 0;
    for (uint32_t c : fi_.counts) sum += (double)c;
    in.kept_per_tx = sum / (double)std::max<int64_t>(global_n_tx_, 1);
  }
  Comm* c = comm_ ? comm_ : shard_comm_;
  auto wait = [&] {
    if (c) c->wait_stream(s);
    else KMLS_HIP(hipStreamSynchronize(s));
  };
  if (shard_comm_ && shard_comm_->world() > 1) {
    kern::PrShard sh{shard_comm_->rank(), shard_comm_->world(),
                     [&](const void* send, void* recv, size_t words) {
                       shard_comm_->all_gather(send, recv, words, CommDtype::U32, s);
                     }};
    return P->count(in, gram, ld, s, wait, &sh);
  }
  return P->count(in, gram, ld, s, wait);
}

bool GpuMiner::pair_counts_csr(uintptr_t out_dev, int64_t ld) {
  KMLS_HIP(hipSetDevice(device_));
  const int64_t F = (int64_t)fi_.ids.size();
  KMLS_CHECK(ld >= F, "pair_counts_csr: ld >= F");
  KMLS_CHECK(!subset_active(), "pair_counts_csr: a use_frequent_subset() set is active; "
                               "select() again first");
  hipStream_t s = (hipStream_t)stream_;
  prows_fresh_ = false;
  if (pair_rows_ok(F)) {
    if (!d_cooc_) KMLS_HIP(hipMalloc((void**)&d_cooc_, 4 * sizeof(unsigned long long)));
    KMLS_HIP(hipMemsetAsync(d_cooc_ + 2, 0, sizeof(unsigned long long), s));  // cooc_check: clean
    if (pair_rows_count((uint32_t*)out_dev, ld)) {
      hl_pairs_est_ = static_cast<kern::PairRows*>(prows_.get())->pairs();  // exact now
      return prows_fresh_ = true;
    }
  }
  const CoocStats st = cooc_stats();
  if (st.max_k > (uint64_t)kern::cooc_max_k()) return false;
  KMLS_HIP(hipMemsetAsync((void*)out_dev, 0, (size_t)F * ld * sizeof(uint32_t), s));
  KMLS_HIP(hipMemsetAsync(d_cooc_ + 2, 0, sizeof(unsigned long long), s));
  kern::cooc_count(d_tx_ptr_, d_items_, n_tx_, d_rank_of_, d_fmask_, F, (uint32_t*)out_dev, ld,
                   (unsigned*)(d_cooc_ + 2), n_cus_, s);
  return true;
}

void GpuMiner::cooc_check() {
  KMLS_CHECK(d_cooc_ != nullptr, "cooc_check: no horizontal count ran");
  hipStream_t s = (hipStream_t)stream_;
  unsigned long long f = 0;
  KMLS_HIP(hipMemcpyAsync(&f, d_cooc_ + 2, sizeof f, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  KMLS_CHECK(!(f & 1ull), "cooc_count: a transaction held more frequent items than the entry "
                          "buffer (its pairs were not counted)");
  KMLS_CHECK(!(f & 2ull), "cooc_count: a transaction holds the same frequent item twice "
                          "(load_csr requires duplicate-free rows)");
}

bool GpuMiner::cooc_cheaper(int64_t F, int64_t Wp, int64_t nnz, const CoocStats& st) {
  if (st.max_k > (uint64_t)kern::cooc_max_k()) return false;
  // rates: the bit-GEMM ~2.7e15 bit-ANDs/s (config 5, profiles/r3_n_config5_w1.json.log); the
  // horizontal count ~1.5e10 pair atomics/s + two CSR passes (rank gathers) at ~5e9 items/s
  const double gemm_ms = 0.5 * (double)F * (double)F * (double)Wp * 64.0 / 2.7e12;
  const double cooc_ms = (double)st.pairs / 1.5e7 + 2.0 * (double)nnz / 5e6;
  return cooc_ms < gemm_ms;
}

// tx-DP level 2: the shard grams are summed by a reduce-scatter of row blocks (rank g owns rows
// [g*per, (g+1)*per), all F columns: (N-1)/N of the gram per rank instead of an all-reduce's
// 2(N-1)/N), each rank keeps the frequent upper entries of its rows, and one all-gather of those
// (row, col, count) triples — a few thousand at configs 3/5 — rebuilds on every rank a dense gram
// holding only the frequent pairs (the level loop reads gram[a][b] >= minsup, nothing else).
// sum_t k_t(k_t-1)/2 estimated from the first 1/16 of the shard's transactions (>= 65536)
int64_t GpuMiner::cooc_pairs_sampled() {
  hipStream_t s = (hipStream_t)stream_;
  if (n_tx_ <= 0 || fi_.ids.empty()) return 0;
  const int64_t ns = std::min<int64_t>(n_tx_, std::max<int64_t>(65536, n_tx_ / 16));
  if (!d_cooc_) KMLS_HIP(hipMalloc((void**)&d_cooc_, 4 * sizeof(unsigned long long)));
  KMLS_HIP(hipMemsetAsync(d_cooc_, 0, 2 * sizeof(unsigned long long), s));
  kern::cooc_stats(d_tx_ptr_, d_items_, ns, d_rank_of_, d_fmask_, d_cooc_, n_cus_, s);
  KMLS_HIP(hipMemcpyAsync(h_scalar_, d_cooc_, 8, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  return (int64_t)((double)h_scalar_[0] * (double)n_tx_ / (double)ns);
}

// Horizontal levels instead of bitmaps: the shard is long (>= 1024 bitmap words, as for the
// level-2 cooc choice) and the cost model picks the horizontal pair count.  Every tx-DP rank must
// take the same path (the two run different collectives): the shard votes are all-reduced.
// KMLS_HLEVELS=0 (or test hook hlevels=0) keeps the bitmap levels.
bool GpuMiner::hlevels_plan(const MineConfig& cfg, int64_t F, int64_t Wp, Comm* comm,
                            bool need_rows) {
  static const long long env_dflt = [] {
    const char* e = std::getenv("KMLS_HLEVELS");
    return e ? std::atoll(e) : 1ll;
  }();
  bool want = test_hook("hlevels", env_dflt) != 0 && cfg.level2_gram && F >= 2 &&
              F <= kern::kSparseMaxF && Wp >= 1024 && test_hook("cooc", 1) != 0 && !subset_active();
  if (want && pair_rows_ok(F)) {
    // the row count has no per-transaction bound: a sampled pair estimate feeds the cost model
    // (a full statistics pass cost as much as a tenth of the config-3 step)
    hl_pairs_est_ = cooc_pairs_sampled();
    CoocStats st;
    st.pairs = (uint64_t)hl_pairs_est_;
    st.max_k = 0;
    want = test_hook("cooc", 1) == 2 || cooc_cheaper(F, Wp, nnz_, st);
  } else if (want && need_rows) {
    want = false;  // folded into the vote below, so every rank declines together
  } else if (want) {
    const CoocStats st = cooc_stats();
    hl_pairs_est_ = (int64_t)st.pairs;
    want = st.max_k <= (uint64_t)kern::cooc_max_k() &&
           (test_hook("cooc", 1) == 2 || cooc_cheaper(F, Wp, nnz_, st));
  }
  if (comm && comm->world() > 1) {
    hipStream_t s = (hipStream_t)stream_;
    const size_t mark = arena_->mark();
    uint32_t* d = (uint32_t*)arena_->push(256);
    const uint32_t v = want ? 1u : 0u;
    KMLS_HIP(hipMemcpyAsync(d, &v, 4, hipMemcpyHostToDevice, s));
    comm->all_reduce(d, d, 1, CommDtype::U32, false, s);
    KMLS_HIP(hipMemcpyAsync(h_scalar_, d, 4, hipMemcpyDeviceToHost, s));
    comm->wait_stream(s);
    arena_->pop_to(mark);
    want = (int)((uint32_t*)h_scalar_)[0] == comm->world();
  }
  return want;
}

void GpuMiner::txdp_gram_combine(uint32_t* gram, int64_t F, int64_t per, uint32_t minsup) {
  hipStream_t s = (hipStream_t)stream_;
  const int W = comm_->world(), R = comm_->rank();
  if (!d_cooc_) KMLS_HIP(hipMalloc((void**)&d_cooc_, 4 * sizeof(unsigned long long)));
  const size_t mark = arena_->mark();
  uint32_t* rows = (uint32_t*)arena_->push((size_t)std::max<int64_t>(per, 1) * F * sizeof(uint32_t));
  comm_->reduce_scatter(gram, rows, (size_t)per * F, CommDtype::U32, false, s);
  const int64_t r0 = std::min<int64_t>(F, (int64_t)R * per);
  const int64_t nrows = std::max<int64_t>(0, std::min<int64_t>(F, r0 + per) - r0);
  KMLS_HIP(hipMemsetAsync(d_cooc_, 0, sizeof(unsigned long long), s));
  kern::gram_frequent(rows, F, r0, nrows, F, minsup, d_cooc_, nullptr, s);
  // every rank's count -> the padded triple block size
  uint64_t* d_n = (uint64_t*)arena_->push((size_t)W * sizeof(uint64_t));
  comm_->all_gather(d_cooc_, d_n, 1, CommDtype::U64, s);
  std::vector<uint64_t> ns((size_t)W);
  KMLS_HIP(hipMemcpyAsync(ns.data(), d_n, (size_t)W * 8, hipMemcpyDeviceToHost, s));
  comm_->wait_stream(s);
  const uint64_t cap = std::max<uint64_t>(1, *std::max_element(ns.begin(), ns.end()));
  uint32_t* mine = (uint32_t*)arena_->push((size_t)cap * 3 * sizeof(uint32_t));
  uint32_t* all = (uint32_t*)arena_->push((size_t)cap * 3 * W * sizeof(uint32_t));
  KMLS_HIP(hipMemsetAsync(mine, 0, (size_t)cap * 3 * sizeof(uint32_t), s));
  KMLS_HIP(hipMemsetAsync(d_cooc_, 0, sizeof(unsigned long long), s));
  kern::gram_frequent(rows, F, r0, nrows, F, minsup, d_cooc_, mine, s);
  comm_->all_gather(mine, all, (size_t)cap * 3, CommDtype::U32, s);
  KMLS_HIP(hipMemsetAsync(gram, 0, (size_t)F * F * sizeof(uint32_t), s));
  kern::gram_scatter(all, (int64_t)cap * W, gram, F, s);
  KMLS_HIP(hipStreamSynchronize(s));  // the arena scratch is released below
  arena_->pop_to(mark);
}

bool GpuMiner::cooc_preferred() {
  if (words_local() < 1024 || fi_.ids.empty() || subset_active()) return false;
  const long long h = test_hook("cooc", 1);
  if (h == 0) return false;
  const CoocStats st = cooc_stats();
  if (st.max_k > (uint64_t)kern::cooc_max_k()) return false;
  return h == 2 || cooc_cheaper((int64_t)fi_.ids.size(), words_local(), nnz_, st);
}

bool GpuMiner::cooc_likely() {
  if (words_local() < 1024 || fi_.ids.empty() || subset_active()) return false;
  const long long h = test_hook("cooc", 1);
  if (h == 0) return false;
  if (h == 2) return true;
  double sum = 0;
  for (uint32_t c : fi_.counts) sum += (double)c;
  const double kbar = sum / (double)std::max<int64_t>(global_n_tx_, 1);
  CoocStats st;
  // sum_t k_t(k_t-1)/2 ~ T kbar^2 / 2 (x1.5 for the spread of k_t: the model's margin)
  st.pairs = (uint64_t)(1.5 * (double)n_tx_ * kbar * kbar / 2.0);
  st.max_k = 0;
  return cooc_cheaper((int64_t)fi_.ids.size(), words_local(), nnz_, st);
}

bool GpuMiner::pair_counts_csr_direct(uintptr_t out_dev, int64_t ld) {
  KMLS_HIP(hipSetDevice(device_));
  const int64_t F = (int64_t)fi_.ids.size();
  KMLS_CHECK(ld >= F, "pair_counts_csr_direct: ld >= F");
  KMLS_CHECK(!subset_active(), "pair_counts_csr_direct: a use_frequent_subset() set is active; "
                               "select() again first");
  hipStream_t s = (hipStream_t)stream_;
  if (!d_cooc_) KMLS_HIP(hipMalloc((void**)&d_cooc_, 4 * sizeof(unsigned long long)));
  prows_fresh_ = false;
  if (pair_rows_ok(F) && pair_rows_count((uint32_t*)out_dev, ld)) return prows_fresh_ = true;
  KMLS_HIP(hipMemsetAsync((void*)out_dev, 0, (size_t)F * ld * sizeof(uint32_t), s));
  KMLS_HIP(hipMemsetAsync(d_cooc_ + 2, 0, sizeof(unsigned long long), s));
  kern::cooc_count(d_tx_ptr_, d_items_, n_tx_, d_rank_of_, d_fmask_, F, (uint32_t*)out_dev, ld,
                   (unsigned*)(d_cooc_ + 2), n_cus_, s);
  unsigned long long f = 0;
  KMLS_HIP(hipMemcpyAsync(&f, d_cooc_ + 2, sizeof f, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  KMLS_CHECK(!(f & 2ull), "cooc_count: a transaction holds the same frequent item twice "
                          "(load_csr requires duplicate-free rows)");
  return !(f & 1ull);
}

GpuMiner::RuleMap GpuMiner::rule_map_from_gram(uintptr_t gram_dev, int64_t ld, uint32_t minsup) {
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  const int64_t F = (int64_t)fi_.ids.size();
  KMLS_CHECK(F > 0 && ld >= F, "rule_map_from_gram: select() first, ld >= F");
  KMLS_CHECK(!subset_active(), "rule_map_from_gram: a use_frequent_subset() set is active; "
                               "select() again first");
  if (!big_lds_) {
    kern::pairs_enable_big_lds();
    big_lds_ = true;
  }
  // exact entry count first (2 x the frequent pairs), so one pass fills buffers of that size
  const int64_t I = n_items_;
  std::vector<void*> bufs;
  auto dalloc = [&](size_t b) {
    void* p = nullptr;
    KMLS_HIP(hipMalloc(&p, std::max<size_t>(b, 256)));
    bufs.push_back(p);
    return p;
  };
  RuleMap out;
  try {
    int64_t cap = std::max<int64_t>(F, 1024);
    for (int attempt = 0; attempt < 3; ++attempt) {
      for (void* p : bufs) (void)hipFree(p);
      bufs.clear();
      kern::PairsArgs pa{};
      pa.gram = (const uint32_t*)gram_dev;
      pa.ld = ld;
      pa.dF = nullptr;
      pa.F_host = F;
      pa.F_max = F;
      pa.minsup = minsup;
      pa.ids = d_ids_;
      pa.rank_of = d_rank_of_;
      pa.n_items = I;
      pa.tie = d_tie_;
      pa.inv_tie = d_inv_tie_;
      pa.scratch_bytes = kern::pairs_scratch_bytes(F, I);
      pa.scratch = dalloc(pa.scratch_bytes);
      pa.row_ptr = (int64_t*)dalloc((size_t)(I + 1) * 8);
      pa.ent = (unsigned long long*)dalloc((size_t)cap * 8);
      pa.ent_cap = cap;
      pa.cons = (int32_t*)dalloc((size_t)cap * 4);
      pa.cnt = (uint32_t*)dalloc((size_t)cap * 4);
      pa.host = nullptr;
      kern::pairs_to_csr(pa, s);
      out.row_ptr.resize((size_t)I + 1);
      KMLS_HIP(hipMemcpyAsync(out.row_ptr.data(), pa.row_ptr, (size_t)(I + 1) * 8,
                              hipMemcpyDeviceToHost, s));
      KMLS_HIP(hipMemcpyAsync(&out.status, pa.scratch, 4, hipMemcpyDeviceToHost, s));
      KMLS_HIP(hipStreamSynchronize(s));
      out.nnz = out.row_ptr[(size_t)I];
      if (out.nnz > cap && (out.status & 1u)) {  // sized from the exact total, retry once
        cap = out.nnz;
        continue;
      }
      out.cons.resize((size_t)out.nnz);
      out.cnt.resize((size_t)out.nnz);
      if (out.nnz) {
        KMLS_HIP(hipMemcpyAsync(out.cons.data(), pa.cons, (size_t)out.nnz * 4,
                                hipMemcpyDeviceToHost, s));
        KMLS_HIP(hipMemcpyAsync(out.cnt.data(), pa.cnt, (size_t)out.nnz * 4,
                                hipMemcpyDeviceToHost, s));
      }
      KMLS_HIP(hipStreamSynchronize(s));
      break;
    }
  } catch (...) {
    for (void* p : bufs) (void)hipFree(p);
    throw;
  }
  for (void* p : bufs) (void)hipFree(p);
  return out;
}

void GpuMiner::gram_mirror(uintptr_t gram_dev, int64_t ld, int64_t F) {
  KMLS_HIP(hipSetDevice(device_));
  KMLS_CHECK(F >= 0 && ld >= F, "gram_mirror: ld >= F");
  kern::gram_mirror((uint32_t*)gram_dev, ld, F, (hipStream_t)stream_);
}

void GpuMiner::rows_union(uintptr_t rows, int64_t Wp, uintptr_t idx, int n, int64_t W,
                          uintptr_t mask) {
  KMLS_HIP(hipSetDevice(device_));
  KMLS_CHECK(n >= 0 && W >= 0 && Wp >= W, "rows_union: Wp >= W, n >= 0");
  kern::rows_union((const uint64_t*)rows, Wp, (const int32_t*)idx, n, W, (uint64_t*)mask,
                   (hipStream_t)stream_);
}

void GpuMiner::word_popc(uintptr_t mask, int64_t W, uintptr_t cnt) {
  KMLS_HIP(hipSetDevice(device_));
  kern::word_popc((const uint64_t*)mask, W, (int32_t*)cnt, (hipStream_t)stream_);
}

void GpuMiner::compact_rows(uintptr_t rows, int64_t R, int64_t Wp_in, uintptr_t mask,
                            uintptr_t nzw, uintptr_t off, int64_t n_nz, uintptr_t out,
                            int64_t Wp_out) {
  KMLS_HIP(hipSetDevice(device_));
  KMLS_CHECK(R >= 0 && n_nz >= 0 && n_nz <= Wp_in && Wp_out * 64 >= 0,
             "compact_rows: bad shape");
  kern::compact_rows((const uint64_t*)rows, R, Wp_in, (const uint64_t*)mask,
                     (const int64_t*)nzw, (const int64_t*)off, n_nz, (uint64_t*)out, Wp_out,
                     (hipStream_t)stream_);
}

GpuMiner::RuleMap GpuMiner::rule_map_rows(uintptr_t rows_dev, int64_t ld, int64_t r0, int64_t nrows,
                                          uint32_t minsup) {
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  const int64_t F = (int64_t)fi_.ids.size();
  KMLS_CHECK(ld >= F && r0 >= 0 && nrows >= 0 && r0 + nrows <= F,
             "rule_map_rows: select() first; rows [r0, r0 + nrows) within F, ld >= F");
  if (!big_lds_) {
    kern::pairs_enable_big_lds();
    big_lds_ = true;
  }
  RuleMap out;
  out.row_ptr.assign((size_t)nrows + 1, 0);
  if (nrows == 0) return out;
  std::vector<void*> bufs;
  auto dalloc = [&](size_t b) {
    void* p = nullptr;
    KMLS_HIP(hipMalloc(&p, std::max<size_t>(b, 256)));
    bufs.push_back(p);
    return p;
  };
  try {
    // [status, n_long] | len_r[nrows] | long_rows[nrows] | row_ptr[nrows + 1]
    char* meta = (char*)dalloc(256 + (size_t)nrows * 8 + (size_t)(nrows + 1) * 8 + 256);
    unsigned* status = (unsigned*)meta;
    unsigned* n_long = status + 1;
    uint32_t* len_r = (uint32_t*)(meta + 256);
    int32_t* long_rows = (int32_t*)(len_r + nrows);
    int64_t* row_ptr = (int64_t*)(meta + 256 + (size_t)nrows * 8);
    KMLS_HIP(hipMemsetAsync(meta, 0, 256, s));
    kern::rows_count((const uint32_t*)rows_dev, ld, nrows, F, r0, minsup, len_r, n_long, long_rows, s);
    std::vector<uint32_t> len((size_t)nrows);
    unsigned hn[2] = {0, 0};
    KMLS_HIP(hipMemcpyAsync(len.data(), len_r, (size_t)nrows * 4, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipMemcpyAsync(hn, meta, 8, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipStreamSynchronize(s));
    for (int64_t r = 0; r < nrows; ++r) out.row_ptr[(size_t)r + 1] = out.row_ptr[(size_t)r] + len[(size_t)r];
    out.nnz = out.row_ptr[(size_t)nrows];
    const int64_t cap = std::max<int64_t>(out.nnz, 1);
    KMLS_HIP(hipMemcpyAsync(row_ptr, out.row_ptr.data(), (size_t)(nrows + 1) * 8,
                            hipMemcpyHostToDevice, s));
    auto* ent = (unsigned long long*)dalloc((size_t)cap * 8);
    auto* cons = (int32_t*)dalloc((size_t)cap * 4);
    auto* cnt = (uint32_t*)dalloc((size_t)cap * 4);
    kern::rows_fill_sort((const uint32_t*)rows_dev, ld, nrows, F, r0, minsup, d_ids_, d_tie_,
                         d_inv_tie_, len_r, row_ptr, ent, cap, cons, cnt, status, n_long,
                         long_rows, hn[1] > 0, s);
    out.cons.resize((size_t)out.nnz);
    out.cnt.resize((size_t)out.nnz);
    if (out.nnz) {
      KMLS_HIP(hipMemcpyAsync(out.cons.data(), cons, (size_t)out.nnz * 4, hipMemcpyDeviceToHost, s));
      KMLS_HIP(hipMemcpyAsync(out.cnt.data(), cnt, (size_t)out.nnz * 4, hipMemcpyDeviceToHost, s));
    }
    KMLS_HIP(hipMemcpyAsync(&out.status, status, 4, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipStreamSynchronize(s));
  } catch (...) {
    for (void* p : bufs) (void)hipFree(p);
    throw;
  }
  for (void* p : bufs) (void)hipFree(p);
  return out;
}

void GpuMiner::ring_pair_rows(Comm* comm, uintptr_t X, int64_t F, int64_t Ws, uintptr_t out,
                              int64_t ldo) {
  KMLS_HIP(hipSetDevice(device_));
  KMLS_CHECK(comm != nullptr && F >= 0 && Ws >= 0 && ldo >= F, "ring_pair_rows: comm, ldo >= F");
  hipStream_t s = (hipStream_t)stream_;
  const int W = comm->world(), R = comm->rank();
  const int64_t fb = (F + W - 1) / std::max(W, 1);
  const int64_t r0 = std::min<int64_t>(F, (int64_t)R * fb), r1 = std::min<int64_t>(F, r0 + fb);
  KMLS_HIP(hipMemsetAsync((void*)out, 0, (size_t)std::max<int64_t>(r1 - r0, 0) * ldo * 4, s));
  const uint64_t* x = (const uint64_t*)X;
  if (W == 1) {
    kern::bitgemm_rect(x + r0 * Ws, r1 - r0, x, F, Ws, (uint32_t*)out, ldo, s);
    return;
  }
  if (!comm_s_) KMLS_HIP(hipStreamCreateWithFlags((hipStream_t*)&comm_s_, hipStreamNonBlocking));
  hipStream_t cs = (hipStream_t)comm_s_;
  const size_t blk = (size_t)F * (size_t)Ws;
  const size_t mark = arena_->mark();
  uint64_t* buf[2] = {(uint64_t*)arena_->push(std::max<size_t>(blk, 1) * 8),
                      (uint64_t*)arena_->push(std::max<size_t>(blk, 1) * 8)};
  Event ready, comp, recv;  // shard X written (encode on s) / count k done / shard k+1 landed
  KMLS_HIP(hipEventRecord(ready.e, s));
  KMLS_HIP(hipStreamWaitEvent(cs, ready.e, 0));
  const uint64_t* cur = x;
  for (int k = 0; k < W; ++k) {
    uint64_t* nxt = buf[k & 1];
    if (k + 1 < W) {
      // nxt was the block counted at step k - 1: its count must be done before it is overwritten
      if (k > 0) KMLS_HIP(hipStreamWaitEvent(cs, comp.e, 0));
      comm->sendrecv(cur, (R + 1) % W, nxt, (R + W - 1) % W, blk, CommDtype::U64, cs);
      KMLS_HIP(hipEventRecord(recv.e, cs));
    }
    kern::bitgemm_rect(cur + r0 * Ws, r1 - r0, cur, F, Ws, (uint32_t*)out, ldo, s);
    KMLS_HIP(hipEventRecord(comp.e, s));
    if (k + 1 < W) {
      KMLS_HIP(hipStreamWaitEvent(s, recv.e, 0));
      cur = nxt;
    }
  }
  KMLS_HIP(hipStreamSynchronize(s));  // the scratch shards are released below
  comm->wait_stream(cs);
  arena_->pop_to(mark);
}

void GpuMiner::bitgemm_rect(uintptr_t A, int64_t Fa, uintptr_t B, int64_t Fb, int64_t Wp,
                            uintptr_t C, int64_t ldc) {
  KMLS_HIP(hipSetDevice(device_));
  kern::bitgemm_rect((const uint64_t*)A, Fa, (const uint64_t*)B, Fb, Wp, (uint32_t*)C, ldc,
                     (hipStream_t)stream_);
}

GpuMineResult GpuMiner::mine_bitmaps(uintptr_t bm_dev, int64_t Wp, const MineConfig& cfg,
                                     const uint8_t* owned_mask, bool emit_level1,
                                     bool download) {
  drain_prefetch();  // a launched-ahead resident call shares the device buffers
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  GpuMineResult res;
  const int64_t F = (int64_t)fi_.ids.size();
  Event e0, e1, e2, e3;
  const size_t mark = arena_->mark();
  KMLS_HIP(hipEventRecord(e0.e, s));
  std::unique_ptr<MineRun> runp;
  for (int attempt = 0;; ++attempt) {
  if (!out_) out_ = std::make_unique<OutBufs>();
  runp = std::make_unique<MineRun>(out_.get());
  MineRun& run = *runp;
  run.comm = comm_;
  run.n_cus = n_cus_;
  run.s = s;
  run.arena = arena_.get();
  run.Wp = Wp;
  run.minsup = fi_.minsup2;
  run.max_len = cfg.pairs_only ? 2 : cfg.max_len;
  run.d_ids = d_ids_;
  run.F = F;
  run.h_scalar = h_scalar_;  // persistent: a per-call hipHostFree costs ~200 us (it syncs)
  run.d_pair = d_pair_;
  // level-1 nodes: gid = Eclat rank
  run.ensure_out(std::max<int64_t>({F * 8, (int64_t)1 << 16, last_nodes_ + (last_nodes_ >> 3)}));
  if (download) {  // pinned host arrays sized from the previous trie; levels stream into them
    run.host_cap = std::max<int64_t>({F * 8, (int64_t)1 << 16, last_nodes_ + (last_nodes_ >> 3)});
    res.h_parent = pinned_->get((size_t)run.host_cap * sizeof(int64_t));
    res.h_item = pinned_->get((size_t)run.host_cap * sizeof(int32_t));
    res.h_count = pinned_->get((size_t)run.host_cap * sizeof(uint32_t));
    res.h_depth = pinned_->get((size_t)run.host_cap * sizeof(uint8_t));
    run.ht = kern::HostTrie{res.h_parent.get(), res.h_item.get(), res.h_count.get(),
                            (uint8_t*)res.h_depth.get(), run.host_cap, 8, 4, 4};
    run.stream_dl = true;
  }
  {
    std::vector<int64_t> par((size_t)F, -1);
    std::vector<uint8_t> dep((size_t)F, 1);
    if (F) {
      KMLS_HIP(hipMemcpyAsync(run.out_parent.p, par.data(), F * sizeof(int64_t), hipMemcpyHostToDevice, s));
      KMLS_HIP(hipMemcpyAsync(run.out_item.p, fi_.ids.data(), F * sizeof(int32_t), hipMemcpyHostToDevice, s));
      KMLS_HIP(hipMemcpyAsync(run.out_count.p, fi_.counts.data(), F * sizeof(uint32_t), hipMemcpyHostToDevice, s));
      KMLS_HIP(hipMemcpyAsync(run.out_depth.p, dep.data(), F * sizeof(uint8_t), hipMemcpyHostToDevice, s));
      KMLS_HIP(hipStreamSynchronize(s));  // par/dep are pageable and die at scope end
    }
    run.out_size = F;
    run.stream_out();
  }
  if (F >= 2 && run.max_len != 1) {
    // root level: one class of all F frequent items
    std::vector<int32_t> rank((size_t)F), row_end((size_t)F, (int32_t)F);
    std::vector<int64_t> gid((size_t)F), root_len((size_t)F + 1, 0);
    int64_t root_total = 0;
    for (int64_t a = 0; a < F; ++a) {
      rank[a] = (int32_t)a;
      gid[a] = a;
      const bool own = owned_mask == nullptr || owned_mask[a];
      root_len[a] = own ? (F - a - 1) : 0;
      root_total += root_len[a];
    }
    int32_t* d_rank = (int32_t*)arena_->push(F * sizeof(int32_t));
    int64_t* d_gid = (int64_t*)arena_->push(F * sizeof(int64_t));
    int32_t* d_end = (int32_t*)arena_->push(F * sizeof(int32_t));
    KMLS_HIP(hipMemcpyAsync(d_rank, rank.data(), F * sizeof(int32_t), hipMemcpyHostToDevice, s));
    KMLS_HIP(hipMemcpyAsync(d_gid, gid.data(), F * sizeof(int64_t), hipMemcpyHostToDevice, s));
    KMLS_HIP(hipMemcpyAsync(d_end, row_end.data(), F * sizeof(int32_t), hipMemcpyHostToDevice, s));
    int64_t* d_len = (int64_t*)arena_->push((F + 1) * sizeof(int64_t));
    KMLS_HIP(hipMemcpyAsync(d_len, root_len.data(), (F + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    // level 2 through the bit-GEMM (LDS-tiled, 64x64 tiles) when the dense F x F fits
    if (F <= kern::kSparseMaxF && cfg.level2_gram) {
      // tx-DP: room for world row blocks of `per` rows (the reduce-scatter's send layout)
      const int cw = comm_ ? comm_->world() : 1;
      const int64_t per = (F + cw - 1) / cw;
      uint32_t* gram = (uint32_t*)arena_->push((size_t)std::max<int64_t>(per * cw, F) * F * sizeof(uint32_t));
      if (per * cw > F)
        KMLS_HIP(hipMemsetAsync(gram + (size_t)F * F, 0, (size_t)(per * cw - F) * F * sizeof(uint32_t), s));
      // sparse large data: count the pairs where they occur (pairrows.hip, cooc.hip fallback) when the cost model says
      // so (only for bitmaps of this miner's own CSR shard: mine_txdp / the host path of mine)
      bool sparse = false;
      if (hl_plan_) {  // decided (globally) before the encode: there is no bitmap
        sparse = true;
        res.level2_method = "cooc";
        res.cooc_pairs = hl_pairs_est_;
      } else if (gram_csr_ok_ && Wp >= 1024 && test_hook("cooc", 1) != 0) {
        const CoocStats st = cooc_stats();
        sparse = test_hook("cooc", 1) == 2 || cooc_cheaper(F, Wp, nnz_, st);
        res.level2_method = sparse ? "cooc" : "gram";
        res.cooc_pairs = (int64_t)st.pairs;
      }
      if (!(sparse && pair_counts_csr((uintptr_t)gram, F))) {
        if (hl_plan_) throw std::logic_error("kmls: horizontal plan but cooc declined");
        if (sparse) res.level2_method = "gram (cooc declined)";
        KMLS_HIP(hipMemsetAsync(gram, 0, (size_t)F * F * sizeof(uint32_t), s));
        // matrix cores for long rows (large T): the masked-nibble FP4 MFMA gram
        // (v_mfma_scale_f32_32x32x64_f8f6f4, gram_mfma.hip) beats the VALU popcount gram there.
        // No BASELINE config reaches this branch today: ds1 rows are short (popcount gram),
        // configs 3 and 5 count pairs horizontally (pairrows.hip)
        const bool mfma = gram_popcount_forced() ? cfg.level2_mfma : (cfg.level2_mfma || Wp >= 4096);
        if (mfma)
          kern::pair_gram_mfma((const uint64_t*)bm_dev, Wp, F, gram, s);
        else
          kern::pair_gram_popcount((const uint64_t*)bm_dev, Wp, F, gram, s);
        if (res.level2_method.empty() || res.level2_method == "gram")
          res.level2_method = mfma ? "gram_mfma" : "gram_popcount";
      }
      if (hl_plan_) res.cooc_pairs = hl_pairs_est_;  // exact after the row count
      if (comm_ && cw > 1) {
        txdp_gram_combine(gram, F, per, run.minsup);
        res.level2_comm = "reduce_scatter+frequent_allgather";
      } else if (comm_) {
        comm_->all_reduce(gram, gram, (size_t)F * F, CommDtype::U32, false, s);
      }
      run.gram = gram;
    }
    KMLS_HIP(hipEventRecord(e1.e, s));
    Level root;
    root.n = F;
    root.bm = (const uint64_t*)bm_dev;
    root.rank = d_rank;
    root.gid = d_gid;
    root.row_end = d_end;
    bool done = false;
    if (hl_plan_) {
      // levels >= 2 from the gram and a filtered CSR (hlevels.hip): no bitmap anywhere
      if (!hl_) hl_ = std::make_shared<kern::HLevels>();
      auto* H = static_cast<kern::HLevels*>(hl_.get());
      kern::HlInput in{d_tx_ptr_, d_items_, n_tx_, n_items_, d_rank_of_, d_fmask_, d_ids_, run.gram, F, F,
                       run.minsup, run.max_len, n_cus_};
      kern::HlHooks hk;
      hk.reserve = [&](int64_t n) {
        run.ensure_out(run.out_size + n);
        return kern::HlTrieOut{run.out_parent.p, run.out_item.p, run.out_count.p,
                               run.out_depth.p, run.out_size, nullptr};
      };
      hk.commit = [&](int64_t n) {
        run.out_size += n;
        run.stream_out();
      };
      if (comm_)
        hk.allreduce = [&](uint32_t* c, int64_t n) {
          comm_->all_reduce(c, c, (size_t)n, CommDtype::U32, false, s);
        };
      hk.wait = [&]() {
        if (comm_) comm_->wait_stream(s);
        else KMLS_HIP(hipStreamSynchronize(s));
      };
      if (prows_ && prows_fresh_) {  // level 2 came from the row count: reuse its rank CSR
        auto* P = static_cast<kern::PairRows*>(prows_.get());
        in.f_txrec = P->txrec();
        in.f_fit = P->fit();
        in.f_rows = P->n_rows();
      }
      kern::HlStats hs;
      H->run(in, hk, s, hs);
      run.max_depth = hs.max_depth;
      run.n_candidates = hs.candidates;
      res.hl_tx_kept = hs.n_tx_kept;
      res.hl_nnz_kept = hs.nnz_kept;
      res.hl_per_level = hs.per_level;
      res.hl_hits = hs.hits;
      done = true;
    } else if (comm_ == nullptr && fused_levels_enabled()) {
      // the fused levels take the root rows in descending rank, each owning its pairs with
      // the rows before it (levels.hip header): row r = rank F-1-r, root class of rank F-1-r
      std::vector<int32_t> rrank((size_t)F);
      std::vector<int64_t> rgid((size_t)F), off((size_t)F + 1, 0);
      for (int64_t r = 0; r < F; ++r) {
        rrank[(size_t)r] = (int32_t)(F - 1 - r);
        rgid[(size_t)r] = F - 1 - r;
        off[(size_t)r + 1] = off[(size_t)r] + (root_len[(size_t)(F - 1 - r)] ? r : 0);
      }
      int32_t* d_rrank = (int32_t*)arena_->push(F * sizeof(int32_t));
      int64_t* d_rgid = (int64_t*)arena_->push(F * sizeof(int64_t));
      KMLS_HIP(hipMemcpyAsync(d_rrank, rrank.data(), F * sizeof(int32_t), hipMemcpyHostToDevice, s));
      KMLS_HIP(hipMemcpyAsync(d_rgid, rgid.data(), F * sizeof(int64_t), hipMemcpyHostToDevice, s));
      Level froot = root;
      froot.rank = d_rrank;
      froot.gid = d_rgid;
      run.pinned = pinned_;
      run.fast_hint = std::max<int64_t>({last_nodes_ + (last_nodes_ >> 2), 16ll << 20, fused_need_});
      done = run.run_fast(froot, off, off[(size_t)F]);
      fused_need_ = std::max(fused_need_, run.need_nodes);
      KMLS_HIP(hipStreamSynchronize(s));  // the pageable staging vectors die at scope end
    }
    if (!done) run.process(root, 1, d_len, root_total);
    res.levels_path = hl_plan_ ? "horizontal" : done ? "fused" : (comm_ ? "chunked-txdp" : "chunked");
    if (!done && !run.fallback_reason.empty()) res.levels_path += " (fused fallback: " + run.fallback_reason + ")";
    KMLS_HIP(hipStreamSynchronize(s));  // host staging vectors die at scope end
    if (res.level2_method == "cooc") cooc_check();
  } else {
    KMLS_HIP(hipEventRecord(e1.e, s));
  }
  break;  // one pass (the loop scopes the run's state)
  }
  MineRun& run = *runp;
  KMLS_HIP(hipEventRecord(e2.e, s));
  const int64_t N = run.out_size;
  res.n_nodes = N;
  last_nodes_ = N;
  // the overflow hint is a high-water mark of one (earlier, larger) problem: a call that fit
  // with 8x room to spare releases it, so later small calls stop sizing for that one
  if (run.need_nodes == 0 && N < (fused_need_ >> 3)) fused_need_ = 0;
  if (download && run.stream_dl) {
    run.stream_out();  // tail (normally empty: every chunk streamed itself)
  } else if (download) {  // the trie outgrew the pinned arrays: one full copy
    KMLS_HIP(hipStreamSynchronize(out_->copy_s));
    res.h_parent = pinned_->get((size_t)N * sizeof(int64_t));
    res.h_item = pinned_->get((size_t)N * sizeof(int32_t));
    res.h_count = pinned_->get((size_t)N * sizeof(uint32_t));
    res.h_depth = pinned_->get((size_t)N * sizeof(uint8_t));
    if (N) {
      KMLS_HIP(hipMemcpyAsync(res.h_parent.get(), run.out_parent.p, N * sizeof(int64_t), hipMemcpyDeviceToHost, s));
      KMLS_HIP(hipMemcpyAsync(res.h_item.get(), run.out_item.p, N * sizeof(int32_t), hipMemcpyDeviceToHost, s));
      KMLS_HIP(hipMemcpyAsync(res.h_count.get(), run.out_count.p, N * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      KMLS_HIP(hipMemcpyAsync(res.h_depth.get(), run.out_depth.p, N * sizeof(uint8_t), hipMemcpyDeviceToHost, s));
    }
  }
  KMLS_HIP(hipEventRecord(e3.e, s));
  KMLS_HIP(hipStreamSynchronize(s));
  KMLS_HIP(hipStreamSynchronize(out_->copy_s));
  res.phases.push_back({"level2_gram", elapsed(e0, e1)});
  res.phases.push_back({"levels_3plus", elapsed(e1, e2)});
  res.phases.push_back({"download", elapsed(e2, e3)});
  res.stats.n_frequent_items = F;
  res.stats.n_itemsets = emit_level1 ? N : N - F;
  res.stats.n_candidates = run.n_candidates;
  res.stats.max_depth = F ? run.max_depth : 0;
  res.arena_high_water = (int64_t)arena_->high_water();
  arena_->pop_to(mark);
  return res;
}


// Single-GPU mining with a device-resident prologue: supports, frequent-item selection, bitmap
// encode, level-2 gram and the root descriptor are all produced on the device, so together with
// the fused level loop one mining call has no host round trip before the final one.  Returns
// false (nothing committed) when the fused loop overflowed; mine() then runs the host path.
bool GpuMiner::mine_resident(const MineConfig& cfg, bool download, GpuMineResult& res, int part_rank,
                             int part_world, bool prefetch) {
  hipStream_t s = (hipStream_t)stream_;
  trace::Range rg_call("kmls.mine_resident");
  auto t0 = std::chrono::steady_clock::now();
  // a call launched ahead by the previous mine(prefetch): adopted below if its launch key matches
  std::unique_ptr<Prefetch> adopt = std::move(pre_);
  struct AdoptGuard {  // leaving with an un-consumed launched-ahead call (exception, early
    hipStream_t s;     // return): wait for it before its pinned buffers go back to the pool
    std::unique_ptr<Prefetch>& a;
    ~AdoptGuard() {
      if (a) (void)hipStreamSynchronize(s);
    }
  } adopt_guard{s, adopt};
  const int64_t I = n_items_;
  const int64_t Wp = words_local();
  constexpr int kMaxLv = 64;
  Event e0, e1, e2;
  KMLS_HIP(hipEventRecord(e0.e, s));
  const size_t mark = arena_->mark();
  uint32_t* d_cnt = (uint32_t*)arena_->push((size_t)I * 4);
  const int64_t tab_stride = (I + 63) & ~(int64_t)63;  // ids | counts | rank_of, one D2H copy
  int32_t* d_ids = (int32_t*)arena_->push((size_t)tab_stride * 12);
  uint32_t* d_fcnt = (uint32_t*)(d_ids + tab_stride);
  int32_t* d_rank_of = d_ids + 2 * tab_stride;
  uint32_t* d_gram = (uint32_t*)arena_->push((size_t)I * I * 4);
  int32_t* d_rrank = (int32_t*)arena_->push((size_t)I * 4);
  int64_t* d_rgid = (int64_t*)arena_->push((size_t)I * 8);
  int64_t* d_roff = (int64_t*)arena_->push((size_t)(I + 1) * 8);
  int32_t* d_m = (int32_t*)arena_->push((size_t)I * 4);         // gram-driven root (levels.hip)
  int64_t* d_soff = (int64_t*)arena_->push((size_t)(I + 1) * 8);
  int64_t* d_coff = (int64_t*)arena_->push((size_t)(I + 1) * 8);
  kern::FLevel* d_desc = (kern::FLevel*)arena_->push(kMaxLv * sizeof(kern::FLevel));
  kern::FCtl* d_ctl = (kern::FCtl*)arena_->push(sizeof(kern::FCtl));
  // rule map (O10 pairs_to_csr) scratch and output, from the same arena
  kern::PairsArgs pa{};
  const int64_t icap = idx_cap_;
  if (cfg.rule_index) {
    if (!big_lds_) {
      kern::pairs_enable_big_lds();
      big_lds_ = true;
    }
    if (!idx_scan_bytes_) idx_scan_bytes_ = kern::pairs_scratch_bytes(I, I);
    pa.gram = d_gram;
    pa.ld = I;
    pa.dF = &d_desc[1].n_rows;
    pa.F_max = I;
    pa.minsup = level2_threshold((uint64_t)n_tx_, cfg.min_support);
    pa.ids = d_ids;
    pa.rank_of = d_rank_of;
    pa.n_items = I;
    pa.tie = d_tie_;
    pa.inv_tie = d_inv_tie_;
    pa.scratch = arena_->push(idx_scan_bytes_);
    pa.scratch_bytes = idx_scan_bytes_;
    pa.row_ptr = (int64_t*)arena_->push((size_t)(I + 1) * 8);
    pa.ent = (unsigned long long*)arena_->push((size_t)icap * 8);
    pa.ent_cap = icap;
    pa.cons = (int32_t*)arena_->push((size_t)icap * 4);
    pa.cnt = (uint32_t*)arena_->push((size_t)icap * 4);
    pa.host = &d_ctl->ph;
  }
  const size_t need = (size_t)std::max<int64_t>(I, 1) * Wp * sizeof(uint64_t);
  if (need > own_bm_bytes_) {
    if (d_own_bm_) KMLS_HIP(hipFree(d_own_bm_));
    KMLS_HIP(hipMalloc((void**)&d_own_bm_, need));
    own_bm_bytes_ = need;
  }
  if (!out_) out_ = std::make_unique<OutBufs>();
  MineRun run(out_.get());
  run.s = s;
  run.root_from_gram = true;  // the resident prologue builds level 2 from the gram
  run.arena = arena_.get();
  run.Wp = Wp;
  run.minsup = level2_threshold((uint64_t)n_tx_, cfg.min_support);
  run.max_len = cfg.max_len;
  run.d_ids = d_ids;
  run.F = I;  // gram row stride
  run.gram = d_gram;
  run.pinned = pinned_;
  run.n_cus = n_cus_;
  run.h_scalar = h_scalar_;
  const int64_t cap_nodes = std::max<int64_t>({last_nodes_ + (last_nodes_ >> 2), 16ll << 20, fused_need_});
  run.ensure_out(cap_nodes);
  const int64_t out_cap = std::min<int64_t>({run.out_parent.cap, run.out_item.cap, run.out_count.cap, run.out_depth.cap});
  bool adopt_bufs = adopt && !download && !adopt->download;  // the host trie it writes is ours
  if (download) {
    run.host_cap = std::max<int64_t>({I * 8, (int64_t)1 << 16, last_nodes_ + (last_nodes_ >> 3)});
    // compact element widths (kernels.hpp HostTrie): the download is PCIe-bound on the
    // headline shape (0.25 ms of 1.1 ms at 17 B/itemset)
    constexpr bool compact = true;
    const int pw = compact && run.host_cap < (int64_t)INT32_MAX ? 4 : 8;
    const int iw = compact && I <= 65536 ? 2 : 4;
    const int cw = compact && n_tx_ <= 65535 ? 2 : 4;
    adopt_bufs = adopt && adopt->download && adopt->host_cap == run.host_cap && adopt->pw == pw &&
                 adopt->iw == iw && adopt->cw == cw;
    if (adopt_bufs) {
      res.h_parent = adopt->h_parent;
      res.h_item = adopt->h_item;
      res.h_count = adopt->h_count;
      res.h_depth = adopt->h_depth;
    } else {
      res.h_parent = pinned_->get((size_t)run.host_cap * pw);
      res.h_item = pinned_->get((size_t)run.host_cap * iw);
      res.h_count = pinned_->get((size_t)run.host_cap * cw);
      res.h_depth = pinned_->get((size_t)run.host_cap * sizeof(uint8_t));
    }
    run.ht = kern::HostTrie{res.h_parent.get(), res.h_item.get(), res.h_count.get(),
                            (uint8_t*)res.h_depth.get(), run.host_cap, pw, iw, cw};
    res.par_w = pw;
    res.item_w = iw;
    res.cnt_w = cw;
    run.stream_dl = true;
  }
  const size_t rem = arena_->capacity() - arena_->used();
  if (rem < (512ull << 20)) {
    if (adopt) KMLS_HIP(hipStreamSynchronize(s));
    arena_->pop_to(mark);
    res = GpuMineResult();
    return false;
  }
  const size_t bump_bytes = fused_bump_cap(rem - (64ull << 20));
  char* bump_base = (char*)arena_->push(bump_bytes);
  // prologue, all on the device: one init launch (histogram + bitmap buffer zeroed, level
  // descriptors zeroed, control block set), supports, selection (small vocabularies: one launch
  // that also writes the frequent-item tables to pinned host memory), bitmaps, gram
  // frequent-item tables for the frequent() API (ids | counts | rank_of, tab_stride apart)
  const size_t back_bytes = kMaxLv * sizeof(kern::FLevel) + sizeof(kern::FCtl);
  std::shared_ptr<void> fstage = adopt ? adopt->fstage : pinned_->get((size_t)tab_stride * 12);
  run.back = adopt ? adopt->back : pinned_->get(back_bytes);
  // pinned rule-map CSR of this call (the launched-ahead call gets its own set)
  struct IdxHost {
    std::shared_ptr<void> rp, cons, cnt, meta;
    kern::PairsHost ph() const {
      if (!meta) return kern::PairsHost{};
      return kern::PairsHost{(int64_t*)rp.get(), (int32_t*)cons.get(), (uint32_t*)cnt.get(), cap,
                             (int64_t*)meta.get()};
    }
    int64_t cap = 0;
  };
  auto new_idx_host = [&]() {
    IdxHost h;
    if (cfg.rule_index) {
      h.cap = icap;
      h.rp = pinned_->get((size_t)(I + 1) * 8);
      h.cons = pinned_->get((size_t)icap * 4);
      h.cnt = pinned_->get((size_t)icap * 4);
      h.meta = pinned_->get(64);
    }
    return h;
  };
  IdxHost ih;
  if (adopt && cfg.rule_index && adopt->i_meta) {
    ih.rp = adopt->i_rp;
    ih.cons = adopt->i_cons;
    ih.cnt = adopt->i_cnt;
    ih.meta = adopt->i_meta;
    ih.cap = icap;
  } else {
    ih = new_idx_host();
  }
  // the control block of a call: slot (call index & 1) of the pinned parameter pair (the init
  // kernel copies it into d_ctl); `bump`/`status` are the same for every call
  auto fill_params = [&](kern::FCtl& init, const kern::HostTrie& ht, void* tab, void* back,
                         const IdxHost& ixh) {
    std::memset(&init, 0, sizeof(init));
    init.ph = ixh.ph();
    init.bump_base = bump_base;
    init.bump_cap = bump_bytes;
    init.status_cap = (unsigned long long)out_->status_cap;
    init.epoch_base = out_->begin_call(s);
    init.h = ht;
    init.host_tab = (int32_t*)tab;
    init.tab_stride = tab_stride;
    init.rb_dst = back;
  };
  const auto t_launch = std::chrono::steady_clock::now();
  const uint32_t c1 = level1_threshold((uint64_t)n_tx_, cfg.min_support);
  const bool fused_select = I <= kern::kSelectFusedMax;
  // The call's launches (prologue + the first batch of levels) are invariant once the data,
  // configuration, buffers and per-level launch plan repeat: they are captured once as a
  // hipGraph and replayed, which takes ~35 kernel launches off the host path of every
  // steady-state call (level tracing runs uncaptured).  All per-call state reaches the kernels
  // through the pinned parameter block read by the init kernel.
  static const bool tracing = std::getenv("KMLS_LEVEL_TRACE") != nullptr;
  const bool use_graph = fused_select && !tracing;
  std::vector<uint64_t> key;
  if (use_graph) {
    auto u = [](const void* p) { return (uint64_t)(uintptr_t)p; };
    key = {u(d_desc), u(d_cnt), u(d_own_bm_), (uint64_t)need, u(d_items_), u(d_tx_ptr_),
           (uint64_t)nnz_, (uint64_t)n_tx_, (uint64_t)I, (uint64_t)Wp, run.minsup, c1,
           (uint64_t)cfg.max_len, (uint64_t)run.stream_dl, (uint64_t)deferred_dl(), (uint64_t)copy_blocks(), (uint64_t)copy_last(),
           (uint64_t)part_rank, (uint64_t)part_world, u(run.out_parent.p), u(run.out_item.p),
           u(run.out_count.p), u(run.out_depth.p), (uint64_t)out_cap, u(out_->status),
           u(out_->tile_row), (uint64_t)n_cus_, (uint64_t)out_->depth_hint, u(call_params_),
           (uint64_t)out_->cand_hint.size()};
    for (int64_t v : out_->cand_hint) key.push_back((uint64_t)v);
    key.push_back((uint64_t)cfg.rule_index);
    if (cfg.rule_index) {
      key.push_back((uint64_t)icap);
      key.push_back(u(pa.ent));
      key.push_back(u(pa.scratch));
      key.push_back(u(d_tie_));
    }
  }
  const bool replay = use_graph && graph_ && graph_->exec && graph_->key == key;
  // the rule map forks off the captured prologue (joined before the capture ends)
  const bool fork_idx = cfg.rule_index && use_graph && !replay;
  if (fork_idx && !idx_s_) {
    KMLS_HIP(hipStreamCreateWithFlags((hipStream_t*)&idx_s_, hipStreamNonBlocking));
    for (auto& e : idx_ev_) KMLS_HIP(hipEventCreateWithFlags((hipEvent_t*)&e, hipEventDisableTiming));
  }
  // Node order of the captured graph: the rule-map branch depends only on the gram, but with its
  // nodes created before the levels' the level branch started ~44 µs after the gram (the
  // profiled step timeline, profiles/r2_s12_ds1_step_timeline.md); creating them last lets the
  // root level start right behind the gram: 0.2566 -> 0.2485 ms/step (medians of 4 interleaved
  // runs, profiles/r2_s15_graph_interleaved.log)
  constexpr bool rulemap_late = true;
  bool pairs_pending = false;
  auto enqueue_prologue = [&]() {
    kern::level_prologue_init(d_cnt, I, d_own_bm_, (int64_t)(need / 8), d_desc, kMaxLv, d_ctl,
                              call_params_, d_call_seq_, s);
    support_counts(d_items_, nnz_, d_cnt, s);
    if (fused_select)
      kern::level_select_fused(d_cnt, I, c1, d_ids, d_fcnt, d_rank_of, d_desc, d_ctl, s);
    else
      kern::level_select(d_cnt, I, c1, d_ids, d_fcnt, d_rank_of, d_rrank /* scratch until root setup */,
                         d_desc, s);
    kern::encode_bitmap(d_tx_ptr_, d_items_, n_tx_, d_rank_of, d_own_bm_, Wp, 0, s);
    if (kern::pair_gram_dev_needs_zero(Wp, I)) KMLS_HIP(hipMemsetAsync(d_gram, 0, (size_t)I * I * 4, s));
    kern::pair_gram_popcount_dev(d_own_bm_, Wp, &d_desc[1].n_rows, I, d_gram, s);
    if (cfg.rule_index) {
      if (fork_idx) {  // captured: the rule map runs on a side branch of the graph, beside the levels
        KMLS_HIP(hipEventRecord((hipEvent_t)idx_ev_[0], s));
        KMLS_HIP(hipStreamWaitEvent((hipStream_t)idx_s_, (hipEvent_t)idx_ev_[0], 0));
        if (rulemap_late) {
          pairs_pending = true;  // its nodes are created after the levels' (end_capture)
        } else {
          kern::pairs_to_csr(pa, (hipStream_t)idx_s_);
          KMLS_HIP(hipEventRecord((hipEvent_t)idx_ev_[1], (hipStream_t)idx_s_));
        }
      } else {
        kern::pairs_to_csr(pa, s);
      }
    }
    int32_t* d_prank = nullptr;
    if (part_world > 1) {  // replicated-data partition of the root classes, computed on device
      int64_t* d_cost = (int64_t*)arena_->push((size_t)I * 8);
      d_prank = (int32_t*)arena_->push((size_t)I * 4);
      kern::level_partition(d_gram, I, d_desc, run.minsup, I, d_cost, d_prank, s);
    }
    // level 2 straight from the gram: frequent pairs per root row, offsets, then the rows
    kern::level_root_rows(d_gram, I, d_desc, run.minsup, d_prank, part_world, part_rank, I, d_m, s);
    kern::RootSetupArgs ra{d_own_bm_, d_rrank, d_rgid, d_roff, d_ids, d_fcnt, run.out_parent.p,
                           run.out_item.p, run.out_count.p, run.out_depth.p, Wp, out_cap,
                           d_prank, part_world, part_rank,
                           run.stream_dl && !deferred_dl(), fused_select, d_m, d_soff, d_coff,
                           cfg.max_len == 2, kern::level_rows_interleaved(Wp), run.stream_dl};
    kern::level_root_setup(d_desc, d_ctl, ra, s);
    kern::level_root_fill(d_desc, d_ctl, d_gram, I, run.minsup, ra, out_->tile_row, I, s);
    if (!fused_select)  // staged to pinned memory while the levels run
      KMLS_HIP(hipMemcpyAsync(fstage.get(), d_ids, (size_t)tab_stride * 12, hipMemcpyDeviceToHost, s));
  };
  auto abort_capture = [&]() {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(s, &g);
    if (g) (void)hipGraphDestroy(g);
  };
  trace::push("kmls.prologue(enqueue)");
  const bool adopted = adopt && adopt_bufs && replay && adopt->key == key;
  if (adopt && !adopted) {  // launched ahead under another plan: let it finish, then drop it
    KMLS_HIP(hipStreamSynchronize(s));
    adopt.reset();
  }
  if (!adopted) {
    fill_params(call_params_[call_seq_ & 1], run.ht, fstage.get(), run.back.get(), ih);
    // eager and capture calls re-sync the device call counter (slot parity) with the host's
    if (!replay) KMLS_HIP(hipMemsetD32Async((hipDeviceptr_t)d_call_seq_, (int)(uint32_t)call_seq_, 1, s));
  }
  if (adopted) {  // already on the stream, behind the call that launched it
    run.graph_replay = true;
    run.graph_last = graph_->last;
    out_->launch_idx = graph_->launch_idx;
  } else if (replay) {
    run.graph_replay = true;
    run.graph_last = graph_->last;
    out_->launch_idx = graph_->launch_idx;  // later (non-graph) launches of this call continue
    KMLS_HIP(hipGraphLaunch(graph_->next(), s));
    ++call_seq_;
  } else if (use_graph) {
    KMLS_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    try {
      enqueue_prologue();
    } catch (...) {
      abort_capture();
      if (graph_) graph_->reset(nullptr, {}, 0, 0);
      throw;
    }
    run.graph_capture = true;
    run.end_capture = [&](int last) {
      if (pairs_pending) {  // the rule-map branch, created after the levels' nodes
        kern::pairs_to_csr(pa, (hipStream_t)idx_s_);
        KMLS_HIP(hipEventRecord((hipEvent_t)idx_ev_[1], (hipStream_t)idx_s_));
        pairs_pending = false;
      }
      if (fork_idx) KMLS_HIP(hipStreamWaitEvent(s, (hipEvent_t)idx_ev_[1], 0));  // join
      hipGraph_t g = nullptr;
      KMLS_HIP(hipStreamEndCapture(s, &g));
      hipGraphExec_t ex = nullptr, tw = nullptr;
      const hipError_t ie = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
      if (ie == hipSuccess && graph_twin_enabled() &&
          hipGraphInstantiate(&tw, g, nullptr, nullptr, 0) != hipSuccess)
        tw = nullptr;
      (void)hipGraphDestroy(g);
      KMLS_HIP(ie);
      if (!graph_) graph_ = std::make_unique<GraphCache>();
      graph_->reset(ex, key, last, out_->launch_idx, tw);
      KMLS_HIP(hipGraphLaunch(graph_->next(), s));
    };
  } else {
    enqueue_prologue();
    KMLS_HIP(hipEventRecord(e1.e, s));
  }
  if (!adopted && !replay) ++call_seq_;  // the eager / captured init launch
  // Launch the next identical call before waiting for this one (steady-state replay only): its
  // GPU work then overlaps this call's completion on the host (readback, result assembly,
  // Python) and the launch latency of the next call.  This call's end is marked by an event.
  Event ev_cur;
  if (prefetch && (replay || adopted) && graph_ && graph_->exec && graph_->key == key) {
    auto p = std::make_unique<Prefetch>();
    p->key = key;
    p->download = download;
    kern::HostTrie ht2 = run.ht;
    if (download) {
      p->host_cap = run.host_cap;
      p->pw = res.par_w;
      p->iw = res.item_w;
      p->cw = res.cnt_w;
      p->h_parent = pinned_->get((size_t)run.host_cap * p->pw);
      p->h_item = pinned_->get((size_t)run.host_cap * p->iw);
      p->h_count = pinned_->get((size_t)run.host_cap * p->cw);
      p->h_depth = pinned_->get((size_t)run.host_cap);
      ht2 = kern::HostTrie{p->h_parent.get(), p->h_item.get(), p->h_count.get(),
                           (uint8_t*)p->h_depth.get(), run.host_cap, p->pw, p->iw, p->cw};
    }
    p->fstage = pinned_->get((size_t)tab_stride * 12);
    p->back = pinned_->get(back_bytes);
    const IdxHost ih2 = new_idx_host();
    p->i_rp = ih2.rp;
    p->i_cons = ih2.cons;
    p->i_cnt = ih2.cnt;
    p->i_meta = ih2.meta;
    KMLS_HIP(hipEventRecord(ev_cur.e, s));
    fill_params(call_params_[call_seq_ & 1], ht2, p->fstage.get(), p->back.get(), ih2);
    KMLS_HIP(hipGraphLaunch(graph_->next(), s));
    ++call_seq_;
    out_->launch_idx = graph_->launch_idx;
    p->t_launch = std::chrono::steady_clock::now();
    pre_ = std::move(p);
    run.wait_ev = ev_cur.e;
    run.no_more_batches = true;  // a later batch would run behind the launched-ahead call
  }
  const bool pipelined = adopted || pre_;
  trace::pop();
  bool ok;
  {
    trace::Range rg("kmls.levels");
    try {
      ok = run.levels_loop(d_desc, d_ctl, out_cap);
      fused_need_ = std::max(fused_need_, run.need_nodes);
    } catch (...) {
      if (run.graph_capture) {
        hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone)
          abort_capture();
      }
      // the host call counter may now be ahead of the device's: no replay until a re-sync
      if (graph_) graph_->reset(nullptr, {}, 0, 0);
      throw;
    }
  }
  // A pipelined call that cannot finish within its replayed plan (more levels than last time,
  // a device overflow, a host-trie overflow needing the full-width copy) is redone on its own:
  // the launched-ahead call has reused the device buffers by now.
  if (pre_ && (!ok || (download && !run.stream_dl))) {
    drain_prefetch();
    arena_->pop_to(mark);
    res = GpuMineResult();
    if (graph_) graph_->reset(nullptr, {}, 0, 0);
    return mine_resident(cfg, download, res, part_rank, part_world, false);
  }
  if (!ok) {
    fused_fallback_ = run.fallback_reason;
    arena_->pop_to(mark);
    res = GpuMineResult();
    return false;
  }
  const int64_t F = run.last_desc[1].n_rows;
  // frequent items to the host (frequent() API); small
  {
    const int32_t* hs = (const int32_t*)fstage.get();
    fi_.ids.assign(hs, hs + F);
    fi_.counts.assign((const uint32_t*)(hs + tab_stride), (const uint32_t*)(hs + tab_stride) + F);
    fi_.rank_of.assign(hs + 2 * tab_stride, hs + 2 * tab_stride + I);
  }
  fi_.minsup2 = run.minsup;
  global_n_tx_ = n_tx_;
  if (!pipelined) KMLS_HIP(hipEventRecord(e2.e, s));
  const int64_t N = run.out_size;
  res.n_nodes = N;
  last_nodes_ = N;
  // the overflow hint is a high-water mark of one (earlier, larger) problem: a call that fit
  // with 8x room to spare releases it, so later small calls stop sizing for that one
  if (run.need_nodes == 0 && N < (fused_need_ >> 3)) fused_need_ = 0;
  if (download && !run.stream_dl) {
    KMLS_HIP(hipStreamSynchronize(out_->copy_s));
    res.par_w = 8;
    res.item_w = 4;
    res.cnt_w = 4;
    res.h_parent = pinned_->get((size_t)N * sizeof(int64_t));
    res.h_item = pinned_->get((size_t)N * sizeof(int32_t));
    res.h_count = pinned_->get((size_t)N * sizeof(uint32_t));
    res.h_depth = pinned_->get((size_t)N * sizeof(uint8_t));
    if (N) {
      KMLS_HIP(hipMemcpyAsync(res.h_parent.get(), run.out_parent.p, N * sizeof(int64_t), hipMemcpyDeviceToHost, s));
      KMLS_HIP(hipMemcpyAsync(res.h_item.get(), run.out_item.p, N * sizeof(int32_t), hipMemcpyDeviceToHost, s));
      KMLS_HIP(hipMemcpyAsync(res.h_count.get(), run.out_count.p, N * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      KMLS_HIP(hipMemcpyAsync(res.h_depth.get(), run.out_depth.p, N * sizeof(uint8_t), hipMemcpyDeviceToHost, s));
    }
  } else if (!download) {
    res.h_parent.reset();
  }
  if (!pre_) KMLS_HIP(hipStreamSynchronize(s));  // else: waited for this call's end event
  KMLS_HIP(hipStreamSynchronize(out_->copy_s));
  if (cfg.rule_index) {
    const int64_t* meta = (const int64_t*)ih.meta.get();
    const int64_t nnz = meta[0], st = meta[1];
    if (st != 0) {  // entry or host capacity exceeded: grow and redo this call on its own
      KMLS_CHECK(!(st & 2), "rule map: a row exceeds the device sort capacity");
      drain_prefetch();
      arena_->pop_to(mark);
      res = GpuMineResult();
      if (graph_) graph_->reset(nullptr, {}, 0, 0);
      idx_cap_ = std::max<int64_t>(idx_cap_ * 2, nnz + (nnz >> 3) + 1024);
      return mine_resident(cfg, download, res, part_rank, part_world, false);
    }
    res.idx_nnz = nnz;
    res.n_items_idx = I + 1;
    res.h_idx_row_ptr = ih.rp;
    res.h_idx_cons = ih.cons;
    res.h_idx_cnt = ih.cnt;
  }
  if (pipelined) {  // GPU events would span the neighbouring call: host clock instead
    res.phases.push_back({adopted ? "mine(graph replay, adopted)" : "mine(graph replay, launched next)",
                          std::chrono::duration<double, std::milli>(
                              std::chrono::steady_clock::now() - (adopted ? adopt->t_launch : t_launch)).count()});
  } else if (use_graph) {
    res.phases.push_back({replay ? "mine(graph replay)" : "mine(graph capture)", elapsed(e0, e2)});
  } else {
    res.phases.push_back({"prologue(support+select+encode+gram)", elapsed(e0, e1)});
    res.phases.push_back({"levels", elapsed(e1, e2)});
  }
  {  // host-side profile (ms): before the first launch, enqueue until the sync, after the sync
    const auto t_end = std::chrono::steady_clock::now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    res.phases.push_back({"host_pre_launch", ms(t0, t_launch)});
    res.phases.push_back({"host_enqueue_to_sync", ms(t_launch, run.t_presync)});
    res.phases.push_back({"host_sync_wait", ms(run.t_presync, run.t_postsync)});
    res.phases.push_back({"host_post_sync", ms(run.t_postsync, t_end)});
  }
  res.stats.n_frequent_items = F;
  // level-1 nodes are replicated on every rank of a partition; rank 0 counts them
  res.stats.n_itemsets = (part_world > 1 && part_rank != 0) ? N - F : N;
  res.stats.n_candidates = run.n_candidates;
  res.stats.max_depth = F ? run.max_depth : 0;
  res.stats.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  res.arena_high_water = (int64_t)arena_->high_water();
  res.levels_path = part_world > 1 ? "fused-resident-partition" : "fused-resident";
  adopt.reset();  // consumed: its buffers now belong to `res`
  arena_->pop_to(mark);
  return true;
}

bool GpuMiner::resident_ok(const MineConfig& cfg) const {
  return fused_levels_enabled() && cfg.level2_gram && !cfg.level2_mfma &&
         !cfg.pairs_only && cfg.max_len != 1 && n_items_ >= 2 &&
         n_items_ <= kern::kSelectMaxItems && (size_t)n_items_ * words_local() * 8 <= (1ull << 30) &&
         n_tx_ > 0;
}

GpuMineResult GpuMiner::mine_partition(const MineConfig& cfg, bool download, int rank, int world,
                                       bool prefetch) {
  KMLS_HIP(hipSetDevice(device_));
  fused_fallback_.clear();
  GpuMineResult r;
  if (!resident_ok(cfg))
    throw std::runtime_error("mine_partition: data not eligible for the device-resident path");
  if (!mine_resident(cfg, download, r, rank, world, prefetch)) {
    const bool retry = arena_limited(fused_fallback_) && grow_arena(0);
    if (!retry || !mine_resident(cfg, download, r, rank, world))
      throw std::runtime_error("mine_partition: fused path overflowed (" + fused_fallback_ + ")");
  }
  return r;
}

GpuMineResult GpuMiner::mine(const MineConfig& cfg, bool download, bool prefetch) {
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  fused_fallback_.clear();
  if (resident_ok(cfg)) {
    GpuMineResult r;
    if (mine_resident(cfg, download, r, 0, 1, prefetch)) return r;
    if (arena_limited(fused_fallback_) && grow_arena(0)) {  // retry once with a bigger arena
      fused_fallback_.clear();
      if (mine_resident(cfg, download, r, 0, 1)) return r;
    }
  }
  drain_prefetch();
  auto t0 = std::chrono::steady_clock::now();
  Event e0, e1, e2;
  KMLS_HIP(hipEventRecord(e0.e, s));
  const size_t mark = arena_->mark();
  uint32_t* d_cnt = (uint32_t*)arena_->push((size_t)std::max<int64_t>(n_items_, 1) * sizeof(uint32_t));
  item_support((uintptr_t)d_cnt);
  std::vector<uint32_t> cnt((size_t)n_items_);
  KMLS_HIP(hipMemcpyAsync(cnt.data(), d_cnt, cnt.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  arena_->pop_to(mark);
  const int64_t F = select(cnt.data(), n_tx_, cfg.min_support);
  KMLS_HIP(hipEventRecord(e1.e, s));
  const int64_t Wp = words_local();
  const bool hl = hlevels_plan(cfg, F, Wp, nullptr);
  if (!hl) {
    const size_t need = (size_t)std::max<int64_t>(F, 1) * Wp * sizeof(uint64_t);
    if (need > own_bm_bytes_) {
      if (d_own_bm_) KMLS_HIP(hipFree(d_own_bm_));
      KMLS_HIP(hipMalloc((void**)&d_own_bm_, need));
      own_bm_bytes_ = need;
    }
    encode_bitmaps_fresh(d_own_bm_, F, Wp);
  }
  KMLS_HIP(hipEventRecord(e2.e, s));
  GpuMineResult r;
  for (int attempt = 0;; ++attempt) {
    const size_t mark = arena_->mark();
    try {
      struct CsrFlag {  // the bitmaps are this miner's own CSR (level-2 cooc allowed)
        bool& f;
        explicit CsrFlag(bool& x, bool v = true) : f(x) { f = v; }
        ~CsrFlag() { f = false; }
      } flag(gram_csr_ok_), plan(hl_plan_, hl);
      r = mine_bitmaps(hl ? 0 : (uintptr_t)d_own_bm_, Wp, cfg, nullptr, true, download);
      break;
    } catch (const ArenaExhausted& ex) {
      // a default-sized arena grows (up to its maximum) and the chunked search reruns
      KMLS_HIP(hipStreamSynchronize(s));
      arena_->pop_to(mark);
      if (attempt >= 3 || mark != 0 || !grow_arena(ex.needed + (ex.needed >> 1))) throw;
    }
  }
  if (!fused_fallback_.empty() && r.levels_path.find("fallback") == std::string::npos)
    r.levels_path += " (resident fallback: " + fused_fallback_ + ")";
  std::vector<Phase> ph;
  ph.push_back({"support+select", elapsed(e0, e1)});
  ph.push_back({hl ? "cooc_stats" : "encode_bitmap", elapsed(e1, e2)});
  for (auto& p : r.phases) ph.push_back(p);
  r.phases = ph;
  r.stats.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return r;
}


// Steps 1-2 of the tx-DP call (and of the item-sharded one): supports of the shard in K tiles,
// all-reduced over the ranks (tile k's all-reduce on the comm stream overlaps tile k+1's
// histogram), then the frequent-item selection on the device.  Returns F.
int64_t GpuMiner::txdp_select(Comm* comm, int64_t global_n_tx, const MineConfig& cfg,
                              int support_tiles) {
  hipStream_t s = (hipStream_t)stream_;
  const size_t mark = arena_->mark();
  // 1. supports in K tiles; tile k's all-reduce (comm stream) overlaps tile k+1's histogram.
  //    The comm stream and the tile events live as long as the miner (no per-call creation).
  //    One rank has no all-reduce to overlap: one tile, so the partitioned histogram's fixed
  //    per-pass costs (per-block bin flushes, scans) are paid once.
  int K = std::max(1, std::min(64, support_tiles));
  if (!comm || comm->world() <= 1) K = 1;
  const size_t vec = (size_t)std::max<int64_t>(n_items_, 1) * sizeof(uint32_t);
  uint32_t* d_part = (uint32_t*)arena_->push(vec * K);
  KMLS_HIP(hipMemsetAsync(d_part, 0, vec * K, s));
  if (!comm_s_) KMLS_HIP(hipStreamCreateWithFlags((hipStream_t*)&comm_s_, hipStreamNonBlocking));
  hipStream_t cs = (hipStream_t)comm_s_;
  while ((int)tile_ev_.size() < K + 1) {
    hipEvent_t e;
    KMLS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    tile_ev_.push_back((void*)e);
  }
  for (int k = 0; k < K; ++k) {
    const int64_t a = tile_nnz_[(size_t)(64 * k / K)], b = tile_nnz_[(size_t)(64 * (k + 1) / K)];
    uint32_t* part = d_part + (size_t)k * (size_t)std::max<int64_t>(n_items_, 1);
    support_counts(d_items_ + a, b - a, part, s);
    KMLS_HIP(hipEventRecord((hipEvent_t)tile_ev_[(size_t)k], s));
    KMLS_HIP(hipStreamWaitEvent(cs, (hipEvent_t)tile_ev_[(size_t)k], 0));
    if (comm) comm->all_reduce(part, part, (size_t)n_items_, CommDtype::U32, false, cs);
  }
  hipEvent_t done = (hipEvent_t)tile_ev_[(size_t)K];
  KMLS_HIP(hipEventRecord(done, cs));
  KMLS_HIP(hipStreamWaitEvent(s, done, 0));
  for (int k = 1; k < K; ++k)
    kern::add_u32(d_part, d_part + (size_t)k * (size_t)std::max<int64_t>(n_items_, 1), n_items_, s);
  // the selection (rank by support over up to millions of items) runs on the host: one 4 B/item
  // readback per call, the same on every rank
  // 2. selection from the global supports (identical on every rank), on the device: only the
  //    frequent ids/counts come back
  constexpr bool dev_select = true;
  int64_t F;
  if (dev_select) {
    F = select_device(d_part, global_n_tx, cfg.min_support, comm);
    arena_->pop_to(mark);
  } else {
    std::vector<uint32_t> cnt((size_t)n_items_);
    KMLS_HIP(hipMemcpyAsync(cnt.data(), d_part, cnt.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (comm) comm->wait_stream(s);
    else KMLS_HIP(hipStreamSynchronize(s));
    arena_->pop_to(mark);
    F = select(cnt.data(), global_n_tx, cfg.min_support);
  }
  return F;
}

GpuMineResult GpuMiner::mine_txdp(Comm* comm, int64_t global_n_tx, const MineConfig& cfg,
                                  bool download, int support_tiles) {
  drain_prefetch();  // a launched-ahead resident call shares the device buffers
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  auto t0 = std::chrono::steady_clock::now();
  Event e0, e1, e2;
  KMLS_HIP(hipEventRecord(e0.e, s));
  const int64_t F = txdp_select(comm, global_n_tx, cfg, support_tiles);
  KMLS_HIP(hipEventRecord(e1.e, s));
  // 3. shard-local bitmaps (none when every level is counted horizontally from the CSR)
  const int64_t Wp = words_local();
  const bool hl = hlevels_plan(cfg, F, Wp, comm);
  if (!hl) {
    const size_t need = (size_t)std::max<int64_t>(F, 1) * Wp * sizeof(uint64_t);
    if (need > own_bm_bytes_) {
      if (d_own_bm_) KMLS_HIP(hipFree(d_own_bm_));
      KMLS_HIP(hipMalloc((void**)&d_own_bm_, need));
      own_bm_bytes_ = need;
    }
    encode_bitmaps_fresh(d_own_bm_, F, Wp);
  }
  KMLS_HIP(hipEventRecord(e2.e, s));
  // the dense level-2 gram (mine_bitmaps) lives in the arena: a default-sized arena grows ahead
  // of it — every rank computes the same F, so no rank re-runs alone inside a collective (at
  // 60k frequent items the gram alone is 14.4 GB, past the 8 GB first guess)
  if (cfg.level2_gram && F >= 2 && F <= kern::kSparseMaxF) {
    const int cw = comm ? comm->world() : 1;
    const size_t gram = (size_t)((F + cw - 1) / cw * cw) * (size_t)F * sizeof(uint32_t);
    const size_t want = gram + gram / 4 + ((size_t)256 << 20);
    if (arena_->capacity() < want) grow_arena(want);
  }
  // 4. level loop with all-reduced candidate counts
  comm_ = comm;
  gram_csr_ok_ = true;
  hl_plan_ = hl;
  GpuMineResult r;
  try {
    r = mine_bitmaps(hl ? 0 : (uintptr_t)d_own_bm_, Wp, cfg, nullptr, true, download);
  } catch (...) {
    comm_ = nullptr;
    gram_csr_ok_ = false;
    hl_plan_ = false;
    throw;
  }
  comm_ = nullptr;
  gram_csr_ok_ = false;
  hl_plan_ = false;
  std::vector<Phase> ph;
  ph.push_back({"support_tiles+allreduce+select", elapsed(e0, e1)});
  ph.push_back({hl ? "cooc_stats" : "encode_bitmap", elapsed(e1, e2)});
  for (auto& p : r.phases) ph.push_back(p);
  r.phases = ph;
  r.stats.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return r;
}

// Item-sharded mining without bitmaps (the horizontal plan): supports/selection as in tx-DP,
// then every rank all-gathers the frequent-rank CSR (PairRows, PrShard) and counts the pair rows
// of its own items (rank a % world == r) and the horizontal levels of their subtrees — complete
// counts from every transaction, so nothing else is reduced.  The result is this rank's
// sub-trie (level 1 + its roots' subtrees); the caller gathers them (dist_miner.gather_trie).
// declined = true (nothing mined) when the shard is not long and sparse enough for the plan.
GpuMineResult GpuMiner::mine_shard(Comm* comm, int64_t global_n_tx, const MineConfig& cfg,
                                   bool download, int support_tiles, bool* declined) {
  drain_prefetch();
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  auto t0 = std::chrono::steady_clock::now();
  Event e0, e1;
  KMLS_HIP(hipEventRecord(e0.e, s));
  const int64_t F = txdp_select(comm, global_n_tx, cfg, support_tiles);
  const int64_t Wp = words_local();
  // only the row form counts complete pairs from the all-gathered CSR (pair_rows_count's PrShard);
  // without it (KMLS_PAIR_ROWS=0, F > 65535) every rank declines and the caller falls back
  *declined = !hlevels_plan(cfg, F, Wp, comm, /*need_rows=*/true);
  KMLS_HIP(hipEventRecord(e1.e, s));
  if (*declined) return GpuMineResult{};
  shard_comm_ = comm;
  gram_csr_ok_ = true;
  hl_plan_ = true;
  GpuMineResult r;
  try {
    r = mine_bitmaps(0, Wp, cfg, nullptr, true, download);
  } catch (...) {
    shard_comm_ = nullptr;
    gram_csr_ok_ = false;
    hl_plan_ = false;
    throw;
  }
  shard_comm_ = nullptr;
  gram_csr_ok_ = false;
  hl_plan_ = false;
  std::vector<Phase> ph;
  ph.push_back({"support_tiles+allreduce+select", elapsed(e0, e1)});
  for (auto& p : r.phases) ph.push_back(p);
  r.phases = ph;
  r.levels_path = "horizontal-item-shard";
  r.stats.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return r;
}

}  // namespace gpu
}  // namespace kmls
