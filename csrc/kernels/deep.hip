// Count-only deep FP-Growth mining on CDNA4: every frequent itemset of every size is found and its
// support computed, the per-size totals and the content digest (kmls/digest.hpp) accumulated on
// the device, and nothing is materialised for the host.  For the reference's datasets (short
// transactions, T <= 4096, i.e. <= 64 bitmap words) at supports where the output has 1e9-1e10
// itemsets (BASELINE config 2, ds1 @ 0.01-0.02), a level-wise miner cannot hold one level in HBM.
//
// Design (one wave = one depth-first worker; idle waves take work from busy ones inside the launch):
// * A class (prefix P, members P∪{x_k}) lives in a BLOCK: WT bitmap words x `pad` slots stored
//   word-major ([w][slot]), then one item-hash word per slot.  Lanes that read consecutive
//   member slots of one word row read contiguous memory, so every bitmap load is coalesced.
// * TID PROJECTION: every member row of a class is a subset of tid(P).  When a class is created
//   from the row of member a (root classes from the item's own row, row steps from member s0),
//   its rows are stored COMPRESSED onto the positions of that row's set bits (parallel bit
//   extract with per-word move masks computed once per class, Hacker's Delight 7-4), so a class
//   whose prefix has support s holds ceil(s/64) words (rounded up to a width tier) instead of
//   ceil(T/64).  At ds1 @0.02 the 36-word rows become 1-10 words at the root and shrink further
//   down the tree: the bytes every AND+popcount reads and every survivor writes drop with them.
//   The width of a block travels in its frames; one launch dispatches each step on the frame's
//   tier (wave-uniform switch), so the words of a candidate stay in VGPRs with unguarded loads.
// * A FRAME is (block, first slot, members, prefix hash, prefix size | width).  Each wave keeps a
//   frame stack and a LIFO stack of blocks in its own HBM region; a block is freed when the
//   frames that reference it are done and it is on top.
// * Row step (big frames, > kCap pairs): member s0 against every later member, lane = candidate:
//   the member's words are a broadcast, the candidates' words one coalesced row per word.
// * Batch step (small frames, the deep levels): the top frames are popped together until their
//   member PAIRS fill up to kCap lanes, so a wave64 instruction still carries 64 candidates when
//   classes have 5-20 members.  Survivors of one (frame, member) group stay contiguous in the
//   child block (lane order = pair order), so each group becomes a child frame.
// * Load balance: tasks are dequeued by ticket, heaviest first (deep_order.hip's cost order).
//   Steal mode (the default): a wave whose ticket finds the queue drained opens its inbox and
//   asks busy waves, one mailbox at a time; a busy wave past its step budget that finds a request
//   in its mailbox hands its bottom (oldest, largest) open class straight to that inbox — a
//   large one split: the upper members go, the lower first members stay (frame lead).  Without
//   steal mode a wave past its budget SPILLS its frames to a heap as new tasks and the host runs
//   another round.
// Counts are exact (popcount of at most 4096 bits per row, u32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "kernels.hpp"
#include "kmls/digest.hpp"
#include <kmls/wave.hpp>

namespace kmls {
namespace kern {

namespace {

constexpr int kWaves = 4;            // independent waves per workgroup
constexpr int kRootChunk = 256;      // level-2 candidates per wave of k_deep_root
constexpr int kCap = 512;            // candidate pairs per batch step (256: 42.7 ms, 512: 39.6, 1024 with 16-bit group fields: 43.9 at ds1 @0.02)
constexpr int kBatchFrames = 64;     // frames one batch step may take
constexpr int kBStack = 96;          // blocks on one wave's memory stack
static_assert(kBStack < 127, "block-stack index + 1 must fit the 7 meta bits");
constexpr unsigned kSingle = 1u << 6;  // frame flag: expand only its first member
constexpr unsigned kMaxLead = 2047;    // frame lead field (11 bits)
// (hand-offs split a class of >= DeepArgs::split_firsts first members, keeping split_keep16/16)
constexpr unsigned kDone = 1u << 31;   // steal mode: ready-flag value epoch ^ kDone = no task
constexpr unsigned kNodeChunk = 4096;  // emit mode: node ids a wave takes from ctl->node_top

// frame meta: bits 0..5 prefix size, bit 6 single, bits 7..13 block width (words), bits 14..20
// block-stack index + 1 (0 = external), bits 21..31 lead: how many of the class's members, from
// s0 on, are still to be expanded as first members (0 = all; every member stays a candidate).  A
// hand-off of a large class gives away its upper members as a class of their own and keeps
// the first `lead` (halving instead of one member per hop: the tail of a split launch).
__device__ __forceinline__ unsigned meta_depth(unsigned m) { return m & 0x3fu; }
__device__ __forceinline__ unsigned meta_width(unsigned m) { return (m >> 7) & 0x7fu; }
__device__ __forceinline__ unsigned meta_bidx(unsigned m) { return (m >> 14) & 0x7fu; }
__device__ __forceinline__ unsigned meta_lead(unsigned m) { return m >> 21; }
__device__ __forceinline__ unsigned meta_with_lead(unsigned m, unsigned lead) {
  return (m & 0x1fffffu) | (lead << 21);
}
__host__ __device__ constexpr unsigned make_meta(unsigned depth, bool single, unsigned width,
                                                 unsigned bidx, unsigned lead = 0) {
  return depth | (single ? kSingle : 0u) | (width << 7) | (bidx << 14) | (lead << 21);
}
// the first members a frame still expands (single: 1; lead: lead; else all but the last)
__device__ __forceinline__ unsigned frame_firsts(unsigned meta, unsigned m) {
  const unsigned lead = meta_lead(meta);
  return (meta & kSingle) ? 1u : lead ? lead : m - 1u;
}

// block widths the kernels are instantiated for (words); tier(n) = smallest >= n
__host__ __device__ constexpr unsigned tier_of(unsigned n) {
  return n <= 1 ? 1 : n <= 2 ? 2 : n <= 3 ? 3 : n <= 4 ? 4 : n <= 6 ? 6 : n <= 8 ? 8
       : n <= 12 ? 12 : n <= 16 ? 16 : n <= 24 ? 24 : n <= 32 ? 32 : n <= 48 ? 48 : 64;
}

constexpr unsigned long long roundup16(unsigned long long x) { return (x + 15) & ~15ull; }

// every lane gets frame `p` (read as 8 dwords by lanes 0-7: a vector load, then broadcast)
__device__ __forceinline__ DeepFrame load_frame(const DeepFrame* p, int lane) {
  const unsigned* w = (const unsigned*)p;
  const unsigned v = lane < 8 ? w[(lane & 7) + vzero()] : 0u;
  DeepFrame f;
  f.blk = ((unsigned long long)__shfl(v, 1, 64) << 32) | __shfl(v, 0, 64);
  f.hash = ((unsigned long long)__shfl(v, 3, 64) << 32) | __shfl(v, 2, 64);
  f.pad = __shfl(v, 4, 64);
  f.s0 = __shfl(v, 5, 64);
  f.m = __shfl(v, 6, 64);
  f.meta = __shfl(v, 7, 64);
  f.blk = uni64(f.blk);
  f.hash = uni64(f.hash);
  f.pad = uni(f.pad);
  f.s0 = uni(f.s0);
  f.m = uni(f.m);
  f.meta = uni(f.meta);
  return f;
}

// the same frame through agent-scope loads (a frame another wave published in this launch:
// its 128-byte line may hold older frames this CU already read)
__device__ __forceinline__ DeepFrame load_frame_agent(const DeepFrame* p, int lane) {
  const unsigned* w = (const unsigned*)p;
  const unsigned v = lane < 8 ? ld_agent(w + (lane & 7)) : 0u;
  DeepFrame f;
  f.blk = uni64(((unsigned long long)__shfl(v, 1, 64) << 32) | __shfl(v, 0, 64));
  f.hash = uni64(((unsigned long long)__shfl(v, 3, 64) << 32) | __shfl(v, 2, 64));
  f.pad = uni(__shfl(v, 4, 64));
  f.s0 = uni(__shfl(v, 5, 64));
  f.m = uni(__shfl(v, 6, 64));
  f.meta = uni(__shfl(v, 7, 64));
  return f;
}

// a frame handed to another wave: write-through stores (see kmls/wave.hpp)
__device__ __forceinline__ void publish_frame(DeepFrame* p, const DeepFrame& f) {
  unsigned long long* w = (unsigned long long*)p;
  st_agent(w + 0, f.blk);
  st_agent(w + 1, f.hash);
  st_agent(w + 2, ((unsigned long long)f.s0 << 32) | f.pad);
  st_agent(w + 3, ((unsigned long long)f.meta << 32) | f.m);
}

__device__ __forceinline__ void store_frame(DeepFrame* p, const DeepFrame& f) {
  p->blk = f.blk;
  p->hash = f.hash;
  p->pad = f.pad;
  p->s0 = f.s0;
  p->m = f.m;
  p->meta = f.meta;
}

// ---- tid projection ----
// Per-word move masks of the compress-right network for a fixed mask R (Hacker's Delight 7-4):
// compress(x) = 6 rounds of  t = x & mv[i];  x = (x ^ t) | (t >> 2^i),  for x already inside R.
template <int NW>
struct ProjLds {
  unsigned long long mv[6][NW];  // [round][word]
  unsigned n[NW];                // popcount of R's word
};

// lanes w < WT: word w of the uniform row R = blk[w][ia]; returns |R| (uniform)
template <int WT, int NW>
__device__ __forceinline__ unsigned proj_setup(ProjLds<NW>& P, gptr<const unsigned long long> blk,
                                               unsigned long long pad, unsigned ia, int lane) {
  static_assert(WT <= NW && NW <= 64, "projection words");
  unsigned n = 0;
  if (lane < WT) {
    unsigned long long m = blk[(unsigned long long)lane * pad + ia];
    n = (unsigned)__popcll(m);
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
      P.mv[i][lane] = mv;
      m = (m ^ mv) | (mv >> (1u << i));
      mk &= ~mp;
    }
    P.n[lane] = n;
  }
  for (int off = 32; off; off >>= 1) n += __shfl_xor(n, off, 64);
  __builtin_amdgcn_wave_barrier();
  return uni(n);
}

// candidate (slot sa, slot sb) of one block: AND of every word (kept in v) and its popcount.
// blk and pad are wave-uniform, so each word row's base is an SGPR pair and the two slot offsets
// are the only address VGPRs (global_load saddr + voffset form).  WT is the block's exact width
// (rows are padded with zero words up to their tier), so the loads are unrolled without guards
// and all 2*WT of them can be in flight.
template <int WT>
__device__ __forceinline__ unsigned and_count(gptr<const unsigned long long> blk,
                                              unsigned long long pad, unsigned sa, unsigned sb,
                                              unsigned long long (&v)[WT]) {
  unsigned c = 0;
#pragma unroll
  for (int w = 0; w < WT; ++w) {
    const gptr<const unsigned long long> row = blk + (unsigned long long)w * pad;
    v[w] = row[sa] & row[sb];
  }
#pragma unroll
  for (int w = 0; w < WT; ++w) c += (unsigned)__popcll(v[w]);
  return c;
}

template <int WT>
__device__ __forceinline__ void write_row(unsigned long long* cb, unsigned long long cpad,
                                          unsigned pos, const unsigned long long (&v)[WT],
                                          unsigned long long ih) {
#pragma unroll
  for (int w = 0; w < WT; ++w) cb[(unsigned long long)w * cpad + pos] = v[w];
  cb[(unsigned long long)WT * cpad + pos] = ih;
}

// the survivor's row compressed onto R (v inside R word by word), written as wt_out words
// (zero-padded) + the item hash.  The bit offsets depend on R only, so the loop is uniform and
// the stores are predicated on `surv`.
template <int WT, int NW>
__device__ __forceinline__ void write_proj(unsigned long long* cb, unsigned long long cpad,
                                           unsigned pos, bool surv,
                                           const unsigned long long (&v)[WT],
                                           const ProjLds<NW>& P, unsigned wt_out,
                                           unsigned long long ih) {
  unsigned long long acc = 0;
  unsigned fill = 0, q = 0;
  // (the masks are re-read from LDS per call: hoisted out of the caller's candidate loop they
  // would hold 12 VGPRs per word)
  const unsigned z = vzero();
#pragma unroll
  for (int w = 0; w < WT; ++w) {
    const unsigned n = uni(P.n[w + z]);
    if (n == 0) continue;
    unsigned long long x = v[w];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const unsigned long long t = x & P.mv[i][w + z];
      x = (x ^ t) | (t >> (1u << i));
    }
    acc |= x << fill;
    if (fill + n >= 64) {
      if (surv) cb[(unsigned long long)q * cpad + pos] = acc;
      ++q;
      acc = fill ? (x >> (64 - fill)) : 0ull;
      fill = fill + n - 64;
    } else {
      fill += n;
    }
  }
  if (fill) {
    if (surv) cb[(unsigned long long)q * cpad + pos] = acc;
    ++q;
  }
  for (; q < wt_out; ++q)
    if (surv) cb[(unsigned long long)q * cpad + pos] = 0ull;
  if (surv) cb[(unsigned long long)wt_out * cpad + pos] = ih;
}

template <int MAXT>
struct WaveLds {
  unsigned long long f_hash[kBatchFrames];
  unsigned f_s0[kBatchFrames], f_m[kBatchFrames], f_meta[kBatchFrames];
  unsigned P[kBatchFrames + 1], G[kBatchFrames + 1];
  // member-group tables in 16 bits (every value < kCap; frames of a batch have <= 32 members):
  // with the u32 block bases, 8 KB of LDS per wave instead of 12.5, so four 4-wave workgroups
  // fit a CU's 160 KB
  unsigned short g_cnt[kCap], g_start[kCap];
  unsigned short g_pos[kCap];       // first pair of member group g (its run start)
  unsigned short g_fi[kCap];        // frame << 8 | member of group g
  unsigned long long g_flag[kCap / 64];  // bit p: a group starts at pair p
  unsigned b_base[kBStack];         // byte offset in the wave's stack region (< 4 GB)
  unsigned b_live[kBStack];
  unsigned long long depth_cnt[64];
  ProjLds<MAXT> proj;
};

struct WaveState {
  unsigned nf;                 // frames on the stack
  unsigned nb;                 // blocks on the memory stack
  unsigned long long mem_top;  // bytes used in the wave's stack region
  unsigned long long ncur, nend;  // emit mode: the wave's current chunk of node ids
};

// emit mode: n consecutive node ids (uniform); a new chunk of the global counter when the
// wave's current one is used up (the tail of the old chunk stays unused: size 0)
__device__ __forceinline__ unsigned long long alloc_nodes(const DeepArgs& a, WaveState& st,
                                                          unsigned n, int lane) {
  if (st.ncur + n > st.nend) {
    const unsigned long long chunk = n > kNodeChunk ? n : kNodeChunk;
    unsigned long long b = 0;
    if (lane == 0) b = atomicAdd(&a.ctl->node_top, chunk);
    b = uni64(bcast64(b, 0));
    st.ncur = b;
    st.nend = b + chunk;
  }
  const unsigned long long r = st.ncur;
  st.ncur += n;
  return r;
}

// emit mode: one trie node (ids past the arena are counted by node_top but not written)
__device__ __forceinline__ void put_node(const DeepArgs& a, unsigned long long id,
                                         unsigned long long parent, unsigned item, unsigned count,
                                         unsigned depth) {
  if (id < a.node_cap) {
    a.node_parent[id] = (unsigned)parent;
    a.node_item[id] = item;
    a.node_count[id] = count;
    a.node_depth[id] = (unsigned char)depth;
  }
}

// A wave's block stack in two parts: the first seg0 bytes in a region where the waves' segments
// are packed next to each other, the rest in a 4 MiB-scale region of its own.  A wave works near
// the bottom of its stack almost all the time, so the hot blocks of all waves sit in a few hundred
// 2 MiB pages instead of one page per wave (4096 waves: more pages than the TLBs map).
struct WaveStack {
  char* s0;  // this wave's dense segment (n0 bytes)
  char* s1;  // the rest of its stack
  unsigned long long n0;
};
// the block of `bytes` at the stack top; no block straddles the two parts (one that would goes to
// the start of the second part: the skipped tail returns when the block below it is freed)
__device__ __forceinline__ unsigned long long* stack_block(const WaveStack& ws,
                                                           unsigned long long& mem_top,
                                                           unsigned long long bytes) {
  if (mem_top < ws.n0 && mem_top + bytes > ws.n0) mem_top = ws.n0;
  return (unsigned long long*)(mem_top < ws.n0 ? ws.s0 + mem_top : ws.s1 + (mem_top - ws.n0));
}

struct WaveAcc {
  unsigned long long dsum, dxor, cands, chunks, budget_used;
};

// pop the top frame: its block loses a live frame
template <int MAXT>
__device__ __forceinline__ void release_frame(WaveLds<MAXT>& L, unsigned meta, int lane) {
  const unsigned b = meta_bidx(meta);
  if (b && lane == 0) L.b_live[b - 1] -= 1;
}

template <int MAXT>
__device__ __forceinline__ void free_blocks(WaveLds<MAXT>& L, WaveState& st) {
  __builtin_amdgcn_wave_barrier();
  while (st.nb > 0) {
    const unsigned live = uni(L.b_live[st.nb - 1 + vzero()]);
    if (live) break;
    st.mem_top = (unsigned long long)uni(L.b_base[st.nb - 1 + vzero()]);
    st.nb -= 1;
  }
}

// drop the bottom `ns` frames (spilled or handed over): their blocks lose a reference, frames
// ns.. move down by ns (64 at a time, low to high: a chunk's loads happen before its stores, and
// it only overwrites frames an earlier chunk already moved)
template <int MAXT>
__device__ __forceinline__ void drop_bottom(DeepFrame* fst, WaveState& st, WaveLds<MAXT>& L,
                                            int lane, unsigned ns) {
  if ((unsigned)lane < ns) {
    const unsigned b = meta_bidx(fst[lane].meta);
    if (b) atomicSub(&L.b_live[b - 1], 1u);
  }
  const unsigned rest = st.nf - ns;
  for (unsigned c0 = 0; c0 < rest; c0 += 64) {
    const bool act = c0 + lane < rest;
    DeepFrame fr{};
    if (act) fr = fst[ns + c0 + lane];
    __builtin_amdgcn_wave_barrier();
    if (act) store_frame(fst + c0 + lane, fr);
    __builtin_amdgcn_wave_barrier();
  }
  st.nf = rest;
}

// Copy the bottom `ns` frames of the stack (all of them: ns = nf) to the spill heap and queue
// them as task(s): frames of more than split_min members become one single-member task each
// (over one shared copy).  Heap bytes and queue slots are reserved for all of them before
// anything is written, so a spill either happens completely or not at all.  Returns 0 (spilled),
// 1 (optional spill skipped: no room, the wave keeps its frames) or -1 (a required spill found
// no room: error set).  Steal mode publishes every task by its ready flag.  A partial spill
// (ns < nf: the oldest, largest open classes handed to waiting waves) drops the spilled frames'
// block references and moves the remaining frames down; the wave keeps working on them.
template <int MAXT, bool EMIT>
__device__ __forceinline__ int spill_frames(const DeepArgs& a, DeepFrame* fst, WaveState& st,
                                            WaveLds<MAXT>& L, int lane, bool optional,
                                            unsigned ns, long long fixed = -1) {
  constexpr unsigned E = EMIT ? 1u : 0u;  // emit mode: the node-word row
  unsigned long long bytes_tot = 0, nt_tot = 0;
  for (unsigned f = 0; f < ns; ++f) {
    const DeepFrame fr = load_frame(fst + f, lane);
    bytes_tot += (unsigned long long)(meta_width(fr.meta) + 1 + E) * roundup16(fr.m) * 8ull;
    const bool single = (fr.meta & kSingle) != 0;
    nt_tot += (!single && fr.m > a.split_min) ? frame_firsts(fr.meta, fr.m) : 1;
  }
  unsigned long long hbase = 0;
  if (fixed >= 0) {  // pre-split: the host laid out every task's heap bytes and queue slots
    hbase = a.split_heap[fixed];
  } else {
    if (lane == 0) hbase = atomicAdd(&a.ctl->heap_top, bytes_tot);  // overshoot is harmless
    hbase = uni64(bcast64(hbase, 0));
  }
  if (hbase + bytes_tot > a.heap_cap) {
    if (!optional && lane == 0) atomicOr(&a.ctl->error, 2u);
    return optional ? 1 : -1;
  }
  // queue slots: never reserved past the capacity (steal-mode readers wait on reserved slots)
  const unsigned long long qcap = (unsigned long long)a.out_cap - (a.steal ? (unsigned long long)a.n_in : 0ull);
  unsigned long long t0 = 0;
  if (fixed >= 0) {
    t0 = (unsigned long long)a.split_q[fixed];
    if (t0 + nt_tot > qcap) t0 = ~0ull;
  } else if (lane == 0) {
    unsigned long long old = ld_agent(&a.ctl->n_out);
    for (;;) {
      if (old + nt_tot > qcap) { old = ~0ull; break; }
      const unsigned long long seen = atomicCAS(&a.ctl->n_out, old, old + nt_tot);
      if (seen == old) break;
      old = seen;
    }
    t0 = old;
    if (t0 != ~0ull && a.steal) atomicAdd(&a.ctl->pending, nt_tot);
  }
  t0 = uni64(bcast64(t0, 0));
  if (t0 == ~0ull) {
    if (!optional && lane == 0) atomicOr(&a.ctl->error, 1u);
    return optional ? 1 : -1;
  }
  DeepFrame* out = a.out + (a.steal ? a.n_in : 0ll);
  unsigned long long hoff = hbase, q = t0;
  for (unsigned f = 0; f < ns; ++f) {
    const DeepFrame fr = load_frame(fst + f, lane);
    const unsigned m = fr.m;
    const unsigned wt = meta_width(fr.meta);
    const unsigned long long npad = roundup16(m);
    const unsigned long long* src = (const unsigned long long*)fr.blk;
    unsigned long long* dst = (unsigned long long*)(a.heap + hoff);
    const unsigned long long tot = (unsigned long long)(wt + 1 + E) * m;
    for (unsigned long long e = lane; e < tot; e += 64) {
      const unsigned long long w = e / m, k = e - w * m;
      if (a.steal)
        st_agent(dst + w * npad + k, src[w * fr.pad + fr.s0 + k]);
      else
        dst[w * npad + k] = src[w * fr.pad + fr.s0 + k];
    }
    const bool single = (fr.meta & kSingle) != 0;
    const bool split = !single && m > a.split_min;
    const unsigned nt = split ? frame_firsts(fr.meta, m) : 1;
    for (unsigned k = lane; k < nt; k += 64) {
      DeepFrame o;
      o.blk = (unsigned long long)dst;
      o.hash = fr.hash;
      o.pad = (unsigned)npad;
      o.s0 = split ? k : 0u;
      o.m = split ? m - k : m;
      o.meta = make_meta(meta_depth(fr.meta), split || single, wt, 0,
                         (split || single) ? 0u : meta_lead(fr.meta));
      if (a.steal)
        publish_frame(out + q + k, o);
      else
        store_frame(out + q + k, o);
    }
    hoff += (unsigned long long)(wt + 1 + E) * npad * 8ull;
    q += nt;
  }
  if (a.steal) {
    wait_stores();  // the write-through copies and frames above are complete before the flags
    __builtin_amdgcn_wave_barrier();
    for (unsigned long long k = lane; k < nt_tot; k += 64) atomicExch(&a.ready[t0 + k], a.epoch);
  }
  if (ns == st.nf) {
    st.nf = 0;
    st.nb = 0;
    st.mem_top = 0;
    return 0;
  }
  drop_bottom<MAXT>(fst, st, L, lane, ns);  // partial: the wave keeps the rest
  return 0;
}

// Direct hand-off to the inbox of the wave that asked (`req`): claim its inbox (open ->
// filling), copy a class block to the heap and the frame to the inbox with write-through stores,
// count the task, mark the inbox full.  The bottom frame (the oldest, largest open class) goes
// whole when it is small; a class of >= split_firsts first members is split instead: its upper
// members become the handed-off class (with the first members past the kept ones) and the wave
// keeps expanding the lower split_keep16/16 of the first members (lead), which pair with more candidates
// each — a large class spreads over the waves in a logarithmic number of hand-offs, not one
// member per hop.  False (nothing changed) when the requester is no longer waiting or the heap
// is full.
template <int MAXT, bool EMIT>
__device__ __forceinline__ bool donate_bottom(const DeepArgs& a, DeepFrame* fst, WaveState& st,
                                              WaveLds<MAXT>& L, int lane, unsigned req,
                                              unsigned k_open, unsigned k_filling,
                                              unsigned k_full) {
  if ((long long)req >= a.nwaves) return false;
  const DeepFrame fr = load_frame(fst, lane);
  const unsigned m = fr.m, wt = meta_width(fr.meta);
  const bool single = (fr.meta & kSingle) != 0;
  const unsigned lead = meta_lead(fr.meta);
  const unsigned firsts = frame_firsts(fr.meta, m);
  unsigned h = 0;  // first members kept (0: the whole frame goes)
  if (!single && a.split_keep16 && firsts >= a.split_firsts) {
    h = firsts * a.split_keep16 / 16u;
    h = h < 1u ? 1u : h > kMaxLead ? kMaxLead : h;
  }
  if (h == 0 && st.nf < 2) return false;  // a lone small frame stays
  unsigned ok = 0;
  if (lane == 0) ok = atomicCAS(&a.inbox_state[req], k_open, k_filling) == k_open;
  if (!uni(__shfl(ok, 0, 64))) return false;
  const unsigned mo = m - h;  // members [s0 + h, s0 + m) go
  constexpr unsigned E = EMIT ? 1u : 0u;
  const unsigned long long npad = roundup16(mo);
  const unsigned long long bytes = (unsigned long long)(wt + 1 + E) * npad * 8ull;
  unsigned long long base = 0;
  if (lane == 0) base = atomicAdd(&a.ctl->heap_top, bytes);
  base = uni64(bcast64(base, 0));
  if (base + bytes > a.heap_cap) {
    if (lane == 0) st_agent(&a.inbox_state[req], k_open);
    return false;
  }
  const unsigned long long* src = (const unsigned long long*)fr.blk;
  unsigned long long* dst = (unsigned long long*)(a.heap + base);
  const unsigned long long tot = (unsigned long long)(wt + 1 + E) * mo;
  for (unsigned long long e = lane; e < tot; e += 64) {
    const unsigned long long w = e / mo, k = e - w * mo;
    st_agent(dst + w * npad + k, src[w * fr.pad + fr.s0 + h + k]);
  }
  if (lane == 0) {
    DeepFrame o;
    o.blk = (unsigned long long)dst;
    o.hash = fr.hash;
    o.pad = (unsigned)npad;
    o.s0 = 0;
    o.m = mo;
    // the given class expands its own first members: all of them, or (a frame with a lead:
    // also when it goes whole) those up to the old lead
    o.meta = make_meta(meta_depth(fr.meta), single, wt, 0, lead ? lead - h : 0u);
    publish_frame(a.inbox + req, o);
    atomicAdd(&a.ctl->pending, 1ull);
    atomicAdd(&a.ctl->handoffs, 1ull);
  }
  wait_stores();  // block and frame complete before the inbox turns full
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) atomicExch(&a.inbox_state[req], k_full);
  if (h) {  // the wave keeps the bottom class's first h members (still paired with all of them)
    if (lane == 0) {
      DeepFrame kf = fr;
      kf.meta = meta_with_lead(fr.meta, h);
      store_frame(fst, kf);
    }
    __builtin_amdgcn_wave_barrier();
  } else {
    drop_bottom<MAXT>(fst, st, L, lane, 1);
  }
  return true;
}

// ---- row step: member s0 against members s0+1 .. s0+m-1 (lane = candidate) ----
// The child class (prefix P ∪ {a}) is projected onto row a when that narrows its tier.
template <int WT, int MAXT, bool EMIT>
__device__ __forceinline__ void row_step(const DeepArgs& a, DeepFrame* fst, WaveState& st,
                                         WaveLds<MAXT>& L, DeepFrame top, const WaveStack& stack,
                                         int lane, WaveAcc& acc) {
  const unsigned long long lanelt = (1ull << lane) - 1ull;
  const unsigned m = top.m;
  const unsigned depth = meta_depth(top.meta);  // prefix size: members are depth+1 itemsets
  const bool deeper = a.max_len == 0 || (int)depth + 3 <= a.max_len;  // children expandable
  const unsigned nc = m - 1;
  const unsigned long long cpad = roundup16(nc);
  const gptr<const unsigned long long> blk = as_global_addr<const unsigned long long>(top.blk);
  const gptr<const unsigned long long> ihp = blk + (unsigned long long)WT * top.pad;
  const unsigned ia = top.s0;
  const unsigned long long ih_a = ihp[ia + vzero()];
  const unsigned long long h_a = top.hash + ih_a;
  constexpr unsigned E = EMIT ? 1u : 0u;
  const gptr<const unsigned long long> nwp = ihp + top.pad;  // emit mode: node words
  const unsigned long long node_a = E ? uni64(nwp[ia + vzero()] & kDeepNodeMask) : 0ull;
  unsigned wt_out = WT;
  if (WT > 1 && deeper && nc >= 2) {
    const unsigned s = proj_setup<WT>(L.proj, blk, top.pad, ia, lane);
    wt_out = tier_of((s + 63) / 64);
  }
  const bool proj = wt_out < (unsigned)WT;
  unsigned long long* cb =
      stack_block(stack, st.mem_top, (unsigned long long)(wt_out + 1 + E) * cpad * 8ull);
  unsigned S = 0;
  for (unsigned c0 = 0; c0 < nc; c0 += 64) {
    const bool act = c0 + lane < nc;
    const unsigned jb = act ? ia + 1 + c0 + lane : ia;
    unsigned long long v[WT];
    // the candidate's item hash is loaded with its row words (96 % of the candidates survive
    // at the headline): one round trip per chunk instead of a second one after the count
    const unsigned long long ih_ld = ihp[jb];
    const unsigned c = and_count<WT>(blk, top.pad, ia + vzero(), jb, v);
    const bool surv = act && c >= a.minsup;
    const unsigned long long mask = __ballot(surv);
    const unsigned pos = S + (unsigned)__popcll(mask & lanelt);
    unsigned long long ih_b = 0;
    if (surv) {
      ih_b = ih_ld;
      const DigestTerms dt = digest_terms(h_a + ih_b, c);
      acc.dsum += dt.sum;
      acc.dxor ^= dt.xr;
    }
    if (deeper) {
      if (proj) {
        write_proj<WT>(cb, cpad, pos, surv, v, L.proj, wt_out, ih_b);
      } else if (surv) {
        write_row<WT>(cb, cpad, pos, v, ih_b);
      }
    }
    if (E && mask) {
      const unsigned long long nb0 = alloc_nodes(a, st, (unsigned)__popcll(mask), lane);
      if (surv) {
        const unsigned long long id = nb0 + (unsigned long long)__popcll(mask & lanelt);
        const unsigned long long nw_b = nwp[jb];
        put_node(a, id, node_a, (unsigned)(nw_b >> 40), c, depth + 2);
        if (deeper) cb[(unsigned long long)(wt_out + 1) * cpad + pos] = ((nw_b >> 40) << 40) | id;
      }
    }
    S += (unsigned)__popcll(mask);
    ++acc.chunks;
  }
  acc.cands += nc;
  if (lane == 0 && S) L.depth_cnt[depth + 2] += S;
  acc.budget_used += (nc + 63) / 64;
  // parent: done with member s0 (a frame with a lead: with its last first member)
  const unsigned lead = meta_lead(top.meta);
  if ((top.meta & kSingle) || m <= 2 || lead == 1u) {
    release_frame(L, top.meta, lane);
    st.nf -= 1;
  } else {
    top.s0 += 1;
    top.m -= 1;
    if (lead) top.meta = meta_with_lead(top.meta, lead - 1u);
    if (lane == 0) store_frame(fst + st.nf - 1, top);
  }
  if (S >= 2 && deeper) {
    if (lane == 0) {
      L.b_base[st.nb] = (unsigned)st.mem_top;
      L.b_live[st.nb] = 1;
      DeepFrame c;
      c.blk = (unsigned long long)cb;
      c.hash = h_a;
      c.pad = (unsigned)cpad;
      c.s0 = 0;
      c.m = S;
      c.meta = make_meta(depth + 1, false, wt_out, st.nb + 1);
      store_frame(fst + st.nf, c);
    }
    st.nb += 1;
    st.nf += 1;
    st.mem_top += (unsigned long long)(wt_out + 1 + E) * cpad * 8ull;
  }
}

// ---- batch step: the top frames' member pairs, up to kCap lanes ----
// (frames of the top frame's block only: sibling classes, so the block base and width stay
// uniform)
template <int WT, int MAXT, bool EMIT>
__device__ __forceinline__ void batch_step(const DeepArgs& a, DeepFrame* fst, WaveState& st,
                                           WaveLds<MAXT>& L, DeepFrame top, const DeepFrame& lf,
                                           const WaveStack& stack, int lane, WaveAcc& acc) {
  const unsigned long long lanelt = (1ull << lane) - 1ull;
  unsigned long long* cb = nullptr;  // (the child block: placed once P is known, below)
  unsigned k = 0, P = 0;
  {
    // frame f (from the top) came with lane f's registers (the step's one round of frame
    // loads, k_deep_count), then two wave scans
    static_assert(kBatchFrames == 64, "one batch frame per lane");
    unsigned fm = 0, fmeta = kSingle;
    if ((unsigned)lane < st.nf) {
      fm = lf.m;
      fmeta = lf.meta;
      // another block, or a frame with a lead (expanded row by row): ends the batch
      if (lf.blk != top.blk || meta_lead(lf.meta)) fmeta |= kSingle;
      L.f_hash[lane] = lf.hash;
      L.f_s0[lane] = lf.s0;
      L.f_m[lane] = fm;
      L.f_meta[lane] = fmeta;
    }
    const unsigned fp = (fmeta & kSingle) ? 0xffffffffu : fm * (fm - 1) / 2;
    // inclusive scan of pairs over lanes (lanes >= nf carry "infinite")
    unsigned incl = fp;
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned o = __shfl_up(incl, off, 64);
      if (lane >= off) incl = (o == 0xffffffffu || incl == 0xffffffffu || o + incl < o)
                                  ? 0xffffffffu : o + incl;
    }
    const unsigned long long okm = __ballot(incl <= (unsigned)kCap && (unsigned)lane < st.nf);
    // frames 0 .. k-1 fit (prefix property: the first failing lane ends the run)
    k = okm == ~0ull ? 64u : (unsigned)__builtin_ctzll(~okm);
    if (k == 0) k = 1;  // top frame always fits (pairs <= kCap, not single)
    k = uni(k);
    P = uni(__shfl(incl, (int)k - 1, 64));
    const unsigned excl = incl - fp;
    if ((unsigned)lane < k) L.P[lane] = excl;
    if (lane == 0) L.P[k] = P;
    // member-group prefix (m - 1 per frame)
    unsigned gm = ((unsigned)lane < k) ? fm - 1 : 0u;
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned o = __shfl_up(gm, off, 64);
      if (lane >= off) gm += o;
    }
    const unsigned gtot = __shfl(gm, (int)k - 1, 64);
    if ((unsigned)lane < k) L.G[lane] = gm - (fm - 1);
    if (lane == 0) L.G[k] = gtot;
  }
  __builtin_amdgcn_wave_barrier();
  const unsigned NG = uni(L.G[k + vzero()]);
  if (lane < (int)(kCap / 64)) L.g_flag[lane] = 0ull;
  __builtin_amdgcn_wave_barrier();
  // member groups once per batch (not per pair): frame, member, first pair, start flag; a pair's
  // group is then the number of group starts at or before it
  for (unsigned g = lane; g < NG; g += 64) {
    L.g_cnt[g] = 0;
    L.g_start[g] = 0xffffu;
    unsigned f = 0;
    for (unsigned step = 32; step; step >>= 1)
      if (f + step < k && L.G[f + step] <= g) f += step;
    const unsigned i = g - L.G[f], fmm = L.f_m[f];
    const unsigned pos = L.P[f] + i * fmm - i * (i + 1) / 2;
    L.g_pos[g] = (unsigned short)pos;
    L.g_fi[g] = (unsigned short)((f << 8) | i);
    atomicOr(&L.g_flag[pos >> 6], 1ull << (pos & 63));
  }
  __builtin_amdgcn_wave_barrier();
  const unsigned long long cpad = roundup16(P);
  cb = stack_block(stack, st.mem_top, (unsigned long long)(WT + 1 + (EMIT ? 1u : 0u)) * cpad * 8ull);
  const gptr<const unsigned long long> bblk = as_global_addr<const unsigned long long>(top.blk);
  const unsigned long long bpad = top.pad;
  const gptr<const unsigned long long> ihp = bblk + (unsigned long long)WT * bpad;
  constexpr unsigned E = EMIT ? 1u : 0u;
  const gptr<const unsigned long long> nwp = ihp + bpad;  // emit mode: node words
  unsigned S = 0, gbase = 0;
  for (unsigned c0 = 0; c0 < P; c0 += 64) {
    const unsigned p = c0 + lane;
    const bool act = p < P;
    // group of pair p (row-major pairs: group (f, i) holds (i, j), j > i): starts up to p
    const unsigned long long gw = uni64(L.g_flag[(c0 >> 6) + vzero()]);
    const unsigned g = gbase + (unsigned)__popcll(gw & ((2ull << lane) - 1ull)) - 1u;
    unsigned f = 0, i = 0, j = 0;
    if (act) {
      const unsigned fi = L.g_fi[g];
      f = fi >> 8;
      i = fi & 0xffu;
      j = i + 1 + (p - L.g_pos[g]);
    }
    gbase += (unsigned)__popcll(gw);
    const unsigned sa = L.f_s0[f] + i, sb = L.f_s0[f] + (act ? j : i);
    unsigned long long v[WT];
    // item hashes in flight with the row words (see row_step)
    const unsigned long long ih_la = ihp[sa], ih_lb = ihp[sb];
    const unsigned c = and_count<WT>(bblk, bpad, sa, sb, v);
    const bool surv = act && c >= a.minsup;
    const unsigned long long mask = __ballot(surv);
    // member groups are runs of consecutive lanes: the first lane of each run updates its
    // group once, instead of one LDS atomic per survivor on the same address
    const bool head = act && (lane == 0 || ((gw >> lane) & 1ull));
    const unsigned long long hmask = __ballot(head);
    if (surv) {
      const unsigned pos = S + (unsigned)__popcll(mask & lanelt);
      const unsigned long long ih_a = ih_la, ih_b = ih_lb;
      write_row<WT>(cb, cpad, pos, v, ih_b);
      const DigestTerms dt = digest_terms(L.f_hash[f] + ih_a + ih_b, c);
      acc.dsum += dt.sum;
      acc.dxor ^= dt.xr;
    }
    if (E && mask) {
      const unsigned long long nb0 = alloc_nodes(a, st, (unsigned)__popcll(mask), lane);
      if (surv) {
        const unsigned pos = S + (unsigned)__popcll(mask & lanelt);
        const unsigned long long id = nb0 + (unsigned long long)__popcll(mask & lanelt);
        const unsigned long long nw_b = nwp[sb];
        put_node(a, id, nwp[sa] & kDeepNodeMask, (unsigned)(nw_b >> 40), c,
                 meta_depth(top.meta) + 2);
        cb[(unsigned long long)(WT + 1) * cpad + pos] = ((nw_b >> 40) << 40) | id;
      }
    }
    if (head) {
      const unsigned long long after = hmask & ~((2ull << lane) - 1ull);  // later run heads
      const unsigned long long below_end = after ? ((1ull << __builtin_ctzll(after)) - 1ull) : ~0ull;
      const unsigned long long rs = mask & below_end & ~lanelt;  // this run's survivors
      if (rs) {
        // one head per group in a chunk (its run of lanes), chunks in program order: plain
        // read-modify-writes, no two lanes on one group
        L.g_cnt[g] = (unsigned short)(L.g_cnt[g] + (unsigned)__popcll(rs));
        if (L.g_start[g] == 0xffffu) {
          const unsigned first = (unsigned)__builtin_ctzll(rs);
          L.g_start[g] = (unsigned short)(S + (unsigned)__popcll(mask & ((1ull << first) - 1ull)));
        }
      }
    }
    // the batch's frames are siblings of one block: one depth
    if (lane == 0 && mask) L.depth_cnt[meta_depth(top.meta) + 2] += (unsigned long long)__popcll(mask);
    S += (unsigned)__popcll(mask);
    ++acc.chunks;
  }
  acc.cands += P;
  acc.budget_used += (P + 63) / 64;
  // the k consumed frames leave the stack
  if ((unsigned)lane < k) {
    const unsigned b = meta_bidx(L.f_meta[lane]);
    if (b) atomicSub(&L.b_live[b - 1], 1u);
  }
  st.nf -= k;
  __builtin_amdgcn_wave_barrier();
  // child frames: groups with >= 2 survivors
  unsigned pushed = 0;
  const unsigned nbi = st.nb;
  for (unsigned g0 = 0; g0 < NG; g0 += 64) {
    const unsigned g = g0 + lane;
    bool mk = false;
    unsigned f = 0;
    if (g < NG) {
      for (unsigned step = 32; step; step >>= 1)
        if (f + step < k && L.G[f + step] <= g) f += step;
      mk = L.g_cnt[g] >= 2 && (a.max_len == 0 || (int)meta_depth(L.f_meta[f]) + 3 <= a.max_len);
    }
    const unsigned long long mask = __ballot(mk);
    if (mk) {
      const unsigned slot = st.nf + pushed + (unsigned)__popcll(mask & lanelt);
      const unsigned i = g - L.G[f];
      const unsigned long long ih_a = ihp[L.f_s0[f] + i];
      DeepFrame c;
      c.blk = (unsigned long long)cb;
      c.hash = L.f_hash[f] + ih_a;
      c.pad = (unsigned)cpad;
      c.s0 = L.g_start[g];
      c.m = L.g_cnt[g];
      c.meta = make_meta(meta_depth(L.f_meta[f]) + 1, false, WT, nbi + 1);
      store_frame(fst + slot, c);
    }
    pushed += (unsigned)__popcll(mask);
  }
  pushed = uni(pushed);
  if (pushed) {
    if (lane == 0) {
      L.b_base[st.nb] = (unsigned)st.mem_top;
      L.b_live[st.nb] = pushed;
    }
    st.nb += 1;
    st.nf += pushed;
    st.mem_top += (unsigned long long)(WT + 1 + E) * cpad * 8ull;
  }
}

// one step of the top frame, dispatched on its block width (wave-uniform)
template <int MAXT, bool EMIT, int T0, int... Ts>
__device__ __forceinline__ void step_tier(unsigned wt, bool row_mode, const DeepArgs& a,
                                          DeepFrame* fst, WaveState& st, WaveLds<MAXT>& L,
                                          const DeepFrame& top, const DeepFrame& lf,
                                          const WaveStack& stack, int lane, WaveAcc& acc) {
  if constexpr (T0 <= MAXT) {
    if (wt == (unsigned)T0) {
      if (row_mode)
        row_step<T0, MAXT, EMIT>(a, fst, st, L, top, stack, lane, acc);
      else
        batch_step<T0, MAXT, EMIT>(a, fst, st, L, top, lf, stack, lane, acc);
      return;
    }
  }
  if constexpr (sizeof...(Ts) > 0)
    step_tier<MAXT, EMIT, Ts...>(wt, row_mode, a, fst, st, L, top, lf, stack, lane, acc);
}

// waves per SIMD the count kernel is compiled for by default (blocks_per_cu may select the other
// instance of a width class).  4 up to MAXT 16: 128 VGPRs with ~20 spilled to scratch, and 8 KB
// of LDS tables per wave so four workgroups fit the CU — 33.2 vs 36.1 ms at ds1 @0.02 against
// 3 waves/SIMD at 162 VGPRs (profiles/r4p_*); the wider tiers keep their registers.
template <int MAXT>
constexpr int deep_waves_per_simd() { return MAXT <= 16 ? 4 : 2; }

template <int MAXT, int WPS, bool EMIT>
__global__ __launch_bounds__(256, WPS) __attribute__((amdgpu_waves_per_eu(WPS))) void k_deep_count(DeepArgs a) {
  __shared__ WaveLds<MAXT> lds[kWaves];
  const int lane = threadIdx.x & 63;
  const int wid = (int)uni(threadIdx.x >> 6);  // (uniform: the wave's pointers live in SGPRs)
  WaveLds<MAXT>& L = lds[wid];
  const unsigned long long gw = (unsigned long long)blockIdx.x * kWaves + wid;
  DeepFrame* fst = a.fstacks + gw * (unsigned long long)a.fcap;
  const WaveStack stack{a.stacks0 ? a.stacks0 + gw * a.seg0 : nullptr,
                        a.stacks + gw * a.stack_bytes, a.stacks0 ? a.seg0 : 0ull};

  for (int d = lane; d < 64; d += 64) L.depth_cnt[d] = 0;
  WaveAcc acc{0, 0, 0, 0, 0};
  __builtin_amdgcn_wave_barrier();

  WaveState st{0, 0, 0, 0, 0};
  constexpr unsigned E = EMIT ? 1u : 0u;
  bool failed = false;
  const unsigned long long t_start = wall_clock64();
  auto timed_out = [&]() {
    if (wall_clock64() - t_start <= a.timeout_ticks) return false;
    if (lane == 0) atomicOr(&a.ctl->error, 4u);
    return true;
  };
  // steal mode: this wave's inbox (direct hand-off from a wave it asked for work)
  const unsigned kOpen = (a.epoch << 2) | 1u, kFilling = (a.epoch << 2) | 2u,
                 kFull = (a.epoch << 2) | 3u, kClosed = a.epoch << 2;
  bool holding = false, inbox_open = false;
  unsigned long long t = 0;
  // instrumentation (a.trace != nullptr, zeroed by the host): kept in the wave's trace record,
  // not in registers held across the whole loop
  unsigned long long* tr = a.trace ? a.trace + gw * (unsigned long long)kDeepTraceWords : nullptr;
  unsigned victim = (unsigned)((gw * 7919ull + 1) % (unsigned long long)(a.nwaves > 0 ? a.nwaves : 1));
  while (!failed) {
    // ---- the next task: queue ticket t, or (steal mode, while t is not published) a class
    // another wave handed over on request ----
    if (!holding) {
      if (lane == 0) t = atomicAdd(&a.ctl->next_task, 1ull);
      t = uni64(bcast64(t, 0));
      holding = true;
    }
    DeepFrame tf;
    bool task_from_inbox = false;
    unsigned long long task_ticket = t;
    if (!a.steal) {
      if (t >= (unsigned long long)a.n_in) break;
      tf = load_frame(a.in + t, lane);
      holding = false;
    } else {
      if (tr && lane == 0 && t + 1 == (unsigned long long)a.n_in) a.ctl->t_drain = wall_clock64();
      // ticket t: wait on its own flag (waiting waves poll distinct addresses: one address
      // polled by thousands of waves serialises every device-scope access to it) until the task
      // is published (epoch) or the launch is over (epoch ^ kDone, written by the wave that
      // finished the last task over every ticket that can still be outstanding).  Meanwhile it
      // opens its inbox and asks busy waves, one mailbox at a time, for their oldest open class.
      bool done = false, from_inbox = false;
      for (unsigned n = 0;; ++n) {
        unsigned rdy = 0, fin = 0, inb = 0;
        if (lane == 0) {
          if (t < (unsigned long long)a.n_in) {
            rdy = 1u;
          } else if (t < (unsigned long long)a.out_cap) {
            const unsigned v = ld_agent(&a.ready[t - a.n_in]);
            rdy = v == a.epoch;
            fin = v == (a.epoch ^ kDone);
          } else if ((n & 63) == 63) {  // past the queue's capacity: never published
            fin = ld_agent(&a.ctl->pending) == 0ull;
          }
          if (inbox_open) {
            const unsigned sv = ld_agent(&a.inbox_state[gw]);
            inb = sv == kFull;
            // a hand-off in flight: finish receiving it before anything else
            if (sv == kFilling) rdy = fin = 0;
            if (rdy && !inb) {  // close the inbox before taking the ticket's task
              const unsigned old = atomicCAS(&a.inbox_state[gw], kOpen, kClosed);
              if (old != kOpen) rdy = 0;  // a donor claimed it meanwhile: receive that first
            }
          }
          // a failed wave never finishes its task: its error ends the wait of the others
          if (!rdy && !fin && !inb && (n & 255) == 255) fin = ld_agent(&a.ctl->error) != 0u;
        }
        inb = uni(__shfl(inb, 0, 64));
        if (inb) {
          from_inbox = true;
          break;
        }
        if (uni(__shfl(rdy, 0, 64))) break;
        if (uni(__shfl(fin, 0, 64))) { done = true; break; }
        if (!inbox_open) {  // not published yet: open the inbox, then start asking
          if (lane == 0) st_agent(&a.inbox_state[gw], kOpen);
          inbox_open = true;
        } else if ((n & a.ask_mask) == 1) {
          // (ask_fanout victims per ask: the first donor fills the inbox, the others find it
          // taken and keep their frames)
          if ((unsigned)lane < a.ask_fanout) {
            const unsigned v = (unsigned)((victim + 97ull * (unsigned)lane) % (unsigned long long)a.nwaves);
            if (v != (unsigned)gw)
              atomicExch(&a.req[v], ((unsigned long long)a.epoch << 32) | (unsigned long long)(gw + 1));
          }
          victim = (unsigned)((victim + 97ull * a.ask_fanout) % (unsigned long long)a.nwaves);
        }
        if (timed_out()) { failed = true; break; }
        wait_short(n < a.sleep_n ? n : a.sleep_n);
      }
      if (done || failed) break;
      task_from_inbox = from_inbox;
      task_ticket = t;
      if (from_inbox) {
        tf = load_frame_agent(a.inbox + gw, lane);
        if (lane == 0) st_agent(&a.inbox_state[gw], kClosed);
        inbox_open = false;  // ticket t is still held
      } else {
        inbox_open = false;
        holding = false;
        tf = t >= (unsigned long long)a.n_in ? load_frame_agent(a.in + t, lane)
                                             : load_frame(a.in + t, lane);
      }
    }
    {
      if (lane == 0) store_frame(fst, tf);
      // lanes exchange frames through memory: coherent within a wave in program order (one L1);
      // the wave barriers mark those hand-offs (the CPU emulator synchronises its lanes there)
      __builtin_amdgcn_wave_barrier();
      st.nf = 1;
      st.nb = 0;
      st.mem_top = 0;
    }
    acc.budget_used = 0;
    const unsigned long long tr_t0 = tr ? wall_clock64() : 0ull;
    if (tr && lane == 0 && tr[1] == 0) tr[1] = tr_t0;
    // ---- run the task ----
    unsigned steps = 0;
    while (st.nf > 0) {
      __builtin_amdgcn_wave_barrier();
      // bounded: a launch that runs past its deadline gives up (error bit 2) instead of holding
      // the GPU; the host reports it (the clock is read every 32 steps: s_memrealtime is a
      // scalar-memory round trip the step would otherwise wait for)
      if ((++steps & 31u) == 0u && timed_out()) {
        failed = true;
        break;
      }
      // the top min(nf, 64) frames, lane f holding frame nf-1-f, in ONE round of vector loads:
      // lane 0's is the top frame, and a batch step takes its frames from these registers (a
      // separate top-frame load was a dependent round trip of its own every step)
      DeepFrame lf;
      lf.blk = 0;
      lf.hash = 0;
      lf.pad = 0;
      lf.s0 = 0;
      lf.m = 0;
      lf.meta = kSingle;
      if ((unsigned)lane < st.nf) {
        const gptr<const DeepFrame> fp = as_global((const DeepFrame*)fst) + (st.nf - 1 - lane);
        lf.blk = fp->blk;
        lf.hash = fp->hash;
        lf.pad = fp->pad;
        lf.s0 = fp->s0;
        lf.m = fp->m;
        lf.meta = fp->meta;
      }
      DeepFrame top;
      top.blk = lane0_64(lf.blk);
      top.hash = lane0_64(lf.hash);
      top.pad = lane0(lf.pad);
      top.s0 = lane0(lf.s0);
      top.m = lane0(lf.m);
      top.meta = lane0(lf.meta);
      const unsigned m = top.m;
      const unsigned wt = meta_width(top.meta);
      const unsigned long long pairs = (unsigned long long)m * (m - 1) / 2;
      const bool row_mode = (top.meta & kSingle) || meta_lead(top.meta) ||
                            pairs > (unsigned long long)kCap;
      const unsigned long long need =
          (unsigned long long)(wt + 1 + E) * roundup16(row_mode ? m : kCap) * 8ull;
      const unsigned long long top_at =  // (a block never straddles the two stack parts)
          (st.mem_top < stack.n0 && st.mem_top + need > stack.n0) ? stack.n0 : st.mem_top;
      if (top_at + need > stack.n0 + a.stack_bytes || st.nf + kCap + 2 > (unsigned)a.fcap ||
          st.nb + 1 >= (unsigned)kBStack || (!a.steal && acc.budget_used >= a.budget)) {
        if (spill_frames<MAXT, EMIT>(a, fst, st, L, lane, false, st.nf,
                                     a.split_q ? (long long)task_ticket : -1ll) < 0)
          failed = true;
        break;
      }
      if (a.steal && acc.budget_used >= a.budget) {
        acc.budget_used = 0;
        if (a.steal_eager == 1) {
          // tests: the bottom frame to the shared queue at every check (a lone frame whole)
          if (spill_frames<MAXT, EMIT>(a, fst, st, L, lane, true, 1) == 0) {
            free_blocks(L, st);
            if (st.nf == 0) break;
            continue;
          }
        } else if (st.nf >= 2 ||
                   (a.split_keep16 && frame_firsts(top.meta, top.m) >= a.split_firsts)) {
          // a waiting wave asked (this wave's own mailbox): hand the bottom (oldest, largest)
          // open class straight to its inbox — split when large (donate_bottom) — and keep the
          // rest.  A lone small frame stays (handing the whole stack over just moves the class
          // to a wave that is asked in turn).
          unsigned long long r = 0;
          if (a.steal_eager == 2) {  // tests: offer to the partner wave whenever it waits
            r = (gw ^ 1ull) < (unsigned long long)a.nwaves ? (gw ^ 1ull) + 1ull : 0ull;
          } else if (lane == 0) {
            r = ld_agent(&a.req[gw]);
            if ((r >> 32) == (unsigned long long)a.epoch) st_agent(&a.req[gw], 0ull);
            else r = 0;
          }
          r = uni64(bcast64(r, 0));
          if (r && donate_bottom<MAXT, EMIT>(a, fst, st, L, lane, (unsigned)(r & 0xffffffffull) - 1u,
                                       kOpen, kFilling, kFull)) {
            free_blocks(L, st);
            continue;
          }
        }
      }
      if (wt == 0 || wt > (unsigned)MAXT) {  // never produced by the host or the steps
        if (lane == 0) atomicOr(&a.ctl->error, 8u);
        failed = true;
        break;
      }
      step_tier<MAXT, EMIT, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64>(wt, row_mode, a, fst, st, L, top,
                                                               lf, stack, lane, acc);
      free_blocks(L, st);
    }
    if (tr && !failed && lane == 0) {
      const unsigned long long now = wall_clock64();
      if (a.trace_bucket) {  // the busy interval spread over the time buckets
        constexpr unsigned long long kLast = (unsigned long long)(kDeepTraceBuckets - 1);
        unsigned long long x0 = tr_t0 - t_start;
        const unsigned long long x1 = now - t_start;
        while (x0 < x1) {
          const unsigned long long b0 = x0 / a.trace_bucket;
          const unsigned long long bk = b0 < kLast ? b0 : kLast;
          const unsigned long long e =
              bk == kLast ? x1 : ((bk + 1) * a.trace_bucket < x1 ? (bk + 1) * a.trace_bucket : x1);
          tr[6 + bk] += e - x0;
          x0 = e;
        }
      }
      tr[4] += now - tr_t0;
      tr[2] = now;
      tr[5] += (1ull << 32) | (task_from_inbox ? 1ull : 0ull);
      if (a.task_ticks && !task_from_inbox && task_ticket < (unsigned long long)a.n_in)
        a.task_ticks[task_ticket] = now - tr_t0;
    }
    if (a.steal && !failed) {  // the task is done
      unsigned long long left = 0;
      if (lane == 0) left = atomicSub(&a.ctl->pending, 1ull);
      left = uni64(bcast64(left, 0));
      if (left == 1) {
        // the last task: nothing can be spilled or handed over any more, so the tail is final
        // and every ticket at or past it is dead; each wave holds at most one, so nwaves flags
        // cover them
        unsigned long long tail = 0;
        if (lane == 0) tail = (unsigned long long)a.n_in + ld_agent(&a.ctl->n_out);
        tail = uni64(bcast64(tail, 0));
        for (unsigned long long k = lane; k < (unsigned long long)a.nwaves; k += 64)
          if (tail + k < (unsigned long long)a.out_cap)
            atomicExch(&a.ready[tail + k - a.n_in], a.epoch ^ kDone);
      }
    }
  }
  // flush: wave reduction of the digest terms, per-depth counts from LDS
  for (int off = 32; off; off >>= 1) {
    acc.dsum += shfl_xor64(acc.dsum, off);
    acc.dxor ^= shfl_xor64(acc.dxor, off);
  }
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    atomicAdd(&a.ctl->digest_sum, acc.dsum);
    atomicXor(&a.ctl->digest_xor, acc.dxor);
    atomicAdd(&a.ctl->candidates, acc.cands);
    atomicAdd(&a.ctl->chunks, acc.chunks);
  }
  for (int d = lane; d < 64; d += 64)
    if (L.depth_cnt[d]) atomicAdd(&a.ctl->per_depth[d], L.depth_cnt[d]);
  if (tr && lane == 0) {
    tr[0] = t_start;
    tr[3] = wall_clock64();
  }
}

// ---- root level: level-2 classes (deterministic, so every rank builds the same task list) ----

// bm [F][Wp] row-major -> root block [W][Fpad] word-major + item hashes [Fpad]
// (rows padded with zero words from W_real up to the instantiated width W)
__global__ void k_deep_transpose(const unsigned long long* bm, long long Wp, long long F, int W,
                                 int W_real, const int32_t* ids, unsigned long long* root,
                                 long long Fpad) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long tot = (long long)(W + 1) * Fpad;
  if (e >= tot) return;
  const long long w = e / Fpad, i = e - w * Fpad;
  unsigned long long v = 0;
  if (i < F) v = w == W ? item_mix((unsigned long long)ids[i]) : (w < W_real ? bm[i * Wp + w] : 0ull);
  root[e] = v;
}

// one wave per (root item i, chunk c of kRootChunk later items j) (lane = candidate): the
// level-2 class of i is counted / filled by ceil((F-1-i) / kRootChunk) waves instead of one, so
// the first classes (F-1 candidates) no longer set the launch's length (one wave per class:
// 144 + 339 us for the two passes at F = 2032, profiles/r4r_ktrace_headline.md).
// fill == false: count only, part[i * maxch + c] = the chunk's survivors;
// fill == true: part holds the chunk's exclusive base inside the class (k_deep_root_scan), block i
// (slots in j order) is written, projected onto row i (the block's width comes from its byte
// size: blk_off[i+1] - blk_off[i]) and, when ctl != nullptr, the level-2 digest terms added
template <int WT>
__global__ __launch_bounds__(256) void k_deep_root(const unsigned long long* root, long long Fpad,
                                                   long long F, int maxch, unsigned minsup,
                                                   const int32_t* m_in, int32_t* part,
                                                   const long long* blk_off, char* base,
                                                   DeepCtl* ctl, int fill, DeepNodes nodes,
                                                   const uint32_t* gram) {
  __shared__ ProjLds<WT> projs[kWaves];
  const int lane = threadIdx.x & 63;
  const long long gw = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long long i = gw / maxch;
  const long long ch = gw - i * maxch;
  if (i >= F) return;  // wave-uniform
  const long long nc = F - 1 - i;
  const long long cbeg = ch * kRootChunk;
  if (cbeg >= nc) {  // wave-uniform: past the class's candidates (an empty chunk)
    if (!fill && lane == 0) part[gw] = 0;
    return;
  }
  const long long cend = cbeg + kRootChunk < nc ? cbeg + kRootChunk : nc;
  ProjLds<WT>& PL = projs[threadIdx.x >> 6];
  const unsigned long long* ihp = root + (unsigned long long)WT * Fpad;
  const unsigned long long h_a = ihp[i];
  unsigned long long* cb = nullptr;
  unsigned long long cpad = 0;
  unsigned wt_out = WT;
  unsigned S = 0;
  const unsigned E = nodes.parent != nullptr;  // emit mode: node-word row + level-2 nodes
  if (fill) {
    cpad = roundup16((unsigned long long)m_in[i]);
    if (cpad == 0) return;  // wave-uniform: no frequent pair
    S = (unsigned)part[gw];  // this chunk's first slot
    // the chunk's survivors = the next chunk's first slot (or the class size) - S
    const long long nx = (ch + 1) * kRootChunk < nc ? (long long)part[gw + 1] : (long long)m_in[i];
    if (nx == (long long)S) return;  // wave-uniform: nothing to write
    cb = (unsigned long long*)(base + blk_off[i]);
    wt_out = (unsigned)((blk_off[i + 1] - blk_off[i]) / (long long)(8 * cpad)) - 1u - E;
    if (wt_out < (unsigned)WT) proj_setup<WT>(PL, as_global(root), (unsigned long long)Fpad, (unsigned)i, lane);
  }
  const bool proj = wt_out < (unsigned)WT;
  const unsigned S0 = S;
  unsigned long long dsum = 0, dxor = 0;
  const unsigned long long lanelt = (1ull << lane) - 1ull;
  for (long long c0 = cbeg; c0 < cend; c0 += 64) {
    const bool act = c0 + lane < cend;
    const long long jb = act ? i + 1 + c0 + lane : i;
    // with the pair gram (fill pass): 64 candidates without a survivor cost one coalesced read,
    // and only the survivors' lanes load their rows
    const bool pre = gram == nullptr || (act && gram[i * F + jb] >= minsup);
    if (gram != nullptr && __ballot(pre) == 0ull) continue;
    unsigned long long v[WT];
    unsigned c = 0;
    if (pre) c = and_count<WT>(as_global(root), (unsigned long long)Fpad, (unsigned)i + vzero(), (unsigned)jb, v);
    const bool surv = act && c >= minsup;
    const unsigned long long mask = __ballot(surv);
    if (fill) {
      const unsigned pos = S + (unsigned)__popcll(mask & lanelt);
      const unsigned long long ih_b = surv ? ihp[jb] : 0ull;
      if (proj)
        write_proj<WT>(cb, cpad, pos, surv, v, PL, wt_out, ih_b);
      else if (surv)
        write_row<WT>(cb, cpad, pos, v, ih_b);
      if (ctl && surv) {
        const DigestTerms dt = digest_terms(h_a + ih_b, c);
        dsum += dt.sum;
        dxor ^= dt.xr;
      }
      if (E && surv) {  // level-2 node (i, jb): id F + node_off[i] + slot
        const unsigned long long id = (unsigned long long)(F + nodes.node_off[i] + pos);
        nodes.parent[id] = (unsigned)i;
        nodes.item[id] = (unsigned)jb;
        nodes.count[id] = c;
        nodes.depth[id] = 2;
        cb[(unsigned long long)(wt_out + 1) * cpad + pos] = ((unsigned long long)jb << 40) | id;
      }
    }
    S += (unsigned)__popcll(mask);
  }
  if (!fill) {
    if (lane == 0) part[gw] = (int32_t)S;
    return;
  }
  if (ctl) {
    for (int off = 32; off; off >>= 1) {
      dsum += shfl_xor64(dsum, off);
      dxor ^= shfl_xor64(dxor, off);
    }
    if (lane == 0 && S > S0) {
      atomicAdd(&ctl->digest_sum, dsum);
      atomicXor(&ctl->digest_xor, dxor);
    }
  }
}

// the count pass from the level-2 pair gram (upper triangle, row-major F x F, rank order): one
// wave per (class i, chunk of kRootChunk candidates), part[i * maxch + c] = the chunk's pairs
// with support >= minsup (one coalesced read per 64 candidates instead of their AND rows)
__global__ __launch_bounds__(256) void k_deep_root_gcount(const uint32_t* gram, long long F,
                                                          int maxch, unsigned minsup,
                                                          int32_t* part) {
  const int lane = threadIdx.x & 63;
  const long long gw = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long long i = gw / maxch;
  const long long ch = gw - i * maxch;
  if (i >= F) return;  // wave-uniform
  const long long nc = F - 1 - i;
  const long long cbeg = ch * kRootChunk;
  const long long cend = cbeg + kRootChunk < nc ? cbeg + kRootChunk : nc;
  unsigned S = 0;
  for (long long c0 = cbeg; c0 < cend; c0 += 64) {
    const bool act = c0 + lane < cend;
    S += (unsigned)__popcll(__ballot(act && gram[i * F + i + 1 + c0 + lane] >= minsup));
  }
  if (lane == 0) part[gw] = (int32_t)S;  // (0 for a chunk past the class's candidates)
}

// one wave: inclusive prefix sums of three int64 arrays of n entries, in place (the level-2
// layout: block byte offsets, task offsets, node ids; n = F + 1, a few thousand)
__global__ __launch_bounds__(64) void k_deep_prefix3(long long* a, long long* b, long long* c,
                                                     long long n) {
  __shared__ long long sh[3][64];
  const int t = threadIdx.x & 63;
  const long long per = (n + 63) / 64;
  const long long lo = (long long)t * per;
  const long long hi = lo + per < n ? lo + per : n;
  long long sa = 0, sb = 0, sc = 0;
  // 8 independent loads of each array in flight per lane (a serial chain of dependent loads
  // took 27 us at n = 2033)
  long long k = lo;
  for (; k + 8 <= hi; k += 8) {
    long long va[8], vb[8], vc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      va[u] = a[k + u];
      vb[u] = b[k + u];
      vc[u] = c[k + u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      sa += va[u];
      sb += vb[u];
      sc += vc[u];
    }
  }
  for (; k < hi; ++k) {
    sa += a[k];
    sb += b[k];
    sc += c[k];
  }
  sh[0][t] = sa;
  sh[1][t] = sb;
  sh[2][t] = sc;
  __builtin_amdgcn_wave_barrier();
  if (t < 3) {  // exclusive scan of the 64 partials of one array
    long long run = 0;
    for (int q = 0; q < 64; ++q) {
      const long long v = sh[t][q];
      sh[t][q] = run;
      run += v;
    }
  }
  __builtin_amdgcn_wave_barrier();
  long long ra = sh[0][t], rb = sh[1][t], rc = sh[2][t];
  for (long long q = lo; q < hi; q += 8) {
    const int cnt = hi - q < 8 ? (int)(hi - q) : 8;
    long long va[8], vb[8], vc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (u < cnt) {
        va[u] = a[q + u];
        vb[u] = b[q + u];
        vc[u] = c[q + u];
      }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (u < cnt) {
        ra += va[u];
        a[q + u] = ra;
        rb += vb[u];
        b[q + u] = rb;
        rc += vc[u];
        c[q + u] = rc;
      }
  }
}

// per root class i (thread): the chunk counts of the count pass -> exclusive chunk bases (in
// place), m[i], and the three per-class sizes whose prefix sums lay out the level-2 blocks (byte
// offsets from the class's projected width tier wt[i]), the level-3 tasks and (emit) the level-2
// node ids: sz[k][i + 1] (sz[k][0] = the first offset: root block bytes / 0 / 0)
__global__ void k_deep_root_scan(int32_t* part, int maxch, long long F, const int32_t* wt,
                                 unsigned extra, long long root_blk, int32_t* m,
                                 long long* sz_blk, long long* sz_task, long long* sz_node) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    sz_blk[0] = root_blk;
    sz_task[0] = 0;
    sz_node[0] = 0;
  }
  if (i >= F) return;
  int32_t tot = 0;
  for (int c = 0; c < maxch; ++c) {
    const int32_t v = part[i * maxch + c];
    part[i * maxch + c] = tot;
    tot += v;
  }
  m[i] = tot;
  sz_blk[i + 1] = (long long)(wt[i] + 1 + (int)extra) * (long long)roundup16((unsigned long long)tot) * 8;
  sz_task[i + 1] = tot > 1 ? tot - 1 : 0;
  sz_node[i + 1] = tot;
}

// this rank's level-3 tasks: out[q] = task order[q] (order == nullptr: task q*world + rank, the
// interleaved split); task t = (root i, member k), t = task_off[i] + k
__global__ void k_deep_root_tasks(const long long* blk_off, const int32_t* m, const long long* task_off,
                                  long long F, char* base, const unsigned long long* root,
                                  long long Fpad, int W, int rank, int world,
                                  const long long* order, long long n, DeepFrame* out,
                                  unsigned extra) {
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n;
       q += (long long)gridDim.x * blockDim.x) {
    const long long t = order ? order[q] : q * world + rank;
    // root i: the last with task_off[i] <= t (empty classes share their offset with the next)
    long long lo = 0, hi = F - 1;
    while (lo < hi) {
      const long long mid = (lo + hi + 1) >> 1;
      if (task_off[mid] <= t) lo = mid;
      else hi = mid - 1;
    }
    const long long i = lo;
    const int mi = m[i];
    const long long k = t - task_off[i];
    const unsigned long long pad = roundup16((unsigned long long)mi);
    const unsigned wt = (unsigned)((blk_off[i + 1] - blk_off[i]) / (long long)(8 * pad)) - 1u - extra;
    DeepFrame f;
    f.blk = (unsigned long long)(base + blk_off[i]);
    f.hash = root[(unsigned long long)W * Fpad + i];
    f.pad = (unsigned)pad;
    f.s0 = (unsigned)k;
    f.m = (unsigned)(mi - k);
    f.meta = make_meta(1, true, wt, 0);
    store_frame(out + q, f);
  }
}

// cost[task_off[i] + k] = members j > k of root class i with |row_k & row_j| >= minsup: the size
// of the class task (i, k) expands (one wave per task, lanes over j; block widths are runtime)
__global__ __launch_bounds__(256) void k_deep_task_cost(const long long* blk_off, const int32_t* m,
                                                        const long long* task_off, long long F,
                                                        const char* base, unsigned minsup,
                                                        unsigned* cost, unsigned extra,
                                                        unsigned* key, int key_mode) {
  const long long i = blockIdx.x;
  if (i >= F) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int mi = m[i];
  if (mi < 2) return;
  const unsigned long long pad = roundup16((unsigned long long)mi);
  const unsigned wt = (unsigned)((blk_off[i + 1] - blk_off[i]) / (long long)(8 * pad)) - 1u - extra;
  const unsigned long long* blk = (const unsigned long long*)(base + blk_off[i]);
  for (int k = wid; k < mi - 1; k += (int)(blockDim.x >> 6)) {
    unsigned c = 0;
    unsigned long long mass = 0;  // (key_mode 1) the survivors' supports above minsup - 1
    for (int j0 = k + 1; j0 < mi; j0 += 64) {
      const int j = j0 + lane;
      unsigned pc = 0;
      if (j < mi)
        for (unsigned w = 0; w < wt; ++w)
          pc += (unsigned)__popcll(blk[(unsigned long long)w * pad + k] & blk[(unsigned long long)w * pad + j]);
      const bool surv = j < mi && pc >= minsup;
      c += (unsigned)__popcll(__ballot(surv));
      if (key_mode == 1) {
        unsigned long long x = surv ? (unsigned long long)(pc - minsup + 1u) : 0ull;
        for (int o = 32; o; o >>= 1) x += __shfl_xor(x, o, 64);
        mass += x;
      }
    }
    if (lane == 0) {
      cost[task_off[i] + k] = c;
      // the deal's sort key: the class size (0), its support mass (1) or its square (2)
      if (key)
        key[task_off[i] + k] =
            key_mode == 1 ? (unsigned)(mass < 0xFFFFFFFFull ? mass : 0xFFFFFFFFull)
            : key_mode == 2 ? (c < 65535u ? c * c : 0xFFFFFFFFu) : c;
    }
  }
}

// emit-mode verification, one pass per itemset size d: every node of size d takes its set hash
// from its parent's (size d-1, hashed in the previous pass) plus its item's mix, then adds its
// digest terms; out = [sum, xor, per_depth[64]]
__global__ __launch_bounds__(256) void k_arena_digest(const unsigned* parent, const unsigned* item,
                                                      const unsigned* count,
                                                      const unsigned char* depth, long long n,
                                                      const int32_t* ids, int d, int count_it,
                                                      unsigned long long* hash,
                                                      unsigned long long* out) {
  unsigned long long sum = 0, xr = 0, cnt = 0;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < n;
       v += (long long)gridDim.x * blockDim.x) {
    if (depth[v] != d) continue;
    const unsigned long long h = (d == 1 ? 0ull : hash[parent[v]]) + item_mix((unsigned long long)ids[item[v]]);
    hash[v] = h;
    if (!count_it) continue;
    const DigestTerms t = digest_terms(h, count[v]);
    sum += t.sum;
    xr ^= t.xr;
    cnt += 1;
  }
  for (int off = 32; off; off >>= 1) {
    sum += shfl_xor64(sum, off);
    xr ^= shfl_xor64(xr, off);
    cnt += shfl_xor64(cnt, off);
  }
  if ((threadIdx.x & 63) == 0 && cnt) {
    atomicAdd(out, sum);
    atomicXor(out + 1, xr);
    atomicAdd(out + 2 + d, cnt);
  }
}

// instantiated widths: the tiers (root blocks, and the count kernel's widest tier)
template <typename Fn>
void by_tier(int W, Fn&& fn) {
  switch (W) {
    case 1: fn(std::integral_constant<int, 1>{}); break;
    case 2: fn(std::integral_constant<int, 2>{}); break;
    case 3: fn(std::integral_constant<int, 3>{}); break;
    case 4: fn(std::integral_constant<int, 4>{}); break;
    case 6: fn(std::integral_constant<int, 6>{}); break;
    case 8: fn(std::integral_constant<int, 8>{}); break;
    case 12: fn(std::integral_constant<int, 12>{}); break;
    case 16: fn(std::integral_constant<int, 16>{}); break;
    case 24: fn(std::integral_constant<int, 24>{}); break;
    case 32: fn(std::integral_constant<int, 32>{}); break;
    case 48: fn(std::integral_constant<int, 48>{}); break;
    case 64: fn(std::integral_constant<int, 64>{}); break;
    default: break;  // deep_tier() never returns another width
  }
}

}  // namespace

void deep_arena_digest(const unsigned* parent, const unsigned* item, const unsigned* count,
                       const unsigned char* depth, int64_t n, const int32_t* ids, int max_depth,
                       int min_depth, uint64_t* hash, unsigned long long* out, hipStream_t s) {
  if (n <= 0) return;
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
  for (int d = 1; d <= max_depth && d < 62; ++d)
    hipLaunchKernelGGL(k_arena_digest, dim3(grid), dim3(256), 0, s, parent, item, count, depth,
                       (long long)n, ids, d, d >= min_depth ? 1 : 0, (unsigned long long*)hash, out);
}

int deep_max_words() { return 64; }
int deep_tier(int words) { return (int)tier_of((unsigned)std::max(words, 1)); }
int deep_row_words(int W) { return deep_tier(W); }
int deep_count_maxt(int widest) { return widest <= 8 ? 8 : widest <= 16 ? 16 : widest <= 32 ? 32 : 64; }
int deep_waves_per_simd(int maxt) {
  return maxt <= 8 ? deep_waves_per_simd<8>() : maxt <= 16 ? deep_waves_per_simd<16>()
       : maxt <= 32 ? deep_waves_per_simd<32>() : deep_waves_per_simd<64>();
}
int deep_waves_per_block() { return kWaves; }
int deep_min_fcap() { return kCap + 64; }
int deep_node_chunk() { return (int)kNodeChunk; }

size_t deep_row_block_bytes(int W, int64_t m, int extra) {
  return (size_t)(W + 1 + extra) * (size_t)roundup16((unsigned long long)std::max<int64_t>(m, kCap)) * 8;
}

void deep_transpose(const uint64_t* bm, int64_t Wp, int64_t F, int W, int W_real,
                    const int32_t* ids, uint64_t* root, int64_t Fpad, hipStream_t s) {
  const int64_t tot = (int64_t)(W + 1) * Fpad;
  hipLaunchKernelGGL(k_deep_transpose, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                     (const unsigned long long*)bm, (long long)Wp, (long long)F, W, W_real, ids,
                     (unsigned long long*)root, (long long)Fpad);
}

int deep_root_chunks(int64_t F) { return (int)std::max<int64_t>(1, (F - 1 + kRootChunk - 1) / kRootChunk); }

void deep_root(const uint64_t* root, int64_t Fpad, int64_t F, int W, uint32_t minsup,
               const int32_t* m, int32_t* part, const int64_t* blk_off, char* base, DeepCtl* ctl,
               bool fill, hipStream_t s, const DeepNodes* nodes, const uint32_t* gram) {
  if (F <= 0) return;
  const int maxch = deep_root_chunks(F);
  const unsigned grid = (unsigned)((F * maxch + kWaves - 1) / kWaves);
  if (gram != nullptr && !fill) {
    hipLaunchKernelGGL(k_deep_root_gcount, dim3(grid), dim3(64 * kWaves), 0, s, gram,
                       (long long)F, maxch, minsup, part);
    return;
  }
  DeepNodes nd{};
  if (nodes && fill) nd = *nodes;
  by_tier(W, [&](auto wt) {
    hipLaunchKernelGGL(k_deep_root<decltype(wt)::value>, dim3(grid), dim3(64 * kWaves), 0, s,
                       (const unsigned long long*)root, (long long)Fpad, (long long)F, maxch,
                       minsup, m, part, (const long long*)blk_off, base, ctl, fill ? 1 : 0, nd,
                       gram);
  });
}

void deep_root_scan(int32_t* part, int64_t F, const int32_t* wt, int extra, int64_t root_blk,
                    int32_t* m, int64_t* off, int64_t* task_off, int64_t* node_off, hipStream_t s) {
  if (F <= 0) return;
  hipLaunchKernelGGL(k_deep_root_scan, dim3((unsigned)((F + 255) / 256)), dim3(256), 0, s, part,
                     deep_root_chunks(F), (long long)F, wt, (unsigned)extra, (long long)root_blk,
                     m, (long long*)off, (long long*)task_off, (long long*)node_off);
  hipLaunchKernelGGL(k_deep_prefix3, dim3(1), dim3(64), 0, s, (long long*)off,
                     (long long*)task_off, (long long*)node_off, (long long)(F + 1));
}

void deep_root_tasks(const int64_t* blk_off, const int32_t* m, const int64_t* task_off, int64_t F,
                     char* base, const uint64_t* root, int64_t Fpad, int W, int rank, int world,
                     const int64_t* order, int64_t n, DeepFrame* out, hipStream_t s, int extra) {
  if (F <= 0 || n <= 0) return;
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_deep_root_tasks, dim3(grid), dim3(256), 0, s,
                     (const long long*)blk_off, m, (const long long*)task_off, (long long)F, base,
                     (const unsigned long long*)root, (long long)Fpad, W, rank, world,
                     (const long long*)order, (long long)n, out, (unsigned)extra);
}

void deep_task_cost(const int64_t* blk_off, const int32_t* m, const int64_t* task_off, int64_t F,
                    const char* base, uint32_t minsup, uint32_t* cost, hipStream_t s, int extra,
                    uint32_t* key, int key_mode) {
  if (F <= 0) return;
  hipLaunchKernelGGL(k_deep_task_cost, dim3((unsigned)F), dim3(256), 0, s,
                     (const long long*)blk_off, m, (const long long*)task_off, (long long)F, base,
                     minsup, cost, (unsigned)extra, key, key_mode);
}

int deep_count_wps(int maxt, int want, bool emit) {
  const int mt = deep_count_maxt(maxt);
  // emit at MAXT 16: 4 waves/SIMD since the wave id is uniform (the wave's pointers in SGPRs:
  // 44.0-44.8 vs 45.6-46.0 ms at 3 waves, profiles/r6s_*); 3 on request
  if (emit) return mt == 8 ? 4 : mt == 16 ? (want == 3 ? 3 : 4) : 2;  // (launched instances)
  if (mt == 8 && (want == 4 || want == 5)) return want;
  if (mt == 16 && (want == 3 || want == 4)) return want;
  if (mt == 32 && (want == 2 || want == 3)) return want;
  return deep_waves_per_simd(mt);
}

void deep_count(const DeepArgs& a, int maxt, int wps, int grid, hipStream_t s) {
  const int mt = deep_count_maxt(maxt);
  const int w = deep_count_wps(mt, wps, a.node_parent != nullptr);
  const dim3 g((unsigned)grid), b(64 * kWaves);
  if (a.node_parent != nullptr) {  // emit mode: the default occupancy of each width class
    // (round 4 kept emit at 3 waves/SIMD for MAXT 16: its node-id bookkeeping pushed a 128-VGPR
    // build into heavy spills, 56.7 vs 51.5 ms, profiles/r4r_*; with the wave id uniform the
    // 4-wave build spills little and wins)
    if (mt == 8) hipLaunchKernelGGL((k_deep_count<8, 4, true>), g, b, 0, s, a);
    else if (mt == 16 && w == 4) hipLaunchKernelGGL((k_deep_count<16, 4, true>), g, b, 0, s, a);
    else if (mt == 16) hipLaunchKernelGGL((k_deep_count<16, 3, true>), g, b, 0, s, a);
    else if (mt == 32) hipLaunchKernelGGL((k_deep_count<32, 2, true>), g, b, 0, s, a);
    else hipLaunchKernelGGL((k_deep_count<64, 2, true>), g, b, 0, s, a);
    return;
  }
  if (mt == 8 && w == 5) hipLaunchKernelGGL((k_deep_count<8, 5, false>), g, b, 0, s, a);
  else if (mt == 8) hipLaunchKernelGGL((k_deep_count<8, 4, false>), g, b, 0, s, a);
  else if (mt == 16 && w == 4) hipLaunchKernelGGL((k_deep_count<16, 4, false>), g, b, 0, s, a);
  else if (mt == 16) hipLaunchKernelGGL((k_deep_count<16, 3, false>), g, b, 0, s, a);
  else if (mt == 32 && w == 3) hipLaunchKernelGGL((k_deep_count<32, 3, false>), g, b, 0, s, a);
  else if (mt == 32) hipLaunchKernelGGL((k_deep_count<32, 2, false>), g, b, 0, s, a);
  else hipLaunchKernelGGL((k_deep_count<64, 2, false>), g, b, 0, s, a);
}

}  // namespace kern
}  // namespace kmls
