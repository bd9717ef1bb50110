// kernels.hpp -- the BFS level kernels for MI355X (gfx950).
//
// k_level<P, ROUTE>: ONE launch per BFS level (Search.java:448-504 with the level barrier of
// :452-455 made explicit). Each workgroup takes a chunk of PB consecutive frontier states:
//   1. the chunk (contiguous rows, PB x S bytes) and its fingerprints are copied to LDS with
//      16-byte coalesced loads -- every parent is read from HBM exactly once;
//   2. one lane per parent counts its enabled events (SearchState.events), a workgroup-local
//      exclusive scan turns the counts into work-item offsets (no global scan pass);
//   3. the chunk's work items (parent j, event k) are listed per parent and counting-sorted by
//      handler class (ballots), so a wavefront mostly runs one handler; every lane takes one:
//      the successor is computed as a DELTA in registers (one node's words + a short send
//      list), its fingerprint incrementally from the parent's (nodestate.hpp), then one 64-byte
//      visited-table bucket probe / CAS insert (discovered.add, Search.java:485). Only a NEW
//      successor is judged (checkState over a node view: parent words in LDS + the changed
//      node); terminal candidates fold into the level's exact best (fold_terminals);
//      An event that changes neither its node nor the network (most redeliveries: the network
//      is a set, every message stays deliverable) leads back to the parent: no fingerprint, no
//      probe. A VALID successor reserves a row (one returning atomic per wavefront) and the
//      wavefront writes its rows cooperatively (row + fingerprint + parent pointer + event).
//   ROUTE (multi-shard): a successor is not probed here; its 16-byte fingerprint goes to its owner's
//      outgoing region instead (bfs_engine.hpp runs the other phases).
#pragma once
#include "nodestate.hpp"

namespace dsl {

constexpr int kBlock = 256;
// k_level workgroup: 4 wavefronts share a chunk of parents staged in LDS (measured: one
// wavefront per workgroup is slower -- its smaller chunks sort into more handler classes per
// wavefront -- despite having no cross-wavefront barrier waits).
constexpr int kLevelBlock = 256;
constexpr uint32_t kTermCap = 1024;  // default TerminalRec entries per shard (DSL_TERM_CAP)
constexpr int kMaxShards = 16;
#ifndef DSL_KWIN
#define DSL_KWIN 1024
#endif
constexpr int kWin = DSL_KWIN;  // work items per class-sorted window of k_level
// a located event in 16 bits: record indices < kNetCap, timers -1 - (node * 256 + j) >= -4096
constexpr int kEvNone = -32768;
// The next frontier is written into up to kSegs segments, one reservation counter each (a
// workgroup appends to segment blockIdx % nseg), so every wavefront reserves its rows with one
// returning atomic and no workgroup barrier, and no counter word carries more than 1/kSegs of
// the level's reservations. A frontier is then a short list of row ranges: the segments, the
// spill range and (multi-shard) the received range.
constexpr int kSegs = 32;
// LDS budget for a k_level chunk's staged parent rows: with the kernel's ~11 KB of static LDS, 4
// resident workgroups per CU (the 4 waves/SIMD the register budget allows) fit in 160 KB.
#ifndef DSL_ROWS_LDS_KB
#define DSL_ROWS_LDS_KB 24
#endif
#ifndef DSL_ROWS_LDS_BYTES  // the same budget in bytes (measurement builds set it between whole KB)
#define DSL_ROWS_LDS_BYTES (DSL_ROWS_LDS_KB * 1024)
#endif
// 1: the parents' node hashes are computed once per chunk and kept in LDS (80 B per Multi-Paxos
// parent); 0: every probing lane hashes its changed node's old words itself (more parents per chunk)
#ifndef DSL_NH_LDS
#define DSL_NH_LDS 1
#endif
// Row stride of the staged parents in LDS (dwords). A packed row is a multiple of 16 B, and
// Multi-Paxos's is 160 dwords = 0 mod 32: at stride kWords every lane-per-parent access of word c
// (node hashes, event counts, classification, the handlers' parent reads) hits bank c mod 32, a
// 32-way conflict per ds_read_b32 group (2.9 extra LDS cycles per LDS instruction on
// C5). A row stride padded by DSL_LDS_PAD dwords spreads consecutive parents over the banks:
//   pad 4 (16-B aligned rows): staged by LDS-DMA, one global_load_lds_dwordx4 per row (lanes over
//     the row's 16-byte units), 8 distinct banks per 32 parents;
//   pad 1 / 2: 32 / 16 distinct banks, staged through registers (LDS-DMA writes lane x 16 B);
//   pad 0: the rows back to back, one DMA instruction per 1 KiB.
// Default: pad 4 for a protocol whose row is 0 mod 32 dwords and has at least 64 words (one DMA
// instruction per row is then at least 16 active lanes), else 0.
template <class P>
struct LdsRow {
  static constexpr int kWords = Layout<P>::kWords;
#ifdef DSL_LDS_PAD
  static constexpr int kPad = DSL_LDS_PAD;
#else
  static constexpr int kPad = (kWords % 32 == 0 && kWords >= 64) ? 4 : 0;
#endif
  static constexpr int kStride = kWords + kPad;
  // dwords of a chunk's row image (rounded to 16 B, so the fingerprints after it stay aligned)
  static constexpr int image(int pb) { return (pb * kStride + 3) / 4 * 4; }
};
constexpr int kMaxSegs = kSegs + 2;
constexpr int kSegStride = 16;  // u64 words between segment counters (one 128-byte line each)
constexpr int kCtrSegOff = 4096;                                  // segment counters inside a counter set
constexpr int kCtrSet = kCtrSegOff + kSegs * kSegStride * 8;      // bytes of one counter set

struct SegTable {
  int32_t n;
  int32_t pb;                     // parents per chunk
  uint64_t base[kMaxSegs];
  uint64_t cnt[kMaxSegs];
  uint64_t chunk0[kMaxSegs + 1];  // first chunk of each segment; chunk0[n] = chunks of the level
};

struct LevelCounters {
  unsigned long long new_states;    // newly discovered successors (all verdicts)
  unsigned long long next_size;     // VALID successors appended to the next frontier
  unsigned long long successors;    // events applied (non-null successors)
  unsigned long long n_terminals;   // terminal candidates of the level
  unsigned long long err_overflow;  // STEP_OVERFLOW count
  unsigned long long err_table;     // INS_FULL count
  unsigned long long err_frontier;  // appends beyond capacity
  unsigned long long work_items;    // (state, event) pairs of this level
  unsigned long long next_work;     // enabled events of the appended states (= next level's work)
  unsigned long long spilled;       // VALID states beyond the next frontier's capacity (spill list)
  unsigned long long term_best;     // ~(best terminal key) of the level (atomicMax; 0 = none)
  unsigned long long n_term_rec;    // TerminalRec entries written (improvements of term_best)
  unsigned long long probes;        // visited-table probes (successors that are not no-ops)
  unsigned long long cum_before;    // queued levels: new states of the queue's earlier levels
  unsigned long long time_up;       // the search's deadline passed during this level (it is partial)
  unsigned long long route_spilled; // routed successors past their destination region (rspill list)
  unsigned long long unspilled;     // rows k_unspill appended (multi-shard fast path: device count)
  unsigned long long deduped;       // successors found in the chunk's LDS set (ChunkDedup): not probed / routed
  unsigned long long phase[12];     // DSL_PHASES builds only: shader cycles per k_level phase
  unsigned long long phcls[32];     // DSL_PHASES: handler cycles per class [0, 16), wave-passes [16, 32)
};

// Phase timing (instrumented builds, -DDSL_PHASES): wave-level shader-clock deltas per phase of
// k_level, summed per workgroup and flushed once. Product builds compile it away.
#ifdef DSL_PHASES
#define PH_DECL unsigned long long ph_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long ph_t = clock64();
#define PH_MARK(i) do { const unsigned long long ph_n = clock64(); ph_acc[i] += ph_n - ph_t; ph_t = ph_n; } while (0)
#define PH_FLUSH(red, ctr) do { for (int ph_i = 0; ph_i < 12; ph_i++) block_flush<kLevelBlock>(red, &(ctr)->phase[ph_i], __lane_id() == 0 ? ph_acc[ph_i] : 0ull); } while (0)
#define PH_CLS_DECL __shared__ unsigned long long s_phcls[32]; if (threadIdx.x < 32) s_phcls[threadIdx.x] = 0;
#define PH_CLS_T0 const unsigned long long ph_c0 = clock64();
#define PH_CLS_ADD(cls, active) do { const unsigned long long ph_c1 = clock64(); if (__lane_id() == 0 && (active)) { atomicAdd(&s_phcls[(cls) & 15], ph_c1 - ph_c0); atomicAdd(&s_phcls[16 + ((cls) & 15)], 1ull); } } while (0)
#define PH_CLS_FLUSH(ctr) do { __syncthreads(); if (threadIdx.x < 32 && s_phcls[threadIdx.x]) atomicAdd(&(ctr)->phcls[threadIdx.x], s_phcls[threadIdx.x]); } while (0)
#elif defined(DSL_TIMELINE)
// Timeline builds (-DDSL_TIMELINE): the real-time clock (s_memrealtime, 100 MHz) at each phase mark
// of workgroup 0's first thread (phcls[0..31] = mark id << 56 | time), the earliest workgroup
// entry (phase[0], complemented) and the latest exit (phase[1]) of every workgroup, WG 0's entry
// (phase[2]).
#define PH_DECL                                                                                   \
  const bool tl_on = blockIdx.x == 0 && threadIdx.x == 0;                                         \
  unsigned tl_n = 0;                                                                              \
  {                                                                                               \
    const unsigned long long tl_t = __builtin_amdgcn_s_memrealtime();                             \
    if (threadIdx.x == 0 && (kTlAll || blockIdx.x == 0)) atomicMax(&a.ctr->phase[0], ~tl_t);     \
    if (tl_on) a.ctr->phase[2] = tl_t;                                                            \
  }
#define PH_MARK(i) do { if (tl_on && tl_n < 32) a.ctr->phcls[tl_n++] = ((unsigned long long)(i) << 56) | (__builtin_amdgcn_s_memrealtime() & ((1ull << 56) - 1)); } while (0)
#define PH_FLUSH(red, ctr) do { __syncthreads(); if (threadIdx.x == 0 && (kTlAll || blockIdx.x == 0)) atomicMax(&(ctr)->phase[1], __builtin_amdgcn_s_memrealtime()); } while (0)
// -DDSL_TIMELINE_WG0: only workgroup 0 touches the entry / exit words (the 1,024 entry atomics of
// the default on one word serialize and add several microseconds to a small level's prologue)
#ifdef DSL_TIMELINE_WG0
constexpr bool kTlAll = false;
#else
constexpr bool kTlAll = true;
#endif
#define PH_CLS_DECL
#define PH_CLS_T0
#define PH_CLS_ADD(cls, active) do { } while (0)
#define PH_CLS_FLUSH(ctr) do { } while (0)
#else
#define PH_CLS_DECL
#define PH_CLS_T0
#define PH_CLS_ADD(cls, active) do { } while (0)
#define PH_CLS_FLUSH(ctr) do { } while (0)
#define PH_DECL
#define PH_MARK(i) do { } while (0)
#define PH_FLUSH(red, ctr) do { } while (0)
#endif

static_assert(sizeof(LevelCounters) <= kCtrSegOff, "LevelCounters must fit before the segment counters");

struct TerminalRec {
  int32_t verdict;  // V_TERM_*
  int32_t pred_index;
  uint32_t event;   // event index within the parent's enabled events
  uint32_t pad;
  uint64_t parent;  // index of the parent in the current frontier
  uint64_t key;     // term_key: priority rank << 62 | fingerprint bits (deterministic tie-break)
};

// Route counters of a sharded level: per destination shard d, kRouteSegs counters (a workgroup
// reserves in counter blockIdx % kRouteSegs), each on its own 128-byte line -- one counter per
// destination was a single hot word that every workgroup's returning atomic hit once per pass.
// Region d of a shard's routed records: a header of kRouteHdr 16-byte records (the kRouteSegs
// counts, one u64 each), then kRouteSegs sub-slabs of `cs` records (sub-slab q holds the records
// of counter q); the whole region is one slab of the exchange.
constexpr int kRouteSegs = 32;
constexpr int kRouteStride = 16;
constexpr int kRouteHdr = kRouteSegs / 2;
// The same regions as they cross the links (round A): 12-byte packed records {lo[0, 32), hi} --
// all an owner's probe reads of a fingerprint (the home bucket and key bits of lo are below bit
// 32, kKeyBits; the owner bits, lo's top 32, are implied by the destination) -- after a header of
// kPkHdr records holding the 32 counts (64 words). A region is kPkWords * (kPkHdr + 32 cs) words.
constexpr int kPkWords = 3;
constexpr int kPkHdr = (2 * kRouteSegs + kPkWords - 1) / kPkWords;
__host__ __device__ inline uint64_t pk_region_words(uint64_t cs) { return (uint64_t)kPkWords * (kPkHdr + kRouteSegs * cs); }
struct RouteCounters {
  unsigned long long out[kMaxShards * kRouteSegs * kRouteStride];
};
__host__ __device__ inline int rc_idx(int d, int q) { return (d * kRouteSegs + q) * kRouteStride; }



__device__ __forceinline__ uint32_t rl32(uint32_t v, int src) { return (uint32_t)__builtin_amdgcn_readlane((int)v, src); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int src) {
  return (uint64_t)rl32((uint32_t)v, src) | ((uint64_t)rl32((uint32_t)(v >> 32), src) << 32);
}

// Wave-wide inclusive prefix sum over the 64 lanes on DPP (GFX9 row_shr 1/2/4/8 inside each row of
// 16 lanes, then row_bcast:15 and row_bcast:31 across rows): no LDS crossbar traffic
// (ds_bpermute) and no per-lane source-address registers kept live. Every lane must be active.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 (rows 1, 3)
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 (rows 2, 3)
  return x;
}
// The same inside each row of 16 lanes only (a scan of at most 16 values held by lanes 0-15).
__device__ __forceinline__ uint32_t row_incl_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  return x;
}
// Sum over the wave, in every lane (a scalar).
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) { return rl32(wave_incl_sum(x), 63); }

__device__ __forceinline__ unsigned long long wave_reserve(unsigned long long* ctr, bool pred) {
  const unsigned long long mask = __ballot(pred);
  if (mask == 0) return 0;
  const int lane = __lane_id();
  const int leader = __ffsll((long long)mask) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(mask));
  base = rl64(base, leader);
  const unsigned long long lt = (lane == 0) ? 0ull : (mask & ((1ull << lane) - 1ull));
  return base + (unsigned long long)__popcll(lt);
}

// Workgroup-wide slot reservation on per-destination counters (W <= kMaxShards; W = 1 for a
// plain append): a lane with `pred` gets a unique index in ctrs[dest]. One returning atomic per
// destination per call per workgroup, not per wave -- a single device-scope counter word
// saturates near 90 returning atomics/us on MI355X, so per-wave reservations from every CU
// serialize the whole level on that word. Has barriers: every thread of the block calls it.
template <int BS = kBlock>
struct BlockResv {
  int cnt[BS / 64][kMaxShards];
  unsigned long long off[BS / 64][kMaxShards];
};

template <int BS = kBlock>
__device__ __forceinline__ unsigned long long block_reserve(BlockResv<BS>& s, unsigned long long* ctrs, bool pred,
                                                            int dest, int W, int stride = 1) {
  const int wid = threadIdx.x >> 6, lane = __lane_id();
  const unsigned long long lt = (1ull << lane) - 1ull;
  unsigned long long mine = 0;
  for (int d = 0; d < W; d++) {
    const bool me = pred && dest == d;
    const unsigned long long m = __ballot(me);
    if (lane == 0) s.cnt[wid][d] = __popcll(m);
    if (me) mine = m;
  }
  __syncthreads();
  if ((int)threadIdx.x < W) {
    const int d = threadIdx.x;
    unsigned long long tot = 0;
    for (int w = 0; w < BS / 64; w++) tot += (unsigned long long)s.cnt[w][d];
    unsigned long long base = tot ? atomicAdd(&ctrs[(size_t)d * stride], tot) : 0ull;
    for (int w = 0; w < BS / 64; w++) {
      s.off[w][d] = base;
      base += (unsigned long long)s.cnt[w][d];
    }
  }
  __syncthreads();
  return pred ? s.off[wid][dest] + (unsigned long long)__popcll(mine & lt) : 0ull;
}

// Wave-level slot reservation on per-destination counters (ctrs[d * stride], d < W <= kMaxShards):
// one ballot per destination, then lane d issues destination d's returning atomic -- the W atomics
// of a wave are in flight together, one memory round trip, and no barrier (k_level's routed passes
// then take dynamic groups like the unrouted ones). Must be called by all lanes of the wave.
__device__ __forceinline__ unsigned long long wave_reserve_dest(unsigned long long* ctrs, bool pred, int dest, int W,
                                                                int stride) {
  const int lane = __lane_id();
  unsigned long long mine = 0;
  uint32_t cnt = 0;
  for (int d = 0; d < W; d++) {
    const bool me = pred && dest == d;
    const unsigned long long m = __ballot(me);
    if (lane == d) cnt = (uint32_t)__popcll(m);
    if (me) mine = m;
  }
  unsigned long long base = 0;
  if (lane < W && cnt) base = atomicAdd(&ctrs[(size_t)lane * stride], (unsigned long long)cnt);
  base = __shfl(base, pred ? dest : 0);
  return pred ? base + (unsigned long long)__popcll(mine & ((1ull << lane) - 1ull)) : 0ull;
}

// Sums a per-thread value over the workgroup and adds it to *ctr with one atomic (kernel exit).
template <int BS = kBlock>
__device__ __forceinline__ void block_flush(unsigned long long* red, unsigned long long* ctr, unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if (__lane_id() == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < BS / 64; w++) t += red[w];
    if (t) atomicAdd(ctr, t);
  }
}

// Wave-cooperative row emission: every lane with `active` has a successor (its parent row
// `base + pidx * STRIDE`, its canonical delta `d`) to be written to `dst`. The rows are written one
// after another by the whole wavefront; the destination is never read back. Per row:
//   - header words (node words, the record count, padding): lane o copies parent word o, or the
//     replaced node's word, and writes it -- one coalesced 4-byte store per 64 words;
//   - records: the merged record array is the parent's sorted records (lane q holds record q)
//     plus the kept sends, placed in the lanes after them; an element's slot in the merged array
//     is its rank: a parent record's is q + the new records below it (one compare per new record),
//     a new record's is ONE ballot + popcount over all the elements (the parent's records below
//     it plus the new records below it). Every lane then stores its element at its rank, and the
//     free slots their zero -- one store instruction per 64 records, all within the row's record
//     region (the memory pipeline coalesces by address, not lane order).
// The source lane's delta is read with v_readlane into scalar registers (no LDS round trip per
// field); everything is branch-free per lane (the per-word select chains of the r02 emitter
// compiled to ~1,300 exec-mask instructions per Multi-Paxos row). Stores go through
// address-space-1 pointers: a pointer that came through v_readlane would otherwise be a FLAT
// store, which also counts in lgkmcnt. Must be called by all lanes of the wave.
// Returns true (wave-uniform) when two kept sends of one row were equal: they would share a rank
// and leave a record slot unwritten. Only a protocol whose Sender skips its duplicate check
// (P::kSendsDistinct, asserted on the explored steps of tests/hostcheck) can get there; the caller
// raises an error instead of writing a wrong row silently.
// nw_lds (k_level): the changed nodes' words already in LDS, kNodeWords per lane of the workgroup
// (s_nodew; `lane0` = the wave's first lane there): a header word then comes from one LDS read
// instead of kNodeWords readlanes and selects per row.
template <class P, int STRIDE = Layout<P>::kWords>
__device__ __forceinline__ bool wave_emit(bool active, const uint32_t* base, uint64_t pidx, const Delta<P>& d,
                                          uint32_t* dst, const uint32_t* nw_lds = nullptr) {
  bool collision = false;
  using L = Layout<P>;
  using Rec = typename P::Rec;
  typedef __attribute__((address_space(1))) uint32_t g32;
  typedef __attribute__((address_space(1))) Rec grec;
  constexpr int NW = L::kWords;
  constexpr int TH = (L::kRecBase + 63) / 64;                         // header words per lane
  constexpr int TR = (P::kNetCap + 63) / 64;                          // records per lane
  constexpr int TAIL0 = L::kRecBase + P::kNetCap * L::kRecWords;      // padding after the records
  static_assert(NW - TAIL0 <= 64, "at most 64 padding words after the records");
  unsigned long long mask = __ballot(active);
  const int lane = __lane_id();
  while (mask) {
    const int src = __ffsll((long long)mask) - 1;
    mask &= mask - 1;
    const uint32_t* pw = base + rl64(pidx, src) * STRIDE;
    g32* ow = (g32*)(rl64((uint64_t)(uintptr_t)dst, src));
    const int node = (int)rl32((uint32_t)d.node, src);
    const uint32_t keep = rl32(d.keep, src);
    const int m = __builtin_popcount(keep);
    const int n = Net<P>::size(pw);
    // header
    if (nw_lds) {
      const uint32_t* nws = nw_lds + src * P::kNodeWords;
#pragma unroll
      for (int t = 0; t < TH; t++) {
        const int o = lane + 64 * t;
        if (o < L::kRecBase) {
          const int rel = o - node * P::kNodeWords;
          const uint32_t v = o < L::kNetCount ? ((unsigned)rel < (unsigned)P::kNodeWords ? nws[rel] : pw[o])
                                              : o == L::kNetCount ? (uint32_t)(n + m) : 0u;
          ow[o] = v;
        }
      }
    } else {
      uint32_t nw[P::kNodeWords];
#pragma unroll
      for (int i = 0; i < P::kNodeWords; i++) nw[i] = rl32(d.nw[i], src);
#pragma unroll
      for (int t = 0; t < TH; t++) {
        const int o = lane + 64 * t;
        if (o < L::kRecBase) {
          uint32_t v = o < L::kNetCount ? pw[o] : o == L::kNetCount ? (uint32_t)(n + m) : 0u;
          const int rel = o - node * P::kNodeWords;
#pragma unroll
          for (int i = 0; i < P::kNodeWords; i++) v = rel == i ? nw[i] : v;
          ow[o] = v;
        }
      }
    }
    // records: the parent's in lanes [0, n), the kept sends in lanes [n, n + m)
    Rec e[TR];
    int rk[TR];
#pragma unroll
    for (int t = 0; t < TR; t++) {
      const int q = lane + 64 * t;
      e[t] = q < n ? Net<P>::at(pw, q) : ~(Rec)0;
      rk[t] = q;
    }
    // the kept sends, one pass: send i goes to lane q (the next free one) with rank pos = the
    // elements already placed below it (parents and earlier sends; free lanes hold ~0, never
    // below), and every placed element above it moves up one -- a later, smaller send then raises
    // the earlier sends' ranks the same way, so the ranks end as the merged order's slots (one
    // readlane per kept send and one scalar test per possible send; it was two of each)
    {
      int q = n;
#pragma unroll
      for (int i = 0; i < P::kMaxSends; i++) {  // constant indices: the send list stays in VGPRs
        if ((keep >> i) == 0u) break;  // no kept send left (sends are kept mostly from the front)
        if ((keep >> i) & 1u) {
          Rec r;
          if constexpr (sizeof(Rec) == 8) r = (Rec)rl64((uint64_t)d.out.r[i], src);
          else r = (Rec)rl32((uint32_t)d.out.r[i], src);
          int pos = 0;
#pragma unroll
          for (int t = 0; t < TR; t++) pos += __popcll(__ballot(e[t] < r));
          if constexpr (SendsDistinct<P>::value) {  // an earlier kept send equal to r
            int eq = 0;
#pragma unroll
            for (int t = 0; t < TR; t++) eq += __popcll(__ballot(lane + 64 * t < q && e[t] == r));
            collision |= eq != 0;
          }
#pragma unroll
          for (int t = 0; t < TR; t++) {
            const int x = lane + 64 * t;
            rk[t] += (x < q && r < e[t]) ? 1 : 0;
            rk[t] = x == q ? pos : rk[t];
            e[t] = x == q ? r : e[t];
          }
          q++;
        }
      }
    }
    // only the row's n + m records are stored: the free slots after them (and the padding) keep
    // whatever the buffer held, since every reader of a row reads its records below the count
    // (Net::at for j < size; rows never leave the device: host states are rebuilt by replay)
    grec* orec = (grec*)(ow + L::kRecBase);
#pragma unroll
    for (int t = 0; t < TR; t++) {
      const int q = lane + 64 * t;
      if (q < n + m) orec[rk[t]] = e[t];
    }
  }
  return collision;
}

// Lane-parallel row emission for small rows (LaneEmit<P>: at most 64 words and 3 sends per step,
// e.g. the synthetic C3's 64-byte rows): every active lane writes its OWN row, 16 bytes per store,
// instead of the wavefront writing its rows one after another (wave_emit: ~100 wave-instructions
// per row, the same for a 64-byte row as for a 640-byte one). The row is streamed in 16-byte units
// with compile-time word offsets: header words from the parent row `pw` (LDS) with the changed
// node's words and the new record count patched in; the records as the merge of the parent's
// sorted records with the kept sends, sorted first by a compare-exchange network (at most 3).
// Returns true (wave-uniform) when two kept sends of one row were equal (see wave_emit).
template <class P, class = void>
struct LaneEmit : std::integral_constant<bool, (Layout<P>::kWords <= 64 && P::kMaxSends <= 3)> {};

template <class P>
__device__ __forceinline__ bool lane_emit(bool active, const uint32_t* pw, const Delta<P>& d, uint32_t* dst) {
  using L = Layout<P>;
  using Rec = typename P::Rec;
  constexpr int NW = L::kWords, RW = L::kRecWords, M = P::kMaxSends, NWd = P::kNodeWords;
  bool coll = false;
  if (active) {
    const int n = Net<P>::size(pw);
    Rec sv[M];
#pragma unroll
    for (int i = 0; i < M; i++) sv[i] = ((d.keep >> i) & 1u) ? d.out.r[i] : ~(Rec)0;
    const int m = __builtin_popcount(d.keep);
    // compare-exchange network (M <= 3): ascending, the unkept sentinels last
    auto cx = [&](int a, int b) {
      const Rec lo = sv[a] < sv[b] ? sv[a] : sv[b], hi = sv[a] < sv[b] ? sv[b] : sv[a];
      sv[a] = lo;
      sv[b] = hi;
    };
    if constexpr (M >= 2) cx(0, 1);
    if constexpr (M >= 3) {
      cx(1, 2);
      cx(0, 1);
    }
    if constexpr (SendsDistinct<P>::value) {  // two kept sends equal: they would share a slot
#pragma unroll
      for (int i = 0; i + 1 < M; i++) coll |= i + 1 < m && sv[i] == sv[i + 1];
    }
    const int rel0 = d.node * NWd;
    int i = 0, j = 0;  // the merge: next send, next parent record
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) v4u g128;
    g128* o4 = (g128*)dst;
#pragma unroll
    for (int u = 0; u < NW / 4; u++) {
      uint32_t w4[4];
      Rec cur = 0;
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int o = 4 * u + t;
        uint32_t v = 0;
        if (o < L::kNetCount) {
          v = pw[o];
          const int rel = o - rel0;
#pragma unroll
          for (int x = 0; x < NWd; x++) v = rel == x ? d.nw[x] : v;
        } else if (o == L::kNetCount) {
          v = (uint32_t)(n + m);
        } else if (o >= L::kRecBase && o < L::kRecBase + P::kNetCap * RW) {
          if ((o - L::kRecBase) % RW == 0) {  // the next merged record
            const Rec s = M == 1 ? sv[0] : M == 2 ? (i == 0 ? sv[0] : sv[1 < M ? 1 : 0])
                                              : (i == 0 ? sv[0] : i == 1 ? sv[1 < M ? 1 : 0] : sv[2 < M ? 2 : 0]);
            const Rec p = j < n ? Net<P>::at(pw, j) : ~(Rec)0;
            const bool take_s = i < m && (j >= n || s < p);
            cur = take_s ? s : j < n ? p : (Rec)0;
            i += take_s ? 1 : 0;
            j += (!take_s && j < n) ? 1 : 0;
          }
          v = RW == 2 && (o - L::kRecBase) % RW == 1 ? (uint32_t)((uint64_t)cur >> 32) : (uint32_t)cur;
        }
        w4[t] = v;
      }
      o4[u] = v4u{w4[0], w4[1], w4[2], w4[3]};
    }
  }
  return __ballot(coll) != 0ull;
}

// In-chunk duplicate filter (P::kChunkDedup): a chunk's parents are consecutive frontier rows,
// so siblings sit together, and two interleavings of two independent events of one grandparent
// (a diamond) reach the same state inside one chunk -- 18 % of the C3 synthetic protocol's probes
// (tools/cpu_bfs.cpp DSL_CPU_CHUNK_CENSUS, profiles/r06_chunk_census.txt). Every probing lane
// first inserts its fingerprint's high word into an LDS set of the chunk (a 64-bit LDS CAS,
// linear probing, at most 8 slots): a lane that finds it there is a successor of this chunk
// already probed (or routed) by another lane -- the same state (63 fingerprint bits), so not new
// (Search.java:485: discovered.add returns false) and neither probed nor routed again. A crowded
// set only lets a duplicate through to the global probe, which answers exactly. A false merge needs
// two distinct states of one chunk with equal high words: about (items per chunk)^2 / 2^64 per
// chunk, 3e-8 for the whole C3 d10 search, within the visited table's own bound.
// P::kChunkDedup enables it on unrouted levels, P::kRouteDedup on sharded (routed) levels, where a
// duplicate also costs 16 bytes over the links and an owner probe.
template <class P, class = void>
struct ChunkDedup : std::false_type {};
template <class P>
struct ChunkDedup<P, std::void_t<decltype(P::kChunkDedup)>> : std::integral_constant<bool, P::kChunkDedup> {};
template <class P, class = void>
struct RouteDedup : std::false_type {};
template <class P>
struct RouteDedup<P, std::void_t<decltype(P::kRouteDedup)>> : std::integral_constant<bool, P::kRouteDedup> {};
#ifndef DSL_DEDUP_SLOTS
#define DSL_DEDUP_SLOTS 1024
#endif
constexpr int kDedupSlots = DSL_DEDUP_SLOTS;  // a power of two
__device__ __forceinline__ bool chunk_seen(unsigned long long* set, const Fp& f) {
  const unsigned long long key = f.hi | 1ull;  // never 0 (an empty slot)
  uint32_t h = (uint32_t)f.lo & (uint32_t)(kDedupSlots - 1);
#pragma unroll 1
  for (int i = 0; i < 8; i++) {
    const unsigned long long old = atomicCAS(set + h, 0ull, key);
    if (old == 0ull) return false;
    if (old == key) return true;
    h = (h + 1u) & (uint32_t)(kDedupSlots - 1);
  }
  return false;
}

template <class P>
struct LevelArgs {
  const uint32_t* cur;       // frontier rows of kWords (row ranges in `segs`)
  const Fp* cur_fp;
  SegTable segs;
  int32_t PB;                // parents per chunk
  int32_t depth;             // depth of the successors
  int32_t incremental;       // parents are expanded non-initial states (judge_view)
  uint32_t* next;            // next frontier rows
  Fp* next_fp;
  uint64_t* next_parent;     // history arena slice of the next level
  uint32_t* next_event;
  unsigned long long* seg_ctr;  // nseg counters, kSegStride apart
  uint4* zero_next;             // the next level's counter set (kCtrSet bytes), zeroed by workgroup 0
  int32_t nseg;
  uint64_t segcap;              // rows per next-frontier segment
  LevelCounters* ctr;
  TerminalRec* terms;
  Table table;
  uint64_t* spill;           // (parent << 20 | event) of VALID states past next_cap
  uint64_t spill_cap;
  int32_t W, me;             // shards (ROUTE only)
  int32_t owner_filter;      // expand only parents this shard owns (first hash-sharded level)
  // W regions of cap_fp routed successors (ROUTE only): the fingerprints, which go to the owner (16 B
  // each; record 0 of a region its header), and beside them the (parent << 20 | event) items,
  // which stay at the source for the materialization
  Fp* out_key;
  uint64_t* out_item;
  uint32_t* out_pk;          // the regions of the other shards packed for the links (kPkWords per record; null: none)
  uint64_t cap_pk;           // words per packed region (pk_region_words(route_cs))
  uint64_t cap_fp;           // records per region (kRouteHdr + kRouteSegs * route_cs)
  uint64_t route_cs;         // records per sub-slab
  RouteCounters* rc;
  uint64_t* rspill;          // routed successors past their region: (parent << 20 | event)
  uint64_t rspill_cap;
  int32_t judge_routed;      // the maxDepth level: routed successors are judged at the source
  // Queued levels (single shard, BfsEngine::enqueue_queue): the frontier's table is derived from
  // the previous queued level's counters instead of `segs`, by the rule the host applies.
  const LevelCounters* qprev;        // null: the table is `segs`
  const unsigned long long* qprev_seg;
  uint64_t qflimit, qwlimit;         // the queue stops above these frontier / work sizes
  uint64_t qroom;                    // ... and before a level whose estimated new states would take
  uint64_t qroom_half;               // the table past half full, or twice them past 3/4 of its slots
  int32_t qspread;                   // resident workgroups (BfsEngine::level_slots): a level of at most
                                     // this many chunks is one round; queued: pb = balanced_chunk(F, PB, qspread)
  uint32_t term_cap;                 // TerminalRec entries of `terms`
  int32_t find;                      // find mode (no table, no rows): the successor whose terminal
  uint64_t find_key;                 // key equals find_key is recorded in terms[0]
  // SearchSettings.maxTimeSecs inside a level (Search.java:127-133: the workers check the deadline
  // continuously): budget_rt > 0 = the search's deadline in s_memrealtime ticks (100 MHz) after
  // *t0_rt, the clock when the search started (k_clock); a workgroup checks it before every chunk
  // and a level past it stops, marked LevelCounters::time_up
  const uint64_t* t0_rt;
  uint64_t budget_rt;
};

// The device clock at the start of a time-limited search (the reference point of the deadline).
__global__ void k_clock(uint64_t* t0) {
  if (threadIdx.x == 0) *t0 = __builtin_amdgcn_s_memrealtime();
}

// Parents per chunk of a level of F parents: at most pbmax, and the chunks come in whole rounds
// of `slots` (the workgroups resident at once) -- R = ceil(F / (slots pbmax)) rounds of equal
// chunks, so the level has no partly filled last round (a round lasts as long as its chunks).
// The frontier is up to kMaxSegs row ranges, each rounded up to whole chunks, so the rounds are
// sized for slots - kMaxSegs chunks: a one-round level never spills a few chunks into a second
// round (measured: C5 level 8, 4,050 parents in 32 segments, took 45 or 80 us by that rounding).
__host__ __device__ inline int balanced_chunk(uint64_t F, int pbmax, int slots) {
  if (slots > 2 * kMaxSegs) slots -= kMaxSegs;
  const uint64_t per_round = (uint64_t)slots * (uint64_t)(pbmax > 0 ? pbmax : 1);
  const uint64_t R = F ? (F + per_round - 1) / per_round : 1;
  const uint64_t pb = (F + (uint64_t)slots * R - 1) / ((uint64_t)slots * R);
  return (int)(pb < 1 ? 1 : pb > (uint64_t)pbmax ? (uint64_t)pbmax : pb);
}

// New states a level of `work` work items may insert, from the previous level's new / work ratio
// (x1.25, plus a floor): the growth rule's estimate (BfsEngine::ensure_table). At most `work`.
__host__ __device__ inline uint64_t est_new_states(uint64_t work, uint64_t prev_new, uint64_t prev_work) {
  // the last level's new states per work item, with a 25 % margin (the ratio falls with depth in
  // every protocol here; the table is then kept at most half full of the estimate)
  const double r = prev_work ? (double)prev_new / (double)prev_work : 1.0;
  const double e = 1.25 * r * (double)work + 1024.0;
  return e < (double)work ? (uint64_t)e : work;
}

// The queue's stop rule: after a level with any of these, the host must act before the next one.
// The visited table's headroom when the queue started (BfsEngine::table_room / table_room_queue):
// the next level runs only if the queue's inserted states so far plus its estimate keep the table
// at most half full -- the rule ensure_table applies between unqueued levels -- AND plus TWICE the
// estimate at most 3/4 full: the estimate assumes the new / work ratio does not rise, and a level
// that overfills the table restarts the whole search with a larger one, so the queue,
// which runs up to twelve levels without the host, stays within 3/4 even when a level doubles.
__host__ __device__ inline bool queue_continues(const LevelCounters& c, uint64_t F, uint64_t flimit,
                                                uint64_t wlimit, uint64_t room34, uint64_t room_half) {
  const uint64_t est = est_new_states(c.next_work, c.new_states, c.work_items);
  return !(c.spilled | c.n_terminals | c.err_overflow | c.err_table | c.err_frontier | c.time_up) && F > 0 &&
         F <= flimit &&
         c.next_work <= wlimit &&
         c.cum_before + c.new_states + 2 * est <= room34 && c.cum_before + c.new_states + est <= room_half;
}

// Copies n16 16-byte units from global memory to LDS with LDS-DMA: wave w issues units
// [64 (w + 4 r), +64) for r = 0, 1, ...; the destination of one wave-instruction is its
// wave-uniform base + lane x 16. No wait here: the caller waits (vmcnt) before its barrier.
__device__ __forceinline__ void stage_lds(const uint4* src, uint4* dst, int n16) {
  const int lane = __lane_id();
  for (int b = (int)(threadIdx.x >> 6) * 64; b < n16; b += (int)blockDim.x) {
    if (b + lane < n16)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + b + lane),
                                       (__attribute__((address_space(3))) void*)(dst + b), 16, 0, 0);
  }
}

// Copies a chunk's rows (pb rows of NW dwords, contiguous in global memory) into an LDS image of
// row stride SP (a multiple of 4 dwords) with LDS-DMA: wave w stages rows w, w + 4, ..., one
// wave-instruction per 64 16-byte units of a row. No wait here (as stage_lds).
template <int NW, int SP>
__device__ __forceinline__ void stage_rows_dma(const uint4* src, uint32_t* dst, int pb) {
  constexpr int U = NW / 4;
  const int lane = __lane_id();
  for (int j = (int)(threadIdx.x >> 6); j < pb; j += (int)(blockDim.x >> 6)) {
#pragma unroll
    for (int b = 0; b < U; b += 64)
      if (b + lane < U)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + j * U + b + lane),
                                         (__attribute__((address_space(3))) void*)(dst + j * SP + 4 * b), 16, 0, 0);
  }
}

// Copies a chunk's rows (pb rows of NW dwords, contiguous in global memory) into an LDS image of
// row stride SP > NW through registers: every thread issues all its 16-byte loads before its first
// LDS store (the chunk is at most DSL_ROWS_LDS_KB, i.e. a fixed number of units per thread).
template <int NW, int SP>
__device__ __forceinline__ void stage_rows_padded(const uint4* src, uint32_t* dst, int pb) {
  constexpr int U = NW / 4;  // 16-byte units per row
  constexpr int kIt = (DSL_ROWS_LDS_BYTES / 16 + kLevelBlock - 1) / kLevelBlock;
  const int n16 = pb * U;
  uint4 v[kIt];
#pragma unroll
  for (int it = 0; it < kIt; it++) {
    const int u = (int)threadIdx.x + it * kLevelBlock;
    if (u < n16) v[it] = src[u];
  }
#pragma unroll
  for (int it = 0; it < kIt; it++) {
    const int u = (int)threadIdx.x + it * kLevelBlock;
    if (u < n16) {
      const int j = u / U, c = u - j * U;
      uint32_t* o = dst + j * SP + 4 * c;
      if constexpr (SP % 2 == 0) {
        reinterpret_cast<uint2*>(o)[0] = make_uint2(v[it].x, v[it].y);
        reinterpret_cast<uint2*>(o)[1] = make_uint2(v[it].z, v[it].w);
      } else {
        o[0] = v[it].x;
        o[1] = v[it].y;
        o[2] = v[it].z;
        o[3] = v[it].w;
      }
    }
  }
}

// Terminal candidates of a level are reduced EXACTLY by priority (EXCEPTION > INVARIANT > GOAL,
// Search.java:370-385), then by the successor's fingerprint (a deterministic tie-break): a wave
// takes the minimum key of its candidates and folds it into LevelCounters::term_best with one
// 64-bit atomicMax of the complemented key (counter sets start zeroed); a wave whose key improved
// the running best records that candidate in the level's TerminalRec list. The final best key was
// recorded by the last improvement, so it is in the list unless the list overflowed (>term_cap
// improvements); the host then re-runs the level in find mode (LevelArgs::find_key), which
// records the successor whose key matches.
__device__ __forceinline__ uint64_t term_key(int verdict, uint64_t fphi) {
  return ((uint64_t)(verdict - V_TERM_EXCEPTION) << 62) | (fphi >> 2);
}

// The tie-break bits of an exceptional successor (never equal to another state, so it has no
// fingerprint of its own): its parent's fingerprint mixed with the event index, so two throwing
// events of one parent have distinct keys and the level's choice never depends on arrival order.
__device__ __forceinline__ uint64_t exception_key(const Fp& parent, int k) {
  return parent.hi ^ fmix64(parent.lo + 0x9E3779B97F4A7C15ull * (uint64_t)(k + 1));
}

__device__ __forceinline__ void fold_terminals(bool term, uint64_t key, int v, int pi, uint32_t k, uint64_t parent,
                                               LevelCounters* ctr, TerminalRec* terms, uint32_t cap) {
  const unsigned long long tm = __ballot(term);
  if (!tm) return;
  // the wave's minimum key: a scalar walk over the (few) terminal lanes
  unsigned long long m = ~0ull;
  for (unsigned long long r = tm; r; r &= r - 1) {
    const unsigned long long y = rl64(key, __ffsll((long long)r) - 1);
    m = y < m ? y : m;
  }
  const int who = __ffsll((long long)__ballot(term && key == m)) - 1;
  if (__lane_id() == who) {
    atomicAdd(&ctr->n_terminals, (unsigned long long)__popcll(tm));
    const unsigned long long old = atomicMax(&ctr->term_best, ~m);
    if (old < ~m) {
      const unsigned long long slot = atomicAdd(&ctr->n_term_rec, 1ull);
      if (slot < cap) terms[slot] = TerminalRec{v, pi, k, 0u, parent, (uint64_t)m};
    }
  }
}

// Occupancy floor of 4 waves/SIMD (<= 128 VGPRs): a latency-bound kernel (r01 on C5 Multi-Paxos:
// 2 waves/SIMD 1.5x slower, 3 waves/SIMD 7-11 % slower at d12/d14, 5 waves/SIMD 1.5-1.65x slower).
// A protocol with small states and short handlers (P::kLevelWaves, e.g. the synthetic C3) asks for
// more waves per SIMD: its instantiation then fits in fewer registers and more workgroups are
// resident (BfsEngine::level_slots sizes the grid from the occupancy).
template <class P, class = void>
struct LevelWaves : std::integral_constant<int, 4> {};
template <class P>
struct LevelWaves<P, std::void_t<decltype(P::kLevelWaves)>> : std::integral_constant<int, P::kLevelWaves> {};
#ifndef DSL_KLEVEL_ATTR
#define DSL_KLEVEL_ATTR __attribute__((amdgpu_waves_per_eu(LevelWaves<P>::value)))
#endif
template <class P, bool ROUTE>
__global__ void __launch_bounds__(kLevelBlock) DSL_KLEVEL_ATTR k_level(LevelArgs<P> a, typename P::Params prm, DevSettings set) {
  constexpr int NW = Layout<P>::kWords;
  constexpr int SP = LdsRow<P>::kStride;  // row stride of the staged parents in LDS
  constexpr int NWAVE = kLevelBlock / 64;
  // handler classes: messages, timers, then the events whose handler surely changes nothing
  // (NoopFilter: counted as successors and never run; they sort last and the passes stop before them)
  constexpr int NC = Classes<P>::kCount;
  constexpr bool kDD = ROUTE ? RouteDedup<P>::value : ChunkDedup<P>::value;  // the in-chunk duplicate filter
  static_assert(P::kNodes * 256 < 32768 && P::kNetCap < 32768, "a located event fits s_ev's 16 bits");
  extern __shared__ __align__(16) uint32_t lds[];
  uint32_t* rows = lds;                                           // a.PB (max) rows, stride SP
  Fp* fps = reinterpret_cast<Fp*>(rows + LdsRow<P>::image(a.PB));  // a.PB
  constexpr int kNhPer = DSL_NH_LDS ? P::kNodes : 0;
  Fp* nh = fps + a.PB;                                     // a.PB * kNodes: the parents' node hashes
  int* off = reinterpret_cast<int*>(nh + a.PB * kNhPer);   // a.PB + 1
  __shared__ SegTable s_segs;
  __shared__ BlockResv<kLevelBlock> s_resv;
  __shared__ uint32_t s_nodew[kLevelBlock * P::kNodeWords];
  __shared__ typename P::Rec s_sends[NetPreds<P>::value ? kLevelBlock * P::kMaxSends : 1];
#ifdef DSL_PHASES
  __shared__ unsigned long long s_red[NWAVE];  // PH_FLUSH (instrumented builds)
#endif
  __shared__ unsigned long long s_red5[NWAVE * 6];
  __shared__ int s_wsum[NWAVE];
#ifndef DSL_SORT_BALLOT
  // the window's class counts (LDS atomics in step 3a, each item's rank within its class in s_rnk)
  __shared__ int s_ccnt[16], s_cbase0[16];
  __shared__ uint16_t s_rnk[kWin];
  __shared__ int s_cbase[1][NC];
#else
  __shared__ int s_cbase[kWin / 64][NC];
#endif
  __shared__ uint8_t s_par[kWin], s_cls[kWin];
  __shared__ uint16_t s_perm[kWin];
  __shared__ int16_t s_ev[kWin];  // each item's located event (locate_event code; kEvNone: none)
  __shared__ int s_stop, s_weff, s_gnext, s_tup;
  __shared__ uint64_t s_t0;
  __shared__ unsigned long long s_dd[kDD ? kDedupSlots : 1];
  const int tid = threadIdx.x, lane = __lane_id(), wid = tid >> 6;
  const bool find = a.find != 0;
  // per-thread statistics, flushed once per workgroup (no per-wave atomics on shared words)
  uint32_t c_succ = 0, c_new = 0, c_next_work = 0, c_work = 0, c_probe = 0, c_dup = 0;
  PH_DECL
  PH_CLS_DECL
#ifdef DSL_KWARM
  {  // (measurement variant) every 64-byte line of the kernel arguments, independent scalar loads
    uint32_t acc = 0;
    const uint32_t* ks = reinterpret_cast<const uint32_t*>(&set);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(DevSettings) / 4); i += 16) acc += ks[i];
    const uint32_t* kp = reinterpret_cast<const uint32_t*>(&prm);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(prm) / 4); i += 16) acc += kp[i];
    const uint32_t* ka = reinterpret_cast<const uint32_t*>(&a);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(a) / 4); i += 16) acc += ka[i];
    asm volatile("" ::"s"(acc));
  }
#endif
  if (a.qprev) {
    // queued level: this frontier is the previous level's segments; every workgroup derives the
    // table (and whether the queue stopped) from those counters, as the host does afterwards
    if (tid < 64) {
      const int q = tid;
      // (32-bit sums: a frontier's rows are far fewer than 2^32 in any device memory)
      const uint64_t c = q < a.nseg ? min<uint64_t>(a.qprev_seg[q * kSegStride], a.segcap) : 0ull;
      const uint64_t F = wave_sum((uint32_t)c);
      const int pb = balanced_chunk(F, a.PB, a.qspread);
      const uint64_t inc = wave_incl_sum((uint32_t)((c + pb - 1) / pb));
      if (q < a.nseg) {
        s_segs.base[q] = (uint64_t)q * a.segcap;
        s_segs.cnt[q] = c;
        s_segs.chunk0[q + 1] = inc;
      }
      if (q == 0) {
        s_segs.n = a.nseg;
        s_segs.pb = pb;
        s_segs.chunk0[0] = 0;
        s_stop = queue_continues(*a.qprev, F, a.qflimit, a.qwlimit, a.qroom, a.qroom_half) ? 0 : 1;
      }
    }
  } else {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&a.segs);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&s_segs);
    for (int i = tid; i < (int)(sizeof(SegTable) / 4); i += blockDim.x) dst[i] = src[i];
    if (tid == 0) s_stop = 0;
  }
  if (a.budget_rt && tid == 0) s_t0 = *a.t0_rt;
#ifndef DSL_SORT_BALLOT
  if (tid < 16) s_ccnt[tid] = 0;
#endif
  __syncthreads();
  if (s_stop) return;  // an earlier queued level stopped the queue
  PH_MARK(8);  // prologue: the frontier's segment table (+ the queue rule)
  if (blockIdx.x == 0) {
    for (int i = tid; i < kCtrSet / 16; i += blockDim.x) a.zero_next[i] = make_uint4(0, 0, 0, 0);
    if (tid == 0 && a.qprev) a.ctr->cum_before = a.qprev->cum_before + a.qprev->new_states;
  }
  const int PB = s_segs.pb;
  const uint64_t nchunks = s_segs.chunk0[s_segs.n];
  const bool spread = nchunks <= (uint64_t)a.qspread;  // at most one round of resident workgroups
  const int seg = (int)(blockIdx.x % (unsigned)a.nseg);
  int g = 0;
  int npass = 0;  // this workgroup's passes so far (ROUTE: its sub-slab rotates with them)
  for (uint64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
#ifndef DSL_NO_LANE_REMAT
    // the lane indices as values opaque to the compiler, once per chunk: the per-lane addresses
    // derived from them are recomputed where used instead of held live (and spilled) across
    // chunks (C5 d12 scratch 36 -> 20 B/lane, C3 d10 60 -> 12 B/lane and +1.1 %:
    // profiles/r06_remat_ab.txt)
    int tid_c = tid, lane_c = lane;
    asm volatile("" : "+v"(tid_c), "+v"(lane_c));
    const int tid = tid_c, lane = lane_c, wid = tid_c >> 6;
#endif
    if (a.budget_rt) {  // the deadline, before every chunk (one workgroup-uniform decision)
      if (tid == 0) s_tup = __builtin_amdgcn_s_memrealtime() - s_t0 > a.budget_rt ? 1 : 0;
      __syncthreads();
      if (s_tup) {
        if (tid == 0) atomicOr(&a.ctr->time_up, 1ull);
        break;
      }
    }
    while (chunk >= s_segs.chunk0[g + 1]) g++;  // chunks ascend: the segment index only grows
    const uint64_t p0 = s_segs.base[g] + (chunk - s_segs.chunk0[g]) * (uint64_t)PB;
    const int pb = (int)min<uint64_t>((uint64_t)PB, s_segs.base[g] + s_segs.cnt[g] - p0);
    // 1. stage the parents (contiguous rows) and their fingerprints in LDS: LDS-DMA
    //    (global_load_lds_dwordx4, 1 KiB per wave-instruction, no VGPRs), every load in flight
    //    before the one wait
    if constexpr (SP == NW)
      stage_lds(reinterpret_cast<const uint4*>(a.cur + p0 * NW), reinterpret_cast<uint4*>(rows), pb * NW / 4);
    else if constexpr (SP % 4 == 0)
      stage_rows_dma<NW, SP>(reinterpret_cast<const uint4*>(a.cur + p0 * NW), rows, pb);
    else
      stage_rows_padded<NW, SP>(reinterpret_cast<const uint4*>(a.cur + p0 * NW), rows, pb);
    stage_lds(reinterpret_cast<const uint4*>(a.cur_fp + p0), reinterpret_cast<uint4*>(fps), pb);
    if constexpr (kDD)  // the chunk's duplicate filter starts empty (the staging barrier publishes it)
      for (int i = tid; i < kDedupSlots; i += kLevelBlock) s_dd[i] = 0ull;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    PH_MARK(9);  // staging (LDS-DMA + wait + barrier)
    // 2. every parent's node hashes, once per parent instead of once per successor (the old-node
    //    term of the incremental fingerprint: fp ^ H(i, old) ^ H(i, new) ^ ...), one lane per
    //    (parent, node); then the enabled events per parent (SearchState.events) and a workgroup
    //    exclusive scan (wave scans); the scan's barrier also publishes the hashes
#ifndef DSL_CNT_SERIAL  // a chunk of <= 64 parents: waves 1-3 hash while wave 0 counts (+0.7 % on C5 d12)
    if (!DSL_NH_LDS) {
    } else if (pb <= 64) {
      for (int x = tid - 64; x >= 0 && x < pb * P::kNodes; x += kLevelBlock - 64) {
        const int jj = x / P::kNodes, ii = x - jj * P::kNodes;
        nh[x] = node_hash<P>(ii, rows + jj * SP + ii * P::kNodeWords);
      }
    } else
#endif
    for (int x = tid; x < pb * kNhPer; x += kLevelBlock) {
      const int jj = x / P::kNodes, ii = x - jj * P::kNodes;
      nh[x] = node_hash<P>(ii, rows + jj * SP + ii * P::kNodeWords);
    }
    int total;
    if (pb <= 64) {  // one wave's worth of parents: wave 0 scans them alone, one barrier
      if (wid == 0) {
        int x = 0;
        if (lane < pb)
          x = (ROUTE && a.owner_filter && owner_of(fps[lane], a.W) != a.me) ? 0
                                                                           : count_events<P>(rows + lane * SP, prm, set);
        x = (int)wave_incl_sum((uint32_t)x);
        if (lane < pb) off[lane + 1] = x;
        if (lane == 0) off[0] = 0;
        if (lane == 63) s_wsum[0] = x;
      }
      __syncthreads();
      total = s_wsum[0];
      if (tid == 0) c_work += (uint32_t)total;
    } else {
      int x = 0;
      if (tid < pb)
        x = (ROUTE && a.owner_filter && owner_of(fps[tid], a.W) != a.me) ? 0
                                                                        : count_events<P>(rows + tid * SP, prm, set);
      x = (int)wave_incl_sum((uint32_t)x);
      if (lane == 63) s_wsum[wid] = x;
      __syncthreads();
      int pre = 0;
      total = 0;
#pragma unroll
      for (int q = 0; q < NWAVE; q++) {
        const int v = s_wsum[q];
        pre += q < wid ? v : 0;
        total += v;
      }
      if (tid < pb) off[tid + 1] = pre + x;
      if (tid == 0) {
        off[0] = 0;
        c_work += (uint32_t)total;
      }
      __syncthreads();
    }
    PH_MARK(0);  // event count + scan
    // 3. the chunk's work items in windows of kWin, grouped by handler class (counting sort in
    //    LDS) so that a wavefront mostly runs one handler; one lane per (parent, event)
    for (int w0 = 0; w0 < total; w0 += kWin) {
      const int wn = min(kWin, total - w0);
      // 3a. (parent, handler class) of every item of the window: a team of TPP threads per
      //     parent writes its events' entries (no search, no atomics). (Measured: one thread per
      //     item -- a binary search for the first item's parent, then runs of ceil(wn / 256) items
      //     -- was 3 % slower on C5 d12, profiles/r06_classify_ab.txt.)
      {
        const int tpp = pb > 128 ? 1 : pb > 64 ? 2 : pb > 32 ? 4 : pb > 16 ? 8 : pb > 8 ? 16 : 32;
        const int j = tid / tpp, sub = tid - j * tpp;
        if (j < pb) {
          const int e0 = off[j];
          const int lo = max(e0, w0), hi = min(off[j + 1], w0 + wn);
          const uint32_t* w = rows + j * SP;
          int q = lo + sub;
#ifndef DSL_CLS_ONE_LOOP  // message events first, by a branch-free body, then the timers (+1.3 % on C5 d12)
          if (set.all_deliver) {  // event k < size is record k (SearchState.events: messages first)
            const int mhi = min(hi, e0 + (int)Net<P>::size(w));
            const int nn = P::num_nodes(prm);
            for (; q < mhi; q += tpp) {
              const auto r = Net<P>::at(w, q - e0);
              const int i = P::rec_to(r);
              const bool skip = i < nn && NoopFilter<P>::msg(i < nn ? i : 0, w, r, prm);
              const int cls = skip ? Classes<P>::kSkip : P::msg_class(r);
              s_par[q - w0] = (uint8_t)j;
              s_cls[q - w0] = (uint8_t)cls;
#ifndef DSL_SORT_BALLOT
              s_rnk[q - w0] = (uint16_t)atomicAdd(&s_ccnt[cls], 1);
#endif
              s_ev[q - w0] = (int16_t)(q - e0);
            }
          }
#endif
          for (; q < hi; q += tpp) {
            int ev;
            s_par[q - w0] = (uint8_t)j;
#ifndef DSL_SORT_BALLOT
            const int cls = event_class_skip<P>(w, prm, set, q - e0, &ev);
            s_cls[q - w0] = (uint8_t)cls;
            s_rnk[q - w0] = (uint16_t)atomicAdd(&s_ccnt[cls], 1);
#else
            s_cls[q - w0] = (uint8_t)event_class_skip<P>(w, prm, set, q - e0, &ev);
#endif
            s_ev[q - w0] = (int16_t)(ev == INT32_MIN ? kEvNone : ev);
          }
        }
      }
      __syncthreads();
#ifdef DSL_PH_SPLIT_CLS  // phase builds: slot 8 (the prologue's) also takes step 3a, slot 7 only the sort
      PH_MARK(8);
#endif
      // 3b. the window sorted by class: one 64-item group is ranked by wave 0 alone with ballots;
      //     a larger window by its LDS-atomic class counts (step 3a: each item's rank within its
      //     class, s_rnk), the class bases by one wave, then one scatter pass -- two barriers and
      //     no per-group ballots (C5 d12 1.54 -> 1.60e9 states/s, profiles/r06_sort_atomic_ab.txt;
      //     the per-group ballot sort of rounds 2-5 stays as -DDSL_SORT_BALLOT)
      const int ng = (wn + 63) >> 6;
      if (ng == 1) {
        // one group (every small level): wave 0 sorts it alone, in registers, with one barrier
        if (wid == 0) {
          const int c = lane < wn ? (int)s_cls[lane] : -1;
          int mine = 0, rank = 0;
#pragma unroll
          for (int q = 0; q < NC; q++) {
            const unsigned long long mq = __ballot(c == q);
            if (lane == q) mine = __popcll(mq);
            if (c == q) rank = __popcll(mq & ((1ull << lane) - 1ull));
          }
          const int inc = (int)row_incl_sum((uint32_t)mine);
          const int run = inc - mine;  // lane q < NC: the first position of class q
          if (lane == NC - 1) {        // the skipped events: counted, never run
            s_weff = run;
            s_gnext = 0;
            c_succ += (uint32_t)mine;
          }
          const int b = __shfl(run, c < 0 ? 0 : c);
          if (lane < wn) s_perm[b + rank] = (uint16_t)lane;
#ifndef DSL_SORT_BALLOT
          if (lane < 16) s_ccnt[lane] = 0;
#endif
        }
        __syncthreads();
      } else {
#ifndef DSL_SORT_BALLOT
      // counting sort from the LDS-atomic class counts of step 3a: bases by one wave, then every
      // item to its class base + its rank (the order within a class is the atomics' order)
      if (tid < 64) {
        const int cnt = lane < NC ? s_ccnt[lane] : 0;
        const int inc = (int)row_incl_sum((uint32_t)cnt);
        const int run = inc - cnt;
        if (lane == NC - 1) {  // the skipped events: counted, never run
          s_weff = run;
          s_gnext = 0;
          c_succ += (uint32_t)cnt;
        }
        if (lane < 16) {
          s_cbase0[lane] = run;
          s_ccnt[lane] = 0;
        }
      }
      __syncthreads();
      for (int t = tid; t < wn; t += kLevelBlock) s_perm[s_cbase0[s_cls[t]] + s_rnk[t]] = (uint16_t)t;
      __syncthreads();
#else
      for (int gr = wid; gr < ng; gr += NWAVE) {
        const int t = gr * 64 + lane;
        const int c = t < wn ? (int)s_cls[t] : -1;
        int mine = 0;
#pragma unroll
        for (int q = 0; q < NC; q++) {
          const int n = __popcll(__ballot(c == q));
          if (lane == q) mine = n;
        }
        if (lane < NC) s_cbase[gr][lane] = mine;
      }
      __syncthreads();
      if (tid < 64) {
        int tot = 0;
        if (lane < NC)
          for (int gr = 0; gr < ng; gr++) tot += s_cbase[gr][lane];
        const int inc = (int)row_incl_sum((uint32_t)tot);
        int run = inc - tot;
        if (lane == NC - 1) {  // the skipped events: counted, never run
          s_weff = run;
          s_gnext = 0;
          c_succ += (uint32_t)tot;
        }
        if (lane < NC)
          for (int gr = 0; gr < ng; gr++) {
            const int v = s_cbase[gr][lane];
            s_cbase[gr][lane] = run;
            run += v;
          }
      }
      __syncthreads();
      // 3c. the permutation: class base + rank among the group's lanes of the same class
      for (int gr = wid; gr < ng; gr += NWAVE) {
        const int t = gr * 64 + lane;
        const int c = t < wn ? (int)s_cls[t] : -1;
        int rank = 0;
#pragma unroll
        for (int q = 0; q < NC; q++) {
          const unsigned long long mq = __ballot(c == q);
          if (c == q) rank = __popcll(mq & ((1ull << lane) - 1ull));
        }
        if (t < wn) s_perm[s_cbase[gr][c] + rank] = (uint16_t)t;
      }
      __syncthreads();
#endif
      }
      PH_MARK(7);  // classify + sort
      const int wrun = s_weff;  // the window's events whose handler runs (a prefix of s_perm)
      // In a level of at most one round of chunks (latency-bound: every chunk runs at once) each
      // pass of r <= 256 items is split into four equal contiguous shares, one per wave -- a short
      // pass spread over all four waves has fewer handler classes, probes and emitted rows per
      // wave, so a shorter critical path. In a larger level (throughput-bound) each wave takes the
      // next group of 64 class-sorted items from an LDS counter until the window is done, so the
      // waves finish the window together whatever their handlers cost (a fixed share per wave
      // left the others waiting at the window's barrier). ROUTE levels too: their reservations are
      // per wave (wave_reserve_dest).
#ifdef DSL_NO_DYN  // measurement variant: fixed shares in every level
      const bool dyn = false;
#else
#ifdef DSL_ROUTE_BLOCK  // measurement variant: workgroup-wide route reservations, fixed shares
      const bool dyn = !ROUTE && !spread;
#else
      const bool dyn = !spread;
#endif
#endif
      for (int base = 0;;) {
        int t;
        bool live;
        if (dyn) {
          int gi = 0;
          if (lane == 0) gi = atomicAdd(&s_gnext, 1);
          gi = __builtin_amdgcn_readfirstlane(gi);
          if (gi * 64 >= wrun) break;
          t = gi * 64 + lane;
          live = t < wrun;
        } else {
          if (base >= wrun) break;
          const int r = min(kLevelBlock, wrun - base);
          const int per = spread ? (r + NWAVE - 1) / NWAVE : 64;
          t = base + wid * per + lane;
          live = lane < per && t < base + r;
          base += kLevelBlock;
        }
        bool is_valid = false, route = false;
        int dest = 0, j = 0, k = 0, tv = 0, tpi = -1;
        uint64_t tkey = ~0ull;  // terminal candidate
        Fp f{0, 0};
        Delta<P> d;  // the successor as a canonical delta of its parent
        d.node = 0;
        d.out.n = 0;
        d.keep = 0;
        if (live) {
          const int u = s_perm[t];
          j = s_par[u];
          k = w0 + u - off[j];
          const uint32_t* w = rows + j * SP;
          uint32_t* my_nw = s_nodew + tid * P::kNodeWords;  // the changed node's words, for the judge
          int rc, dnode = 0, dn = 0;
          bool noop = false;
          // an event that changes neither its node nor the network (a redelivered message most
          // often) leads back to the parent, which is in the visited set: no probe
          {
            PH_CLS_T0
            const int ev = s_ev[u];
            rc = delta_step_located<P>(w, ev == kEvNone ? INT32_MIN : ev, d, prm, set);
            PH_CLS_ADD(s_cls[u], true);
            PH_MARK(1);  // decode + handler + canonical sends
            if (rc == STEP_OK) {
              dnode = d.node;
              dn = delta_new_count<P>(d);
              noop = dn == 0 && same_words<P::kNodeWords>(d.nw, w + dnode * P::kNodeWords);
              if (!noop) {
                if constexpr (DSL_NH_LDS) f = delta_fingerprint_cached<P>(fp_xor(fps[j], nh[j * P::kNodes + dnode]), d);
                else f = delta_fingerprint<P>(w, fps[j], d);
                // the changed node's words go through LDS: a view pointing at the register
                // array would take its address and push the whole delta into scratch
#pragma unroll
                for (int q = 0; q < P::kNodeWords; q++) my_nw[q] = d.nw[q];
              }
            }
          }
          if (rc == STEP_OK) c_succ++;
          if (rc == STEP_OK && !noop) {
            PH_MARK(2);  // fingerprint
            // a successor of this chunk seen before (ChunkDedup): the same state, not new; it was
            // probed or routed once already
            bool dup = false;
            if constexpr (kDD) dup = !find && chunk_seen(s_dd, f);
            c_dup += dup ? 1u : 0u;
            if (ROUTE) dest = owner_of(f, a.W);
            bool judge = false;
            bool spec = false;  // judged while the home slot's CAS is in flight (DSL_JUDGE_OVERLAP)
            unsigned long long spec_old = 0ull, spec_key = 0ull;
            if (dup) {
            } else if (ROUTE) {
              // a sharded level routes EVERY successor, its own shard's too: the owner probes them
              // all in one interleaved pass (k_probe_slab), so which source wins a state generated
              // by several is a fair race, and the shards' frontiers stay balanced (a local insert
              // first would let every shard win all of its own, and the busiest shard grow busier)
              route = true;
              // the maxDepth level (no successor is expanded): judged here, at the source, so the
              // owner only answers nothing -- no round B, no k_materialize (a routed successor that
              // is not new was judged when it was first inserted, and checkState is a function of
              // the state: its verdict cannot be terminal, Search.java:468-504)
              judge = a.judge_routed != 0;
            } else {
              c_probe++;
#ifdef DSL_JUDGE_OVERLAP
              if (!find && !a.table.load_first) {
                // the home slot's CAS is issued now and its answer used after the judge, which every
                // probing lane runs meanwhile (its verdict counts only for a new state)
                spec_key = table_key0(a.table, f);
                spec_old = atomicCAS(a.table.slots + table_home(a.table, f), 0ull, spec_key);
                spec = true;
                judge = true;
              } else
#endif
              {
                const int ins = find ? INS_NEW : table_insert(a.table, f);
                PH_MARK(3);  // visited-table probe / insert
                if (ins == INS_NEW) {
                  c_new++;
                  judge = true;
                } else if (ins == INS_FULL) {
                  atomicAdd(&a.ctr->err_table, 1ull);
                }
              }
            }
            if (judge) {
              {
                int pi = -1;
                NodeView view{w, P::kNodeWords, dnode, my_nw};
                if constexpr (NetPreds<P>::value) {  // the new records through LDS (no register addresses)
                  typename P::Rec* ms = s_sends + tid * P::kMaxSends;
                  int c = 0;
#pragma unroll
                  for (int q = 0; q < P::kMaxSends; q++)
                    if ((d.keep >> q) & 1u) ms[c++] = d.out.r[q];
                  view.sends = ms;
                  view.nsends = dn;
                }
#ifdef DSL_X0_JUDGE  // cost probe (measurement builds): no judge (every new state VALID below maxDepth)
                const int v = set.max_depth >= 0 && a.depth >= set.max_depth ? V_PRUNED : V_VALID;
                (void)view;
#else
                const int v = judge_view<P>(view, prm, set, a.depth, &pi, a.incremental != 0);
#endif
                bool use = true;
                if (spec) {  // the probe's answer: the home slot held nothing (new), this key, or another one
                  const int ins = spec_old == 0ull ? INS_NEW : spec_old == spec_key ? INS_EXISTS : table_insert(a.table, f, 1);
                  if (ins == INS_NEW) c_new++;
                  else if (ins == INS_FULL) atomicAdd(&a.ctr->err_table, 1ull);
                  use = ins == INS_NEW;
                }
                if (!use) {
                } else if (v == V_VALID) {
                  if (route) {
                  } else if (Net<P>::size(w) + dn <= P::kNetCap) {
                    is_valid = !find;
                  } else {
                    atomicAdd(&a.ctr->err_overflow, 1ull);
                  }
                } else if (v >= V_TERM_EXCEPTION) {
                  tv = v;
                  tpi = pi;
                  tkey = term_key(v, f.hi);
                }
              }
            }
          } else if (rc == STEP_EXCEPTION) {
            // exceptional states never equal another (Throwable identity): new and terminal
            c_succ++;
            c_new++;
            tv = V_TERM_EXCEPTION;
            tkey = term_key(V_TERM_EXCEPTION, exception_key(fps[j], k));
          } else if (rc == STEP_OVERFLOW) {
            atomicAdd(&a.ctr->err_overflow, 1ull);
          }
        }
        PH_MARK(4);  // judge (+ divergence wait)
        const bool term = tkey != ~0ull;
        if (find) {
          if (term && tkey == a.find_key) a.terms[0] = TerminalRec{tv, tpi, (uint32_t)k, 0u, p0 + j, tkey};
        } else {
          fold_terminals(term, tkey, tv, tpi, (uint32_t)k, p0 + j, a.ctr, a.terms, a.term_cap);
        }
        {
          // a VALID successor reserves a row of its workgroup's segment (one returning atomic per
          // wavefront), then the wavefront writes its rows cooperatively
          const unsigned long long li = wave_reserve(&a.seg_ctr[seg * kSegStride], is_valid);
          PH_MARK(5);  // terminal fold + reservation
          const bool fits = is_valid && li < a.segcap;
          const uint64_t idx = (uint64_t)seg * a.segcap + li;
          if (fits) {
            const uint32_t* w = rows + j * SP;
            a.next_fp[idx] = f;
            a.next_parent[idx] = ((uint64_t)a.me << 48) | (p0 + j);
            a.next_event[idx] = (uint32_t)k;
            c_next_work += (uint32_t)delta_event_count<P>(w, off[j + 1] - off[j], d, prm, set);
          }
          bool coll;
          if constexpr (LaneEmit<P>::value) coll = lane_emit<P>(fits, rows + j * SP, d, a.next + idx * NW);
          else coll = wave_emit<P, SP>(fits, rows, (uint64_t)j, d, a.next + idx * NW, s_nodew + (tid - lane) * P::kNodeWords);
          if (coll && lane == 0)
            atomicAdd(&a.ctr->err_overflow, 1ull);  // two equal kept sends (see wave_emit)
#ifdef DSL_X2_EMIT  // cost probe (measurement builds): the same rows written twice
          wave_emit<P, SP>(fits, rows, (uint64_t)j, d, a.next + idx * NW);
#endif
          PH_MARK(6);  // history + row emission
          // beyond the segment's rows: spill (parent, event); materialized after the level (rare)
          const bool spill = is_valid && !fits;
          if (__ballot(spill)) {
            const unsigned long long sidx = wave_reserve(&a.ctr->spilled, spill);
            if (spill) {
              if (sidx < a.spill_cap) a.spill[sidx] = ((p0 + j) << 20) | (uint64_t)k;
              else atomicAdd(&a.ctr->err_frontier, 1ull);
            }
          }
        }
        if (ROUTE) {
          // region `dest`, sub-slab `sub` (see RouteCounters); a record past its sub-slab goes to
          // the route-spill list (parent, event), which the host re-routes after the level
          // (BfsEngine::complete_sharded; rare)
          // the workgroup's sub-slab rotates with its passes, so one workgroup's records (a small
          // level has few workgroups) spread over every sub-slab
#ifdef DSL_ROUTE_BLOCK
          const int sub = (int)((blockIdx.x + (unsigned)npass++) % kRouteSegs);
          const unsigned long long ridx = block_reserve<kLevelBlock>(s_resv, a.rc->out + rc_idx(0, sub), route, dest,
                                                                     a.W, kRouteSegs * kRouteStride);
#else
          // by wave: the wave's sub-slab rotates with its passes and with the workgroup, so every
          // sub-slab takes records of all four waves of many workgroups (blockIdx * 4 + wid gave
          // sub-slab q only wave q % 4's records: in a one-round level each wave routes its own
          // share of the class-sorted items, so the sub-slabs of one wave index filled 1.6x the
          // mean and overflowed into the completion phase)
          const int sub = (int)((blockIdx.x + (unsigned)wid * (kRouteSegs / NWAVE) + (unsigned)npass++) % kRouteSegs);
          const unsigned long long ridx = wave_reserve_dest(a.rc->out + rc_idx(0, sub), route, dest, a.W,
                                                            kRouteSegs * kRouteStride);
#endif
          if (route) {
            const uint64_t item = ((p0 + j) << 20) | (uint64_t)k;
            if (ridx < a.route_cs) {
              const uint64_t o = (uint64_t)dest * a.cap_fp + kRouteHdr + (uint64_t)sub * a.route_cs + ridx;
              a.out_item[o] = item;
              if (!a.out_pk) a.out_key[o] = f;
              if (a.out_pk) {  // what the owner probes (its own region's too): 12 bytes
                uint32_t* pk = a.out_pk + (uint64_t)dest * a.cap_pk +
                               (uint64_t)kPkWords * (kPkHdr + (uint64_t)sub * a.route_cs + ridx);
                pk[0] = (uint32_t)f.lo;
                pk[1] = (uint32_t)f.hi;
                pk[2] = (uint32_t)(f.hi >> 32);
              }
            } else {
              const unsigned long long x = atomicAdd(&a.ctr->route_spilled, 1ull);
              if (x < a.rspill_cap) a.rspill[x] = item;
              else atomicAdd(&a.ctr->err_frontier, 1ull);
            }
          }
        }
      }
      PH_MARK(10);  // the pass loop's exit
      if (w0 + kWin < total) __syncthreads();  // the window's LDS arrays are reused by the next window
    }
    __syncthreads();  // LDS is reused by the next chunk
    PH_MARK(10);  // end-of-window / end-of-chunk barrier waits
  }
  {  // the statistics in one workgroup reduction (one barrier pair, one atomic each)
    constexpr int NS = kDD ? 6 : 5;
    uint32_t v[NS];
    v[0] = wave_sum(c_succ);
    v[1] = wave_sum(c_new);
    v[2] = wave_sum(c_next_work);
    v[3] = wave_sum(c_work);
    v[4] = wave_sum(c_probe);
    if constexpr (NS > 5) v[5] = wave_sum(c_dup);
    __syncthreads();
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < NS; i++) s_red5[wid * 6 + i] = v[i];
    __syncthreads();
    if (tid < NS) {
      unsigned long long t = 0;
      for (int w = 0; w < NWAVE; w++) t += s_red5[w * 6 + tid];
      unsigned long long* dst = tid == 0 ? &a.ctr->successors : tid == 1 ? &a.ctr->new_states
                                : tid == 2 ? &a.ctr->next_work : tid == 3 ? &a.ctr->work_items
                                : tid == 4 ? &a.ctr->probes : &a.ctr->deduped;
      if (t) atomicAdd(dst, t);
    }
  }
  PH_MARK(11);  // the statistics reduction
  PH_FLUSH(s_red, a.ctr);
  PH_CLS_FLUSH(a.ctr);
}

// Materializes spilled VALID states (already inserted, counted and judged) at next_size.
// n_dev (multi-shard fast path, the host has not read the counters): n = min(*n_dev, n).
template <class P>
__global__ void __launch_bounds__(kBlock) k_unspill(const uint64_t* items, uint64_t n, const uint32_t* cur,
                                                    const Fp* cur_fp, uint32_t* next, Fp* next_fp,
                                                    uint64_t* next_parent, uint32_t* next_event, uint64_t base_idx,
                                                    int32_t me, LevelCounters* ctr, typename P::Params prm,
                                                    DevSettings set, const unsigned long long* n_dev = nullptr) {
  constexpr int NW = Layout<P>::kWords;
  __shared__ unsigned long long s_red[kBlock / 64];
  unsigned long long c_next_work = 0;
  if (n_dev) n = min<uint64_t>(*n_dev, n);
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
    const uint64_t i = base + threadIdx.x;
    unsigned long long ne = 0;
    bool ok = false;
    uint64_t parent = 0;
    Delta<P> d;
    d.out.n = 0;
    d.keep = 0;
    if (i < n) {
      parent = items[i] >> 20;
      const int k = (int)(items[i] & 0xfffff);
      const uint32_t* w = cur + parent * NW;
      delta_step<P>(w, k, d, prm, set);
      const uint64_t idx = base_idx + i;
      ok = Net<P>::size(w) + delta_new_count<P>(d) <= P::kNetCap;
      if (!ok) atomicAdd(&ctr->err_overflow, 1ull);
      next_fp[idx] = delta_fingerprint<P>(w, cur_fp[parent], d);
      next_parent[idx] = ((uint64_t)me << 48) | parent;
      next_event[idx] = (uint32_t)k;
      ne = (unsigned long long)delta_event_count<P>(w, count_events<P>(w, prm, set), d, prm, set);
    }
    if (wave_emit<P>(ok, cur, parent, d, next + (base_idx + i) * NW) && __lane_id() == 0)
      atomicAdd(&ctr->err_overflow, 1ull);  // two equal kept sends (see wave_emit)
    c_next_work += ne;
  }
  block_flush(s_red, &ctr->next_work, c_next_work);
}

// Search setup in one launch (it replaces three memsets, two copies and k_seed): zeroes the
// visited table, the level counter sets and the route counters, and -- on the shard that holds the
// initial state -- writes the initial row and fingerprint to frontier row 0 and its key into its
// home slot (BFS.initSearch's discovered.add, Search.java:434-440: in an empty table the first
// probe is the home slot). The initial state is judged on the host (bfs_engine.hpp).
template <class P>
struct SetupArgs {
  uint4* table;       // n_table 16-byte units (two slots each)
  uint64_t n_table;
  uint4* ctr;         // n_ctr 16-byte units
  int32_t n_ctr;
  uint4* rc;
  int32_t n_rc;
  int32_t seed;       // this shard holds the initial state
  int32_t clean;      // the table is already zero (cleared when the previous search ended)
  uint64_t home;      // its home slot
  unsigned long long key;
  uint32_t* cur;
  Fp* cur_fp;
  Fp fp;
  uint32_t init[Layout<P>::kWords];
};

template <class P>
__global__ void __launch_bounds__(kBlock) k_setup(SetupArgs<P> a) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t hu = a.seed ? a.home >> 1 : ~0ull;
  // a clean table needs only the seed's unit
  const uint64_t lo = a.clean ? (a.seed ? hu : 0) : 0, hi = a.clean ? (a.seed ? hu + 1 : 0) : a.n_table;
  for (uint64_t u = lo + tid; u < hi; u += stride) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (u == hu) {
      if (a.home & 1) v = make_uint4(0, 0, (uint32_t)a.key, (uint32_t)(a.key >> 32));
      else v = make_uint4((uint32_t)a.key, (uint32_t)(a.key >> 32), 0, 0);
    }
    a.table[u] = v;
  }
  if (blockIdx.x == 0) {
    for (int i = threadIdx.x; i < a.n_ctr; i += blockDim.x) a.ctr[i] = make_uint4(0, 0, 0, 0);
    for (int i = threadIdx.x; i < a.n_rc; i += blockDim.x) a.rc[i] = make_uint4(0, 0, 0, 0);
    if (a.seed) {
      for (int i = threadIdx.x; i < Layout<P>::kWords; i += blockDim.x) a.cur[i] = a.init[i];
      if (threadIdx.x == 0) *a.cur_fp = a.fp;
    }
  }
}

// The queue's counter sets to the pinned host copy (BfsEngine::enqueue_queue), launched on the
// stream right behind the queued levels. A hipMemcpyAsync's blit kernel started ~12 us after the
// last level (rocprofv3 kernel trace); a kernel follows back-to-back like the levels do. The
// system-scope fence makes the stores visible to the host before the kernel completes.
__global__ void __launch_bounds__(kBlock) k_fetch_counters(const uint4* __restrict__ src, uint4* dst, int n16) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) dst[i] = src[i];
  __threadfence_system();
}

// Visited-table growth (a level boundary, BfsEngine::ensure_table): every key of `from` into the
// larger, zeroed table `to` of the same key layout (fingerprint.hpp: the home is recomputed from
// the slot word and its position). All keys are distinct, so a CAS only looks for an empty slot.
__global__ void __launch_bounds__(kBlock) k_rehash(Table from, Table to, unsigned long long* err) {
  const uint64_t n = (from.bucket_mask + 1) * 8, nmask = to.bucket_mask * 8 + 7;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long bad = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t v = from.slots[i];
    if (!v) continue;
    const uint64_t home = table_rehome(from, to, i, v), base = v & ~0xEull;
    uint64_t j = home;
    bool done = false;
    for (int p = 0; p < 8 * (kMaxDisp + 1) && !done; p++) {
      const uint64_t d = ((j >> 3) - (home >> 3)) & to.bucket_mask;
      if (d > (uint64_t)kMaxDisp) break;
      if (atomicCAS(to.slots + j, 0ull, (unsigned long long)(base | (d << 1))) == 0ull) done = true;
      else j = (j + 1) & nmask;
    }
    bad += done ? 0 : 1;
  }
  if (bad) atomicAdd(err, bad);
}

// ---- multi-shard phases (see bfs_engine.hpp) -------------------------------------------------
// Virtual shards' all-to-all round (BfsEngine::xfer without a communicator): every (source,
// destination) segment of the round in ONE launch instead of a device copy per pair. Segment i
// is seg[3i] = source address, seg[3i + 1] = destination address, seg[3i + 2] = bytes.
__global__ void __launch_bounds__(kBlock) k_copy_segments(const uint64_t* seg, int n) {
  for (int i = blockIdx.y; i < n; i += gridDim.y) {
    const uint8_t* src = reinterpret_cast<const uint8_t*>(seg[3 * i]);
    uint8_t* dst = reinterpret_cast<uint8_t*>(seg[3 * i + 1]);
    const uint64_t len = seg[3 * i + 2];
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (uint64_t)gridDim.x * blockDim.x;
    if ((((uintptr_t)src | (uintptr_t)dst | len) & 7) == 0) {
      const uint64_t* s8 = reinterpret_cast<const uint64_t*>(src);
      uint64_t* d8 = reinterpret_cast<uint64_t*>(dst);
      for (uint64_t k = t0; k < len / 8; k += st) d8[k] = s8[k];
    } else {
      for (uint64_t k = t0; k < len; k += st) dst[k] = src[k];
    }
  }
}

// A sharded level's closing record (one per shard, gathered by every rank in ONE collective,
// BfsEngine::run): what the next level and the level's bookkeeping need from every shard. It is
// computed on the device from the shard's counters, so the host reads nothing before it.
enum : int {
  kRecNew = 0, kRecRows, kRecSucc, kRecErrOverflow, kRecErrTable, kRecErrFrontier, kRecWork, kRecParents,
  kRecNextWork, kRecTerm, kRecTimeUp, kRecProbes, kRecLevelTimeUp,
  kRecIncomplete,   // the fast path left work for the host (route spills, row spills past their room)
  kRecCap,          // the records one out_fp region of the shard holds (+1: its header)
  kRecRoute,        // kMaxShards words: records routed to each shard this level
  kRecWords = kRecRoute + kMaxShards
};
struct RecordArgs {
  const LevelCounters* c;
  const unsigned long long* seg_ctr;  // nseg counters, kSegStride apart
  int32_t nseg;
  uint64_t segcap;
  uint64_t extra_rows;     // host-known rows beyond the segments (the completion phase), else 0
  uint64_t uns_cap;        // fast path: unspilled rows = min(spilled, uns_cap)
  uint64_t mat_cap;        // materialized rows = min(next_size, mat_cap)
  uint64_t parents, time_up;
  int32_t gid, W;
  RouteCounters* rc;  // null: no routing this level
  int32_t zero_rc;    // the record is the route counters' last reader: zero them for the next level
  uint64_t cap_fp;
  uint64_t* out;
  uint64_t* ctr_out;  // the shard's LevelCounters and its nseg segment counts (kCtrMirrorWords), so
                      // the host reads records and counters in ONE copy
};
constexpr int kLcWords = (int)(sizeof(LevelCounters) / 8);
constexpr int kCtrMirrorWords = kLcWords + kSegs;
static_assert(sizeof(LevelCounters) % 8 == 0, "LevelCounters mirrored in 8-byte words");
__global__ void __launch_bounds__(64) k_level_record(RecordArgs a) {
  // one wave: the segment counters and the route counters summed lane-parallel (a single thread
  // walking them took ~13 us of dependent loads per launch)
  const int lane = threadIdx.x;
  const LevelCounters* c = a.c;
  uint32_t seg = 0;
  for (int q = lane; q < a.nseg; q += 64) {
    const uint64_t v = a.seg_ctr[q * kSegStride];
    seg += (uint32_t)min<uint64_t>(v, a.segcap);
    a.ctr_out[kLcWords + q] = v;
  }
  for (int i = lane; i < kLcWords; i += 64) a.ctr_out[i] = reinterpret_cast<const uint64_t*>(c)[i];
  uint64_t route[kMaxShards];
#pragma unroll
  for (int d = 0; d < kMaxShards; d++) {
    uint64_t r = 0;
    if (a.rc && d < a.W && lane < kRouteSegs) {
      r = a.rc->out[rc_idx(d, lane)];
      if (a.zero_rc) a.rc->out[rc_idx(d, lane)] = 0;
    }
    for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
    route[d] = r;
  }
  for (int o = 32; o > 0; o >>= 1) seg += __shfl_xor(seg, o);
  if (lane) return;
  uint64_t rows = a.extra_rows + seg;
  rows += min<uint64_t>(c->spilled, a.uns_cap) + min<uint64_t>(c->next_size, a.mat_cap);
  uint64_t* out = a.out;
  out[kRecNew] = c->new_states;
  out[kRecRows] = rows;
  out[kRecSucc] = c->successors;
  out[kRecErrOverflow] = c->err_overflow;
  out[kRecErrTable] = c->err_table;
  out[kRecErrFrontier] = c->err_frontier;
  out[kRecWork] = c->work_items;
  out[kRecParents] = a.parents;
  out[kRecNextWork] = c->next_work;
  out[kRecTerm] = c->term_best ? ((~(uint64_t)c->term_best) & ~(uint64_t)0xff) | (uint64_t)a.gid : ~0ull;
  out[kRecTimeUp] = a.time_up;
  out[kRecProbes] = c->probes;
  out[kRecLevelTimeUp] = c->time_up;  // the level itself stopped at the deadline (partial)
  out[kRecIncomplete] = (c->spilled > a.uns_cap ? 1 : 0) | (c->route_spilled ? 2 : 0);
  out[kRecCap] = a.cap_fp;
#pragma unroll
  for (int d = 0; d < kMaxShards; d++) out[kRecRoute + d] = route[d];
}

// The header of every destination region (the kRouteSegs counts of its sub-slabs, clipped to the
// sub-slab capacity); the owner reads it from the region it receives (k_probe_slab). Also zeroes
// k_new_list's counter for this level (no separate fill launch).
__global__ void k_route_headers(const RouteCounters* rc, Fp* out_key, uint64_t cap_fp, uint64_t cs, int W,
                                unsigned long long* zero_ctr, uint32_t* out_pk, uint64_t cap_pk) {
  const int t = threadIdx.x, d = t / kRouteSegs, q = t - d * kRouteSegs;
  if (t == 0 && zero_ctr) *zero_ctr = 0ull;
  if (d < W) {
    const uint64_t c = min<uint64_t>(rc->out[rc_idx(d, q)], cs);
    reinterpret_cast<uint64_t*>(out_key + (uint64_t)d * cap_fp)[q] = c;
    if (out_pk) {  // the packed region's header: the same counts, two words each
      out_pk[(uint64_t)d * cap_pk + 2 * q] = (uint32_t)c;
      out_pk[(uint64_t)d * cap_pk + 2 * q + 1] = (uint32_t)(c >> 32);
    }
  }
}

// Owner side of the fast path: W regions of cap_fp records (layout: RouteCounters), the received
// ones at in[s * cap_fp], this shard's own in its out_key (`self`). The sources are interleaved
// (consecutive items take consecutive sources), so duplicates of one state from several sources
// race fairly for "new". A record is answered at the same index of reply[s * cap_fp + ...], this
// shard's own at self_reply[...] (its source-side answer array).
struct ProbeSlabArgs {
  const Fp* in;
  const uint32_t* in_pk;  // the other sources' regions as received: packed (kPkWords per record); null: `in`
  const uint32_t* self_pk;  // this shard's own region, packed (its out_pk)
  uint64_t cap_pk;
  const Fp* self;
  uint64_t cap_fp, cs;
  int32_t W, me;
  Table table;
  uint8_t* reply;       // null: no answers (the maxDepth level)
  uint8_t* self_reply;
  LevelCounters* ctr;
};
// Grid: x = the W * kRouteSegs (source, sub-slab) groups, y = 256-record blocks of a sub-slab
// (grid-stride). x varies fastest in the dispatch order, so the sources' records are probed
// interleaved in time; no 64-bit division per record.
__global__ void __launch_bounds__(kBlock) k_probe_slab(ProbeSlabArgs a) {
  __shared__ unsigned long long s_red[kBlock / 64];
  const int g = blockIdx.x, src = g / kRouteSegs, q = g - src * kRouteSegs;
  const bool self = src == a.me;
  const bool pk = a.in_pk != nullptr;  // packed regions: the received ones in in_pk, this shard's own in self_pk
  const Fp* region = self ? a.self : a.in + (uint64_t)src * a.cap_fp;
  const uint32_t* pregion = pk ? (self ? a.self_pk : a.in_pk + (uint64_t)src * a.cap_pk) : nullptr;
  const uint64_t n = min<uint64_t>(pk ? ((uint64_t)pregion[2 * q] | ((uint64_t)pregion[2 * q + 1] << 32))
                                      : reinterpret_cast<const uint64_t*>(region)[q], a.cs);
  uint8_t* rep = a.reply ? (self ? a.self_reply : a.reply + (uint64_t)src * a.cap_fp) : nullptr;
  const uint64_t base = kRouteHdr + (uint64_t)q * a.cs;  // the answers keep the 16-byte layout's indexes
  const uint64_t pbase = (uint64_t)kPkWords * (kPkHdr + (uint64_t)q * a.cs);
  unsigned long long c_new = 0;
  for (uint64_t j = (uint64_t)blockIdx.y * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.y * blockDim.x) {
    Fp f;
    if (pk) {  // lo's owner bits (above kKeyBits) are not needed by the probe
      const uint32_t* r = pregion + pbase + (uint64_t)kPkWords * j;
      f = Fp{(uint64_t)r[1] | ((uint64_t)r[2] << 32), (uint64_t)r[0]};
    } else {
      f = region[base + j];
    }
    const int ins = table_insert(a.table, f);
    if (ins == INS_FULL) atomicAdd(&a.ctr->err_table, 1ull);
    c_new += ins == INS_NEW;
    if (rep) rep[base + j] = ins == INS_NEW ? 1 : 0;
  }
  block_flush(s_red, &a.ctr->new_states, c_new);
}

// Route-spilled successors (k_level's rspill list) re-fingerprinted and laid out per destination
// (completion phase): region d of `out` (cap records, no header) gets those owned by d.
template <class P>
__global__ void __launch_bounds__(kBlock) k_respill(const uint64_t* items, uint64_t n, const uint32_t* cur,
                                                    const Fp* cur_fp, int32_t W, Fp* out_key, uint64_t* out_item, uint64_t cap,
                                                    unsigned long long* cnt, LevelCounters* ctr, typename P::Params prm,
                                                    DevSettings set) {
  constexpr int NW = Layout<P>::kWords;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t parent = items[i] >> 20;
    const int k = (int)(items[i] & 0xfffff);
    const uint32_t* w = cur + parent * NW;
    Delta<P> d;
    delta_step<P>(w, k, d, prm, set);  // deterministic: the successor k_level fingerprinted
    const Fp f = delta_fingerprint<P>(w, cur_fp[parent], d);
    const int dest = owner_of(f, W);
    const unsigned long long x = atomicAdd(&cnt[dest], 1ull);
    if (x < cap) {
      out_key[(uint64_t)dest * cap + x] = f;
      out_item[(uint64_t)dest * cap + x] = items[i];
    }
    else atomicAdd(&ctr->err_frontier, 1ull);
  }
}

// A sharded level keeps every new state at the shard that generated it; only the visited set is
// partitioned. Routed successors go to their owner as 16-byte fingerprints (round A), the owner probes
// and answers one byte per record, in the order received (round B: its counts are round A's,
// reversed, so no second count exchange), and the source materializes, judges and appends the
// successors its owners found new.
struct ProbeArgs {
  const Fp* in;
  uint64_t n;
  Table table;
  uint8_t* reply;  // 1 = inserted (new), per received record
  LevelCounters* ctr;
};

__global__ void __launch_bounds__(kBlock) k_probe_remote(ProbeArgs a) {
  __shared__ unsigned long long s_red[kBlock / 64];
  unsigned long long c_new = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    const int ins = table_insert(a.table, a.in[i]);
    if (ins == INS_FULL) atomicAdd(&a.ctr->err_table, 1ull);
    c_new += ins == INS_NEW;
    a.reply[i] = ins == INS_NEW ? 1 : 0;
  }
  block_flush(s_red, &a.ctr->new_states, c_new);
}

// The routed records the owners found new, as a compact list of their slots (k_new_list), so
// k_materialize runs one lane per new successor (a lane per routed record left ~4 of 5 lanes
// idle on C3). Fast path: groups (d, q) = sub-slab q of region d, the first min(rc[d][q], cs)
// records at d * cap + kRouteHdr + q * cs; completion phase: groups d, cnt[d] records at d * cap.
struct NewListArgs {
  const uint8_t* reply;
  uint64_t cap;
  int32_t W;
  const RouteCounters* dev_cnt;  // null: the host's cnt[]
  uint64_t cs;
  uint64_t cnt[kMaxShards];
  uint64_t* list;
  unsigned long long* n_list;
};
// Grid: x = the groups, y = blocks of a group (grid-stride). A workgroup counts the new records of
// all its items first and reserves their list slots with ONE atomic (a reservation per wave hit
// the list's counter ~200 K times per shard on C3's level 8), then writes them.
__global__ void __launch_bounds__(kBlock) k_new_list(NewListArgs a) {
  __shared__ uint32_t s_cnt[kBlock / 64];
  __shared__ unsigned long long s_base;
  const int g = blockIdx.x, lane = __lane_id(), wid = threadIdx.x >> 6;
  const bool dev = a.dev_cnt != nullptr;
  if (g >= (dev ? a.W * kRouteSegs : a.W)) return;
  const int d = dev ? g / kRouteSegs : g, q = dev ? g - d * kRouteSegs : 0;
  const uint64_t n = dev ? min<uint64_t>(a.dev_cnt->out[rc_idx(d, q)], a.cs) : a.cnt[g];
  const uint64_t base = dev ? (uint64_t)d * a.cap + kRouteHdr + (uint64_t)q * a.cs : (uint64_t)g * a.cap;
  const uint64_t stride = (uint64_t)gridDim.y * blockDim.x;
  uint32_t mine = 0;  // this wave's new records (wave-uniform)
  for (uint64_t j = (uint64_t)blockIdx.y * blockDim.x + threadIdx.x; j - threadIdx.x < n; j += stride)
    mine += (uint32_t)__popcll(__ballot(j < n && a.reply[base + j] != 0));
  if (lane == 0) s_cnt[wid] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kBlock / 64; w++) t += s_cnt[w];
    s_base = t ? atomicAdd(a.n_list, (unsigned long long)t) : 0ull;
  }
  __syncthreads();
  unsigned long long x = s_base;
  for (int w = 0; w < wid; w++) x += s_cnt[w];
  for (uint64_t j = (uint64_t)blockIdx.y * blockDim.x + threadIdx.x; j - threadIdx.x < n; j += stride) {
    const bool take = j < n && a.reply[base + j] != 0;
    const unsigned long long m = __ballot(take);
    if (take) a.list[x + __popcll(m & ((1ull << lane) - 1ull))] = base + j;
    x += __popcll(m);
  }
}

template <class P>
struct MaterializeArgs {
  const Fp* sent_key;                // (unused since round 6: the fingerprint is recomputed from the parent's)
  const uint64_t* sent_item;         // ... and their (parent << 20 | event) items
  const uint64_t* list;              // the slots of the new ones (k_new_list)
  const unsigned long long* n_list;
  const uint32_t* cur;
  const Fp* cur_fp;
  int32_t me, depth, incremental;
  // the rows' reservation: segmented (seg_ctr non-null: workgroup b appends to segment b % nseg,
  // rows [q * segcap, (q + 1) * segcap), as k_level does -- one counter word took every wave's
  // returning atomic, ~40 us per launch on C5's sharded levels), else next_size from next_base
  unsigned long long* seg_ctr;
  int32_t nseg;
  uint64_t segcap;
  uint32_t* next;                    // rows [next_base, next_base + next_cap) of the next frontier
  Fp* next_fp;
  uint64_t* next_parent;
  uint32_t* next_event;
  uint64_t next_base, next_cap;
  LevelCounters* ctr;                // next_size counts the appended rows
  TerminalRec* terms;
  uint32_t term_cap;
  int32_t per_fixed;                 // states per wave (<= the LDS rows per wave), 0: from the list size
};

// States per wave at most in k_materialize: a wave stages its states' parent rows in LDS (8 KiB
// per wave), so the handler, the judge and the emitter read LDS, not global memory.
template <class P>
constexpr int mat_per_max() {
  constexpr int r = 8192 / (Layout<P>::kWords * 4);
  return r < 8 ? 8 : r > 64 ? 64 : r;
}

template <class P>
__global__ void __launch_bounds__(kBlock) k_materialize(MaterializeArgs<P> a, typename P::Params prm, DevSettings set) {
  constexpr int NW = Layout<P>::kWords;
  constexpr int PMAX = mat_per_max<P>();
  __shared__ uint32_t s_nodew[kBlock * P::kNodeWords];
  __shared__ typename P::Rec s_sends[NetPreds<P>::value ? kBlock * P::kMaxSends : 1];
  __shared__ unsigned long long s_red[kBlock / 64];
  extern __shared__ __align__(16) uint32_t s_mrows[];  // (kBlock / 64) x PMAX parent rows
  unsigned long long c_next_work = 0;
  const uint64_t n = *a.n_list;
  // states per wave: a wave writes its rows one after another (wave_emit), so a short list is
  // spread over about as many waves as the chip holds at once (at least 8 states each) instead of
  // 64 per wave on a few workgroups (C5's sharded levels: ~85 us per launch whatever the size); a
  // long list keeps up to PMAX per wave (C3: the handler's lanes full). The grid is about the
  // resident workgroups (BfsEngine::launch_materialize): every wave of it has work.
  const uint64_t waves = (uint64_t)gridDim.x * (kBlock / 64);
  const int per = a.per_fixed ? a.per_fixed : (int)max<uint64_t>(8, min<uint64_t>(PMAX, (n + waves - 1) / waves));
  const int lane = __lane_id(), wid = threadIdx.x >> 6;
  uint32_t* wrows = s_mrows + wid * per * NW;
#ifdef DSL_PHASES  // per-phase shader cycles of the wave passes: LevelCounters::phcls[10..15], passes in [31]
  unsigned long long mph[6] = {0, 0, 0, 0, 0, 0}, mpass = 0, mt = clock64();
#define MAT_PH(i) do { const unsigned long long t1 = clock64(); mph[i] += t1 - mt; mt = t1; } while (0)
#else
#define MAT_PH(i) do { } while (0)
#endif
  for (uint64_t base = ((uint64_t)blockIdx.x * (kBlock / 64) + wid) * per; base < n; base += waves * per) {
#ifdef DSL_PHASES
    mpass++;
    mt = clock64();
#endif
    const uint64_t i = base + lane;
    const bool act = lane < per && i < n;
    bool ship = false;
    int tv = 0, tpi = -1, k = 0;
    uint64_t parent = 0, tkey = ~0ull, slot = 0;
    if (act) {
      slot = a.list[i];
      const uint64_t item = a.sent_item[slot];
      parent = item >> 20;
      k = (int)(item & 0xfffff);
    }
    MAT_PH(0);  // (the loads' latency shows in the staging phase, their first use)
    // the wave's parent rows into LDS with LDS-DMA (no register round trip: a load-then-store
    // copy waited for each row's load before the next row's, ~9 us per pass on C5's level 11)
    const int nr = (int)min<uint64_t>((uint64_t)per, n - base);
    constexpr int U = NW / 4;  // 16-byte units per row
    if constexpr (U < 64 && 64 % U == 0) {
      // small rows: 64 / U rows per wave-instruction (lane = row * U + unit; LDS row-major)
      constexpr int RPI = 64 / U;
      for (int r0 = 0; r0 < nr; r0 += RPI) {
        const int r = r0 + lane / U;
        const uint64_t pr = __shfl((unsigned long long)parent, r < 64 ? r : 63);
        if (r < nr)
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(reinterpret_cast<const uint4*>(a.cur + pr * NW) + lane % U),
              (__attribute__((address_space(3))) void*)(wrows + r0 * NW), 16, 0, 0);
      }
    } else {
      for (int r = 0; r < nr; r++) {
        const uint4* src = reinterpret_cast<const uint4*>(a.cur + rl64(parent, r) * NW);
#pragma unroll
        for (int b = 0; b < U; b += 64)
          if (b + lane < U)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + b + lane),
                                             (__attribute__((address_space(3))) void*)(wrows + r * NW + 4 * b), 16, 0, 0);
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    MAT_PH(1);
    const uint32_t* w = wrows + (act ? lane : 0) * NW;
    Delta<P> d;
    d.node = 0;
    d.out.n = 0;
    d.keep = 0;
    Fp f{0, 0};
    if (act) {
      delta_step<P>(w, k, d, prm, set);  // deterministic: the successor k_level fingerprinted
    }
    MAT_PH(2);
    if (act) {
      // the fingerprint again from the parent's (the routed records cross the links packed, and the
      // source keeps no 16-byte copy of them)
      f = delta_fingerprint<P>(w, a.cur_fp[parent], d);
      int pi = -1;
      uint32_t* my_nw = s_nodew + threadIdx.x * P::kNodeWords;
#pragma unroll
      for (int q = 0; q < P::kNodeWords; q++) my_nw[q] = d.nw[q];
      NodeView view{w, P::kNodeWords, d.node, my_nw};
      if constexpr (NetPreds<P>::value) {
        typename P::Rec* ms = s_sends + threadIdx.x * P::kMaxSends;
        int c = 0;
#pragma unroll
        for (int q = 0; q < P::kMaxSends; q++)
          if ((d.keep >> q) & 1u) ms[c++] = d.out.r[q];
        view.sends = ms;
        view.nsends = c;
      }
      const int v = judge_view<P>(view, prm, set, a.depth, &pi, a.incremental != 0);
      if (v == V_VALID) {
        if (Net<P>::size(w) + delta_new_count<P>(d) <= P::kNetCap) ship = true;
        else atomicAdd(&a.ctr->err_overflow, 1ull);
      } else if (v >= V_TERM_EXCEPTION) {
        tv = v;
        tpi = pi;
        tkey = term_key(v, f.hi);
      }
    }
    fold_terminals(tkey != ~0ull, tkey, tv, tpi, (uint32_t)k, parent, a.ctr, a.terms, a.term_cap);
    MAT_PH(3);
    // the wave's segment: waves take the list in order, so a short list only reaches the first
    // waves -- by wave, not by workgroup, its rows spread over every segment
    const int seg = a.seg_ctr ? (int)((blockIdx.x * (kBlock / 64) + wid) % (unsigned)a.nseg) : 0;
    const unsigned long long li = wave_reserve(a.seg_ctr ? &a.seg_ctr[seg * kSegStride] : &a.ctr->next_size, ship);
    const bool fits = ship && li < (a.seg_ctr ? a.segcap : a.next_cap);
    if (ship && !fits) atomicAdd(&a.ctr->err_frontier, 1ull);
    const uint64_t idx = a.seg_ctr ? (uint64_t)seg * a.segcap + li : a.next_base + li;
    if (fits) {
      a.next_fp[idx] = f;
      a.next_parent[idx] = ((uint64_t)a.me << 48) | parent;
      a.next_event[idx] = (uint32_t)k;
      c_next_work += (unsigned long long)delta_event_count<P>(w, count_events<P>(w, prm, set), d, prm, set);
    }
    MAT_PH(4);
    bool coll;
    if constexpr (LaneEmit<P>::value) coll = lane_emit<P>(fits, w, d, a.next + idx * NW);
    else coll = wave_emit<P>(fits, wrows, (uint64_t)lane, d, a.next + idx * NW, s_nodew + (threadIdx.x - lane) * P::kNodeWords);
    if (coll && __lane_id() == 0)
      atomicAdd(&a.ctr->err_overflow, 1ull);  // two equal kept sends (see wave_emit)
    __builtin_amdgcn_wave_barrier();  // the rows are overwritten by the next iteration's staging
    MAT_PH(5);
  }
#ifdef DSL_PHASES
  if (lane == 0 && mpass) {
    for (int q = 0; q < 6; q++) atomicAdd(&a.ctr->phcls[10 + q], mph[q]);
    atomicAdd(&a.ctr->phcls[31], mpass);
  }
#endif
#undef MAT_PH
  block_flush(s_red, &a.ctr->next_work, c_next_work);
}

}  // namespace dsl

namespace dsl {

// ---- random depth-first search (RandomDFS.runProbe, Search.java:507-583) -------------------------
// One probe per lane: from the initial state, repeatedly try the current state's enabled events in
// a random order (a random rotation of SearchState.events: Collections.shuffle's role) and move to
// the first successor that is not null and not PRUNED (counting every non-null successor, as
// states.incrementAndGet()); a TERMINAL successor ends the whole search (first lane wins a CAS); a
// state with no such successor ends the probe and the lane starts a new one. There is no visited
// set. Each launch runs a bounded number of steps per lane, so every wavefront exits.
struct DfsArgs {
  const uint32_t* init;
  int32_t init_depth;
  int32_t tcap;              // events a probe may record (a probe at depth tcap is restarted)
  uint32_t* rows;            // 2 rows per probe (current / successor)
  uint32_t* trace;           // tcap events per probe
  int32_t* pdepth;           // steps taken by the probe; -1 = start a new probe
  int32_t* pcur;             // which of its two rows is current
  uint64_t* rng;
  uint64_t nprobe;
  int32_t steps;
  unsigned long long* ctr;   // [states, probes, overflow]
  int32_t* found;            // 0, or 1 + the winning probe
  int32_t* term;             // winner: [verdict, predicate index, depth]
};

__device__ __forceinline__ uint64_t xorshift64s(uint64_t& x) {
  x ^= x >> 12;
  x ^= x << 25;
  x ^= x >> 27;
  return x * 0x2545F4914F6CDD1Dull;
}

template <class P>
__global__ void __launch_bounds__(kBlock) k_dfs(DfsArgs a, typename P::Params prm, DevSettings set) {
  constexpr int NW = Layout<P>::kWords;
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long c_states = 0, c_probes = 0, c_err = 0;
  if (lane < a.nprobe) {
    int dep = a.pdepth[lane], cur = a.pcur[lane];
    uint64_t rng = a.rng[lane];
    uint32_t* const base = a.rows + lane * 2 * NW;
    for (int step = 0; step < a.steps; step++) {
      if (__hip_atomic_load(a.found, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
      if (dep < 0) {  // runProbe: a new probe from the initial state (counted once)
        for (int i = 0; i < NW; i++) base[i] = a.init[i];
        cur = 0;
        dep = 0;
        c_probes++;
        c_states++;
      }
      if (dep >= a.tcap) {  // a successor would be too deep to record: restart before stepping
        dep = -1;
        continue;
      }
      const uint32_t* w = base + cur * NW;
      uint32_t* nxt = base + (cur ^ 1) * NW;
      const int ne = count_events<P>(w, prm, set);
      bool advanced = false, ended = false;
      const int r0 = ne ? (int)(xorshift64s(rng) % (uint64_t)ne) : 0;
      for (int i = 0; i < ne && !advanced && !ended; i++) {
        const int k = r0 + i < ne ? r0 + i : r0 + i - ne;
        Delta<P> d;
        const int rc = delta_step<P>(w, k, d, prm, set);
        if (rc == STEP_NULL) continue;
        c_states++;
        int v, pi = -1;
        if (rc == STEP_EXCEPTION) {
          v = V_TERM_EXCEPTION;
        } else if (rc == STEP_OVERFLOW || !emit_row<P>(w, d, nxt)) {
          c_err++;
          ended = true;
          break;
        } else {
          const NodeView view{nxt, P::kNodeWords, -1, nullptr};
          v = judge_view<P>(view, prm, set, a.init_depth + dep + 1, &pi);
        }
        if (v >= V_TERM_EXCEPTION) {
          a.trace[lane * a.tcap + dep] = (uint32_t)k;
          if (atomicCAS(a.found, 0, (int)(lane + 1)) == 0) {
            a.term[0] = v;
            a.term[1] = pi;
            a.term[2] = dep + 1;
          }
          ended = true;
          break;
        }
        if (v == V_PRUNED) continue;
        a.trace[lane * a.tcap + dep] = (uint32_t)k;
        dep++;
        cur ^= 1;
        advanced = true;
      }
      if (!advanced) dep = -1;  // no non-pruned successor (or ended): the probe is over
    }
    a.pdepth[lane] = dep;
    a.pcur[lane] = cur;
    a.rng[lane] = rng;
  }
  for (int o = 32; o > 0; o >>= 1) {
    c_states += __shfl_xor(c_states, o);
    c_probes += __shfl_xor(c_probes, o);
    c_err += __shfl_xor(c_err, o);
  }
  if (__lane_id() == 0) {
    if (c_states) atomicAdd(&a.ctr[0], c_states);
    if (c_probes) atomicAdd(&a.ctr[1], c_probes);
    if (c_err) atomicAdd(&a.ctr[2], c_err);
  }
}

}  // namespace dsl
