// kernels.hpp -- the BFS level kernels for MI355X (gfx950).
//
// k_level<P, ROUTE>: ONE launch per BFS level (Search.java:448-504 with the level barrier of
// :452-455 made explicit). Each workgroup takes a chunk of PB consecutive frontier states:
//   1. the chunk (contiguous rows, PB x S bytes) and its fingerprints are copied to LDS with
//      16-byte coalesced loads -- every parent is read from HBM exactly once;
//   2. one lane per parent counts its enabled events (SearchState.events), a workgroup-local
//      exclusive scan turns the counts into work-item offsets (no global scan pass);
//   3. every lane takes work items (parent j, event k): the successor is computed as a DELTA
//      in registers (one node's words + a short send list), its fingerprint incrementally from
//      the parent's (nodestate.hpp), then one 64-byte visited-table bucket probe / CAS insert
//      (discovered.add, Search.java:485). Only a NEW successor is judged (checkState over a node
//      view: parent words in LDS + the changed node) and, if VALID, materialized straight into
//      the next frontier (row + fingerprint + parent pointer + event index).
//   ROUTE (multi-shard): a successor owned by another shard is not probed here; a 24-byte
//      FpRec goes to its owner's outgoing region instead (sharded.hpp for the other phases).
#pragma once
#include "nodestate.hpp"

namespace dsl {

constexpr int kBlock = 256;
constexpr uint32_t kTermCap = 1024;
constexpr int kMaxShards = 16;

struct LevelCounters {
  unsigned long long new_states;    // newly discovered successors (all verdicts)
  unsigned long long next_size;     // VALID successors appended to the next frontier
  unsigned long long successors;    // events applied (non-null successors)
  unsigned long long n_terminals;   // terminal candidates recorded
  unsigned long long err_overflow;  // STEP_OVERFLOW count
  unsigned long long err_table;     // INS_FULL count
  unsigned long long err_frontier;  // appends beyond capacity
  unsigned long long work_items;    // (state, event) pairs of this level
  unsigned long long next_work;     // enabled events of the appended states (= next level's work)
  unsigned long long spilled;       // VALID states beyond the next frontier's capacity (spill list)
};

struct TerminalRec {
  int32_t verdict;  // V_TERM_*
  int32_t pred_index;
  uint32_t event;   // event index within the parent's enabled events
  uint32_t pad;
  uint64_t parent;  // index of the parent in the current frontier
  uint64_t key;     // fingerprint high word (deterministic tie-break)
};

struct RouteCounters {
  unsigned long long out[kMaxShards];  // records written per destination
};

struct FpRec {
  uint64_t hi, lo;
  uint64_t item;  // (parent index << 20) | event index, at the source shard
};

__device__ __forceinline__ unsigned long long wave_reserve(unsigned long long* ctr, bool pred) {
  const unsigned long long mask = __ballot(pred);
  if (mask == 0) return 0;
  const int lane = __lane_id();
  const int leader = __ffsll((long long)mask) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(mask));
  base = __shfl(base, leader);
  const unsigned long long lt = (lane == 0) ? 0ull : (mask & ((1ull << lane) - 1ull));
  return base + (unsigned long long)__popcll(lt);
}

__device__ __forceinline__ unsigned long long wave_reserve_dest(unsigned long long* ctrs, bool pred, int dest, int W) {
  unsigned long long idx = 0;
  for (int d = 0; d < W; d++) {
    const bool mine = pred && dest == d;
    const unsigned long long r = wave_reserve(&ctrs[d], mine);
    if (mine) idx = r;
  }
  return idx;
}

template <class P>
struct LevelArgs {
  const uint32_t* cur;       // F rows of kWords
  const Fp* cur_fp;
  uint64_t F;
  int32_t PB;                // parents per chunk
  int32_t depth;             // depth of the successors
  uint32_t* next;            // next frontier rows
  Fp* next_fp;
  uint64_t* next_parent;     // history arena slice of the next level
  uint32_t* next_event;
  uint64_t next_cap;
  LevelCounters* ctr;
  TerminalRec* terms;
  Table table;
  uint64_t* spill;           // (parent << 20 | event) of VALID states past next_cap
  uint64_t spill_cap;
  int32_t W, me;             // shards (ROUTE only)
  FpRec* out_fp;             // W regions of cap_fp records (ROUTE only)
  uint64_t cap_fp;
  RouteCounters* rc;
};

template <class P, bool ROUTE>
__global__ void __launch_bounds__(kBlock) k_level(LevelArgs<P> a, typename P::Params prm, DevSettings set) {
  constexpr int NW = Layout<P>::kWords;
  extern __shared__ __align__(16) uint32_t lds[];
  uint32_t* rows = lds;                                    // PB * NW
  Fp* fps = reinterpret_cast<Fp*>(rows + a.PB * NW);       // PB
  int* off = reinterpret_cast<int*>(fps + a.PB);           // PB + 1
  __shared__ int s_total;

  const uint64_t nchunks = (a.F + a.PB - 1) / a.PB;
  for (uint64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const uint64_t p0 = chunk * a.PB;
    const int pb = (int)min<uint64_t>((uint64_t)a.PB, a.F - p0);
    // 1. stage the parents (contiguous rows) and their fingerprints in LDS
    {
      const uint4* src = reinterpret_cast<const uint4*>(a.cur + p0 * NW);
      uint4* dst = reinterpret_cast<uint4*>(rows);
      const int n16 = pb * NW / 4;
      for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
      for (int i = threadIdx.x; i < pb; i += blockDim.x) fps[i] = a.cur_fp[p0 + i];
    }
    __syncthreads();
    // 2. enabled events per parent, workgroup-local exclusive scan
    if (threadIdx.x < pb) off[threadIdx.x + 1] = count_events<P>(rows + threadIdx.x * NW, prm, set);
    __syncthreads();
    if (threadIdx.x == 0) {
      off[0] = 0;
      for (int j = 0; j < pb; j++) off[j + 1] += off[j];
      s_total = off[pb];
      atomicAdd(&a.ctr->work_items, (unsigned long long)off[pb]);
    }
    __syncthreads();
    const int total = s_total;
    // 3. one lane per (parent, event)
    for (int base = 0; base < total; base += blockDim.x) {
      const int t = base + threadIdx.x;
      bool is_new = false, is_valid = false, is_succ = false, route = false;
      int dest = 0, j = 0, k = 0;
      Fp f{0, 0};
      Delta<P> d;
      if (t < total) {
        int lo = 0, hi = pb;
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (off[mid] <= t) lo = mid; else hi = mid;
        }
        j = lo;
        k = t - off[lo];
        const uint32_t* w = rows + j * NW;
        const int rc = delta_step<P>(w, k, d, prm, set);
        if (rc == STEP_OK) {
          is_succ = true;
          f = delta_fingerprint<P>(w, fps[j], d);
          if (ROUTE) dest = owner_of(f, a.W);
          if (ROUTE && dest != a.me) {
            route = true;
          } else {
            const int ins = table_insert(a.table, f);
            if (ins == INS_NEW) {
              is_new = true;
              int pi = -1;
              const NodeView view{w, P::kNodeWords, d.node, d.nw};
              const int v = judge_view<P>(view, prm, set, a.depth, &pi);
              if (v == V_VALID) {
                is_valid = true;
              } else if (v >= V_TERM_EXCEPTION) {
                const unsigned long long slot = atomicAdd(&a.ctr->n_terminals, 1ull);
                if (slot < kTermCap) a.terms[slot] = TerminalRec{v, pi, (uint32_t)k, 0u, p0 + j, f.hi};
              }
            } else if (ins == INS_FULL) {
              atomicAdd(&a.ctr->err_table, 1ull);
            }
          }
        } else if (rc == STEP_EXCEPTION) {
          // exceptional states never equal another (Throwable identity): new and terminal
          is_succ = true;
          is_new = true;
          const unsigned long long slot = atomicAdd(&a.ctr->n_terminals, 1ull);
          if (slot < kTermCap) a.terms[slot] = TerminalRec{V_TERM_EXCEPTION, -1, (uint32_t)k, 0u, p0 + j, fps[j].hi};
        } else if (rc == STEP_OVERFLOW) {
          atomicAdd(&a.ctr->err_overflow, 1ull);
        }
      }
      const unsigned long long nsucc = __popcll(__ballot(is_succ));
      const unsigned long long nnew = __popcll(__ballot(is_new));
      if (__lane_id() == 0) {
        if (nsucc) atomicAdd(&a.ctr->successors, nsucc);
        if (nnew) atomicAdd(&a.ctr->new_states, nnew);
      }
      const unsigned long long idx = wave_reserve(&a.ctr->next_size, is_valid);
      const bool fits = is_valid && idx < a.next_cap;
      unsigned long long ne = 0;
      if (fits) {
        const uint32_t* w = rows + j * NW;
        if (materialize<P>(w, d, a.next + idx * NW)) {
          a.next_fp[idx] = f;
          a.next_parent[idx] = ((uint64_t)a.me << 48) | (p0 + j);
          a.next_event[idx] = (uint32_t)k;
          ne = (unsigned long long)delta_event_count<P>(w, off[j + 1] - off[j], d, prm, set);
        } else {
          atomicAdd(&a.ctr->err_overflow, 1ull);
        }
      }
      // beyond the estimated capacity: spill (parent, event); materialized after the level
      const unsigned long long sidx = wave_reserve(&a.ctr->spilled, is_valid && !fits);
      if (is_valid && !fits) {
        if (sidx < a.spill_cap) a.spill[sidx] = ((p0 + j) << 20) | (uint64_t)k;
        else atomicAdd(&a.ctr->err_frontier, 1ull);
      }
      {
        unsigned long long s = ne;
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (__lane_id() == 0 && s) atomicAdd(&a.ctr->next_work, s);
      }
      if (ROUTE) {
        const unsigned long long ridx = wave_reserve_dest(a.rc->out, route, dest, a.W);
        if (route) a.out_fp[(uint64_t)dest * a.cap_fp + ridx] = FpRec{f.hi, f.lo, ((p0 + j) << 20) | (uint64_t)k};
      }
    }
    __syncthreads();  // LDS is reused by the next chunk
  }
}

// Materializes spilled VALID states (already inserted, counted and judged) at next_size.
template <class P>
__global__ void __launch_bounds__(kBlock) k_unspill(const uint64_t* items, uint64_t n, const uint32_t* cur,
                                                    const Fp* cur_fp, uint32_t* next, Fp* next_fp,
                                                    uint64_t* next_parent, uint32_t* next_event, uint64_t base_idx,
                                                    int32_t me, LevelCounters* ctr, typename P::Params prm,
                                                    DevSettings set) {
  constexpr int NW = Layout<P>::kWords;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
    const uint64_t i = base + threadIdx.x;
    unsigned long long ne = 0;
    if (i < n) {
      const uint64_t parent = items[i] >> 20;
      const int k = (int)(items[i] & 0xfffff);
      const uint32_t* w = cur + parent * NW;
      Delta<P> d;
      delta_step<P>(w, k, d, prm, set);
      const uint64_t idx = base_idx + i;
      if (!materialize<P>(w, d, next + idx * NW)) atomicAdd(&ctr->err_overflow, 1ull);
      next_fp[idx] = delta_fingerprint<P>(w, cur_fp[parent], d);
      next_parent[idx] = ((uint64_t)me << 48) | parent;
      next_event[idx] = (uint32_t)k;
      ne = (unsigned long long)delta_event_count<P>(w, count_events<P>(w, prm, set), d, prm, set);
    }
    for (int o = 32; o > 0; o >>= 1) ne += __shfl_xor(ne, o);
    if (__lane_id() == 0 && ne) atomicAdd(&ctr->next_work, ne);
  }
}

// Inserts the initial state's fingerprint and judges it (BFS.initSearch + exploreNode's
// initial-state check, Search.java:434-440, :470-480).
template <class P>
__global__ void k_seed(const uint32_t* init, const Fp* fp, typename P::Params prm, DevSettings set, Table table,
                       int depth, int32_t* out /* [verdict, pred_index, insert_rc] */) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[2] = table_insert(table, *fp);
    int pi = -1;
    const NodeView v{init, P::kNodeWords, -1, nullptr};
    out[0] = judge_view<P>(v, prm, set, depth, &pi);
    out[1] = pi;
  }
}

// ---- multi-shard phases (see sharded_engine.hpp) -------------------------------------------------
struct ProbeArgs {
  const FpRec* in;
  uint64_t n;
  uint64_t src_off[kMaxShards + 1];  // records from source s are in [src_off[s], src_off[s+1])
  int32_t W;
  Table table;
  uint64_t* out_items;  // W regions of cap_v items (one per source)
  uint64_t cap_v;
  RouteCounters* rc;
  LevelCounters* ctr;
};

__global__ void __launch_bounds__(kBlock) k_probe_remote(ProbeArgs a) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < a.n; base += stride) {
    const uint64_t i = base + threadIdx.x;
    bool is_new = false;
    int src = 0;
    uint64_t item = 0;
    if (i < a.n) {
      const FpRec r = a.in[i];
      while (src + 1 < a.W && a.src_off[src + 1] <= i) src++;
      const int ins = table_insert(a.table, Fp{r.hi, r.lo});
      if (ins == INS_NEW) {
        is_new = true;
        item = r.item;
      } else if (ins == INS_FULL) {
        atomicAdd(&a.ctr->err_table, 1ull);
      }
    }
    const unsigned long long nnew = __popcll(__ballot(is_new));
    if (__lane_id() == 0 && nnew) atomicAdd(&a.ctr->new_states, nnew);
    const unsigned long long idx = wave_reserve_dest(a.rc->out, is_new, src, a.W);
    if (is_new) a.out_items[(uint64_t)src * a.cap_v + idx] = item;
  }
}

// A routed VALID new state: row, fingerprint, parent pointer, event.
template <class P>
struct StateRec {
  uint32_t w[Layout<P>::kWords];
  Fp fp;
  uint64_t parent;
  uint32_t event;
  uint32_t pad;
};

template <class P>
struct MaterializeArgs {
  const uint64_t* items;  // items of this shard found new at their owner
  uint64_t n;
  const uint32_t* cur;
  const Fp* cur_fp;
  int32_t W, me, depth;
  StateRec<P>* out;  // W regions of cap_s records
  uint64_t cap_s;
  RouteCounters* rc;
  LevelCounters* ctr;
  TerminalRec* terms;
};

template <class P>
__global__ void __launch_bounds__(kBlock) k_materialize(MaterializeArgs<P> a, typename P::Params prm, DevSettings set) {
  constexpr int NW = Layout<P>::kWords;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < a.n; base += stride) {
    const uint64_t i = base + threadIdx.x;
    bool ship = false;
    int dest = 0;
    uint64_t parent = 0;
    int k = 0;
    Delta<P> d;
    Fp f{0, 0};
    if (i < a.n) {
      parent = a.items[i] >> 20;
      k = (int)(a.items[i] & 0xfffff);
      const uint32_t* w = a.cur + parent * NW;
      delta_step<P>(w, k, d, prm, set);  // deterministic: the same successor as in k_level
      f = delta_fingerprint<P>(w, a.cur_fp[parent], d);
      dest = owner_of(f, a.W);
      int pi = -1;
      const NodeView view{w, P::kNodeWords, d.node, d.nw};
      const int v = judge_view<P>(view, prm, set, a.depth, &pi);
      if (v == V_VALID) {
        ship = true;
      } else if (v >= V_TERM_EXCEPTION) {
        const unsigned long long slot = atomicAdd(&a.ctr->n_terminals, 1ull);
        if (slot < kTermCap) a.terms[slot] = TerminalRec{v, pi, (uint32_t)k, 0u, parent, f.hi};
      }
    }
    const unsigned long long idx = wave_reserve_dest(a.rc->out, ship, dest, a.W);
    if (ship) {
      StateRec<P>* r = a.out + (uint64_t)dest * a.cap_s + idx;
      const uint32_t* w = a.cur + parent * NW;
      if (!materialize<P>(w, d, r->w)) atomicAdd(&a.ctr->err_overflow, 1ull);
      r->fp = f;
      r->parent = ((uint64_t)a.me << 48) | parent;
      r->event = (uint32_t)k;
      r->pad = (uint32_t)delta_event_count<P>(w, count_events<P>(w, prm, set), d, prm, set);
    }
  }
}

template <class P>
__global__ void __launch_bounds__(kBlock) k_append_received(const StateRec<P>* in, uint64_t n, uint32_t* next, Fp* next_fp,
                                                            uint64_t* next_parent, uint32_t* next_event,
                                                            uint64_t next_cap, LevelCounters* ctr) {
  constexpr int NW = Layout<P>::kWords;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
    const uint64_t i = base + threadIdx.x;
    const bool ok = i < n;
    const unsigned long long idx = wave_reserve(&ctr->next_size, ok);
    unsigned long long ne = 0;
    if (ok) {
      if (idx < next_cap) {
        const uint4* s = reinterpret_cast<const uint4*>(in[i].w);
        uint4* dd = reinterpret_cast<uint4*>(next + idx * NW);
        for (int q = 0; q < NW / 4; q++) dd[q] = s[q];
        next_fp[idx] = in[i].fp;
        next_parent[idx] = in[i].parent;
        next_event[idx] = in[i].event;
        ne = in[i].pad;  // enabled events of the state (next level's work)
      } else {
        atomicAdd(&ctr->err_frontier, 1ull);
      }
    }
    for (int o = 32; o > 0; o >>= 1) ne += __shfl_xor(ne, o);
    if (__lane_id() == 0 && ne) atomicAdd(&ctr->next_work, ne);
  }
}

}  // namespace dsl
