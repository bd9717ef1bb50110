// sharded.hpp -- hash-partitioned BFS across W shards (GPUs, or virtual shards on one GPU).
//
// Owner of a state = owner_of(fingerprint, W). Each shard keeps the visited-table partition and
// the frontier of the states it owns. One BFS level on shard r:
//   1. k_count + scan over the local frontier (as in the single-shard engine).
//   2. k_expand_route: every successor is fingerprinted; if r owns it, it is inserted, judged
//      and appended locally; otherwise a 24-byte FpRec {fp.hi, fp.lo, work item} goes to the
//      owner's outgoing region (wave-aggregated per-destination reservation).
//   3. exchange #1 (fingerprints) -> k_probe_remote on the owner: table insert; a NEW record's
//      work item id is returned to its source (exchange #2).
//   4. k_materialize on the source: re-derives the successor from (parent, event), judges it
//      (terminal candidates are recorded at the source, which holds the parent), and ships
//      VALID states to their owner (exchange #3) -> k_append_received.
// Only new states cross the links at full size; duplicates cost 24 bytes each way.
// Per-depth counts are the sum over shards of newly inserted keys: shard-count invariant.
#pragma once
#include "engine.hpp"

namespace dsl {

constexpr int kMaxShards = 16;

struct FpRec {
  uint64_t hi, lo;
  uint64_t item;  // work item index at the source
};

template <class P>
struct StateRec {
  typename P::State s;
  uint64_t parent;  // (source shard << 48) | parent index in the source's frontier
  uint32_t event;
  uint32_t pad;
};

struct RouteCounters {
  unsigned long long out[kMaxShards];  // records written per destination
};

__device__ __forceinline__ unsigned long long wave_reserve_dest(unsigned long long* ctrs, bool pred, int dest,
                                                                int W) {
  unsigned long long idx = 0;
  for (int d = 0; d < W; d++) {
    const bool mine = pred && dest == d;
    const unsigned long long r = wave_reserve(&ctrs[d], mine);
    if (mine) idx = r;
  }
  return idx;
}

template <class P>
struct RouteArgs {
  ExpandArgs<P> e;
  int32_t W, me;
  FpRec* out_fp;          // W regions of cap_fp records
  uint64_t cap_fp;
  RouteCounters* rc;
};

template <class P>
__global__ void __launch_bounds__(kBlock) k_expand_route(RouteArgs<P> a, typename P::Params prm, DevSettings set) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const ExpandArgs<P>& e = a.e;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < e.total; base += stride) {
    const uint64_t t = base + threadIdx.x;
    const bool active = t < e.total;
    bool is_new = false, is_valid = false, is_succ = false, route = false;
    int dest = 0;
    uint64_t parent = 0;
    uint32_t ev = 0;
    Fp f{0, 0};
    typename P::State succ;
    if (active) {
      uint64_t lo = 0, hi = e.F;
      while (hi - lo > 1) {
        uint64_t mid = (lo + hi) >> 1;
        if (e.offsets[mid] <= t) lo = mid; else hi = mid;
      }
      parent = lo;
      ev = (uint32_t)(t - e.offsets[lo]);
      const typename P::State s = e.cur[parent];
      const int rc = P::step(s, (int)ev, succ, prm, set);
      if (rc == STEP_OK) {
        is_succ = true;
        f = fingerprint(succ.w);
        dest = owner_of(f, a.W);
        if (dest != a.me) {
          route = true;
        } else {
          const int ins = table_insert(e.table, f);
          if (ins == INS_NEW) {
            is_new = true;
            int pi = -1;
            const int v = judge<P>(succ, prm, set, e.depth, &pi);
            if (v == V_VALID) {
              is_valid = true;
            } else if (v >= V_TERM_EXCEPTION) {
              const unsigned long long slot = atomicAdd(&e.ctr->n_terminals, 1ull);
              if (slot < kTermCap) e.terms[slot] = TerminalRec{v, pi, ev, 0u, parent, f.hi};
            }
          } else if (ins == INS_FULL) {
            atomicAdd(&e.ctr->err_table, 1ull);
          }
        }
      } else if (rc == STEP_EXCEPTION) {
        is_succ = true;
        is_new = true;
        f = fingerprint(succ.w);
        const unsigned long long slot = atomicAdd(&e.ctr->n_terminals, 1ull);
        if (slot < kTermCap) e.terms[slot] = TerminalRec{V_TERM_EXCEPTION, -1, ev, 0u, parent, f.hi};
      } else if (rc == STEP_OVERFLOW) {
        atomicAdd(&e.ctr->err_overflow, 1ull);
      }
    }
    const unsigned long long nsucc = __popcll(__ballot(is_succ));
    const unsigned long long nnew = __popcll(__ballot(is_new));
    if (__lane_id() == 0) {
      if (nsucc) atomicAdd(&e.ctr->successors, nsucc);
      if (nnew) atomicAdd(&e.ctr->new_states, nnew);
    }
    const unsigned long long idx = wave_reserve(&e.ctr->next_size, is_valid);
    if (is_valid) {
      if (idx < e.next_cap) {
        e.next[idx] = succ;
        e.next_parent[idx] = ((uint64_t)a.me << 48) | parent;
        e.next_event[idx] = ev;
      } else {
        atomicAdd(&e.ctr->err_frontier, 1ull);
      }
    }
    const unsigned long long ridx = wave_reserve_dest(a.rc->out, route, dest, a.W);
    if (route) a.out_fp[(uint64_t)dest * a.cap_fp + ridx] = FpRec{f.hi, f.lo, t};
  }
}

struct ProbeArgs {
  const FpRec* in;
  uint64_t n;
  uint64_t src_off[kMaxShards + 1];  // records from source s are in [src_off[s], src_off[s+1])
  int32_t W;
  Table table;
  uint64_t* out_items;  // W regions of cap_v work-item ids (one per source)
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

template <class P>
struct MaterializeArgs {
  const uint64_t* items;  // work items of this shard that are new at their owner
  uint64_t n;
  const typename P::State* cur;
  const unsigned long long* offsets;
  uint64_t F;
  int32_t W, me, depth;
  StateRec<P>* out;  // W regions of cap_s records
  uint64_t cap_s;
  RouteCounters* rc;
  LevelCounters* ctr;
  TerminalRec* terms;
};

template <class P>
__global__ void __launch_bounds__(kBlock) k_materialize(MaterializeArgs<P> a, typename P::Params prm,
                                                        DevSettings set) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < a.n; base += stride) {
    const uint64_t i = base + threadIdx.x;
    bool ship = false;
    int dest = 0;
    uint64_t parent = 0;
    uint32_t ev = 0;
    typename P::State succ;
    if (i < a.n) {
      const uint64_t t = a.items[i];
      uint64_t lo = 0, hi = a.F;
      while (hi - lo > 1) {
        uint64_t mid = (lo + hi) >> 1;
        if (a.offsets[mid] <= t) lo = mid; else hi = mid;
      }
      parent = lo;
      ev = (uint32_t)(t - a.offsets[lo]);
      const typename P::State s = a.cur[parent];
      P::step(s, (int)ev, succ, prm, set);  // deterministic: same successor as in k_expand_route
      const Fp f = fingerprint(succ.w);
      dest = owner_of(f, a.W);
      int pi = -1;
      const int v = judge<P>(succ, prm, set, a.depth, &pi);
      if (v == V_VALID) {
        ship = true;
      } else if (v >= V_TERM_EXCEPTION) {
        const unsigned long long slot = atomicAdd(&a.ctr->n_terminals, 1ull);
        if (slot < kTermCap) a.terms[slot] = TerminalRec{v, pi, ev, 0u, parent, f.hi};
      }
    }
    const unsigned long long idx = wave_reserve_dest(a.rc->out, ship, dest, a.W);
    if (ship) a.out[(uint64_t)dest * a.cap_s + idx] = StateRec<P>{succ, ((uint64_t)a.me << 48) | parent, ev, 0u};
  }
}

template <class P>
__global__ void __launch_bounds__(kBlock) k_append_received(const StateRec<P>* in, uint64_t n,
                                                            typename P::State* next, uint64_t* next_parent,
                                                            uint32_t* next_event, uint64_t next_cap,
                                                            LevelCounters* ctr) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
    const uint64_t i = base + threadIdx.x;
    const bool ok = i < n;
    const unsigned long long idx = wave_reserve(&ctr->next_size, ok);
    if (ok) {
      if (idx < next_cap) {
        next[idx] = in[i].s;
        next_parent[idx] = in[i].parent;
        next_event[idx] = in[i].event;
      } else {
        atomicAdd(&ctr->err_frontier, 1ull);
      }
    }
  }
}

}  // namespace dsl
