// engine.hpp -- level-synchronous BFS engine for MI355X, templated on a protocol P.
//
// One BFS level (Search.java:448-504 with the level barrier of :452-455 made explicit):
//   k_count   : one thread per frontier state -> number of enabled events (SearchState.events)
//   scan      : exclusive prefix sum -> work-item offsets (one work item = one (state, event))
//   k_expand  : one thread per work item: locate parent, apply the event (stepMessage /
//               stepTimer), fingerprint, probe/insert the visited table (discovered.add),
//               count new states (states++ for every newly discovered successor, pruned and
//               terminal ones included), judge (checkState), record terminal candidates, and
//               append VALID successors + parent pointer + event index to the next frontier
//               with a wave-aggregated atomic.
// The host loop reads four counters per level. A TERMINAL state ends the search after its
// level completes (all depth-d successors generated), and the reported terminal is the
// highest-priority one (EXCEPTION > INVARIANT > GOAL, Search.java:370-385).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"
#include "fingerprint.hpp"

namespace dsl {

void set_error(const std::string& msg);

#define DSL_HIP(call)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (call);                                                                     \
    if (e_ != hipSuccess) {                                                                     \
      set_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + __FILE__ + ":" +  \
                std::to_string(__LINE__) + " (" #call ")");                                     \
      return DSL_ERR_HIP;                                                                       \
    }                                                                                           \
  } while (0)

struct LevelCounters {
  unsigned long long new_states;   // newly discovered successors (all verdicts)
  unsigned long long next_size;    // VALID successors appended to the next frontier
  unsigned long long successors;   // events applied (non-null successors)
  unsigned long long n_terminals;  // terminal candidates recorded
  unsigned long long err_overflow; // STEP_OVERFLOW count
  unsigned long long err_table;    // INS_FULL count
  unsigned long long err_frontier; // appends beyond capacity
  unsigned long long pad;
};

struct TerminalRec {
  int32_t verdict;      // V_TERM_*
  int32_t pred_index;
  uint32_t event;       // event index within the parent's enabled events
  uint32_t pad;
  uint64_t parent;      // index of the parent in the current frontier
  uint64_t key;         // fingerprint high word (deterministic tie-break)
};

constexpr int kBlock = 256;
constexpr uint32_t kTermCap = 1024;

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

template <class P>
__global__ void k_init(typename P::State* out, typename P::Params prm) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    typename P::State s;
    P::init(s, prm);
    *out = s;
  }
}

// Inserts the initial state's fingerprint and judges it (BFS.initSearch + exploreNode's
// initial-state check, Search.java:434-440, :470-480).
template <class P>
__global__ void k_seed(const typename P::State* init, typename P::Params prm, DevSettings set, Table table,
                       int depth, int32_t* out /* [verdict, pred_index, insert_rc] */) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    typename P::State s = *init;
    Fp f = fingerprint(s.w);
    out[2] = table_insert(table, f);
    int pi = -1;
    out[0] = judge<P>(s, prm, set, depth, &pi);
    out[1] = pi;
  }
}

template <class P>
__global__ void __launch_bounds__(kBlock) k_count(const typename P::State* __restrict__ cur, uint64_t F,
                                                  typename P::Params prm, DevSettings set,
                                                  unsigned long long* __restrict__ counts) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < F; i += stride) {
    typename P::State s = cur[i];
    counts[i] = (unsigned long long)P::num_events(s, prm, set);
  }
}

template <class P>
struct ExpandArgs {
  const typename P::State* cur;
  const unsigned long long* offsets;  // exclusive scan of per-state event counts
  uint64_t F;
  uint64_t total;
  typename P::State* next;
  uint64_t* next_parent;
  uint32_t* next_event;
  uint64_t next_cap;
  LevelCounters* ctr;
  TerminalRec* terms;
  Table table;
  int32_t depth;  // depth of the successors
};

template <class P>
__global__ void __launch_bounds__(kBlock) k_expand(ExpandArgs<P> a, typename P::Params prm, DevSettings set) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < a.total; base += stride) {
    const uint64_t t = base + threadIdx.x;
    const bool active = t < a.total;
    bool is_new = false, is_valid = false, is_succ = false;
    uint64_t parent = 0;
    uint32_t ev = 0;
    typename P::State succ;
    if (active) {
      // parent = last p with offsets[p] <= t
      uint64_t lo = 0, hi = a.F;
      while (hi - lo > 1) {
        uint64_t mid = (lo + hi) >> 1;
        if (a.offsets[mid] <= t) lo = mid; else hi = mid;
      }
      parent = lo;
      ev = (uint32_t)(t - a.offsets[lo]);
      const typename P::State s = a.cur[parent];
      const int rc = P::step(s, (int)ev, succ, prm, set);
      if (rc == STEP_OK) {
        is_succ = true;
        const Fp f = fingerprint(succ.w);
        const int ins = table_insert(a.table, f);
        if (ins == INS_NEW) {
          is_new = true;
          int pi = -1;
          const int v = judge<P>(succ, prm, set, a.depth, &pi);
          if (v == V_VALID) {
            is_valid = true;
          } else if (v >= V_TERM_EXCEPTION) {
            const unsigned long long slot = atomicAdd(&a.ctr->n_terminals, 1ull);
            if (slot < kTermCap) a.terms[slot] = TerminalRec{v, pi, ev, 0u, parent, f.hi};
          }
        } else if (ins == INS_FULL) {
          atomicAdd(&a.ctr->err_table, 1ull);
        }
      } else if (rc == STEP_EXCEPTION) {
        // Exceptional states never equal another (Throwable identity, SearchState.java:601):
        // always new, always terminal.
        is_succ = true;
        is_new = true;
        const Fp f = fingerprint(succ.w);
        const unsigned long long slot = atomicAdd(&a.ctr->n_terminals, 1ull);
        if (slot < kTermCap) a.terms[slot] = TerminalRec{V_TERM_EXCEPTION, -1, ev, 0u, parent, f.hi};
      } else if (rc == STEP_OVERFLOW) {
        atomicAdd(&a.ctr->err_overflow, 1ull);
      }
    }
    // Converged: wave-aggregated counters and frontier append.
    const unsigned long long nsucc = __popcll(__ballot(is_succ));
    const unsigned long long nnew = __popcll(__ballot(is_new));
    if (__lane_id() == 0) {
      if (nsucc) atomicAdd(&a.ctr->successors, nsucc);
      if (nnew) atomicAdd(&a.ctr->new_states, nnew);
    }
    const unsigned long long idx = wave_reserve(&a.ctr->next_size, is_valid);
    if (is_valid) {
      if (idx < a.next_cap) {
        a.next[idx] = succ;
        a.next_parent[idx] = parent;
        a.next_event[idx] = ev;
      } else {
        atomicAdd(&a.ctr->err_frontier, 1ull);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Host side.
// ------------------------------------------------------------------------------------------
struct EngineBase {
  virtual ~EngineBase() = default;
  virtual int set_settings(const dsl_settings& s) = 0;
  virtual int set_initial(const uint8_t* p, size_t len, int depth) = 0;
  virtual int get_initial(uint8_t* p, size_t len) = 0;
  virtual int run(dsl_result** out) = 0;
  virtual int state_bytes() const = 0;
  volatile unsigned long long progress_states = 0;
  volatile int progress_depth = 0;
  dsl_stats stats{};
};

int resolve_settings(const dsl_settings& in, int num_nodes, bool (*known)(int), DevSettings* out);

template <class P>
struct Engine : EngineBase {
  using State = typename P::State;
  typename P::Params prm;
  dsl_engine_config cfg;
  dsl_settings hset{};
  DevSettings dset{};
  State init{};
  int init_depth = 0;
  bool have_init = false;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, evc0 = nullptr, evc1 = nullptr;

  // device memory
  unsigned long long* d_table = nullptr;
  uint64_t table_buckets = 0;
  State* d_cur = nullptr;
  State* d_next = nullptr;
  uint64_t cur_cap = 0, next_cap = 0;
  unsigned long long* d_counts = nullptr;
  unsigned long long* d_offsets = nullptr;
  uint64_t counts_cap = 0, offsets_cap = 0;
  void* d_scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;
  uint64_t* d_hist_parent = nullptr;  // parent pointers of every frontier entry, all levels
  uint32_t* d_hist_event = nullptr;
  uint64_t hist_parent_cap = 0, hist_event_cap = 0;
  LevelCounters* d_ctr = nullptr;
  TerminalRec* d_terms = nullptr;
  int32_t* d_seed = nullptr;

  Engine(const typename P::Params& p, const dsl_engine_config& c) : prm(p), cfg(c) {
    dsl_settings s{};
    s.max_depth = -1;
    s.max_time_ms = -1;
    s.network_active = 1;
    s.deliver_timers = 1;
    std::memset(s.link_active, -1, sizeof(s.link_active));
    std::memset(s.sender_active, -1, sizeof(s.sender_active));
    std::memset(s.receiver_active, -1, sizeof(s.receiver_active));
    std::memset(s.timers_active, -1, sizeof(s.timers_active));
    hset = s;
    resolve_settings(hset, P::num_nodes(prm), &P::known_predicate, &dset);
  }

  ~Engine() override { release(); }

  void release() {
    hipFree(d_table);
    hipFree(d_cur);
    hipFree(d_next);
    hipFree(d_counts);
    hipFree(d_offsets);
    hipFree(d_scan_tmp);
    hipFree(d_hist_parent);
    hipFree(d_hist_event);
    hipFree(d_ctr);
    hipFree(d_terms);
    hipFree(d_seed);
    if (ev0) hipEventDestroy(ev0);
    if (ev1) hipEventDestroy(ev1);
    if (evc0) hipEventDestroy(evc0);
    if (evc1) hipEventDestroy(evc1);
    if (stream) hipStreamDestroy(stream);
    d_table = nullptr;
    d_cur = d_next = nullptr;
    d_counts = d_offsets = nullptr;
    d_scan_tmp = nullptr;
    d_hist_parent = nullptr;
    d_hist_event = nullptr;
    d_ctr = nullptr;
    d_terms = nullptr;
    d_seed = nullptr;
    stream = nullptr;
    ev0 = ev1 = evc0 = evc1 = nullptr;
  }

  int state_bytes() const override { return (int)sizeof(State); }

  int set_settings(const dsl_settings& s) override {
    int rc = resolve_settings(s, P::num_nodes(prm), &P::known_predicate, &dset);
    if (rc == DSL_OK) hset = s;
    return rc;
  }

  int set_initial(const uint8_t* p, size_t len, int depth) override {
    if (len != sizeof(State) || depth < 0) return DSL_ERR_ARG;
    std::memcpy(&init, p, len);
    init_depth = depth;
    have_init = true;
    return DSL_OK;
  }

  int get_initial(uint8_t* p, size_t len) override {
    if (len != sizeof(State)) return DSL_ERR_ARG;
    if (!have_init) {
      P::init(init, prm);  // host execution of the protocol's init handlers
      init_depth = 0;
      have_init = true;
    }
    std::memcpy(p, &init, len);
    return DSL_OK;
  }

  int ensure_stream() {
    if (!stream) {
      if (cfg.device >= 0) DSL_HIP(hipSetDevice(cfg.device));
      DSL_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
      DSL_HIP(hipEventCreate(&ev0));
      DSL_HIP(hipEventCreate(&ev1));
      DSL_HIP(hipEventCreate(&evc0));
      DSL_HIP(hipEventCreate(&evc1));
    }
    return DSL_OK;
  }

  template <class T>
  int grow(T** ptr, uint64_t* cap, uint64_t need, bool keep, uint64_t keep_elems) {
    if (need <= *cap) return DSL_OK;
    uint64_t ncap = std::max<uint64_t>(need, *cap + *cap / 2);
    ncap = std::max<uint64_t>(ncap, 1024);
    T* np = nullptr;
    DSL_HIP(hipMalloc(&np, ncap * sizeof(T)));
    if (keep && *ptr && keep_elems) DSL_HIP(hipMemcpyAsync(np, *ptr, keep_elems * sizeof(T), hipMemcpyDeviceToDevice, stream));
    DSL_HIP(hipStreamSynchronize(stream));
    hipFree(*ptr);
    *ptr = np;
    *cap = ncap;
    return DSL_OK;
  }

  int alloc_table() {
    int log2 = hset.table_log2_slots > 0 ? hset.table_log2_slots : 26;
    if (log2 < 10 || log2 > 40) return DSL_ERR_ARG;
    uint64_t buckets = (1ull << log2) / 8;
    if (buckets != table_buckets) {
      hipFree(d_table);
      d_table = nullptr;
      DSL_HIP(hipMalloc(&d_table, buckets * 64));
      table_buckets = buckets;
    }
    DSL_HIP(hipMemsetAsync(d_table, 0, table_buckets * 64, stream));
    return DSL_OK;
  }

  int run(dsl_result** out) override {
    int rc = ensure_stream();
    if (rc) return rc;
    auto t_start = std::chrono::steady_clock::now();
    stats = dsl_stats{};
    stats.state_bytes = sizeof(State);
    stats.world_size = 1;
    if (!have_init) {
      uint8_t tmp[sizeof(State)];
      get_initial(tmp, sizeof(State));
    }
    if ((rc = alloc_table())) return rc;
    if (!d_ctr) DSL_HIP(hipMalloc(&d_ctr, sizeof(LevelCounters)));
    if (!d_terms) DSL_HIP(hipMalloc(&d_terms, sizeof(TerminalRec) * kTermCap));
    if (!d_seed) DSL_HIP(hipMalloc(&d_seed, 4 * sizeof(int32_t)));
    if ((rc = grow(&d_cur, &cur_cap, 1024, false, 0))) return rc;
    if ((rc = grow(&d_next, &next_cap, 1024, false, 0))) return rc;
    if ((rc = grow(&d_hist_parent, &hist_parent_cap, 1024, false, 0))) return rc;
    if ((rc = grow(&d_hist_event, &hist_event_cap, 1024, false, 0))) return rc;
    Table table{d_table, table_buckets - 1, 64};
    stats.table_slots = table_buckets * 8;

    DSL_HIP(hipMemcpyAsync(d_cur, &init, sizeof(State), hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(k_seed<P>, dim3(1), dim3(64), 0, stream, d_cur, prm, dset, table, init_depth, d_seed);
    int32_t seed[4];
    DSL_HIP(hipMemcpyAsync(seed, d_seed, sizeof(seed), hipMemcpyDeviceToHost, stream));
    DSL_HIP(hipStreamSynchronize(stream));

    std::vector<uint64_t> per_depth{1};
    std::vector<uint64_t> level_base{0};  // history arena offset of each level's frontier
    std::vector<uint64_t> level_size{1};
    uint64_t total_states = 1, successors = 0;
    int end = DSL_SPACE_EXHAUSTED, pred_index = -1, term_depth = -1;
    TerminalRec best{};
    bool have_term = false;
    double level_ms_max = 0;
    progress_states = 1;
    progress_depth = init_depth;
    // the initial state has no parent
    uint64_t zero64 = ~0ull;
    uint32_t zero32 = ~0u;
    DSL_HIP(hipMemcpyAsync(d_hist_parent, &zero64, 8, hipMemcpyHostToDevice, stream));
    DSL_HIP(hipMemcpyAsync(d_hist_event, &zero32, 4, hipMemcpyHostToDevice, stream));

    if (seed[0] >= V_TERM_EXCEPTION) {
      end = seed[0] == V_TERM_INVARIANT ? DSL_INVARIANT_VIOLATED : DSL_GOAL_FOUND;
      pred_index = seed[1];
      term_depth = init_depth;
    } else {
      // A PRUNED initial state is still expanded (Search.java:475).
      uint64_t F = 1;
      int depth = init_depth;
      while (F > 0) {
        if (hset.max_time_ms > 0) {
          double el = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
          if (el > hset.max_time_ms) {
            end = DSL_TIME_EXHAUSTED;
            break;
          }
        }
        auto lt0 = std::chrono::steady_clock::now();
        // 1. count events
        if ((rc = grow(&d_counts, &counts_cap, F, false, 0))) return rc;
        if ((rc = grow(&d_offsets, &offsets_cap, F, false, 0))) return rc;
        const int cblocks = (int)std::min<uint64_t>((F + kBlock - 1) / kBlock, 8192);
        DSL_HIP(hipEventRecord(evc0, stream));
        hipLaunchKernelGGL(k_count<P>, dim3(cblocks), dim3(kBlock), 0, stream, d_cur, F, prm, dset, d_counts);
        // 2. exclusive scan
        size_t need = 0;
        DSL_HIP(scan_bytes(F, &need));
        if (need > scan_tmp_bytes) {
          hipFree(d_scan_tmp);
          d_scan_tmp = nullptr;
          DSL_HIP(hipMalloc(&d_scan_tmp, need));
          scan_tmp_bytes = need;
        }
        DSL_HIP(scan(F));
        DSL_HIP(hipEventRecord(evc1, stream));
        unsigned long long last[2];
        DSL_HIP(hipMemcpyAsync(&last[0], d_offsets + F - 1, 8, hipMemcpyDeviceToHost, stream));
        DSL_HIP(hipMemcpyAsync(&last[1], d_counts + F - 1, 8, hipMemcpyDeviceToHost, stream));
        DSL_HIP(hipMemsetAsync(d_ctr, 0, sizeof(LevelCounters), stream));
        DSL_HIP(hipStreamSynchronize(stream));
        const uint64_t total = last[0] + last[1];
        if (total == 0) break;
        // 3. capacity of the next frontier: at most one new state per work item
        uint64_t cap_limit = hset.max_frontier_states ? hset.max_frontier_states : (1ull << 40);
        uint64_t want = std::min<uint64_t>(total, cap_limit);
        if ((rc = grow(&d_next, &next_cap, want, false, 0))) return rc;
        if ((rc = grow(&d_cur, &cur_cap, want, true, F))) return rc;
        const uint64_t hbase = level_base.back() + level_size.back();
        if ((rc = grow(&d_hist_parent, &hist_parent_cap, hbase + want, true, hbase))) return rc;
        if ((rc = grow(&d_hist_event, &hist_event_cap, hbase + want, true, hbase))) return rc;
        // 4. expand
        ExpandArgs<P> a;
        a.cur = d_cur;
        a.offsets = d_offsets;
        a.F = F;
        a.total = total;
        a.next = d_next;
        a.next_parent = d_hist_parent + hbase;
        a.next_event = d_hist_event + hbase;
        a.next_cap = want;
        a.ctr = d_ctr;
        a.terms = d_terms;
        a.table = table;
        a.depth = depth + 1;
        const int eblocks = (int)std::min<uint64_t>((total + kBlock - 1) / kBlock, 256ull * 32);
        DSL_HIP(hipEventRecord(ev0, stream));
        hipLaunchKernelGGL(k_expand<P>, dim3(eblocks), dim3(kBlock), 0, stream, a, prm, dset);
        DSL_HIP(hipGetLastError());
        DSL_HIP(hipEventRecord(ev1, stream));
        LevelCounters ctr;
        DSL_HIP(hipMemcpyAsync(&ctr, d_ctr, sizeof(ctr), hipMemcpyDeviceToHost, stream));
        DSL_HIP(hipStreamSynchronize(stream));
        float kms = 0, cms = 0;
        hipEventElapsedTime(&kms, ev0, ev1);
        hipEventElapsedTime(&cms, evc0, evc1);
        stats.expand_ms += kms;
        stats.scan_ms += cms;
        stats.expand_launches++;
        stats.parents += F;
        stats.work_items += total;
        stats.new_states += ctr.new_states;
        stats.appended += ctr.next_size;
        if (ctr.err_overflow) {
          set_error("a successor exceeded the packed state's bounds (" + std::to_string(ctr.err_overflow) + " times)");
          return DSL_ERR_STATE_OVERFLOW;
        }
        if (ctr.err_table) {
          set_error("visited table full: raise table_log2_slots");
          return DSL_ERR_TABLE_FULL;
        }
        if (ctr.err_frontier || ctr.next_size > want) {
          set_error("next frontier exceeds capacity: raise max_frontier_states");
          return DSL_ERR_FRONTIER_FULL;
        }
        depth++;
        successors += ctr.successors;
        total_states += ctr.new_states;
        if (ctr.new_states) per_depth.push_back(ctr.new_states);
        progress_states = total_states;
        progress_depth = depth;
        level_base.push_back(hbase);
        level_size.push_back(ctr.next_size);
        double lms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - lt0).count();
        level_ms_max = std::max(level_ms_max, lms);
        if (ctr.n_terminals) {
          uint32_t nt = (uint32_t)std::min<unsigned long long>(ctr.n_terminals, kTermCap);
          std::vector<TerminalRec> terms(nt);
          DSL_HIP(hipMemcpy(terms.data(), d_terms, nt * sizeof(TerminalRec), hipMemcpyDeviceToHost));
          best = terms[0];
          for (auto& t : terms)
            if (t.verdict < best.verdict || (t.verdict == best.verdict && t.key < best.key)) best = t;
          // lower V_TERM_* value = higher priority (EXCEPTION < INVARIANT < GOAL)
          have_term = true;
          end = best.verdict == V_TERM_EXCEPTION ? DSL_EXCEPTION_THROWN
                : best.verdict == V_TERM_INVARIANT ? DSL_INVARIANT_VIOLATED
                                                   : DSL_GOAL_FOUND;
          pred_index = best.verdict == V_TERM_EXCEPTION ? -1 : best.pred_index;
          term_depth = depth;
          break;
        }
        std::swap(d_cur, d_next);
        F = ctr.next_size;
      }
    }
    double elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();

    // Result + trace reconstruction (parent pointers walked back level by level, then the
    // events replayed on the host from the initial state with the same transition code).
    dsl_result* r = (dsl_result*)calloc(1, sizeof(dsl_result));
    r->end_condition = end;
    r->terminal_depth = term_depth;
    r->predicate_index = pred_index;
    r->states = total_states;
    r->initial_depth = init_depth;
    r->max_depth = init_depth + (int)per_depth.size() - 1;
    r->n_levels = (int)per_depth.size();
    r->per_depth = (uint64_t*)malloc(sizeof(uint64_t) * per_depth.size());
    std::memcpy(r->per_depth, per_depth.data(), sizeof(uint64_t) * per_depth.size());
    r->elapsed_s = elapsed;
    r->successors = successors;
    r->new_states_inserted = total_states;
    r->level_ms_max = level_ms_max;
    r->state_bytes = sizeof(State);
    if (term_depth >= 0) {
      std::vector<uint32_t> evs;
      if (have_term) {
        evs.push_back(best.event);
        uint64_t idx = best.parent;  // index in frontier of level L-1
        for (int L = (int)level_base.size() - 2; L >= 1; L--) {
          uint64_t p;
          uint32_t e;
          DSL_HIP(hipMemcpy(&p, d_hist_parent + level_base[L] + idx, 8, hipMemcpyDeviceToHost));
          DSL_HIP(hipMemcpy(&e, d_hist_event + level_base[L] + idx, 4, hipMemcpyDeviceToHost));
          evs.push_back(e);
          idx = p;
        }
        std::reverse(evs.begin(), evs.end());
      }
      r->trace_len = (int)evs.size();
      r->trace = (dsl_event*)calloc(evs.size() + 1, sizeof(dsl_event));
      State s = init, n;
      for (size_t i = 0; i < evs.size(); i++) {
        P::describe(s, prm, dset, (int)evs[i], &r->trace[i]);
        P::step(s, (int)evs[i], n, prm, dset);
        s = n;
      }
      r->terminal_state = (uint8_t*)malloc(sizeof(State));
      std::memcpy(r->terminal_state, &s, sizeof(State));
    }
    *out = r;
    return DSL_OK;
  }

  hipError_t scan_bytes(uint64_t n, size_t* bytes);
  hipError_t scan(uint64_t n);
};

}  // namespace dsl
