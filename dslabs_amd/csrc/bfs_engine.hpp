// bfs_engine.hpp -- host side of the level-synchronous BFS (Search.run + BFS, Search.java:233-505).
//
// W hash shards (owner = owner_of(fingerprint, W)); each holds its visited-table partition and
// a frontier. Deployments:
//   * W = 1: one GPU, one k_level launch per BFS level (or a device-side queue of them);
//   * one process (or thread) per GPU, W = world size, one local shard, exchanges through a Comm
//     (RCCL: grouped ncclSend/ncclRecv = all-to-all over the xGMI links, allgather, broadcast);
//   * virtual shards: W shards on ONE device, exchanges are device-to-device copies (tests).
// A sharded level (sharded_fast): k_level<ROUTE> routes every successor's 16-byte fingerprint to
// its owner's region -> round A: fixed-size slabs to the owners -> k_probe_slab (all sources
// interleaved, one answer byte per record) -> round B: the answers back -> k_materialize at the
// source (judge, append to the source's own next frontier) -> the level records gathered: ONE
// host round trip. Only the visited set is partitioned: a new state stays where it was generated
// (no state row crosses the links); the fair race for "new" keeps the frontiers balanced.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "kernels.hpp"
#include "replay.hpp"

namespace dsl {

void set_error(const std::string& msg);
int resolve_settings(const dsl_settings& in, int num_nodes, bool (*known)(int), DevSettings* out);

#define DSL_HIP(call)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (call);                                                                     \
    if (e_ != hipSuccess) {                                                                     \
      set_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + __FILE__ + ":" +  \
                std::to_string(__LINE__) + " (" #call ")");                                     \
      return DSL_ERR_HIP;                                                                       \
    }                                                                                           \
  } while (0)

#define DSL_TRY(x)     \
  do {                 \
    int r_ = (x);      \
    if (r_) return r_; \
  } while (0)

// Collectives across ranks (one local shard per rank). RCCL / caller transports in engine.hip.
struct Comm {
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual int allgather_u64(const uint64_t* in, int n, uint64_t* out, hipStream_t st) = 0;
  virtual int allreduce_u64(uint64_t* v, int n, bool min, hipStream_t st) = 0;
  virtual int bcast_u64(uint64_t* v, int n, int root, hipStream_t st) = 0;
  virtual int alltoallv(const uint8_t* send, const uint64_t* send_off, const uint64_t* send_bytes, uint8_t* recv,
                        const uint64_t* recv_off, const uint64_t* recv_bytes, hipStream_t st) = 0;
  // Device-side allgather enqueued on `st` (no host synchronization): n words of d_in from every
  // rank into d_out (rank-major). Only transports with device collectives (RCCL) provide it.
  virtual bool device_collectives() const { return false; }
  virtual int allgather_dev(const uint64_t*, int, uint64_t*, hipStream_t) { return DSL_ERR_COMM; }
  virtual int version() const { return 0; }
  // RCCL: the communicator's asynchronous error (ncclCommGetAsyncError: a peer that died, a
  // network failure), polled while the host waits on the stream; abort() ends every outstanding
  // operation of the communicator (ncclCommAbort), so a failed rank ends the search on every rank
  // with DSL_ERR_COMM instead of leaving the others blocked in a collective.
  virtual int async_error() { return DSL_OK; }
  // true once the stream has reached the last collective it enqueued since the last synced():
  // a wait then waits on the collective, and only then does the deadline run (a long local kernel
  // before it is not a stalled peer); false for a transport without stream collectives
  virtual bool collective_reached() { return false; }
  virtual void synced() {}
  virtual void abort() {}
};

struct EngineBase {
  virtual ~EngineBase() = default;
  virtual int set_settings(const dsl_settings& s) = 0;
  virtual int set_initial(const uint8_t* p, size_t len, int depth) = 0;
  virtual int get_initial(uint8_t* p, size_t len) = 0;
  virtual int set_dropped(const uint64_t* recs, int n) = 0;
  virtual int run(dsl_result** out) = 0;
  virtual int run_dfs(const dsl_dfs_config& c, dsl_result** out) = 0;
  virtual int replay(const dsl_event* trace, int n, int minimize, dsl_result** out) = 0;
  virtual int human_readable(const dsl_event* trace, int n, dsl_result** out) = 0;
  virtual int state_bytes() const = 0;
  volatile unsigned long long progress_states = 0;
  volatile int progress_depth = 0;
  dsl_stats stats{};
};

template <class P>
struct BfsEngine : EngineBase {
  static constexpr int NW = Layout<P>::kWords;

  struct Shard {
    int gid = 0;
    unsigned long long* table = nullptr;
    bool table_clean = false;  // zeroed after the last search ended (k_setup then skips the clear)
    uint32_t* cur = nullptr;
    uint32_t* next = nullptr;
    Fp* cur_fp = nullptr;
    Fp* next_fp = nullptr;
    uint64_t cur_cap = 0, next_cap = 0, curfp_cap = 0, nextfp_cap = 0;
    // history: per BFS level of the search (index = depth - initial depth), parent pointer and
    // event of every row of that level's frontier; one buffer pair per level, kept across
    // searches, so a repeated search neither reallocates nor copies history
    std::vector<uint64_t*> hpar;
    std::vector<uint32_t*> hev;
    std::vector<uint64_t> hcap;
    bool flip = false;  // cur/next swapped an odd number of times since the search started
    LevelCounters* ctr = nullptr;
    TerminalRec* terms = nullptr;
    unsigned char* find_ctr = nullptr;  // scratch counter sets of a find-mode k_level
    RouteCounters* rc = nullptr;
    Fp* out_key = nullptr;       // routed successors: W regions of cap_fp fingerprints (header first)
    uint64_t out_fp_cap = 0;
    uint64_t* out_item = nullptr;  // ... and their (parent << 20 | event) items (stay at the source)
    uint64_t out_item_cap = 0;
    Fp* in_fp = nullptr;
    uint64_t in_fp_cap = 0;
    uint32_t* out_pk = nullptr;  // the regions packed for the links (12 B per record), out and in
    uint32_t* in_pk = nullptr;
    uint64_t out_pk_cap = 0, in_pk_cap = 0, cap_pk = 0;
    uint8_t* rep_out = nullptr;  // answers to the received fingerprints (owner side)
    uint64_t rep_out_cap = 0;
    uint8_t* rep_in = nullptr;   // answers to this shard's fingerprints, W regions of cap_fp (source side)
    uint64_t rep_in_cap = 0;
    uint64_t* spill = nullptr;
    uint64_t spill_cap = 0;
    uint64_t F = 0;
    uint64_t work = 0;        // enabled events of the current frontier (exact)
    std::vector<uint64_t> seg_base, seg_cnt;  // row ranges of the current frontier
    unsigned long long* seg_ctr = nullptr;    // kSegs reservation counters (inside the current set)
    // Two counter sets (LevelCounters + segment counters, kCtrSet bytes each): a level uses set
    // cset, and its k_level zeroes the other set for the next level, so no per-level memset;
    // the host reads the whole set with ONE copy into pinned memory.
    unsigned char* ctrbuf = nullptr;
    unsigned char* hctr = nullptr;
    int cset = 0;
    uint64_t segcap = 0;
    int nseg = 1;
    std::vector<uint64_t> level_size;  // rows of each level's frontier (history entries)
    uint64_t cap_fp = 0;
    uint64_t* rspill = nullptr;  // route-spilled successors (k_level ROUTE past a region)
    uint64_t rspill_cap = 0;
    Fp* out2 = nullptr;          // completion phase: re-routed route spills, W regions
    uint64_t out2_cap = 0;
    uint64_t* out2_item = nullptr;
    uint64_t out2_item_cap = 0;
    uint8_t* rep2 = nullptr;     // ... and the owners' answers to them
    uint64_t rep2_cap = 0;
    uint64_t rs_cap = 0;         // records per out2 / rep2 region
    uint64_t route_cs = 0;       // records per sub-slab of this level's regions
    uint64_t* newl = nullptr;    // slots of the routed records found new (k_new_list)
    uint64_t newl_cap = 0;
    void* nl_ctr = nullptr;      // [0]: newl's count, [2, 2 + kMaxShards): k_respill's counts
    // a sharded level's next-frontier layout (rows): [0, seg_span) the segments, [seg_span,
    // + uns_room) rows k_unspill appends (fast path), [seg_span + uns_room, + mat_room) rows
    // k_materialize appends, [ovf_base, + ovf_cnt) spills past uns_room (completion phase)
    uint64_t seg_span = 0, uns_room = 0, mat_room = 0, ovf_base = 0, ovf_cnt = 0;
    LevelCounters lc{};
  };

  typename P::Params prm;
  dsl_engine_config cfg;
  dsl_settings hset{};
  DevSettings dset{};
  typename P::State init{};
  int init_depth = 0;
  bool have_init = false;
  int W = 1;
  std::vector<Shard> sh;
  std::unique_ptr<Comm> comm;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  uint64_t table_buckets = 0;  // buckets of each shard's visited table (it only grows)
  Table tbl{};                 // the table's geometry and key layout (slots: per shard)
  uint64_t inserted = 0;       // states inserted in each shard's table so far (an upper bound)
  unsigned long long* rehash_err = nullptr;
  // multi-rank exchange scratch: the route-count matrix and the level records (kernels.hpp
  // k_level_record), on the device and pinned on the host
  // [0, kMaxShards * kRecWords): the local shards' records; then the gathered records (RCCL);
  // then the completion phase's route-spill counts (kMaxShards x kMaxShards)
  static constexpr int kXRecEnd = 2 * kMaxShards * kRecWords + kMaxShards * kMaxShards;
  static constexpr int kXWords = kXRecEnd + kMaxShards * kCtrMirrorWords;  // + the counters' mirrors
  uint64_t* xdev = nullptr;
  // the device-side deadline of a time-limited search (LevelArgs::budget_rt): the device clock at
  // the search's start (k_clock) and the budget in its ticks; not used in a replicated level of a
  // multi-shard search (every shard must finish it, so the replicas stay identical: the host check,
  // agreed by a collective, ends those)
  uint64_t* t0_rt = nullptr;
  uint64_t budget_rt = 0;
  uint64_t level_budget(bool rep) const { return W > 1 && rep ? 0 : budget_rt; }
  uint64_t* xhost = nullptr;
  uint64_t* segs_dev = nullptr;   // virtual shards: the segment tables of the two exchange rounds
  uint64_t* segs_host = nullptr;
  uint64_t seg_round = 0, seg_since_sync = 0;
  static constexpr int kSegTables = 8;
  // One host round trip (counted in dsl_stats.host_syncs). The host polls the stream instead of
  // blocking in hipStreamSynchronize: a search is ~1 ms of device work with one or two waits, and a
  // blocked thread's wake-up latency (tens of microseconds, varying by host) is paid per search.
  // DSL_BLOCKING_SYNC=1 restores the blocking wait.
  bool spin_sync = !getenv("DSL_BLOCKING_SYNC");
  // With a communicator the wait also polls its asynchronous error and a deadline
  // (DSL_COMM_TIMEOUT_MS, default 300 s, counted once the stream reached its last collective):
  // either aborts the communicator and fails the search.
  const double comm_timeout_ms = getenv("DSL_COMM_TIMEOUT_MS") ? atof(getenv("DSL_COMM_TIMEOUT_MS")) : 300000.0;
  bool comm_failed = false;
  int comm_fail(const std::string& why) {
    comm_failed = true;
    if (comm) comm->abort();
    set_error("multi-GPU exchange failed on rank " + std::to_string(comm ? comm->rank() : 0) + ": " + why +
              " (communicator aborted)");
    return DSL_ERR_COMM;
  }
  int hsync() {
    if (comm) {
      // the deadline counts from the moment the stream reached its last collective (local work
      // before it may take as long as it takes)
      auto t0 = std::chrono::steady_clock::now();
      hipError_t e;
      for (uint64_t it = 0; (e = hipStreamQuery(stream)) == hipErrorNotReady; it++) {
        if ((it & 1023) == 1023) {
          if (comm->async_error() != DSL_OK) return comm_fail("asynchronous communicator error");
          const auto now = std::chrono::steady_clock::now();
          if (!comm->collective_reached()) t0 = now;
          else if (std::chrono::duration<double, std::milli>(now - t0).count() > comm_timeout_ms)
            return comm_fail("no progress within DSL_COMM_TIMEOUT_MS");
        }
      }
      if (e != hipSuccess) DSL_HIP(e);
      comm->synced();
    } else if (spin_sync) {
      seg_since_sync = 0;
      hipError_t e;
      while ((e = hipStreamQuery(stream)) == hipErrorNotReady) {
      }
      if (e != hipSuccess) DSL_HIP(e);
    } else {
      seg_since_sync = 0;
      DSL_HIP(hipStreamSynchronize(stream));
    }
    stats.host_syncs++;
    return DSL_OK;
  }
  uint64_t avg_events_x16 = 16 * 8;  // running estimate of events per state (x16)
  uint32_t term_cap = kTermCap;      // TerminalRec entries per shard (DSL_TERM_CAP)
  uint32_t terms_alloc = 0;
  std::vector<uint32_t> trace_events;

  // ---- queued small levels (single local shard) ------------------------------------------------
  // While the frontier is small, a level's kernel is short and the host round trip between levels
  // (counter copy, sync, next launch) is a large part of its time. Up to kQueue levels are then
  // enqueued back to back; each derives its row ranges from the previous level's counters on the
  // device and stops (with every later one) where the host must act (queue_continues). The host
  // then walks the queued levels' counters with the ordinary per-level bookkeeping.
  // A queue's capacity is `span` next-frontier rows per level (32 segments), sized from the
  // frontier it starts at: 32x its size, at least kQueueRowsMin, at most 1 GiB of rows. It runs
  // while the frontier stays within span/4 states (a level grows it ~3x) and the next level's
  // work items fit the spill list (8 span); past a segment's rows a level spills and stops it.
  static constexpr int kQueue = 12;
  static constexpr uint64_t kQueueRowsMin = 1u << 16;
  uint64_t queue_span_max() const {
    uint64_t s = 1ull << 24;
    while (s > kQueueRowsMin && s * NW * 4 > (1ull << 30)) s >>= 1;
    return s;
  }
  uint64_t queue_span(uint64_t F) const {
    if (q_rows_forced) return q_rows_forced;  // tests: small queues that spill and stop early
    uint64_t s = kQueueRowsMin;
    while ((s < 32 * F || s < q_span_hint || s < q_span_want) && s < queue_span_max()) s <<= 1;
    return s;
  }
  // The span a repeated search of this engine wants: 4x the largest frontier the last search
  // produced, so that one queue covers every level that fits (no host round trip between them);
  // DSL_QSPAN_FIXED keeps the span at 32x the frontier the queue starts from.
  uint64_t q_span_want = 0;
  const bool q_span_adapt = getenv("DSL_QSPAN_FIXED") == nullptr;
  uint64_t q_rows_forced = 0;  // DSL_QUEUE_ROWS (a multiple of 32)
  uint64_t q_span_hint = 0;  // the largest span an earlier queue of this engine used (buffers exist)
  uint64_t queue_flimit(uint64_t span) const {
    return W > 1 && !auto_rep() ? std::min<uint64_t>(span / 4, rep_threshold() - 1) : span / 4;
  }
  double q_ms_per_level = 0;       // the last queue's device time per level
  unsigned char* qctr = nullptr;   // kQueue + 1 counter sets
  bool qctr_clean = false;         // zeroed after the last search ended
  unsigned char* hq = nullptr;     // pinned copy of the kQueue sets
  std::vector<hipEvent_t> qev;     // brackets the whole queue (no event packets between its levels)
  // HIP events bracket the queue: its device time is expand_ms, which bench.py's roofline divides
  // by the launches. DSL_NO_QUEUE_EVENTS times the queue on the host instead (launch to drained
  // stream, ~0.6 % faster per search: profiles/r03_queue_fetch_events.txt)
  const bool q_events = getenv("DSL_NO_QUEUE_EVENTS") == nullptr;
  const bool q_memcpy = getenv("DSL_CTR_KERNEL") == nullptr;  // counters by hipMemcpyAsync (k_fetch_counters measured slower)
  double q_ms_total = 0;           // the last queue's time (expand_ms)
  int q_left = 0, q_pos = 0;
  uint64_t n_reallocs = 0;  // device buffer reallocations (DSL_LEVEL_TRACE)
  uint64_t q_segcap = 0;

  BfsEngine(const typename P::Params& p, const dsl_engine_config& c, int world, Comm* cm)
      : prm(p), cfg(c), W(world), comm(cm) {
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
    set_pred_reads<P>(dset, prm);
    const int nlocal = comm ? 1 : W;
    sh.resize(nlocal);
    for (int i = 0; i < nlocal; i++) sh[i].gid = comm ? comm->rank() : i;
  }

  ~BfsEngine() override {
    for (auto& s : sh) {
      void* ptrs[] = {s.table,     s.cur,      s.next,   s.cur_fp, s.next_fp, s.terms,  s.rc,
                      s.out_key,   s.in_fp,    s.rep_out, s.rep_in, s.spill, s.ctrbuf,
                      s.find_ctr,  s.rspill,   s.out2,    s.rep2,   s.out_item, s.out2_item, s.newl, s.nl_ctr,
                      s.out_pk,    s.in_pk};
      for (void* q : ptrs) (void)hipFree(q);
      for (auto* q : s.hpar) (void)hipFree(q);
      for (auto* q : s.hev) (void)hipFree(q);
      if (s.hctr) (void)hipHostFree(s.hctr);
    }
    (void)hipFree(qctr);
    (void)hipFree(dropped_d);
    (void)hipFree(xdev);
    (void)hipFree(segs_dev);
    if (segs_host) (void)hipHostFree(segs_host);
    (void)hipFree(rehash_err);
    (void)hipFree(t0_rt);
    if (xhost) (void)hipHostFree(xhost);
    if (hq) (void)hipHostFree(hq);
    for (auto e : qev) (void)hipEventDestroy(e);
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    comm.reset();
    if (stream) (void)hipStreamDestroy(stream);
    (void)hipGetLastError();
  }

  int state_bytes() const override { return (int)sizeof(typename P::State); }
  int set_settings(const dsl_settings& s) override {
    int rc = resolve_settings(s, P::num_nodes(prm), &P::known_predicate, &dset);
    if (rc == DSL_OK) {
      hset = s;
      set_pred_reads<P>(dset, prm);
    }
    apply_dropped();
    return rc;
  }
  // The caller's dropped network (dsl_set_dropped): kept in host memory and, for the kernels'
  // network predicates, in a device buffer; DevSettings points at both.
  std::vector<typename P::Rec> dropped_h;
  typename P::Rec* dropped_d = nullptr;
  uint64_t dropped_cap = 0;
  void apply_dropped() {
    dset.dropped_host = dropped_h.empty() ? nullptr : dropped_h.data();
    dset.dropped_dev = dropped_h.empty() ? nullptr : dropped_d;
    dset.n_dropped = (int32_t)dropped_h.size();
  }
  int set_dropped(const uint64_t* recs, int n) override {
    if (n < 0 || (n > 0 && !recs)) return DSL_ERR_ARG;
    dropped_h.assign(n, typename P::Rec{});
    for (int i = 0; i < n; i++) dropped_h[i] = (typename P::Rec)recs[i];
    if (n > 0 && NetPreds<P>::value) {
      if (cfg.device >= 0) DSL_HIP(hipSetDevice(cfg.device));
      DSL_TRY(grow(&dropped_d, &dropped_cap, (uint64_t)n, false, 0));
      DSL_HIP(hipMemcpy(dropped_d, dropped_h.data(), n * sizeof(typename P::Rec), hipMemcpyHostToDevice));
    }
    apply_dropped();
    return DSL_OK;
  }
  int set_initial(const uint8_t* p, size_t len, int depth) override {
    if (len != sizeof(init) || depth < 0) return DSL_ERR_ARG;
    std::memcpy(&init, p, len);
    init_depth = depth;
    have_init = true;
    return DSL_OK;
  }
  int get_initial(uint8_t* p, size_t len) override {
    if (len != sizeof(init)) return DSL_ERR_ARG;
    if (!have_init) {
      if (!init_state<P>(init.w, prm)) {
        set_error("initial state exceeds the packed state's bounds");
        return DSL_ERR_STATE_OVERFLOW;
      }
      init_depth = 0;
      have_init = true;
    }
    std::memcpy(p, &init, len);
    return DSL_OK;
  }

  template <class T>
  int grow(T** ptr, uint64_t* cap, uint64_t need, bool keep, uint64_t keep_elems) {
    if (need <= *cap && *ptr) return DSL_OK;
    const uint64_t ncap = std::max<uint64_t>(std::max<uint64_t>(need, *cap + *cap / 2), 1024);
    T* np = nullptr;
    n_reallocs++;
    if (getenv("DSL_LEVEL_TRACE"))
      fprintf(stderr, "[grow] %zu-byte elements: %llu -> %llu (keep %llu)\n", sizeof(T), (unsigned long long)*cap,
              (unsigned long long)ncap, (unsigned long long)(keep ? keep_elems : 0));
    DSL_HIP(hipMalloc(&np, ncap * sizeof(T)));
    if (keep && *ptr && keep_elems)
      DSL_HIP(hipMemcpyAsync(np, *ptr, keep_elems * sizeof(T), hipMemcpyDeviceToDevice, stream));
    DSL_TRY(hsync());
    (void)hipFree(*ptr);
    *ptr = np;
    *cap = ncap;
    return DSL_OK;
  }
  int grow_rows(uint32_t** ptr, uint64_t* cap, uint64_t rows, bool keep, uint64_t keep_rows) {
    uint64_t cw = *cap * NW;
    DSL_TRY(grow(ptr, &cw, rows * NW, keep, keep_rows * NW));
    *cap = cw / NW;
    return DSL_OK;
  }

  // History of level `lev` with room for `rows` entries, the first `keep` preserved.
  int hist_grow(Shard& S, size_t lev, uint64_t rows, uint64_t keep) {
    if (S.hpar.size() <= lev) {
      S.hpar.resize(lev + 1, nullptr);
      S.hev.resize(lev + 1, nullptr);
      S.hcap.resize(lev + 1, 0);
    }
    uint64_t c = S.hcap[lev];
    DSL_TRY(grow(&S.hpar[lev], &c, rows, keep > 0, keep));
    c = S.hcap[lev];
    DSL_TRY(grow(&S.hev[lev], &c, rows, keep > 0, keep));
    S.hcap[lev] = c;
    return DSL_OK;
  }

  int global_sum(std::vector<uint64_t>& v) {
    if (!comm) return DSL_OK;
    stats.host_syncs++;
    return comm->allreduce_u64(v.data(), (int)v.size(), false, stream);
  }

  // One all-to-all round: local shard l sends sb[l][d] bytes at send[l] + so[l][d] to shard d and
  // receives rb[l][s] bytes from shard s at recv[l] + ro[l][s] (RCCL grouped send/recv across
  // ranks; device-to-device copies between the virtual shards of one device).
  using Mat = std::vector<std::vector<uint64_t>>;
  int xfer(const std::vector<const uint8_t*>& send, const Mat& so, const Mat& sb, const std::vector<uint8_t*>& recv,
           const Mat& ro, const Mat& rb) {
    if (comm) return comm->alltoallv(send[0], so[0].data(), sb[0].data(), recv[0], ro[0].data(), rb[0].data(), stream);
    // virtual shards: the round's segments as one table, copied by one launch (k_copy_segments)
    const int L = (int)sh.size();
    if (!segs_dev) {
      DSL_HIP(hipMalloc(&segs_dev, kSegTables * 3 * kMaxShards * kMaxShards * 8));
      DSL_HIP(hipHostMalloc(&segs_host, kSegTables * 3 * kMaxShards * kMaxShards * 8));
    }
    // rounds take the pinned tables in turn; the host rewrites a table only after a host round
    // trip has drained the copy that read it
    if (seg_since_sync >= kSegTables) DSL_TRY(hsync());
    uint64_t* h = segs_host + (seg_round % kSegTables) * 3 * kMaxShards * kMaxShards;
    uint64_t* dv = segs_dev + (seg_round % kSegTables) * 3 * kMaxShards * kMaxShards;
    seg_round++;
    seg_since_sync++;
    int n = 0;
    uint64_t maxlen = 0;
    for (int s = 0; s < L; s++)
      for (int d = 0; d < L; d++)
        if (sb[s][d]) {
          h[3 * n] = (uint64_t)(uintptr_t)(send[s] + so[s][d]);
          h[3 * n + 1] = (uint64_t)(uintptr_t)(recv[d] + ro[d][s]);
          h[3 * n + 2] = sb[s][d];
          maxlen = std::max<uint64_t>(maxlen, sb[s][d]);
          n++;
        }
    if (!n) return DSL_OK;
    DSL_HIP(hipMemcpyAsync(dv, h, (size_t)n * 24, hipMemcpyHostToDevice, stream));
    const int gx = (int)std::min<uint64_t>(64, std::max<uint64_t>(1, (maxlen / 8 + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(k_copy_segments, dim3(gx, std::min(n, 64)), dim3(kBlock), 0, stream, (const uint64_t*)dv, n);
    DSL_HIP(hipGetLastError());
    return DSL_OK;
  }

  // Replicated or hash-sharded (multi-shard searches, see run()). dsl_engine_config.replicate_below
  // n > 0: a level whose frontier holds fewer than n states runs replicated; 0: every level is
  // sharded; -1 (automatic): a level is sharded once sharding it pays, by the cost model
  //     replicated  T(work)          sharded  T(work / W) + X,   T(w) = max(Tf, c w)
  // i.e. from work = shard_work_min on, with c = k_level ns per work item (the whole GPU), Tf the
  // latency floor of a small level and X =
  // the non-kernel time of a sharded level (exchange rounds, owner probes, materialization, the two
  // host round trips). Both are measured (c: the smallest per-item time of a level of >= 64K items,
  // X: the mean of the sharded levels), kept across searches and agreed by every rank at the start
  // of a search (the maximum, in the collective that judges the initial state), so every rank
  // takes the same decision; before any measurement c = 0.05 ns, X = 100 us. The switch happens
  // once per search: a sharded level's tables no longer hold every state.
  static constexpr double kLevelFloorUs = 20.0;  // a small level's k_level time (profiles/r03_level_times*)
  bool auto_rep() const { return cfg.replicate_below < 0; }
  uint64_t rep_threshold() const { return auto_rep() ? ~0ull : (uint64_t)cfg.replicate_below; }
  double cost_c_ns = 0, cost_x_us = 0;  // this rank's measurements (0: none yet)
  uint64_t shard_work_min = ~0ull;      // agreed for the current search (auto mode)
  bool level_replicated(uint64_t F, uint64_t work) const {
    return auto_rep() ? work <= shard_work_min : F < rep_threshold();
  }
  uint64_t queue_wlimit(uint64_t span) const {
    return W > 1 && auto_rep() ? std::min<uint64_t>(8 * span, shard_work_min) : 8 * span;
  }
  // Parents per chunk at most: about three passes of 256 lanes at the observed branching, within
  // the LDS budget of the staged rows.
  // LDS per staged parent: its row, fingerprint, node hashes (kernels.hpp k_level step 2) and offset
  // (+16 per chunk: LdsRow::image rounds the padded row image up to 16 bytes)
  static constexpr size_t kRowLds = (size_t)LdsRow<P>::kStride * 4 + sizeof(Fp) * (1 + (DSL_NH_LDS ? P::kNodes : 0)) + 4;
  int pb_max() const {
#ifndef DSL_PB_PASSES
#define DSL_PB_PASSES 3
#endif
    const int lds_max = (int)((DSL_ROWS_LDS_BYTES) / kRowLds);
    const int want = (int)((DSL_PB_PASSES * kLevelBlock * 16 + avg_events_x16 - 1) / std::max<uint64_t>(avg_events_x16, 1));
    return std::max(1, std::min({want, lds_max, kLevelBlock}));
  }
  // k_level workgroups resident at once on the device with `lds` bytes of dynamic LDS: the
  // occupancy of the protocol's instantiation (registers, LDS) x the CUs -- 1,024 for C5's
  // Multi-Paxos (128 VGPRs: 4 per CU), more for a protocol with small rows and few registers (the
  // synthetic C3: 48 VGPRs). The grids and the chunk rounds are sized for it. DSL_SLOTS_RT forces it.
  std::vector<std::pair<uint64_t, int>> slot_cache;
  int level_slots(size_t lds, bool route = false) {
    if (const char* e = getenv("DSL_SLOTS_RT")) return stats.level_slots = std::max(64, atoi(e));
    const uint64_t key = lds * 2 + (route ? 1 : 0);
    for (auto& kv : slot_cache)
      if (kv.first == key) {
        stats.level_slots = std::max(stats.level_slots, kv.second);
        return kv.second;
      }
    int occ = 0, cus = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    const hipError_t e = route ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_level<P, true>, kLevelBlock, lds)
                               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_level<P, false>, kLevelBlock, lds);
    if (e != hipSuccess || occ <= 0) occ = 4;
    (void)hipGetLastError();
    const int slots = std::min(8192, std::max(256, occ * cus));
    slot_cache.push_back({key, slots});
    stats.level_slots = std::max(stats.level_slots, slots);
    return slots;
  }
  int chunk_parents(uint64_t F, bool route = false) {
    const int pb = pb_max();
    return balanced_chunk(F, pb, level_slots((size_t)pb * kRowLds + 16, route));
  }

  // Enqueues up to kQueue levels of shard 0 (see the members above); returns how many ran.
  // elapsed_ms: the search's time so far; with a time limit, the queue holds no more levels than
  // the remaining budget covers at the last queue's measured time per level (SearchSettings
  // maxTimeSecs is checked between levels, so a queue never runs far past it).
  int enqueue_queue(int depth, double growth, double elapsed_ms, int* ran) {
    Shard& S = sh[0];
    if (!qctr) {
      DSL_HIP(hipMalloc(&qctr, (size_t)(kQueue + 1) * kCtrSet));
      DSL_HIP(hipHostMalloc(&hq, (size_t)kQueue * kCtrSet));
      qev.resize(2);
      for (auto& e : qev) DSL_HIP(hipEventCreate(&e));
    }
    const int nseg = kSegs;
    const uint64_t span = queue_span(S.F);
    if (span > q_span_hint) {
      // the next search's first queue starts with this span at level 1: size those history
      // levels now, so that a repeated search allocates nothing (the live rows are kept)
      q_span_hint = span;
      for (size_t lv = 1; lv <= (size_t)kQueue; lv++)
        DSL_TRY(hist_grow(S, lv, span, lv < S.level_size.size() ? S.level_size[lv] : 0));
    }
    q_segcap = span / nseg;
    // levels: up to kQueue, none past max_depth (its level's successors are all pruned)
    int nq = hset.max_depth >= 0 ? std::max(1, std::min(kQueue, hset.max_depth - depth)) : kQueue;
    if (hset.max_time_ms > 0 && q_ms_per_level > 0)
      nq = std::max(1, std::min(nq, (int)((hset.max_time_ms - elapsed_ms) / q_ms_per_level)));
    const uint64_t flimit = queue_flimit(span), wlimit = queue_wlimit(span);
    const uint64_t room = table_room_queue(), room_half = table_room();
    uint64_t used = 0;  // rows of the current frontier that must be kept
    for (size_t q = 0; q < S.seg_cnt.size(); q++) used = std::max(used, S.seg_base[q] + S.seg_cnt[q]);
    DSL_TRY(grow_rows(&S.cur, &S.cur_cap, std::max(span, used), true, used));
    DSL_TRY(grow(&S.cur_fp, &S.curfp_cap, std::max(span, used), true, used));
    DSL_TRY(grow_rows(&S.next, &S.next_cap, span, false, 0));
    DSL_TRY(grow(&S.next_fp, &S.nextfp_cap, span, false, 0));
    const size_t lev0 = S.level_size.size();  // the history level of the first queued level's rows
    for (int j = 0; j < nq; j++) DSL_TRY(hist_grow(S, lev0 + j, span, 0));
    DSL_TRY(grow(&S.spill, &S.spill_cap, wlimit, false, 0));
    const size_t per = kRowLds;
    const int pb_max = this->pb_max();
    const int spread = level_slots((size_t)pb_max * per + 16);
    SegTable t0{};
    t0.n = (int32_t)S.seg_cnt.size();
    t0.pb = balanced_chunk(S.F, pb_max, spread);
    for (int q = 0; q < t0.n; q++) {
      t0.base[q] = S.seg_base[q];
      t0.cnt[q] = S.seg_cnt[q];
      t0.chunk0[q + 1] = t0.chunk0[q] + (S.seg_cnt[q] + t0.pb - 1) / t0.pb;
    }
    // every set starts zeroed: the levels after a stop leave theirs untouched, and read zeros
    if (!qctr_clean) DSL_HIP(hipMemsetAsync(qctr, 0, (size_t)(kQueue + 1) * kCtrSet, stream));
    qctr_clean = false;
    const auto tq0 = std::chrono::steady_clock::now();
    const size_t lds = (size_t)pb_max * per + 16;
    for (int j = 0; j < nq; j++) {
      unsigned char* set = qctr + (size_t)j * kCtrSet;
      LevelArgs<P> a{};
      a.cur = (j & 1) ? S.next : S.cur;
      a.cur_fp = (j & 1) ? S.next_fp : S.cur_fp;
      a.segs = t0;
      a.qprev = j ? reinterpret_cast<const LevelCounters*>(set - kCtrSet) : nullptr;
      a.qprev_seg = j ? reinterpret_cast<const unsigned long long*>(set - kCtrSet + kCtrSegOff) : nullptr;
      a.qflimit = flimit;
      a.qwlimit = wlimit;
      a.qroom = room;
      a.qroom_half = room_half;
      a.qspread = spread;
      a.t0_rt = t0_rt;
      a.budget_rt = level_budget(W > 1);
      a.PB = pb_max;
      a.depth = depth + 1 + j;
      a.incremental = depth + j > init_depth ? 1 : 0;
      a.next = (j & 1) ? S.cur : S.next;
      a.next_fp = (j & 1) ? S.cur_fp : S.next_fp;
      a.next_parent = S.hpar[lev0 + j];
      a.next_event = S.hev[lev0 + j];
      a.seg_ctr = reinterpret_cast<unsigned long long*>(set + kCtrSegOff);
      a.zero_next = reinterpret_cast<uint4*>(set + kCtrSet);
      a.nseg = nseg;
      a.segcap = q_segcap;
      a.spill = S.spill;
      a.spill_cap = S.spill_cap;
      a.ctr = reinterpret_cast<LevelCounters*>(set);
      a.terms = S.terms;
      a.term_cap = term_cap;
      a.table = tbl;
      a.table.slots = S.table;
      a.W = W;
      a.me = S.gid;
      a.owner_filter = 0;
      if (j == 0 && q_events) DSL_HIP(hipEventRecord(qev[0], stream));
      // grid: one chunk per workgroup at the predicted frontier size (the kernel loops over more)
      const double fpred = (double)S.F * std::pow(growth, (double)j);
      (void)fpred;
      const int grid = spread;
      hipLaunchKernelGGL((k_level<P, false>), dim3(grid), dim3(kLevelBlock), lds, stream, a, prm, dset);
      DSL_HIP(hipGetLastError());
    }
    if (q_events) DSL_HIP(hipEventRecord(qev[1], stream));
    stats.expand_launches += nq;  // every dispatch, also those after the stop (they return at once)
    if (q_memcpy) {
      DSL_HIP(hipMemcpyAsync(hq, qctr, (size_t)nq * kCtrSet, hipMemcpyDeviceToHost, stream));
    } else {
      static_assert(kCtrSet % 16 == 0, "counter sets are copied in 16-byte units");
      const int n16 = nq * (kCtrSet / 16);
      hipLaunchKernelGGL(k_fetch_counters, dim3((n16 + kBlock - 1) / kBlock), dim3(kBlock), 0, stream,
                         reinterpret_cast<const uint4*>(qctr), reinterpret_cast<uint4*>(hq), n16);
      DSL_HIP(hipGetLastError());
    }
    DSL_TRY(hsync());
    q_ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count();
    // the levels that ran: up to the first whose counters stop the queue (the device's rule)
    *ran = nq;
    for (int j = 0; j + 1 < nq; j++) {
      const unsigned char* set = hq + (size_t)j * kCtrSet;
      LevelCounters c;
      std::memcpy(&c, set, sizeof(c));
      uint64_t F = 0;
      for (int q = 0; q < nseg; q++) {
        unsigned long long v;
        std::memcpy(&v, set + kCtrSegOff + (size_t)q * kSegStride * 8, 8);
        F += std::min<uint64_t>(v, q_segcap);
      }
      if (!queue_continues(c, F, flimit, wlimit, room, room_half)) {
        *ran = j + 1;
        break;
      }
    }
    float qms = 0;
    if (q_events && hipEventElapsedTime(&qms, qev[0], qev[1]) == hipSuccess) q_ms_total = qms;
    q_ms_per_level = q_ms_total / *ran;
    return DSL_OK;
  }

  // ---- visited-table growth (Search.java:406-408: `discovered` grows without bound) -----------
  // Each shard's table is kept at most half full: before a level, its estimated new states
  // (est_new_states) are added to what is inserted so far, and a table too small for twice that is
  // rehashed at once into the next power of two that is large enough (k_rehash). A level whose
  // probes still ran out of room (an estimate far off) makes the search restart with a larger
  // first table (run). The table never shrinks: a repeated search starts at the size reached.
  uint64_t table_room() const { return tbl.bucket_mask * 4 + 4 > inserted ? tbl.bucket_mask * 4 + 4 - inserted : 0; }
  // The queue's second room (queue_continues: twice the estimate, beside the estimate against
  // table_room's half-full rule): up to 3/4 of the slots, so a level whose new / work ratio doubles
  // against the estimate still probes a table at most 3/4 full.
  uint64_t table_room_queue() const {
    const uint64_t cap = (tbl.bucket_mask + 1) * 6;
    return cap > inserted ? cap - inserted : 0;
  }
  uint64_t table_limit_buckets() const {
    uint64_t lim = 1ull << kKeyBits;  // 2^35 slots, 256 GiB per shard
    if (hset.memory_budget_bytes) lim = std::min<uint64_t>(lim, std::max<uint64_t>(16, hset.memory_budget_bytes / 64));
    return lim;
  }
  // The key layout (fingerprint.hpp) pins 60 + b0 fingerprint bits, b0 = log2 of the search's
  // first table: a table of 2^b buckets (at most 2^(b+2) states, half full) keeps the chance of a
  // false merge n^2 / 2^(61 + b0) below 2^-20 while 2b - b0 <= kKeyRisk. A growth past that does
  // not rehash: the search restarts from a first table of the size needed (DSL_RESTART_REKEY), so
  // its keys pin more bits. Every input is identical on every rank, so all ranks restart together.
  static constexpr int kKeyRisk = 37;
  static constexpr int DSL_RESTART_REKEY = 1;
  uint64_t rekey_buckets = 0;
  // Probe mode (fingerprint.hpp table_insert): load first when the tables are well beyond the
  // Infinity Cache (256 MiB); DSL_PROBE_LOAD=0 / 1 forces it.
  int probe_load_first(uint64_t buckets) const {
    if (const char* e = getenv("DSL_PROBE_LOAD")) return atoi(e) ? 1 : 0;
    return buckets * 64 * (uint64_t)sh.size() > (1ull << 30) ? 1 : 0;
  }
  int ensure_table(uint64_t need_states) {
    const uint64_t have = tbl.bucket_mask + 1;
    uint64_t nb = have;
    while (nb * 4 < need_states && nb < table_limit_buckets()) nb <<= 1;  // 8 slots per bucket, half full
    if (nb == have) return DSL_OK;  // large enough, or at the budget (the probes then report a full table)
    {
      int b = 0;
      while ((2ull << b) <= nb) b++;
      const char* kr = getenv("DSL_KEY_RISK");  // tests: a smaller bound forces the restart
      if (2 * b - tbl.b0 > (kr ? atoi(kr) : kKeyRisk)) {
        rekey_buckets = nb;
        if (getenv("DSL_LEVEL_TRACE"))
          fprintf(stderr, "[table] %llu slots would pin too few key bits (b0 %d): restart\n",
                  (unsigned long long)nb * 8, tbl.b0);
        return DSL_RESTART_REKEY;
      }
    }
    if (!rehash_err) DSL_HIP(hipMalloc(&rehash_err, 8));
    DSL_HIP(hipMemsetAsync(rehash_err, 0, 8, stream));
    Table to = tbl;
    to.bucket_mask = nb - 1;
    // every shard allocates first; with several ranks the outcome is agreed (one sum over the
    // ranks) before anything changes, so a failed allocation on one rank ends the search on all
    std::vector<unsigned long long*> fresh(sh.size(), nullptr);
    uint64_t fail = 0;
    for (size_t l = 0; l < sh.size(); l++)
      if (hipMalloc(&fresh[l], nb * 64) != hipSuccess) fail = 1;
    (void)hipGetLastError();
    if (comm) {
      stats.host_syncs++;
      DSL_TRY(comm->allreduce_u64(&fail, 1, false, stream));
    }
    if (fail) {  // out of device memory: not "the estimate was far off", so run() does not restart
      for (auto* q : fresh) (void)hipFree(q);
      set_error("visited table growth: device allocation of " + std::to_string(nb * 64) + " bytes failed");
      return DSL_ERR_HIP;
    }
    std::vector<unsigned long long*> old(sh.size());
    for (size_t l = 0; l < sh.size(); l++) {
      Shard& S = sh[l];
      unsigned long long* nt = fresh[l];
      DSL_HIP(hipMemsetAsync(nt, 0, nb * 64, stream));
      Table from = tbl;
      from.slots = S.table;
      to.slots = nt;
      const int grid = (int)std::min<uint64_t>(8192, std::max<uint64_t>(1, have * 8 / kBlock));
      hipLaunchKernelGGL(k_rehash, dim3(grid), dim3(kBlock), 0, stream, from, to, rehash_err);
      DSL_HIP(hipGetLastError());
      old[l] = S.table;
      S.table = nt;
    }
    unsigned long long bad = 0;
    DSL_HIP(hipMemcpyAsync(&bad, rehash_err, 8, hipMemcpyDeviceToHost, stream));
    DSL_TRY(hsync());
    if (comm) {  // a rehash that found no free slot on one rank ends the search on every rank
      uint64_t b = bad;
      stats.host_syncs++;
      DSL_TRY(comm->allreduce_u64(&b, 1, false, stream));
      bad = b;
    }
    for (auto* q : old) (void)hipFree(q);
    tbl.bucket_mask = nb - 1;
    tbl.load_first = probe_load_first(nb);
    table_buckets = nb;
    stats.table_rehashes++;
    stats.table_slots = nb * 8 * (uint64_t)W;
    if (getenv("DSL_LEVEL_TRACE"))
      fprintf(stderr, "[table] %llu -> %llu slots (%llu inserted, %llu needed)\n", (unsigned long long)have * 8,
              (unsigned long long)nb * 8, (unsigned long long)inserted, (unsigned long long)need_states);
    if (bad) {
      set_error("visited table rehash found no free slot");
      return DSL_ERR_TABLE_FULL;
    }
    return DSL_OK;
  }

  // The TerminalRec of the level's best terminal key: from the list of improvements, or (the list
  // overflowed) by re-running the level's expansion in find mode over the current frontier.
  int resolve_terminal(Shard& S, uint64_t key, int succ_depth, bool incremental, TerminalRec* out) {
    const uint64_t n = std::min<uint64_t>(S.lc.n_term_rec, term_cap);
    std::vector<TerminalRec> recs(n);
    if (n) {
      DSL_HIP(hipMemcpyAsync(recs.data(), S.terms, n * sizeof(TerminalRec), hipMemcpyDeviceToHost, stream));
      DSL_TRY(hsync());
    }
    for (const auto& r : recs)
      if (r.key == key) {
        *out = r;
        return DSL_OK;
      }
    stats.terminal_finds++;
    if (!S.find_ctr) DSL_HIP(hipMalloc(&S.find_ctr, 2 * kCtrSet));
    DSL_HIP(hipMemsetAsync(S.find_ctr, 0, 2 * kCtrSet, stream));
    DSL_HIP(hipMemsetAsync(S.terms, 0, sizeof(TerminalRec), stream));
    uint64_t F = 0;
    for (uint64_t c : S.seg_cnt) F += c;
    const int PB = chunk_parents(F);
    const int slots = level_slots((size_t)pb_max() * kRowLds + 16);
    LevelArgs<P> a{};
    a.cur = S.cur;
    a.cur_fp = S.cur_fp;
    a.segs.n = (int32_t)S.seg_cnt.size();
    a.segs.pb = PB;
    for (int q = 0; q < a.segs.n; q++) {
      a.segs.base[q] = S.seg_base[q];
      a.segs.cnt[q] = S.seg_cnt[q];
      a.segs.chunk0[q + 1] = a.segs.chunk0[q] + (S.seg_cnt[q] + PB - 1) / PB;
    }
    a.PB = PB;
    a.depth = succ_depth;
    a.incremental = incremental ? 1 : 0;
    a.next = S.next;
    a.next_fp = S.next_fp;
    a.next_parent = S.hpar[0];
    a.next_event = S.hev[0];
    a.seg_ctr = reinterpret_cast<unsigned long long*>(S.find_ctr + kCtrSegOff);
    a.zero_next = reinterpret_cast<uint4*>(S.find_ctr + kCtrSet);
    a.nseg = 1;
    a.segcap = 0;
    a.ctr = reinterpret_cast<LevelCounters*>(S.find_ctr);
    a.terms = S.terms;
    a.term_cap = 1;
    a.W = W;
    a.me = S.gid;
    a.find = 1;
    a.find_key = key;
    a.qspread = slots;
    const uint64_t nchunks = a.segs.chunk0[a.segs.n];
    const int blocks = (int)std::max<uint64_t>(1, std::min<uint64_t>(nchunks, (uint64_t)slots));
    const size_t lds = (size_t)PB * kRowLds + 16;
    hipLaunchKernelGGL((k_level<P, false>), dim3(blocks), dim3(kLevelBlock), lds, stream, a, prm, dset);
    DSL_HIP(hipGetLastError());
    DSL_HIP(hipMemcpyAsync(out, S.terms, sizeof(TerminalRec), hipMemcpyDeviceToHost, stream));
    DSL_TRY(hsync());
    if (out->key != key) {
      set_error("terminal state of the level could not be resolved");
      return DSL_ERR_ARG;
    }
    return DSL_OK;
  }

  // ---- sharded levels: the fast path ----------------------------------------------
  // A sharded level moves its routed fingerprints in fixed-size SLABS: per (source, owner) pair
  // one region of kRouteSegs sub-slabs of `cs` records plus a header with their counts
  // (RouteCounters), sized before the level from the busiest rank's work and the last measured
  // routed fraction (route_frac, x1.3). No count crosses to the host before the exchange, so the
  // level is ONE host round trip: k_level<ROUTE> -> k_route_headers -> round A (the regions) ->
  // k_probe_slab (owners: every source interleaved, its own shard's included) -> round B (one
  // answer byte per record) -> k_new_list + k_materialize (sources) -> k_level_record -> the
  // records gathered -> the one synchronization. The maxDepth level has no round B and no
  // materialization (its routed successors were judged at the source: LevelArgs::judge_routed).
  // A record past its sub-slab is route-spilled (k_level keeps its parent and event); every rank
  // then runs the completion phase (complete_sharded: k_respill re-fingerprints them, host-sized
  // rounds). DSL_SLAB=0 routes everything that way (cs = 0: every record spills).
  const bool slab_mode = !(getenv("DSL_SLAB") && atoi(getenv("DSL_SLAB")) == 0);
  double route_frac = 0;  // routed records / work items of the last sharded level (0: none yet)
  uint64_t max_rank_work = 0;  // the next level's work of the busiest rank (0: no sharded level yet)

  // The exchange buffers grow with 1/8 headroom and no further factor: they are the largest
  // buffers of a sharded search (GBs at C3's deep levels), and the next search's slabs differ by a
  // few percent.
  template <class T>
  int grow_x(T** ptr, uint64_t* cap, uint64_t need) {
    if (need <= *cap && *ptr) return DSL_OK;
    const uint64_t want = need + need / 8 + 1024;
    if (*ptr) {
      DSL_TRY(hsync());
      (void)hipFree(*ptr);
      *ptr = nullptr;
      *cap = 0;
    }
    uint64_t c = 0;
    return grow(ptr, &c, want, false, 0) == DSL_OK ? (*cap = c, DSL_OK) : DSL_ERR_HIP;
  }
  int sharded_capacity(Shard& S, uint64_t cs, bool last) {
    S.route_cs = cs;
    S.cap_fp = kRouteHdr + (uint64_t)kRouteSegs * cs;  // the same on every rank
    DSL_TRY(grow_x(&S.out_key, &S.out_fp_cap, S.cap_fp * W));
    DSL_TRY(grow_x(&S.out_item, &S.out_item_cap, S.cap_fp * W));
    DSL_TRY(grow_x(&S.rspill, &S.rspill_cap, std::max<uint64_t>(S.work, 1)));
    DSL_TRY(grow_x(&S.in_fp, &S.in_fp_cap, S.cap_fp * W));
    S.cap_pk = pk_region_words(cs);
    DSL_TRY(grow_x(&S.out_pk, &S.out_pk_cap, std::max<uint64_t>(S.cap_pk * W, 1)));
    DSL_TRY(grow_x(&S.in_pk, &S.in_pk_cap, std::max<uint64_t>(S.cap_pk * W, 1)));
    DSL_TRY(grow_x(&S.rep_out, &S.rep_out_cap, S.cap_fp * W));
    DSL_TRY(grow_x(&S.rep_in, &S.rep_in_cap, S.cap_fp * W));
    // rows: every routed record of this shard may come back new (its own shard's included);
    // k_materialize appends them to the level's kSegs segments (k_level<ROUTE> appends none)
    const uint64_t mat_rows = last ? 0 : (uint64_t)kRouteSegs * cs * W;
    S.nseg = kSegs;
    S.segcap = mat_rows ? (mat_rows + kSegs - 1) / kSegs + 64 : 0;  // + a wave's share of imbalance
    S.seg_span = S.segcap * S.nseg;
    S.uns_room = 0;
    S.mat_room = 0;  // the completion phase's materialized rows, after the segments
    S.ovf_base = S.ovf_cnt = 0;
    DSL_TRY(grow(&S.spill, &S.spill_cap, 1, false, 0));
    DSL_TRY(grow_x(&S.newl, &S.newl_cap, std::max<uint64_t>(mat_rows, 1)));
    const uint64_t rows = S.seg_span + S.uns_room + S.mat_room;
    DSL_TRY(grow_rows(&S.next, &S.next_cap, rows, false, 0));
    DSL_TRY(grow(&S.next_fp, &S.nextfp_cap, rows, false, 0));
    DSL_TRY(hist_grow(S, S.level_size.size(), rows, 0));
    if (!S.nl_ctr) DSL_HIP(hipMalloc(&S.nl_ctr, (2 + kMaxShards) * 8));
    return DSL_OK;
  }

  // One all-to-all round where every (source, owner) pair moves `bytes[s][d]` bytes: local shard
  // l sends from send[l] + soff[l][d], receives at recv[l] + roff[l][s].
  int xround(const std::vector<const uint8_t*>& snd, const Mat& so, const Mat& sb, const std::vector<uint8_t*>& rcv,
             const Mat& ro, const Mat& rb) {
    stats.exchange_rounds++;
    if (comm) {  // the transport moves the other ranks' parts; this rank's own is a device copy
      const int me = sh[0].gid;
      if (sb[0][me])
        DSL_HIP(hipMemcpyAsync(rcv[0] + ro[0][me], snd[0] + so[0][me], sb[0][me], hipMemcpyDeviceToDevice, stream));
      Mat sb2 = sb, rb2 = rb;
      sb2[0][me] = rb2[0][me] = 0;
      return xfer(snd, so, sb2, rcv, ro, rb2);
    }
    return xfer(snd, so, sb, rcv, ro, rb);
  }

  // Every local shard's level record (k_level_record) computed on the device, gathered by every
  // rank, read with the shards' counters in ONE host round trip; recs = W records.
  // zero_rc: the fast path's gather is the route counters' last reader (no fill launch per level).
  int gather_records(const std::vector<uint64_t>& extra_rows, uint64_t time_up, std::vector<uint64_t>& recs,
                     bool zero_rc = false) {
    const int L = (int)sh.size();
    const bool dev_gather = comm && comm->device_collectives();
    for (int l = 0; l < L; l++) {
      Shard& S = sh[l];
      RecordArgs ra{};
      ra.c = S.ctr;
      ra.seg_ctr = S.seg_ctr;
      ra.nseg = S.nseg;
      ra.segcap = S.segcap;
      ra.extra_rows = extra_rows[l];
      ra.uns_cap = S.uns_room;
      ra.mat_cap = S.mat_room;
      ra.parents = S.F;
      ra.time_up = time_up;
      ra.gid = S.gid;
      ra.W = W;
      ra.rc = S.rc;
      ra.zero_rc = zero_rc ? 1 : 0;
      ra.cap_fp = S.cap_fp;
      ra.out = xdev + (size_t)l * kRecWords;
      ra.ctr_out = xdev + kXRecEnd + (size_t)l * kCtrMirrorWords;
      hipLaunchKernelGGL(k_level_record, dim3(1), dim3(64), 0, stream, ra);
      DSL_HIP(hipGetLastError());
    }
    uint64_t* gdev = xdev + (size_t)kMaxShards * kRecWords;
    if (dev_gather) DSL_TRY(comm->allgather_dev(xdev, kRecWords, gdev, stream));
    // ONE copy: the (gathered) records through the local shards' counter mirrors
    const size_t from = dev_gather ? (size_t)kMaxShards * kRecWords : 0;
    DSL_HIP(hipMemcpyAsync(xhost, xdev + from, (kXRecEnd + (size_t)L * kCtrMirrorWords - from) * 8,
                           hipMemcpyDeviceToHost, stream));
    DSL_TRY(hsync());
    for (int l = 0; l < L; l++) {  // the counters as the strided counter set (S.hctr's layout)
      Shard& S = sh[l];
      const uint64_t* m = xhost + (kXRecEnd - from) + (size_t)l * kCtrMirrorWords;
      std::memcpy(S.hctr, m, sizeof(LevelCounters));
      for (int q = 0; q < S.nseg; q++) std::memcpy(S.hctr + kCtrSegOff + (size_t)q * kSegStride * 8, m + kLcWords + q, 8);
    }
    recs.assign((size_t)W * kRecWords, 0);
    if (comm && !dev_gather) {
      stats.host_syncs++;
      DSL_TRY(comm->allgather_u64(xhost, kRecWords, recs.data(), stream));
    } else if (comm) {
      std::memcpy(recs.data(), xhost, recs.size() * 8);
    } else {
      for (int l = 0; l < L; l++)
        std::memcpy(recs.data() + (size_t)sh[l].gid * kRecWords, xhost + (size_t)l * kRecWords, kRecWords * 8);
    }
    for (auto& S : sh) std::memcpy(&S.lc, S.hctr, sizeof(LevelCounters));
    return DSL_OK;
  }

  int sharded_fast(int depth, bool last, uint64_t cs, uint64_t time_up, std::vector<uint64_t>& recs,
                   std::vector<std::vector<uint64_t>>& nbase, std::vector<std::vector<uint64_t>>& ncnt,
                   std::vector<uint64_t>& span) {
    const int L = (int)sh.size();
    Mat so(L, std::vector<uint64_t>(W, 0)), sb = so, ro = so, rb = so;
    std::vector<const uint8_t*> snd(L);
    std::vector<uint8_t*> rcv(L);
    if (cs) {
      for (auto& S : sh) {
        hipLaunchKernelGGL(k_route_headers, dim3(1), dim3(kMaxShards * kRouteSegs), 0, stream,
                           (const RouteCounters*)S.rc, S.out_key, S.cap_fp, cs, W,
                           (unsigned long long*)(last ? nullptr : S.nl_ctr), S.out_pk, S.cap_pk);
        DSL_HIP(hipGetLastError());
      }
      // round A: the regions of every (source, owner) pair, packed (12 bytes per record)
      for (int l = 0; l < L; l++) {
        Shard& S = sh[l];
        const uint64_t PB = S.cap_pk * 4;
        for (int d = 0; d < W; d++) {
          const uint64_t n = d == S.gid ? 0 : PB;
          so[l][d] = (uint64_t)d * PB;
          sb[l][d] = n;
          ro[l][d] = (uint64_t)d * PB;
          rb[l][d] = n;
        }
        snd[l] = reinterpret_cast<const uint8_t*>(S.out_pk);
        rcv[l] = reinterpret_cast<uint8_t*>(S.in_pk);
      }
      DSL_TRY(xround(snd, so, sb, rcv, ro, rb));
      for (auto& S : sh) {
        ProbeSlabArgs pa{};
        pa.in = S.in_fp;
        pa.in_pk = S.in_pk;
        pa.self_pk = S.out_pk + (size_t)S.gid * S.cap_pk;
        pa.cap_pk = S.cap_pk;
        pa.self = S.out_key + (size_t)S.gid * S.cap_fp;
        pa.cap_fp = S.cap_fp;
        pa.cs = cs;
        pa.W = W;
        pa.me = S.gid;
        pa.table = tbl;
        pa.table.slots = S.table;
        pa.reply = last ? nullptr : S.rep_out;
        pa.self_reply = S.rep_in + (size_t)S.gid * S.cap_fp;
        pa.ctr = S.ctr;
        hipLaunchKernelGGL(k_probe_slab, dim3(W * kRouteSegs, slab_gy(W * kRouteSegs, cs)), dim3(kBlock), 0, stream, pa);
        DSL_HIP(hipGetLastError());
      }
      if (!last) {
        // round B: one answer byte per record, back to its source (the regions' layout)
        for (int l = 0; l < L; l++) {
          Shard& S = sh[l];
          for (int d = 0; d < W; d++) {
            const uint64_t n = d == S.gid ? 0 : S.cap_fp;
            so[l][d] = (uint64_t)d * S.cap_fp;
            sb[l][d] = n;
            ro[l][d] = (uint64_t)d * S.cap_fp;
            rb[l][d] = n;
          }
          snd[l] = S.rep_out;
          rcv[l] = S.rep_in;
        }
        DSL_TRY(xround(snd, so, sb, rcv, ro, rb));
        for (auto& S : sh) DSL_TRY(launch_materialize(S, depth, true, nullptr, S.out_key, S.out_item, S.rep_in, S.cap_fp));
      }
    }
    std::vector<uint64_t> extra(L, 0);
    DSL_TRY(gather_records(extra, time_up, recs, true));
    bool incomplete = false, errors = false;
    for (int x = 0; x < W; x++) {
      const uint64_t* r = recs.data() + (size_t)x * kRecWords;
      incomplete |= r[kRecIncomplete] != 0;
      errors |= (r[kRecErrOverflow] | r[kRecErrTable] | r[kRecErrFrontier]) != 0;
    }
    if (getenv("DSL_LEVEL_TRACE")) {
      fprintf(stderr, "[shard] depth %d cs %llu last %d:", depth + 1, (unsigned long long)cs, last ? 1 : 0);
      for (int x = 0; x < W; x++) {
        const uint64_t* r = recs.data() + (size_t)x * kRecWords;
        uint64_t mx = 0;
        for (int d = 0; d < W; d++) mx = std::max<uint64_t>(mx, r[kRecRoute + d]);
        fprintf(stderr, " [%d: work %llu max_route %llu inc %llu]", x, (unsigned long long)r[kRecWork],
                (unsigned long long)mx, (unsigned long long)r[kRecIncomplete]);
      }
      fprintf(stderr, "\n");
    }
    if (incomplete && !errors) {
      stats.completions++;
      // the level's routed counts: the first gather's (it zeroed the route counters)
      std::vector<uint64_t> routes((size_t)W * kMaxShards);
      for (int x = 0; x < W; x++)
        std::memcpy(&routes[(size_t)x * kMaxShards], &recs[(size_t)x * kRecWords + kRecRoute], kMaxShards * 8);
      DSL_TRY(complete_sharded(depth, last, time_up, recs));
      for (int x = 0; x < W; x++)
        std::memcpy(&recs[(size_t)x * kRecWords + kRecRoute], &routes[(size_t)x * kMaxShards], kMaxShards * 8);
    } else {
      stats.fast_levels++;
    }
    // the next frontier of every local shard: the segments k_materialize filled, the completion
    // phase's materialized rows and its row spills (k_level appends none on a sharded level)
    for (int l = 0; l < L; l++) {
      Shard& S = sh[l];
      std::vector<unsigned long long> seg(kSegs * kSegStride);
      std::memcpy(seg.data(), S.hctr + kCtrSegOff, 8 * S.nseg * kSegStride);
      for (int q = 0; q < S.nseg; q++) {
        const uint64_t c = std::min<uint64_t>(seg[(size_t)q * kSegStride], S.segcap);
        if (c) {
          nbase[l].push_back((uint64_t)q * S.segcap);
          ncnt[l].push_back(c);
        }
      }
      const uint64_t mat = std::min<uint64_t>(S.lc.next_size, S.mat_room);
      if (mat) {
        nbase[l].push_back(S.seg_span + S.uns_room);
        ncnt[l].push_back(mat);
      }
      if (S.ovf_cnt) {
        nbase[l].push_back(S.ovf_base);
        ncnt[l].push_back(S.ovf_cnt);
      }
      span[l] = std::max(S.seg_span + S.uns_room + S.mat_room, S.ovf_base + S.ovf_cnt);
    }
    return DSL_OK;
  }

  // Blocks per group of the slab kernels (k_probe_slab, k_new_list: grid x = the groups, y =
  // blocks of a group, grid-stride): about the workgroups resident at once in all. The grid used to
  // be (W * 32, up to 64) = 16,384 workgroups at W = 8, mostly without a record: dispatching them
  // was most of the launch (C5's level 12: 27 us of k_probe_slab per shard).
  static int slab_gy(int groups, uint64_t per) {
    static const int total = getenv("DSL_SLAB_BLOCKS") ? std::max(1, atoi(getenv("DSL_SLAB_BLOCKS"))) : 2048;
    return (int)std::max<uint64_t>(1, std::min<uint64_t>((per + kBlock - 1) / kBlock,
                                                         (uint64_t)std::max(1, total / std::max(1, groups))));
  }

  // k_new_list + k_materialize of shard S: the new ones among its routed records (the fast path's
  // sub-slabs with device counts, or host counts cnt[d] of regions of `cap` records), appended at
  // seg_span + uns_room (next_size counts them across calls).
  int launch_materialize(Shard& S, int depth, bool dev, const uint64_t* cnt, const Fp* sent_key,
                         const uint64_t* sent_item, const uint8_t* reply, uint64_t cap) {
    const size_t lv = S.level_size.size();
    NewListArgs na{};
    na.reply = reply;
    na.cap = cap;
    na.W = W;
    na.dev_cnt = dev ? S.rc : nullptr;
    na.cs = S.route_cs;
    if (cnt)
      for (int d = 0; d < W; d++) na.cnt[d] = cnt[d];
    na.list = S.newl;
    na.n_list = reinterpret_cast<unsigned long long*>(S.nl_ctr);
    const uint64_t per = dev ? S.route_cs : cap, items = per * (uint64_t)W * (dev ? kRouteSegs : 1);
    const uint64_t room = dev ? S.seg_span : S.mat_room;
    if (!items || !room) return DSL_OK;
    if (!dev) DSL_HIP(hipMemsetAsync(S.nl_ctr, 0, 8, stream));  // dev: zeroed by k_route_headers
    const int groups = dev ? W * kRouteSegs : W;
    hipLaunchKernelGGL(k_new_list, dim3(groups, slab_gy(groups, per)), dim3(kBlock), 0, stream, na);
    DSL_HIP(hipGetLastError());
    MaterializeArgs<P> ma{};
    ma.sent_key = sent_key;
    ma.sent_item = sent_item;
    ma.list = S.newl;
    ma.n_list = reinterpret_cast<const unsigned long long*>(S.nl_ctr);
    ma.cur = S.cur;
    ma.cur_fp = S.cur_fp;
    ma.me = S.gid;
    ma.depth = depth + 1;
    ma.incremental = depth > init_depth ? 1 : 0;
    ma.next = S.next;
    ma.next_fp = S.next_fp;
    ma.next_parent = S.hpar[lv];
    ma.next_event = S.hev[lv];
    ma.next_base = S.seg_span + S.uns_room;
    ma.next_cap = S.mat_room;
    ma.seg_ctr = dev ? S.seg_ctr : nullptr;
    ma.nseg = S.nseg;
    ma.segcap = S.segcap;
    ma.ctr = S.ctr;
    ma.terms = S.terms;
    ma.term_cap = term_cap;
    // the grid: the workgroups resident at once (a wave takes 8..PMAX states; more workgroups only
    // launched and left, ~7,000 of 8,192 on C5's sharded levels)
    static const int mat_blocks = getenv("DSL_MAT_BLOCKS") ? std::max(1, atoi(getenv("DSL_MAT_BLOCKS"))) : 1024;
    const int blocks = (int)std::min<uint64_t>((std::min(items, room) + kBlock - 1) / kBlock, (uint64_t)mat_blocks);
    static const int mat_per = getenv("DSL_MAT_PER") ? std::max(1, std::min(mat_per_max<P>(), atoi(getenv("DSL_MAT_PER")))) : 0;
    ma.per_fixed = mat_per;
    const size_t lds = (size_t)(kBlock / 64) * (mat_per ? mat_per : mat_per_max<P>()) * NW * 4;
    hipLaunchKernelGGL(k_materialize<P>, dim3(std::max(1, blocks)), dim3(kBlock), lds, stream, ma, prm, dset);
    DSL_HIP(hipGetLastError());
    return DSL_OK;
  }

  // The completion phase of a sharded level (every rank, when any record is incomplete): the
  // route-spilled successors are re-fingerprinted per owner (k_respill; their counts gathered: a
  // host round trip), go through one host-sized exchange round (probe, answers,
  // materialization), the row spills are materialized, then the records are gathered again.
  // Rare: a sub-slab is 1.3x the records expected in it.
  int complete_sharded(int depth, bool last, uint64_t time_up, std::vector<uint64_t>& recs) {
    const int L = (int)sh.size();
    const size_t R = sizeof(Fp);
    const size_t lv = sh[0].level_size.size();
    Mat rs(W, std::vector<uint64_t>(W, 0));
    {
      std::vector<uint64_t> nrs(L);
      for (int l = 0; l < L; l++) {
        Shard& S = sh[l];
        nrs[l] = std::min<uint64_t>(S.lc.route_spilled, S.rspill_cap);
        S.rs_cap = std::max<uint64_t>(nrs[l], 1);
        unsigned long long* cnt = reinterpret_cast<unsigned long long*>(S.nl_ctr) + 2;
        DSL_HIP(hipMemsetAsync(cnt, 0, kMaxShards * 8, stream));
        if (!nrs[l]) continue;
        DSL_TRY(grow(&S.out2, &S.out2_cap, nrs[l] * W, false, 0));
        DSL_TRY(grow(&S.out2_item, &S.out2_item_cap, nrs[l] * W, false, 0));
        const int blocks = (int)std::min<uint64_t>((nrs[l] + kBlock - 1) / kBlock, 8192);
        hipLaunchKernelGGL(k_respill<P>, dim3(blocks), dim3(kBlock), 0, stream, (const uint64_t*)S.rspill, nrs[l],
                           (const uint32_t*)S.cur, (const Fp*)S.cur_fp, W, S.out2, S.out2_item, S.rs_cap, cnt, S.ctr,
                           prm, dset);
        DSL_HIP(hipGetLastError());
      }
      uint64_t* h = xhost + 2 * (size_t)kMaxShards * kRecWords;
      for (int l = 0; l < L; l++)
        DSL_HIP(hipMemcpyAsync(h + (size_t)l * kMaxShards, reinterpret_cast<unsigned long long*>(sh[l].nl_ctr) + 2,
                               kMaxShards * 8, hipMemcpyDeviceToHost, stream));
      DSL_TRY(hsync());
      std::vector<uint64_t> mine((size_t)L * W), all((size_t)W * W);
      for (int l = 0; l < L; l++)
        for (int d = 0; d < W; d++) mine[(size_t)l * W + d] = h[(size_t)l * kMaxShards + d];
      if (comm) {
        stats.host_syncs++;
        DSL_TRY(comm->allgather_u64(mine.data(), W, all.data(), stream));
      } else {
        for (int l = 0; l < L; l++)
          for (int d = 0; d < W; d++) all[(size_t)sh[l].gid * W + d] = mine[(size_t)l * W + d];
      }
      for (int x = 0; x < W; x++)
        for (int d = 0; d < W; d++) rs[x][d] = all[(size_t)x * W + d];
    }
    // rows: the materialized room grows by everything this shard may still get back
    for (int l = 0; l < L; l++) {
      Shard& S = sh[l];
      uint64_t more = 0;
      for (int d = 0; d < W; d++) more += rs[S.gid][d];
      const uint64_t used = S.seg_span + S.uns_room + S.mat_room;
      const uint64_t ovf = S.lc.spilled > S.uns_room ? std::min<uint64_t>(S.lc.spilled, S.spill_cap) - S.uns_room : 0;
      const uint64_t need = used + more + ovf;
      if (need > used) {
        DSL_TRY(grow_rows(&S.next, &S.next_cap, need, true, used));
        DSL_TRY(grow(&S.next_fp, &S.nextfp_cap, need, true, used));
        DSL_TRY(hist_grow(S, lv, need, used));
      }
      if (!last) S.mat_room += more;
      DSL_TRY(grow(&S.newl, &S.newl_cap, std::max<uint64_t>(more, 1), false, 0));
      S.ovf_base = S.seg_span + S.uns_room + S.mat_room;
      S.ovf_cnt = ovf;
    }
    bool any = false;
    for (int x = 0; x < W; x++)
      for (int d = 0; d < W; d++) any |= rs[x][d] != 0;
    if (any) {
      Mat so(L, std::vector<uint64_t>(W, 0)), sb = so, ro = so, rb = so;
      std::vector<const uint8_t*> snd(L);
      std::vector<uint8_t*> rcv(L);
      std::vector<uint64_t> nin(L, 0);
      for (int l = 0; l < L; l++) {
        Shard& S = sh[l];
        const int g = S.gid;
        uint64_t roff = 0;
        for (int d = 0; d < W; d++) {
          so[l][d] = (uint64_t)d * S.rs_cap * R;
          sb[l][d] = rs[g][d] * R;
          ro[l][d] = roff * R;
          rb[l][d] = rs[d][g] * R;
          roff += rs[d][g];
        }
        nin[l] = roff;
        DSL_TRY(grow(&S.in_fp, &S.in_fp_cap, std::max<uint64_t>(roff, 1), false, 0));
        DSL_TRY(grow(&S.rep_out, &S.rep_out_cap, std::max<uint64_t>(roff, 1), false, 0));
        snd[l] = reinterpret_cast<const uint8_t*>(S.out2);
        rcv[l] = reinterpret_cast<uint8_t*>(S.in_fp);
      }
      DSL_TRY(xround(snd, so, sb, rcv, ro, rb));
      for (int l = 0; l < L; l++) {
        Shard& S = sh[l];
        if (!nin[l]) continue;
        ProbeArgs pa;
        pa.in = S.in_fp;
        pa.n = nin[l];
        pa.table = tbl;
        pa.table.slots = S.table;
        pa.reply = S.rep_out;
        pa.ctr = S.ctr;
        const int blocks = (int)std::min<uint64_t>((nin[l] + kBlock - 1) / kBlock, 8192);
        hipLaunchKernelGGL(k_probe_remote, dim3(blocks), dim3(kBlock), 0, stream, pa);
        DSL_HIP(hipGetLastError());
      }
      if (!last) {  // the maxDepth level: judged at the source, nothing comes back
        for (int l = 0; l < L; l++) {
          Shard& S = sh[l];
          const int g = S.gid;
          DSL_TRY(grow(&S.rep2, &S.rep2_cap, S.rs_cap * W, false, 0));
          uint64_t soff = 0;
          for (int d = 0; d < W; d++) {
            so[l][d] = soff;
            sb[l][d] = rs[d][g];
            soff += rs[d][g];
            ro[l][d] = (uint64_t)d * S.rs_cap;
            rb[l][d] = rs[g][d];
          }
          snd[l] = S.rep_out;
          rcv[l] = S.rep2;
        }
        DSL_TRY(xround(snd, so, sb, rcv, ro, rb));
        for (int l = 0; l < L; l++) {
          Shard& S = sh[l];
          uint64_t cnt[kMaxShards] = {0};
          for (int d = 0; d < W; d++) cnt[d] = rs[S.gid][d];
          DSL_TRY(launch_materialize(S, depth, false, cnt, S.out2, S.out2_item, S.rep2, S.rs_cap));
        }
      }
    }
    // spills past their room
    std::vector<uint64_t> extra(L, 0);
    for (int l = 0; l < L; l++) {
      Shard& S = sh[l];
      if (!S.ovf_cnt) continue;
      const int blocks = (int)std::min<uint64_t>((S.ovf_cnt + kBlock - 1) / kBlock, 8192);
      hipLaunchKernelGGL(k_unspill<P>, dim3(blocks), dim3(kBlock), 0, stream, (const uint64_t*)(S.spill + S.uns_room),
                         S.ovf_cnt, (const uint32_t*)S.cur, (const Fp*)S.cur_fp, S.next, S.next_fp, S.hpar[lv], S.hev[lv],
                         S.ovf_base, S.gid, S.ctr, prm, dset, nullptr);
      DSL_HIP(hipGetLastError());
      extra[l] = S.ovf_cnt;
    }
    DSL_TRY(gather_records(extra, time_up, recs));
    return DSL_OK;
  }

  // ---- GlobalSettings.doErrorChecks / doAllChecks (Search.java:201-220) ------------------------
  // After a level, up to check_sample (0: 256) of its new states, evenly spaced over the shard's
  // next frontier, are re-derived on the host from their parent row and event (full_step, the
  // same transition functions compiled for the host) and compared with the device's row:
  // CheckLogger.notDeterministic (T/utils/CheckLogger.java:104-112). With DSL_CHECKS_ALL a
  // delivered message is also delivered again to the successor (it stays in the network, a set),
  // which must give the successor back: CheckLogger.notIdempotent (:114-121, "not necessarily an
  // error"). The first offending event of each kind is kept (decoded at its parent).
  // Scope: the sample is drawn from the level's device ROWS, i.e. its VALID new states. Pruned and
  // terminal successors, and every state of the maxDepth level, are never written as rows, so there
  // is no device result to compare them with (the reference checks every non-terminal state before
  // its prune test, Search.java:201-220); the handlers that produce them are the same code. A
  // multi-rank search sums the counts over the ranks (allreduce at the end of run_once).
  uint64_t chk_run = 0, chk_nd = 0, chk_ni = 0;
  dsl_event chk_first_nd{}, chk_first_ni{};
  // equal packed states: the header words and the records below the count (a device row's slots
  // past its count keep whatever the buffer held, kernels.hpp wave_emit)
  static bool same_state(const uint32_t* a, const uint32_t* b) {
    using L = Layout<P>;
    if (Net<P>::size(a) != Net<P>::size(b)) return false;
    return std::memcmp(a, b, (size_t)(L::kRecBase + Net<P>::size(a) * L::kRecWords) * 4) == 0;
  }
  int run_checks(Shard& S, const std::vector<uint64_t>& nbase, const std::vector<uint64_t>& ncnt) {
    uint64_t total = 0;
    for (uint64_t c : ncnt) total += c;
    if (!total) return DSL_OK;
    const size_t lv = S.level_size.size() - 1;  // this level's history (pushed above)
    const uint64_t want = hset.check_sample > 0 ? (uint64_t)hset.check_sample : 256;
    const uint64_t step = std::max<uint64_t>(1, total / want);
    const bool flip = getenv("DSL_CHECK_FLIP") != nullptr;  // tests: corrupt the first sampled row
    typename P::State child, parent, again, twice;
    for (uint64_t i = 0; i < total; i += step) {
      uint64_t idx = 0, pre = 0;
      for (size_t r = 0; r < ncnt.size(); r++) {
        if (i < pre + ncnt[r]) {
          idx = nbase[r] + (i - pre);
          break;
        }
        pre += ncnt[r];
      }
      uint64_t hp = 0;
      uint32_t k = 0;
      DSL_HIP(hipMemcpy(child.w, S.next + idx * NW, NW * 4, hipMemcpyDeviceToHost));
      DSL_HIP(hipMemcpy(&hp, S.hpar[lv] + idx, 8, hipMemcpyDeviceToHost));
      DSL_HIP(hipMemcpy(&k, S.hev[lv] + idx, 4, hipMemcpyDeviceToHost));
      const uint64_t pidx = hp & ((1ull << 48) - 1);
      DSL_HIP(hipMemcpy(parent.w, S.cur + pidx * NW, NW * 4, hipMemcpyDeviceToHost));
      if (flip && chk_run == 0) child.w[0] ^= 1u;
      chk_run++;
      const int rc = full_step<P>(parent.w, (int)k, again.w, prm, dset);
      if (rc != STEP_OK || !same_state(again.w, child.w)) {
        if (!chk_nd) describe_event<P>(parent.w, (int)k, prm, dset, &chk_first_nd);
        chk_nd++;
        continue;
      }
      if (hset.do_checks != DSL_CHECKS_ALL) continue;
      const int e = locate_event<P>(parent.w, prm, dset, (int)k);
      if (e < 0) continue;  // timers: not checked (SearchState.stepEvent's e.isMessage())
      const auto rec = Net<P>::at(parent.w, e);
      int e2 = -1;
      for (int j = 0; j < Net<P>::size(child.w); j++)
        if (Net<P>::at(child.w, j) == rec) e2 = j;
      Delta<P> d;
      const int rc2 = e2 < 0 ? STEP_NULL : delta_step_located<P>(child.w, e2, d, prm, dset);
      const bool same = rc2 == STEP_OK && materialize<P>(child.w, d, twice.w) && same_state(twice.w, child.w);
      if (!same) {
        if (!chk_ni) describe_event<P>(parent.w, (int)k, prm, dset, &chk_first_ni);
        chk_ni++;
      }
    }
    return DSL_OK;
  }

  // Search.run for BFS. A search whose visited table ran out of room (est_new_states far off:
  // more new states in one level than twice the estimate) is run again from a first table twice
  // the size it reached -- the table grows instead of failing, up to the memory budget.
  // A search restarted for its key width (ensure_table) starts from the table size it needed.
  // SearchSettings.maxTimeSecs bounds the whole call: a restart gets the time that is left
  // (t_run0 is the first attempt's start).
  uint64_t restart_buckets = 0;
  std::chrono::steady_clock::time_point t_run0;
  int run(dsl_result** out) override {
    restart_buckets = 0;
    t_run0 = std::chrono::steady_clock::now();
    for (int attempt = 0;; attempt++) {
      const int rc = run_once(out);
      if (rc == DSL_ERR_COMM && comm && !comm_failed) {
        // a transport failure (a dead or stalled peer, a caller-transport callback that failed)
        // leaves the ranks out of step: the engine refuses every later search
        comm_failed = true;
        comm->abort();
      }
      if (rc == DSL_RESTART_REKEY && attempt < 8) {
        restart_buckets = rekey_buckets;
        continue;
      }
      if (rc == DSL_RESTART_REKEY) {
        set_error("visited table: no key layout reached the required width");
        return DSL_ERR_TABLE_FULL;
      }
      if (rc != DSL_ERR_TABLE_FULL || table_buckets * 2 > table_limit_buckets() || attempt >= 8) return rc;
      restart_buckets = table_buckets * 2;
      if (getenv("DSL_LEVEL_TRACE")) fprintf(stderr, "[table] full: search restarts with %llu slots\n",
                                              (unsigned long long)restart_buckets * 8);
    }
  }

  int run_once(dsl_result** out) {
    const auto t_start = t_run0;
    if (comm_failed) {
      set_error("the engine's communicator was aborted by an earlier failure: create a new engine");
      return DSL_ERR_COMM;
    }
    (void)hipGetLastError();  // the per-thread sticky error must not blame this search for an older call
    if (!stream) {
      if (cfg.device >= 0) DSL_HIP(hipSetDevice(cfg.device));
      DSL_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
      DSL_HIP(hipEventCreate(&ev0));
      DSL_HIP(hipEventCreate(&ev1));
    }
    stats = dsl_stats{};
    stats.state_bytes = NW * 4;
    stats.world_size = W;
    if (!have_init) {
      uint8_t tmp[sizeof(init)];
      DSL_TRY(get_initial(tmp, sizeof(init)));
    }
    const int L = (int)sh.size();
    // DSL_TERM_CAP (tests): TerminalRec entries per shard; 0 records none, so every terminal level
    // is resolved by the find-mode re-run
    const char* tc = getenv("DSL_TERM_CAP");
    term_cap = tc ? (uint32_t)std::max(0l, strtol(tc, nullptr, 10)) : kTermCap;
    // the first table: 2^table_log2_slots slots (default 2^20), or the size an earlier search of
    // this engine grew it to; it grows during the search (ensure_table)
    const int log2 = hset.table_log2_slots > 0 ? hset.table_log2_slots : 20;
    if (log2 < 10 || log2 > kKeyBits + 3) return DSL_ERR_ARG;
    const uint64_t buckets = std::max<uint64_t>((1ull << log2) / 8, std::max(table_buckets, restart_buckets));
    for (auto& S : sh) {
      if (buckets != table_buckets || !S.table) {
        (void)hipFree(S.table);
        S.table = nullptr;
        DSL_HIP(hipMalloc(&S.table, buckets * 64));
        S.table_clean = false;
      }
      // the table, counter sets and route counters are zeroed by k_setup (below)
      if (!S.ctrbuf) DSL_HIP(hipMalloc(&S.ctrbuf, 2 * kCtrSet));
      if (!S.hctr) DSL_HIP(hipHostMalloc(&S.hctr, kCtrSet + sizeof(RouteCounters)));
      S.cset = 0;
      S.ctr = reinterpret_cast<LevelCounters*>(S.ctrbuf);
      S.seg_ctr = reinterpret_cast<unsigned long long*>(S.ctrbuf + kCtrSegOff);
      if (!S.terms || terms_alloc != term_cap) {
        (void)hipFree(S.terms);
        S.terms = nullptr;
        DSL_HIP(hipMalloc(&S.terms, sizeof(TerminalRec) * std::max<uint32_t>(term_cap, 1)));
      }
      if (!S.rc) DSL_HIP(hipMalloc(&S.rc, sizeof(RouteCounters)));
      S.seg_base.clear();
      S.seg_cnt.clear();
      DSL_TRY(grow_rows(&S.cur, &S.cur_cap, 1024, false, 0));
      DSL_TRY(grow_rows(&S.next, &S.next_cap, 1024, false, 0));
      DSL_TRY(grow(&S.cur_fp, &S.curfp_cap, 1024, false, 0));
      DSL_TRY(grow(&S.next_fp, &S.nextfp_cap, 1024, false, 0));
      // every search starts with the same buffer of each pair as `cur`: the two then take the
      // same roles level by level in every search, so a repeated search reallocates nothing
      if (S.flip) {
        std::swap(S.cur, S.next);
        std::swap(S.cur_cap, S.next_cap);
        std::swap(S.cur_fp, S.next_fp);
        std::swap(S.curfp_cap, S.nextfp_cap);
        S.flip = false;
      }
      DSL_TRY(hist_grow(S, 0, 1, 0));
      S.level_size.assign(1, 0);
      S.F = 0;
      S.work = 0;
    }
    table_buckets = buckets;
    terms_alloc = term_cap;
    budget_rt = 0;
    if (hset.max_time_ms > 0) {
      if (!t0_rt) DSL_HIP(hipMalloc(&t0_rt, 8));
      hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, stream, t0_rt);
      DSL_HIP(hipGetLastError());
      const double left = hset.max_time_ms -
                          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
      budget_rt = (uint64_t)std::max(1.0, left * 1e5);  // s_memrealtime: 100 MHz
    }
    stats.table_slots = buckets * 8 * (uint64_t)W;
    q_left = 0;
    q_pos = 0;
    // do_checks reads every level's rows right after the level: no device-side queue of levels
    const bool use_queue = !getenv("DSL_NO_QUEUE") && hset.do_checks == DSL_CHECKS_NONE;
    chk_run = chk_nd = chk_ni = 0;
    chk_first_nd = chk_first_ni = dsl_event{};
    if (const char* qr = getenv("DSL_QUEUE_ROWS")) q_rows_forced = std::max<uint64_t>(kSegs, strtoull(qr, nullptr, 10) / kSegs * kSegs);
    const bool trace_levels = getenv("DSL_LEVEL_TRACE") != nullptr;
    tbl = Table{nullptr, buckets - 1, 0, 0};
    tbl.load_first = probe_load_first(buckets);
    while ((2ull << tbl.b0) <= buckets) tbl.b0++;  // log2(buckets): the key layout of this search
    inserted = 1;
    uint64_t prev_new = 0, prev_work = 0;  // the last level's new states and work items (est_new_states)
    // the last level's frontier growth (next frontier / frontier, all shards): the next frontier's
    // rows are reserved for 1.25x that growth (at least 4x), so a protocol that grows faster than
    // 4 new states per parent (the synthetic C3: ~5) does not spill every large level
    uint64_t prev_front = 1;
    double front_growth = 0;

    // Seed: the initial state lives on its owner shard (BFS.initSearch, Search.java:434-440).
    const Fp init_fp = full_fingerprint<P>(init.w);
    const int init_owner = owner_of(init_fp, W);
    uint64_t init_enc = ~0ull;
    // Replicated small levels: while the frontier is below rep_threshold, every shard runs the
    // whole level itself (identical work, no exchange; each table then holds every state of
    // those levels, a superset of what it owns, so later owner probes stay exact). The first
    // level above the threshold expands only owned parents, and from there on the search is
    // hash-sharded. Per-level latency of a sharded level is ~3 exchange rounds, so sharding a
    // level pays only once it has enough work.
    bool rep_active = W > 1 && rep_threshold() > 0;
    max_rank_work = 0;
    bool first_sharded = W > 1 && !rep_active;
    // checkState of the initial state: the same judge, on the host (no round trip before the
    // first level); k_setup only inserts its fingerprint
    {
      int pi = -1;
      const NodeView v0{init.w, P::kNodeWords, -1, nullptr};
      const int v = judge_view<P>(v0, prm, dset, init_depth, &pi);
      init_enc = ((uint64_t)v << 32) | (uint32_t)(pi + 1);
    }
    for (auto& S : sh) {
      // one k_setup per shard: zeroes its table and counters; seeds the initial state's owner (or
      // every shard while small levels are replicated)
      const bool seed = S.gid == init_owner || rep_active;
      SetupArgs<P> sa{};
      sa.table = reinterpret_cast<uint4*>(S.table);
      sa.n_table = buckets * 4;
      sa.clean = S.table_clean ? 1 : 0;
      S.table_clean = false;
      sa.ctr = reinterpret_cast<uint4*>(S.ctrbuf);
      sa.n_ctr = 2 * kCtrSet / 16;
      sa.rc = reinterpret_cast<uint4*>(S.rc);
      sa.n_rc = (int32_t)((sizeof(RouteCounters) + 15) / 16);
      static_assert(sizeof(RouteCounters) % 16 == 0, "RouteCounters is zeroed in 16-byte units");
      sa.seed = seed ? 1 : 0;
      sa.home = table_home(tbl, init_fp);  // an empty table: the home slot, displacement 0
      sa.key = (unsigned long long)table_key0(tbl, init_fp);
      sa.cur = S.cur;
      sa.cur_fp = S.cur_fp;
      sa.fp = init_fp;
      std::memcpy(sa.init, init.w, NW * 4);
      const int sgrid = sa.clean ? 1 : (int)std::min<uint64_t>(4096, std::max<uint64_t>(1, sa.n_table / kBlock));
      hipLaunchKernelGGL(k_setup<P>, dim3(sgrid), dim3(kBlock), 0, stream, sa);
      DSL_HIP(hipGetLastError());
      if (!seed) continue;
      S.F = 1;
      S.seg_base.assign(1, 0);
      S.seg_cnt.assign(1, 1);
      S.work = (uint64_t)count_events<P>(init.w, prm, dset);
      S.level_size[0] = 1;
    }
    if (comm) {  // the initial state's verdict and the cost model, agreed by every rank (one collective)
      uint64_t v[3] = {init_enc, ~(uint64_t)(cost_c_ns * 1e6), ~(uint64_t)(cost_x_us * 1e3)};
      DSL_TRY(comm->allreduce_u64(v, 3, true, stream));
      init_enc = v[0];
      stats.cost_c_ns = (double)~v[1] / 1e6;
      stats.cost_x_us = (double)~v[2] / 1e3;
    } else {
      stats.cost_c_ns = cost_c_ns;
      stats.cost_x_us = cost_x_us;
    }
    {
      // a level of w work items takes T(w) = max(Tf, c w) (Tf: the latency floor of a small level);
      // shard iff T(w) - T(w / W) > X, i.e. from the smallest such w
      const double c = stats.cost_c_ns > 0 ? stats.cost_c_ns : 0.05, x = (stats.cost_x_us > 0 ? stats.cost_x_us : 100.0) * 1e3;
      const double tf = kLevelFloorUs * 1e3;
      const double w = x <= (W - 1) * tf ? (x + tf) / c : x / (c * (1.0 - 1.0 / W));
      shard_work_min = W > 1 ? (uint64_t)std::min(w, 1.8e19) : ~0ull;
      stats.shard_work_min = W > 1 ? shard_work_min : 0;
    }
    const int init_verdict = (int)(init_enc >> 32);
    if (trace_levels)
      fprintf(stderr, "[setup] %.4f ms\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());

    if (W > 1 && !xdev) {
      DSL_HIP(hipMalloc(&xdev, kXWords * 8));
      DSL_HIP(hipHostMalloc(&xhost, kXWords * 8));
    }
    stats.rccl_version = comm ? comm->version() : 0;
    // a sharded level's gathered records already hold the next level's global frontier size, work
    // and time-up flag (g below): no collective at the top of that next level
    bool have_g = false;
    std::vector<uint64_t> g_next(3, 0);
    std::vector<uint64_t> per_depth{1};
    uint64_t total_states = 1, successors = 0, exchanged = 0, max_front = 1, x_levels = 0;
    double x_sum_us = 0;
    int end = DSL_SPACE_EXHAUSTED, pred_index = -1, term_depth = -1;
    int depth = init_depth;
    double level_ms_max = 0;
    progress_states = 1;
    progress_depth = depth;
    if (init_verdict >= V_TERM_EXCEPTION) {
      end = init_verdict == V_TERM_INVARIANT ? DSL_INVARIANT_VIOLATED : DSL_GOAL_FOUND;
      pred_index = (int)(init_enc & 0xffffffffu) - 1;
      term_depth = init_depth;
    } else {
      while (true) {
        const auto lt0 = std::chrono::steady_clock::now();
        const uint64_t reallocs0 = n_reallocs + stats.table_rehashes, exchanged0 = exchanged;
        // every shard holds the same frontier in a replicated level: the decision is identical
        const bool rep = rep_active && level_replicated(sh[0].F, sh[0].work);
        if (rep_active && !rep) {
          rep_active = false;
          first_sharded = true;
        }
        const bool route = W > 1 && !rep;
        std::vector<uint64_t> g(3, 0);  // [frontier states, time-up flag, work items]
        if (rep) {
          g[0] = sh[0].F;
          g[2] = sh[0].work;
        } else {
          for (auto& S : sh) g[0] += S.F, g[2] += S.work;
        }
        if (hset.max_time_ms > 0) {
          const double el =
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
          if (el > hset.max_time_ms) g[1] = 1;
        }
        if (have_g) {
          g = g_next;
          have_g = false;
        } else if (!rep || hset.max_time_ms > 0) {
          DSL_TRY(global_sum(g));
        }
        if (g[1]) {
          end = DSL_TIME_EXHAUSTED;
          break;
        }
        if (g[0] == 0) break;

        if (use_queue && q_left == 0 && L == 1 && (W == 1 || rep) && sh[0].F > 0 &&
            sh[0].F <= queue_flimit(queue_span(sh[0].F)) && sh[0].work <= 8 * queue_span(sh[0].F)) {
          // frontier growth per level, for the queued launches' grid sizes
          const size_t nd = per_depth.size();
          const double growth =
              nd >= 2 && per_depth[nd - 2] ? std::max(1.0, (double)per_depth[nd - 1] / per_depth[nd - 2]) : 3.0;
          int ran = 0;
          const auto tq0 = std::chrono::steady_clock::now();
          DSL_TRY(ensure_table(inserted + est_new_states(sh[0].work, prev_new, prev_work)));
          DSL_TRY(enqueue_queue(depth, growth,
                                std::chrono::duration<double, std::milli>(tq0 - t_start).count(), &ran));
          if (trace_levels)
            fprintf(stderr, "[queue] enqueue+run %.4f ms (loop entry %.4f ms after start)\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count(),
                    std::chrono::duration<double, std::milli>(tq0 - t_start).count());
          q_left = ran;
          q_pos = 0;
        }
        const bool queued = q_left > 0;
        if (!queued) {
          // a sharded level inserts about 1/W of its new states into each shard's table (+25 % for
          // the hash's imbalance); a replicated or single-shard level all of them
          const uint64_t est = est_new_states(g[2], prev_new, prev_work);
          DSL_TRY(ensure_table(inserted + (route ? est / W + est / (4 * W) + 1024 : est)));
        }

        // Capacity: the level has exactly S.work work items, an upper bound on its new states.
        // The next frontier gets min(work, 4F) rows (typical growth is ~3 new states per
        // parent) split into nseg equal segments; VALID states beyond a segment's rows are
        // spilled as 8-byte items (room for all `work` of them) and materialized after the
        // kernel, so the estimate never fails and never reserves the worst case.
        uint64_t Fmax = 0;
        for (auto& S : sh) Fmax = std::max(Fmax, S.F);
        const int PB = chunk_parents(Fmax, route);
        // a sharded level: the slab (records per source -> owner pair the fast path moves without
        // the host reading any count), from the global work and the last measured routed fraction;
        // identical on every rank (its inputs are). The maxDepth level expands nothing further.
        // (DSL_LAST_ROUND_B=1, measurement: the maxDepth level like any other, answers back and the
        // new ones judged at the source by k_materialize, which appends none of them: all PRUNED)
        const bool last_level = hset.max_depth >= 0 && depth + 1 >= hset.max_depth && !getenv("DSL_LAST_ROUND_B");
        uint64_t slab = 0;  // records per sub-slab (LevelArgs::route_cs)
        if (route && slab_mode) {
          // the most work one rank has: from the last sharded level's records; after replicated
          // levels every rank expands the parents it owns (hash-balanced, g/W); a search sharded
          // from its first level starts on the initial state's owner alone
          const double per_rank = max_rank_work ? (double)max_rank_work
                                  : rep_threshold() > 0 ? (double)g[2] / W : (double)g[2];
          const double frac = route_frac > 0 ? route_frac : 1.0;
          // 1.15x the expected records per sub-slab + one wave's 64: every sub-slab takes records of
          // all four wave indexes of many workgroups (k_level), so the fill is even (1.3x before
          // round 6, when a sub-slab took one wave index's records)
          static const double factor = getenv("DSL_SLAB_FACTOR") ? atof(getenv("DSL_SLAB_FACTOR")) : 1.15;
          slab = (uint64_t)(factor * frac * per_rank / ((double)W * kRouteSegs)) + 64;
          if (const char* m = getenv("DSL_SLAB_MAX")) slab = std::min<uint64_t>(slab, std::max(1, atoi(m)));  // tests
        }
        const int lslots = level_slots((size_t)pb_max() * kRowLds + 16, route);
        if (queued) {
          sh[0].nseg = kSegs;
          sh[0].segcap = q_segcap;
        } else {
        for (auto& S : sh) {
          S.ctr = reinterpret_cast<LevelCounters*>(S.ctrbuf + S.cset * kCtrSet);
          S.seg_ctr = reinterpret_cast<unsigned long long*>(S.ctrbuf + S.cset * kCtrSet + kCtrSegOff);
          // a shard that launches no k_level this level zeroes its next set here
          if (S.F == 0) DSL_HIP(hipMemsetAsync(S.ctrbuf + (S.cset ^ 1) * kCtrSet, 0, kCtrSet, stream));
          if (route) {  // every successor is routed: the rows come from k_materialize only
            DSL_TRY(sharded_capacity(S, slab, last_level));
            continue;
          }
          uint64_t nchunks = 0;
          for (size_t q = 0; q < S.seg_cnt.size(); q++) nchunks += (S.seg_cnt[q] + PB - 1) / PB;
          const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>(nchunks, (uint64_t)lslots));
          S.nseg = (int)std::min<uint64_t>(kSegs, blocks);
          const uint64_t grown = (uint64_t)(1.25 * front_growth * (double)S.F);
          const uint64_t want = std::min<uint64_t>(S.work, std::max<uint64_t>(std::max<uint64_t>(4 * S.F, grown), 8192)) + 1;
          S.segcap = (want + S.nseg - 1) / S.nseg + 1;
          const uint64_t rows = S.segcap * S.nseg;
          DSL_TRY(grow_rows(&S.next, &S.next_cap, rows, false, 0));
          DSL_TRY(grow(&S.next_fp, &S.nextfp_cap, rows, false, 0));
          DSL_TRY(hist_grow(S, S.level_size.size(), rows, 0));
          DSL_TRY(grow(&S.spill, &S.spill_cap, std::max<uint64_t>(S.work, 1), false, 0));
        }
        }  // !queued (capacity)
        const size_t lds = (size_t)PB * kRowLds + 16;
        if (!queued) {
        DSL_HIP(hipEventRecord(ev0, stream));
        for (auto& S : sh) {
          if (S.F == 0) continue;
          LevelArgs<P> a{};
          a.cur = S.cur;
          a.cur_fp = S.cur_fp;
          a.segs.n = (int32_t)S.seg_cnt.size();
          a.segs.chunk0[0] = 0;
          for (int q = 0; q < a.segs.n; q++) {
            a.segs.base[q] = S.seg_base[q];
            a.segs.cnt[q] = S.seg_cnt[q];
            a.segs.chunk0[q + 1] = a.segs.chunk0[q] + (S.seg_cnt[q] + PB - 1) / PB;
          }
          a.PB = PB;
          a.depth = depth + 1;
          a.incremental = depth > init_depth ? 1 : 0;
          a.next = S.next;
          a.next_fp = S.next_fp;
          a.next_parent = S.hpar[S.level_size.size()];
          a.next_event = S.hev[S.level_size.size()];
          a.seg_ctr = S.seg_ctr;
          a.zero_next = reinterpret_cast<uint4*>(S.ctrbuf + (S.cset ^ 1) * kCtrSet);
          a.nseg = S.nseg;
          a.segcap = S.segcap;
          a.spill = S.spill;
          a.spill_cap = S.spill_cap;
          a.ctr = S.ctr;
          a.terms = S.terms;
          a.term_cap = term_cap;
          a.table = tbl;
          a.table.slots = S.table;
          a.W = W;
          a.me = S.gid;
          a.owner_filter = route && first_sharded ? 1 : 0;
          a.out_key = S.out_key;
          a.out_pk = slab ? S.out_pk : nullptr;
          a.cap_pk = S.cap_pk;
          a.out_item = S.out_item;
          a.cap_fp = S.cap_fp;
          a.route_cs = S.route_cs;
          a.rc = S.rc;
          a.rspill = S.rspill;
          a.rspill_cap = S.rspill_cap;
          a.judge_routed = route && last_level ? 1 : 0;
          a.qprev = nullptr;
          a.qprev_seg = nullptr;
          a.segs.pb = PB;
          a.qspread = lslots;
          a.t0_rt = t0_rt;
          a.budget_rt = level_budget(rep);
          const uint64_t nchunks = a.segs.chunk0[a.segs.n];
          const int blocks = (int)std::min<uint64_t>(nchunks, (uint64_t)lslots);
          if (route)
            hipLaunchKernelGGL((k_level<P, true>), dim3(blocks), dim3(kLevelBlock), lds, stream, a, prm, dset);
          else
            hipLaunchKernelGGL((k_level<P, false>), dim3(blocks), dim3(kLevelBlock), lds, stream, a, prm, dset);
          DSL_HIP(hipGetLastError());
        }
        DSL_HIP(hipEventRecord(ev1, stream));
        }  // !queued (launch)
        // The level's counters. A sharded level runs its exchange first (sharded_fast): the
        // owners' probes, the materialization and every shard's level record, then ONE host round
        // trip; a single-shard or replicated level reads its counters right after k_level.
        std::vector<std::vector<unsigned long long>> segc(L, std::vector<unsigned long long>(kSegs * kSegStride));
        std::vector<std::vector<uint64_t>> nbase(L), ncnt(L);
        std::vector<uint64_t> span(L);
        std::vector<uint64_t> recs;  // sharded: W records of kRecWords (k_level_record), every rank's
        const auto tx0 = std::chrono::steady_clock::now();
        if (route) {
          stats.sharded_levels++;
          uint64_t time_up = 0;
          if (hset.max_time_ms > 0 &&
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count() >
                  hset.max_time_ms)
            time_up = 1;
          DSL_TRY(sharded_fast(depth, last_level, slab, time_up, recs, nbase, ncnt, span));
          // the routed fraction of this level (all shards), for the next level's slab
          uint64_t routed = 0, lw = 0;
          for (int x = 0; x < W; x++) {
            const uint64_t* r = recs.data() + (size_t)x * kRecWords;
            lw += r[kRecWork];
            for (int d = 0; d < W; d++) routed += r[kRecRoute + d];  // its own shard's included
          }
          if (lw) route_frac = std::max(0.05, (double)routed / (double)lw);
          max_rank_work = 0;
          for (int x = 0; x < W; x++) max_rank_work = std::max<uint64_t>(max_rank_work, recs[(size_t)x * kRecWords + kRecNextWork]);
          for (int l = 0; l < L; l++)
            for (int d = 0; d < W; d++)
              if (d != sh[l].gid) exchanged += recs[(size_t)sh[l].gid * kRecWords + kRecRoute + d];
        } else {
        if (queued) {  // this level's counters came back with the queue
          const unsigned char* set = hq + (size_t)q_pos * kCtrSet;
          std::memcpy(&sh[0].lc, set, sizeof(LevelCounters));
          // only the segments' counter words (one per 128-byte line) from the pinned host buffer
          for (int q = 0; q < kSegs; q++)
            std::memcpy(&segc[0][(size_t)q * kSegStride], set + kCtrSegOff + (size_t)q * kSegStride * 8, 8);
        } else {
          for (int l = 0; l < L; l++) {
            Shard& S = sh[l];
            DSL_HIP(hipMemcpyAsync(S.hctr, S.ctrbuf + S.cset * kCtrSet, kCtrSegOff + 8 * S.nseg * kSegStride,
                                   hipMemcpyDeviceToHost, stream));
          }
          DSL_TRY(hsync());
          for (int l = 0; l < L; l++) {
            Shard& S = sh[l];
            std::memcpy(&S.lc, S.hctr, sizeof(LevelCounters));
            std::memcpy(segc[l].data(), S.hctr + kCtrSegOff, 8 * S.nseg * kSegStride);
          }
        }
        // next frontier: the filled part of each segment, then the spill range
        bool unspilled = false;
        for (int l = 0; l < L; l++) {
          Shard& S = sh[l];
          for (int q = 0; q < S.nseg; q++) {
            const uint64_t c = std::min<uint64_t>(segc[l][(size_t)q * kSegStride], S.segcap);
            if (c) {
              nbase[l].push_back((uint64_t)q * S.segcap);
              ncnt[l].push_back(c);
            }
          }
          span[l] = S.segcap * S.nseg;
          const uint64_t ns = std::min<uint64_t>(S.lc.spilled, S.spill_cap);
          if (!ns || S.lc.err_frontier || S.lc.err_overflow) continue;
          unspilled = true;
          const uint64_t keep = span[l], need = keep + ns;
          const size_t lv = S.level_size.size();
          DSL_TRY(grow_rows(&S.next, &S.next_cap, need, true, keep));
          DSL_TRY(grow(&S.next_fp, &S.nextfp_cap, need, true, keep));
          DSL_TRY(hist_grow(S, lv, need, keep));
          const int blocks = (int)std::min<uint64_t>((ns + kBlock - 1) / kBlock, 256ull * 32);
          LevelCounters* uctr = queued ? reinterpret_cast<LevelCounters*>(qctr + (size_t)q_pos * kCtrSet) : S.ctr;
          hipLaunchKernelGGL(k_unspill<P>, dim3(blocks), dim3(kBlock), 0, stream, S.spill, ns, S.cur, S.cur_fp, S.next,
                             S.next_fp, S.hpar[lv], S.hev[lv], keep, S.gid, uctr, prm, dset, nullptr);
          nbase[l].push_back(keep);
          ncnt[l].push_back(ns);
          span[l] = need;
        }
        if (unspilled) {  // counters changed after the first read (next_work)
          for (auto& S : sh) {
            const void* src = queued ? (const void*)(qctr + (size_t)q_pos * kCtrSet) : (const void*)S.ctr;
            DSL_HIP(hipMemcpyAsync(S.hctr, src, sizeof(LevelCounters), hipMemcpyDeviceToHost, stream));
          }
          DSL_TRY(hsync());
          for (auto& S : sh) std::memcpy(&S.lc, S.hctr, sizeof(LevelCounters));
        }
        }  // !route
        if (route)  // the exchange rounds, the owners' probes and the materialization, up to the counters
          stats.exchange_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tx0).count();
        float kms = 0;
        if (!queued || q_pos == 0) {  // a queue is timed as a whole (its dispatches counted there)
          if (queued) kms = (float)q_ms_total;
          else (void)hipEventElapsedTime(&kms, ev0, ev1);
          stats.expand_ms += kms;
        }
        if (!queued) stats.expand_launches++;
#ifdef DSL_PHASES
        for (auto& S : sh) {
          const auto& q = S.lc.phase;
          fprintf(stderr, "[phases] depth %d F=%llu work=%llu new=%llu cycles:", depth + 1, (unsigned long long)S.F,
                  (unsigned long long)S.lc.work_items, (unsigned long long)S.lc.new_states);
          for (int i = 0; i < 12; i++) fprintf(stderr, " %.3g", (double)q[i]);
          fprintf(stderr, "\n[phcls] depth %d", depth + 1);
          for (int c = 0; c < 16; c++)
            if (S.lc.phcls[16 + c])
              fprintf(stderr, " c%d: %.3g cyc / %llu passes (%.0f)", c, (double)S.lc.phcls[c],
                      (unsigned long long)S.lc.phcls[16 + c], (double)S.lc.phcls[c] / S.lc.phcls[16 + c]);
          if (S.lc.phcls[31]) {  // k_materialize (sharded levels): cycles per wave pass by phase
            fprintf(stderr, "\n[matph] depth %d passes %llu cycles/pass: items %.0f stage %.0f handler %.0f judge %.0f "
                    "reserve+count %.0f emit %.0f", depth + 1, (unsigned long long)S.lc.phcls[31],
                    (double)S.lc.phcls[10] / S.lc.phcls[31], (double)S.lc.phcls[11] / S.lc.phcls[31],
                    (double)S.lc.phcls[12] / S.lc.phcls[31], (double)S.lc.phcls[13] / S.lc.phcls[31],
                    (double)S.lc.phcls[14] / S.lc.phcls[31], (double)S.lc.phcls[15] / S.lc.phcls[31]);
          }
          fprintf(stderr, "\n");
        }
#elif defined(DSL_TIMELINE)
        for (auto& S : sh) {
          const auto& q = S.lc.phase;
          const unsigned long long t0 = ~q[0];  // the earliest workgroup entry
          fprintf(stderr, "[timeline] depth %d F=%llu work=%llu | all WGs %.2f us | WG0 entry +%.2f:", depth + 1,
                  (unsigned long long)S.F, (unsigned long long)S.lc.work_items, (q[1] - t0) / 100.0,
                  ((long long)q[2] - (long long)t0) / 100.0);
          for (int i = 0; i < 32 && S.lc.phcls[i]; i++)
            fprintf(stderr, " %llu@%.2f", S.lc.phcls[i] >> 56,
                    ((long long)(S.lc.phcls[i] & ((1ull << 56) - 1)) - (long long)(t0 & ((1ull << 56) - 1))) / 100.0);
          fprintf(stderr, "\n");
        }
#endif
        // global counts, errors, terminal selection
        std::vector<uint64_t> gsum(8, 0);
        uint64_t enc = ~0ull;
        std::vector<TerminalRec> local_best(L);
        uint64_t max_new = 0;  // the most states one shard's table took this level
        bool level_tup = false;  // the level stopped at the deadline: partial
        for (int l = 0; l < (rep ? 1 : L); l++) {  // replicated: every shard has the same counts
          Shard& S = sh[l];
          gsum[0] += S.lc.new_states;
          max_new = std::max<uint64_t>(max_new, S.lc.new_states);
          level_tup |= S.lc.time_up != 0;
          uint64_t fn = 0;
          for (uint64_t c : ncnt[l]) fn += c;
          gsum[1] += fn;
          gsum[2] += S.lc.successors;
          gsum[3] += S.lc.err_overflow;
          gsum[4] += S.lc.err_table;
          gsum[5] += S.lc.err_frontier;
          gsum[6] += S.lc.work_items;
          gsum[7] += S.F;
          stats.parents += S.F;
          stats.work_items += S.lc.work_items;
          stats.new_states += S.lc.new_states;
          stats.probes += S.lc.probes;
          stats.deduped += S.lc.deduped;
          stats.appended += fn;
          if (S.lc.term_best && recs.empty()) {  // the level's exact best terminal (fold_terminals)
            const uint64_t key = ~(uint64_t)S.lc.term_best;
            DSL_TRY(resolve_terminal(S, key, depth + 1, depth > init_depth, &local_best[l]));
            enc = std::min<uint64_t>(enc, (key & ~(uint64_t)0xff) | (uint64_t)S.gid);
          }
        }
        if (!recs.empty()) {  // the gathered records: global sums, the best terminal, the next level's g
          std::fill(gsum.begin(), gsum.end(), 0);
          std::fill(g_next.begin(), g_next.end(), 0);
          max_new = 0;
          for (int x = 0; x < W; x++) {
            const uint64_t* r = recs.data() + (size_t)x * kRecWords;
            gsum[0] += r[kRecNew];
            max_new = std::max<uint64_t>(max_new, r[kRecNew]);
            level_tup |= r[kRecLevelTimeUp] != 0;
            gsum[1] += r[kRecRows];
            gsum[2] += r[kRecSucc];
            gsum[3] += r[kRecErrOverflow];
            gsum[4] += r[kRecErrTable];
            gsum[5] += r[kRecErrFrontier];
            gsum[6] += r[kRecWork];
            gsum[7] += r[kRecParents];
            enc = std::min<uint64_t>(enc, r[kRecTerm]);
            g_next[0] += r[kRecRows];
            g_next[1] = std::max<uint64_t>(g_next[1], r[kRecTimeUp]);
            g_next[2] += r[kRecNextWork];
          }
          have_g = true;
          for (int l = 0; l < L; l++) {
            Shard& S = sh[l];
            if (enc != ~0ull && (int)(enc & 0xff) == S.gid)  // this shard holds the level's best terminal
              DSL_TRY(resolve_terminal(S, ~(uint64_t)S.lc.term_best, depth + 1, depth > init_depth, &local_best[l]));
          }
        } else if (!rep) {
          DSL_TRY(global_sum(gsum));
          if (comm) {
            stats.host_syncs++;
            DSL_TRY(comm->allreduce_u64(&enc, 1, true, stream));
          }
        }
        if (route) first_sharded = false;
        if (gsum[3]) {
          set_error("a successor exceeded the packed state's bounds (" + std::to_string(gsum[3]) + " times)");
          return DSL_ERR_STATE_OVERFLOW;
        }
        if (gsum[4]) {
          set_error("visited table full: raise table_log2_slots");
          return DSL_ERR_TABLE_FULL;
        }
        if (gsum[5]) {
          set_error("next frontier exceeds capacity");
          return DSL_ERR_FRONTIER_FULL;
        }
        if (hset.max_frontier_states > 0 && gsum[1] > hset.max_frontier_states) {
          set_error("the frontier of depth " + std::to_string(depth + 1) + " holds " + std::to_string(gsum[1]) +
                    " states, more than max_frontier_states");
          return DSL_ERR_FRONTIER_FULL;
        }
        if (gsum[7]) avg_events_x16 = std::max<uint64_t>(16, (gsum[6] * 16 + gsum[7] - 1) / gsum[7]);
        if (level_tup && enc == ~0ull) {
          // the deadline passed inside the level (Search.java:313-318): its states count, but it is
          // not a completed depth; a terminal it found is still reported (below)
          successors += gsum[2];
          total_states += gsum[0];
          progress_states = total_states;
          end = DSL_TIME_EXHAUSTED;
          break;
        }
        depth++;
        successors += gsum[2];
        total_states += gsum[0];
        inserted += route ? max_new : gsum[0];  // per shard (an upper bound)
        prev_new = gsum[0];
        prev_work = gsum[6];
        if (gsum[1]) {  // the level's parents: gsum[7] when counted, else the last frontier
          front_growth = (double)gsum[1] / (double)(gsum[7] ? gsum[7] : prev_front);
          prev_front = gsum[1];
        }
        if (gsum[0]) per_depth.push_back(gsum[0]);
        max_front = std::max(max_front, gsum[1]);
        progress_states = total_states;
        progress_depth = depth;
        for (int l = 0; l < L; l++) {
          Shard& S = sh[l];
          S.level_size.push_back(span[l]);
        }
        const double lms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - lt0).count();
        level_ms_max = std::max(level_ms_max, lms);
        // the cost model (auto replicate_below): c from levels in the throughput regime, X from the
        // sharded levels that allocated nothing (a first search grows its buffers)
        if (!queued && kms > 0) {
          uint64_t lw = 0;
          for (auto& S : sh) lw += S.lc.work_items;
          if (lw >= 65536) {
            const double c = (double)kms * 1e6 / (double)lw;
            cost_c_ns = cost_c_ns > 0 ? std::min(cost_c_ns, c) : c;
          }
          if (route && n_reallocs + stats.table_rehashes == reallocs0) {
            x_sum_us += std::max(0.0, (lms - (double)kms) * 1000.0);
            x_levels++;
          }
        }
        if (trace_levels)
          fprintf(stderr, "[level] depth %d F=%llu new=%llu queued=%d wall_ms=%.4f kernel_ms=%.4f sharded=%d "
                  "routed=%llu reallocs=%llu\n", depth, (unsigned long long)gsum[7], (unsigned long long)gsum[0],
                  queued ? 1 : 0, lms, (double)kms, route ? 1 : 0, (unsigned long long)(exchanged - exchanged0),
                  (unsigned long long)n_reallocs);
        if (enc != ~0ull) {
          const int wrank = (int)(enc & 0xff);
          uint64_t rec[4] = {0, 0, 0, 0};
          for (int l = 0; l < L; l++)
            if (sh[l].gid == wrank) {
              const TerminalRec& b = local_best[l];
              rec[0] = ((uint64_t)wrank << 48) | b.parent;
              rec[1] = b.event;
              rec[2] = (uint64_t)b.verdict;
              rec[3] = (uint64_t)(b.pred_index + 1);
            }
          if (comm && !rep) DSL_TRY((stats.host_syncs++, comm->bcast_u64(rec, 4, wrank, stream)));
          const int v = (int)rec[2];
          end = v == V_TERM_EXCEPTION ? DSL_EXCEPTION_THROWN : v == V_TERM_INVARIANT ? DSL_INVARIANT_VIOLATED
                                                                                     : DSL_GOAL_FOUND;
          pred_index = v == V_TERM_EXCEPTION ? -1 : (int)rec[3] - 1;
          term_depth = depth;
          // walk parent pointers back level by level (across shards)
          std::vector<uint32_t> evs{(uint32_t)rec[1]};
          uint64_t ref = rec[0];
          const int nlev = (int)sh[0].level_size.size();
          for (int lev = nlev - 2; lev >= 1; lev--) {
            const int r = (int)(ref >> 48);
            const uint64_t idx = ref & ((1ull << 48) - 1);
            uint64_t hop[2] = {0, 0};
            for (int l = 0; l < L; l++)
              if (sh[l].gid == r) {
                uint64_t p;
                uint32_t e;
                DSL_HIP(hipMemcpy(&p, sh[l].hpar[lev] + idx, 8, hipMemcpyDeviceToHost));
                DSL_HIP(hipMemcpy(&e, sh[l].hev[lev] + idx, 4, hipMemcpyDeviceToHost));
                hop[0] = p;
                hop[1] = e;
              }
            // a terminal of a replicated level has a local chain on every rank: no exchange
            if (comm && !rep) DSL_TRY((stats.host_syncs++, comm->bcast_u64(hop, 2, r, stream)));
            evs.push_back((uint32_t)hop[1]);
            ref = hop[0];
          }
          std::reverse(evs.begin(), evs.end());
          trace_events = evs;
          break;
        }
        if (hset.do_checks != DSL_CHECKS_NONE)
          for (int l = 0; l < L; l++) DSL_TRY(run_checks(sh[l], nbase[l], ncnt[l]));
        if (gsum[1] == 0) break;
        for (int l = 0; l < L; l++) {
          Shard& S = sh[l];
          std::swap(S.cur, S.next);
          std::swap(S.cur_cap, S.next_cap);
          std::swap(S.cur_fp, S.next_fp);
          std::swap(S.curfp_cap, S.nextfp_cap);
          S.flip = !S.flip;
          S.seg_base = nbase[l];
          S.seg_cnt = ncnt[l];
          S.F = 0;
          for (uint64_t c : ncnt[l]) S.F += c;
          S.work = S.lc.next_work;
          if (!queued) S.cset ^= 1;  // queued levels used the queue's counter sets
        }
        if (queued) {
          q_pos++;
          q_left--;
        }
      }
    }
    if (trace_levels)
      fprintf(stderr, "[levels] %.4f ms\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
    // the search is over and no kernel of it is left to read the tables: zero them now, on the
    // stream, while the host assembles the result and the caller prepares the next search (whose
    // k_setup then only writes the seed); an error return above leaves table_clean false
    if (!getenv("DSL_SETUP_CLEAR")) {
      for (auto& S : sh) {
        DSL_HIP(hipMemsetAsync(S.table, 0, table_buckets * 64, stream));
        S.table_clean = true;
      }
      if (qctr) {
        DSL_HIP(hipMemsetAsync(qctr, 0, (size_t)(kQueue + 1) * kCtrSet, stream));
        qctr_clean = true;
      }
    }
    if (trace_levels)
      fprintf(stderr, "[clear] %.4f ms\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
    if (x_levels) cost_x_us = x_sum_us / (double)x_levels;
    if (q_span_adapt && L == 1) {
      uint64_t want = kQueueRowsMin;
      while (want < 4 * max_front && want < queue_span_max()) want <<= 1;
      q_span_want = std::max(q_span_want, want);
    }
    stats.exchanged = exchanged;
    if (comm && hset.do_checks != DSL_CHECKS_NONE) {
      // every rank checked a sample of its own shards' rows: the result carries the sums (the first
      // offending event of each kind stays the one this rank found, if any)
      uint64_t cv[3] = {chk_run, chk_nd, chk_ni};
      DSL_TRY((stats.host_syncs++, comm->allreduce_u64(cv, 3, false, stream)));
      chk_run = cv[0];
      chk_nd = cv[1];
      chk_ni = cv[2];
    }
    const double elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
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
    r->exchanged_states = exchanged;
    r->level_ms_max = level_ms_max;
    r->checks_run = chk_run;
    r->not_deterministic = chk_nd;
    r->not_idempotent = chk_ni;
    r->first_not_deterministic = chk_first_nd;
    r->first_not_idempotent = chk_first_ni;
    r->state_bytes = sizeof(init);
    if (term_depth >= 0) {
      // events replayed on the host from the initial state with the same transition code
      r->trace_len = (int)trace_events.size();
      r->trace = (dsl_event*)calloc(trace_events.size() + 1, sizeof(dsl_event));
      typename P::State s = init, n;
      for (size_t i = 0; i < trace_events.size(); i++) {
        describe_event<P>(s.w, (int)trace_events[i], prm, dset, &r->trace[i]);
        full_step<P>(s.w, (int)trace_events[i], n.w, prm, dset);
        s = n;
      }
      r->terminal_state = (uint8_t*)malloc(sizeof(init));
      std::memcpy(r->terminal_state, &s, sizeof(init));
      trace_events.clear();
    }
    if (trace_levels)
      fprintf(stderr, "[run] %.4f ms\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
    *out = r;
    return DSL_OK;
  }

  // Search.dfs on the device (k_dfs): see dsl_run_dfs in include/dslabs_hip.h.
  int run_dfs(const dsl_dfs_config& c, dsl_result** out) override {
    auto t_start = std::chrono::steady_clock::now();
    (void)hipGetLastError();
    if (W != 1) {
      set_error("random DFS runs on a single shard");
      return DSL_ERR_ARG;
    }
    if (!stream) {
      if (cfg.device >= 0) DSL_HIP(hipSetDevice(cfg.device));
      DSL_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
      DSL_HIP(hipEventCreate(&ev0));
      DSL_HIP(hipEventCreate(&ev1));
    }
    if (!have_init) {
      uint8_t tmp[sizeof(init)];
      DSL_TRY(get_initial(tmp, sizeof(init)));
    }
    const uint64_t np = c.probes > 0 ? (uint64_t)c.probes : 65536;
    const int steps = c.steps_per_launch > 0 ? c.steps_per_launch : 64;
    const int tcap = hset.max_depth >= 0 ? std::max(1, hset.max_depth - init_depth + 1)
                                         : (c.max_trace > 0 ? c.max_trace : 4096);
    struct Bufs {
      void* p[8] = {};
      ~Bufs() {
        for (void* q : p) (void)hipFree(q);
      }
    } b;
    uint32_t *rows, *trace, *dinit;
    int32_t *pdepth, *pcur, *found, *term;
    uint64_t* rng;
    unsigned long long* ctr;
    DSL_HIP(hipMalloc(&b.p[0], np * 2 * NW * 4));
    DSL_HIP(hipMalloc(&b.p[1], np * (uint64_t)tcap * 4));
    DSL_HIP(hipMalloc(&b.p[2], np * 4));
    DSL_HIP(hipMalloc(&b.p[3], np * 4));
    DSL_HIP(hipMalloc(&b.p[4], np * 8));
    DSL_HIP(hipMalloc(&b.p[5], 64));
    DSL_HIP(hipMalloc(&b.p[6], NW * 4));
    rows = (uint32_t*)b.p[0];
    trace = (uint32_t*)b.p[1];
    pdepth = (int32_t*)b.p[2];
    pcur = (int32_t*)b.p[3];
    rng = (uint64_t*)b.p[4];
    ctr = (unsigned long long*)b.p[5];
    found = (int32_t*)((char*)b.p[5] + 32);
    term = (int32_t*)((char*)b.p[5] + 36);
    dinit = (uint32_t*)b.p[6];
    std::vector<uint64_t> seeds(np);
    uint64_t x = c.seed ^ 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < np; i++) {  // splitmix64 per probe, never zero
      uint64_t z = (x += 0x9E3779B97F4A7C15ull);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      seeds[i] = (z ^ (z >> 31)) | 1;
    }
    DSL_HIP(hipMemcpyAsync(rng, seeds.data(), np * 8, hipMemcpyHostToDevice, stream));
    DSL_HIP(hipMemsetAsync(pdepth, 0xff, np * 4, stream));
    DSL_HIP(hipMemsetAsync(pcur, 0, np * 4, stream));
    DSL_HIP(hipMemsetAsync(b.p[5], 0, 64, stream));
    DSL_HIP(hipMemcpyAsync(dinit, init.w, NW * 4, hipMemcpyHostToDevice, stream));
    DfsArgs a{dinit, init_depth, tcap, rows, trace, pdepth, pcur, rng, np, steps, ctr, found, term};
    unsigned long long hc[3] = {0, 0, 0};
    int32_t hf[4] = {0, 0, 0, 0};
    int end = DSL_TIME_EXHAUSTED;
    // the initial state is checked once, as BFS does (RandomDFS.initSearch + the first probe)
    {
      int pi = -1;
      const NodeView v0{init.w, P::kNodeWords, -1, nullptr};
      const int v = judge_view<P>(v0, prm, dset, init_depth, &pi);
      if (v >= V_TERM_EXCEPTION) {
        dsl_result* r = (dsl_result*)calloc(1, sizeof(dsl_result));
        r->end_condition = v == V_TERM_INVARIANT ? DSL_INVARIANT_VIOLATED : DSL_GOAL_FOUND;
        r->terminal_depth = init_depth;
        r->predicate_index = pi;
        r->states = 1;
        r->initial_depth = init_depth;
        r->state_bytes = sizeof(init);
        r->trace = (dsl_event*)calloc(1, sizeof(dsl_event));
        r->terminal_state = (uint8_t*)malloc(sizeof(init));
        std::memcpy(r->terminal_state, &init, sizeof(init));
        *out = r;
        return DSL_OK;
      }
    }
    const int blocks = (int)((np + kBlock - 1) / kBlock);
    while (true) {
      hipLaunchKernelGGL(k_dfs<P>, dim3(blocks), dim3(kBlock), 0, stream, a, prm, dset);
      DSL_HIP(hipGetLastError());
      DSL_HIP(hipMemcpyAsync(hc, ctr, 24, hipMemcpyDeviceToHost, stream));
      DSL_HIP(hipMemcpyAsync(hf, found, 16, hipMemcpyDeviceToHost, stream));
      DSL_TRY(hsync());
      progress_states = hc[0];
      if (hc[2]) {
        set_error("a successor exceeded the packed state's bounds");
        return DSL_ERR_STATE_OVERFLOW;
      }
      if (hf[0]) break;
      if (c.max_probes > 0 && hc[1] >= (uint64_t)c.max_probes) break;
      const double el = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
      if (hset.max_time_ms > 0 && el > hset.max_time_ms) break;
      if (hset.max_time_ms <= 0 && c.max_probes <= 0) {
        set_error("random DFS needs a time limit (maxTimeSecs) or a probe budget");
        return DSL_ERR_ARG;
      }
    }
    const double elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    dsl_result* r = (dsl_result*)calloc(1, sizeof(dsl_result));
    r->states = hc[0];
    r->initial_depth = init_depth;
    r->elapsed_s = elapsed;
    r->successors = hc[0];
    r->state_bytes = sizeof(init);
    r->terminal_depth = -1;
    r->predicate_index = -1;
    if (hf[0]) {
      const int v = hf[1], depth = hf[3];
      end = v == V_TERM_EXCEPTION ? DSL_EXCEPTION_THROWN : v == V_TERM_INVARIANT ? DSL_INVARIANT_VIOLATED
                                                                                 : DSL_GOAL_FOUND;
      r->predicate_index = v == V_TERM_EXCEPTION ? -1 : hf[2];
      const uint64_t who = (uint64_t)(hf[0] - 1);
      std::vector<uint32_t> evs(std::min(depth, tcap));
      DSL_HIP(hipMemcpy(evs.data(), trace + who * tcap, evs.size() * 4, hipMemcpyDeviceToHost));
      r->terminal_depth = init_depth + depth;
      r->max_depth = r->terminal_depth;
      r->trace_len = (int)evs.size();
      r->trace = (dsl_event*)calloc(evs.size() + 1, sizeof(dsl_event));
      typename P::State s = init, n;
      for (size_t i = 0; i < evs.size(); i++) {  // replayed on the host with the same transitions
        describe_event<P>(s.w, (int)evs[i], prm, dset, &r->trace[i]);
        full_step<P>(s.w, (int)evs[i], n.w, prm, dset);
        s = n;
      }
      if (!c.no_minimize) {  // RandomDFS reports the minimized trace (checkState(s, true))
        TraceTool<P> tt(prm, dset);
        std::vector<dsl_event> ev(r->trace, r->trace + r->trace_len);
        typename TraceTool<P>::Step last{s, v == V_TERM_EXCEPTION};
        tt.minimize(typename TraceTool<P>::Step{init, false}, ev, &last,
                    tt.expected(v, hf[2], s));
        std::memcpy(r->trace, ev.data(), ev.size() * sizeof(dsl_event));
        r->trace_len = (int)ev.size();
        r->terminal_depth = r->max_depth = init_depth + (int)ev.size();
        s = last.s;
      }
      r->terminal_state = (uint8_t*)malloc(sizeof(init));
      std::memcpy(r->terminal_state, &s, sizeof(init));
    }
    r->end_condition = end;
    r->new_states_inserted = hc[1];  // probes started
    *out = r;
    return DSL_OK;
  }

  // dsl_human_readable_trace: SearchState.humanReadableTrace on the host (replay.hpp).
  int human_readable(const dsl_event* tr, int n, dsl_result** out) override {
    if (!have_init) {
      uint8_t tmp[sizeof(init)];
      DSL_TRY(get_initial(tmp, sizeof(init)));
    }
    TraceTool<P> tt(prm, dset);
    std::vector<dsl_event> evs(tr, tr + n);
    typename P::State last = init;
    {  // the end state of the trace as given (kept if the reordering cannot be replayed)
      typename TraceTool<P>::Step cur{init, false};
      for (const auto& e : evs) {
        typename TraceTool<P>::Step nx;
        if (tt.step(tt.open, cur.s, e, &nx) != 1) {
          set_error("the trace does not apply to the initial state");
          return DSL_ERR_ARG;
        }
        cur = nx;
      }
      last = cur.s;
    }
    tt.human_readable(init, evs, &last);
    dsl_result* r = (dsl_result*)calloc(1, sizeof(dsl_result));
    r->end_condition = DSL_SPACE_EXHAUSTED;
    r->predicate_index = -1;
    r->terminal_depth = r->max_depth = init_depth + (int)evs.size();
    r->initial_depth = init_depth;
    r->state_bytes = sizeof(init);
    r->trace_len = (int)evs.size();
    r->trace = (dsl_event*)calloc(evs.size() + 1, sizeof(dsl_event));
    if (!evs.empty()) std::memcpy(r->trace, evs.data(), evs.size() * sizeof(dsl_event));
    r->terminal_state = (uint8_t*)malloc(sizeof(init));
    std::memcpy(r->terminal_state, &last, sizeof(init));
    *out = r;
    return DSL_OK;
  }

  // dsl_replay: TraceReplaySearch on the host (replay.hpp).
  int replay(const dsl_event* tr, int n, int minimize, dsl_result** out) override {
    const auto t_start = std::chrono::steady_clock::now();
    if (!have_init) {
      uint8_t tmp[sizeof(init)];
      DSL_TRY(get_initial(tmp, sizeof(init)));
    }
    using Step = typename TraceTool<P>::Step;
    TraceTool<P> tt(prm, dset);
    Step cur{init, false};
    std::vector<dsl_event> evs;
    int pi = -1;
    uint64_t checked = 1;
    int v = tt.judge(cur, init_depth, &pi);  // checkState(initial, false)
    if (v < V_TERM_EXCEPTION) {
      for (int i = 0; i < n; i++) {
        Step nx;
        const int rc = tt.step(dset, cur.s, tr[i], &nx);
        if (rc < 0) {
          set_error("a replayed successor exceeded the packed state's bounds");
          return DSL_ERR_STATE_OVERFLOW;
        }
        if (rc == 0) break;  // cannot be delivered: the replay ends (eventsExhausted)
        cur = nx;
        evs.push_back(tr[i]);
        checked++;
        v = tt.judge(cur, init_depth + (int)evs.size(), &pi);
        if (v >= V_TERM_EXCEPTION) {
          if (minimize) tt.minimize(Step{init, false}, evs, &cur, tt.expected(v, pi, cur.s));
          break;
        }
      }
    }
    const bool term = v >= V_TERM_EXCEPTION;
    dsl_result* r = (dsl_result*)calloc(1, sizeof(dsl_result));
    r->end_condition = !term ? DSL_SPACE_EXHAUSTED
                             : v == V_TERM_EXCEPTION ? DSL_EXCEPTION_THROWN
                                                     : v == V_TERM_INVARIANT ? DSL_INVARIANT_VIOLATED : DSL_GOAL_FOUND;
    r->predicate_index = term && v != V_TERM_EXCEPTION ? pi : -1;
    r->terminal_depth = term ? init_depth + (int)evs.size() : -1;
    r->max_depth = init_depth + (int)evs.size();
    r->initial_depth = init_depth;
    r->states = checked;
    r->state_bytes = sizeof(init);
    r->trace_len = (int)evs.size();
    r->trace = (dsl_event*)calloc(evs.size() + 1, sizeof(dsl_event));
    if (!evs.empty()) std::memcpy(r->trace, evs.data(), evs.size() * sizeof(dsl_event));
    r->terminal_state = (uint8_t*)malloc(sizeof(init));
    std::memcpy(r->terminal_state, &cur.s, sizeof(init));
    r->elapsed_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    *out = r;
    return DSL_OK;
  }
};

}  // namespace dsl
