// engine.hip -- libdslabs_hip.so: C ABI (include/dslabs_hip.h) over the templated engine.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <string>

#include "bfs_engine.hpp"
#include "settings.hpp"
#include "protocols/all.hpp"

#ifdef DSL_WITH_RCCL
#include <rccl/rccl.h>
#endif

namespace dsl {

#ifdef DSL_WITH_RCCL
// One communicator per engine (one rank per GPU). Small host-visible collectives are staged
// through a device scratch buffer on the engine's stream.
struct RcclComm : Comm {
  ncclComm_t c = nullptr;
  int r = 0, n = 1;
  uint64_t* dbuf = nullptr;  // 2 * (kMaxShards * 64) u64
  static constexpr int kScratch = 2 * kMaxShards * 64;
  const double timeout_ms = getenv("DSL_COMM_TIMEOUT_MS") ? atof(getenv("DSL_COMM_TIMEOUT_MS")) : 300000.0;
  hipEvent_t ev = nullptr;  // recorded before each collective: the deadline starts when it is reached
  bool ev_set = false;
  ~RcclComm() override {
    if (c) ncclCommDestroy(c);
    hipFree(dbuf);
    if (ev) hipEventDestroy(ev);
  }
  void mark(hipStream_t st) {
    if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return;
    if (hipEventRecord(ev, st) == hipSuccess) ev_set = true;
  }
  bool collective_reached() override { return ev_set && hipEventQuery(ev) == hipSuccess; }
  void synced() override { ev_set = false; }
  int async_error() override {
    if (!c) return DSL_ERR_COMM;
    ncclResult_t st = ncclSuccess;
    if (ncclCommGetAsyncError(c, &st) != ncclSuccess) return DSL_ERR_COMM;
    if (st != ncclSuccess && st != ncclInProgress) {
      set_error(std::string("RCCL asynchronous error: ") + ncclGetErrorString(st));
      return DSL_ERR_COMM;
    }
    return DSL_OK;
  }
  void abort() override {
    if (c) (void)ncclCommAbort(c);
    c = nullptr;
  }
  // The small host-read collectives wait for their result polling the communicator's error and a
  // deadline (a dead peer aborts the communicator instead of blocking this rank forever); the
  // deadline counts from the moment the stream reached the collective (mark), not from the local
  // kernels enqueued before it.
  int wait(hipStream_t st) {
    auto t0 = std::chrono::steady_clock::now();
    hipError_t e;
    for (uint64_t it = 0; (e = hipStreamQuery(st)) == hipErrorNotReady; it++) {
      if ((it & 1023) == 1023) {
        const auto now = std::chrono::steady_clock::now();
        if (!collective_reached()) t0 = now;
        if (async_error() != DSL_OK || std::chrono::duration<double, std::milli>(now - t0).count() > timeout_ms) {
          abort();
          set_error("RCCL collective failed or timed out on rank " + std::to_string(r) + " (communicator aborted)");
          return DSL_ERR_COMM;
        }
      }
    }
    if (e != hipSuccess) {
      set_error(std::string("HIP error ") + hipGetErrorString(e) + " in an RCCL collective");
      return DSL_ERR_HIP;
    }
    ev_set = false;  // the stream is drained
    return DSL_OK;
  }
  int rank() const override { return r; }
  int size() const override { return n; }
  static int ck(ncclResult_t e, const char* what) {
    if (e != ncclSuccess) {
      set_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(e));
      return DSL_ERR_COMM;
    }
    return DSL_OK;
  }
  int allgather_u64(const uint64_t* in, int k, uint64_t* out, hipStream_t st) override {
    if (!c) return DSL_ERR_COMM;
    if (k * (n + 1) > kScratch) return DSL_ERR_ARG;
    mark(st);
    DSL_HIP(hipMemcpyAsync(dbuf, in, k * 8, hipMemcpyHostToDevice, st));
    int rc = ck(ncclAllGather(dbuf, dbuf + k, k, ncclUint64, c, st), "allgather");
    if (rc) return rc;
    DSL_HIP(hipMemcpyAsync(out, dbuf + k, (size_t)k * n * 8, hipMemcpyDeviceToHost, st));
    return wait(st);
  }
  int allreduce_u64(uint64_t* v, int k, bool min, hipStream_t st) override {
    if (!c) return DSL_ERR_COMM;
    if (k > kScratch) return DSL_ERR_ARG;
    mark(st);
    DSL_HIP(hipMemcpyAsync(dbuf, v, k * 8, hipMemcpyHostToDevice, st));
    int rc = ck(ncclAllReduce(dbuf, dbuf, k, ncclUint64, min ? ncclMin : ncclSum, c, st), "allreduce");
    if (rc) return rc;
    DSL_HIP(hipMemcpyAsync(v, dbuf, k * 8, hipMemcpyDeviceToHost, st));
    return wait(st);
  }
  int bcast_u64(uint64_t* v, int k, int root, hipStream_t st) override {
    if (!c) return DSL_ERR_COMM;
    if (k > kScratch) return DSL_ERR_ARG;
    mark(st);
    DSL_HIP(hipMemcpyAsync(dbuf, v, k * 8, hipMemcpyHostToDevice, st));
    int rc = ck(ncclBroadcast(dbuf, dbuf, k, ncclUint64, root, c, st), "broadcast");
    if (rc) return rc;
    DSL_HIP(hipMemcpyAsync(v, dbuf, k * 8, hipMemcpyDeviceToHost, st));
    return wait(st);
  }
  bool device_collectives() const override { return true; }
  int allgather_dev(const uint64_t* d_in, int k, uint64_t* d_out, hipStream_t st) override {
    if (!c) return DSL_ERR_COMM;
    mark(st);
    return ck(ncclAllGather(d_in, d_out, k, ncclUint64, c, st), "allgather");
  }
  int ver = 0;
  int version() const override { return ver; }
  int alltoallv(const uint8_t* send, const uint64_t* so, const uint64_t* sb, uint8_t* recv, const uint64_t* ro,
                const uint64_t* rb, hipStream_t st) override {
    if (!c) return DSL_ERR_COMM;
    mark(st);
    int rc = ck(ncclGroupStart(), "group start");
    if (rc) return rc;
    for (int p = 0; p < n; p++) {
      if (p == r) continue;
      if (sb[p]) {
        rc = ck(ncclSend(send + so[p], sb[p], ncclUint8, p, c, st), "send");
        if (rc) break;
      }
      if (rb[p]) {
        rc = ck(ncclRecv(recv + ro[p], rb[p], ncclUint8, p, c, st), "recv");
        if (rc) break;
      }
    }
    int rc2 = ck(ncclGroupEnd(), "group end");
    return rc ? rc : rc2;
  }
};

static int make_comm(const dsl_engine_config& cfg, Comm** out) {
  auto* cm = new RcclComm();
  cm->r = cfg.rank;
  cm->n = cfg.world_size;
  if (cfg.device >= 0) {
    hipError_t e = hipSetDevice(cfg.device);
    if (e != hipSuccess) {
      delete cm;
      set_error("hipSetDevice failed");
      return DSL_ERR_HIP;
    }
  }
  if (hipMalloc(&cm->dbuf, RcclComm::kScratch * 8) != hipSuccess) {
    delete cm;
    set_error("hipMalloc failed");
    return DSL_ERR_HIP;
  }
  ncclUniqueId id;
  std::memcpy(&id, cfg.comm_id, sizeof(id));
  int rc = RcclComm::ck(ncclCommInitRank(&cm->c, cfg.world_size, id, cfg.rank), "comm init");
  if (rc) {
    delete cm;
    return rc;
  }
  (void)ncclGetVersion(&cm->ver);  // reported in dsl_stats.rccl_version (which RCCL this process bound)
  *out = cm;
  return DSL_OK;
}
#else
static int make_comm(const dsl_engine_config&, Comm**) {
  set_error("built without RCCL: multi-GPU unavailable");
  return DSL_ERR_COMM;
}
#endif

// Transport provided by the caller through dsl_host_comm (host buffers).
struct HostComm : Comm {
  dsl_host_comm h;
  std::vector<uint8_t> sbuf, rbuf;
  explicit HostComm(const dsl_host_comm& x) : h(x) {}
  int rank() const override { return h.rank; }
  int size() const override { return h.size; }
  int allgather_u64(const uint64_t* in, int n, uint64_t* out, hipStream_t) override {
    return h.allgather_u64(h.ctx, in, n, out) ? DSL_ERR_COMM : DSL_OK;
  }
  int allreduce_u64(uint64_t* v, int n, bool min, hipStream_t) override {
    return h.allreduce_u64(h.ctx, v, n, min ? 1 : 0) ? DSL_ERR_COMM : DSL_OK;
  }
  int bcast_u64(uint64_t* v, int n, int root, hipStream_t) override {
    return h.bcast_u64(h.ctx, v, n, root) ? DSL_ERR_COMM : DSL_OK;
  }
  // DSL_HOST_COMM_DEVICE_COLLECTIVES: the engine runs its RCCL branches (device gathers enqueued on
  // its stream); each device gather is emulated here by a copy of the rank's words to the host, the
  // caller's allgather and a copy of the gathered words back, all before returning. This is test
  // plumbing for the bookkeeping of those branches, not a fast path.
  std::vector<uint64_t> gin, gout;
  bool device_collectives() const override { return (h.flags & DSL_HOST_COMM_DEVICE_COLLECTIVES) != 0; }
  int allgather_dev(const uint64_t* d_in, int k, uint64_t* d_out, hipStream_t st) override {
    if (!device_collectives()) return DSL_ERR_COMM;
    gin.resize(k);
    gout.resize((size_t)k * h.size);
    DSL_HIP(hipMemcpyAsync(gin.data(), d_in, (size_t)k * 8, hipMemcpyDeviceToHost, st));
    DSL_HIP(hipStreamSynchronize(st));
    if (h.allgather_u64(h.ctx, gin.data(), k, gout.data())) return DSL_ERR_COMM;
    DSL_HIP(hipMemcpyAsync(d_out, gout.data(), gout.size() * 8, hipMemcpyHostToDevice, st));
    DSL_HIP(hipStreamSynchronize(st));  // gout is pageable host memory: the copy completes here
    return DSL_OK;
  }
  int alltoallv(const uint8_t* send, const uint64_t* so, const uint64_t* sb, uint8_t* recv, const uint64_t* ro,
                const uint64_t* rb, hipStream_t st) override {
    const int n = h.size;
    std::vector<uint64_t> hso(n), hro(n);
    uint64_t stot = 0, rtot = 0;
    for (int p = 0; p < n; p++) {
      hso[p] = stot;
      stot += sb[p];
      hro[p] = rtot;
      rtot += rb[p];
    }
    sbuf.resize(stot + 1);
    rbuf.resize(rtot + 1);
    for (int p = 0; p < n; p++)
      if (sb[p]) DSL_HIP(hipMemcpyAsync(sbuf.data() + hso[p], send + so[p], sb[p], hipMemcpyDeviceToHost, st));
    DSL_HIP(hipStreamSynchronize(st));
    if (h.alltoallv(h.ctx, sbuf.data(), hso.data(), sb, rbuf.data(), hro.data(), rb)) return DSL_ERR_COMM;
    for (int p = 0; p < n; p++)
      if (rb[p]) DSL_HIP(hipMemcpyAsync(recv + ro[p], rbuf.data() + hro[p], rb[p], hipMemcpyHostToDevice, st));
    DSL_HIP(hipStreamSynchronize(st));
    return DSL_OK;
  }
};

static thread_local const dsl_host_comm* g_pending_host_comm = nullptr;


static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

int resolve_settings(const dsl_settings& in, int num_nodes, bool (*known)(int), DevSettings* out) {
  std::string why;
  const int rc = resolve_settings(in, num_nodes, known, out, &why);
  if (rc) set_error(why);
  return rc;
}

template <class P>
static int make_engine(const dsl_protocol_desc& d, const dsl_engine_config& cfg, EngineBase** out) {
  typename P::Params prm = P::from_desc(d);
  if (!P::valid(prm)) {
    set_error("invalid protocol parameters");
    return DSL_ERR_ARG;
  }
  if (cfg.world_size > 1 || (cfg.flags & DSL_CFG_RCCL_AT_WORLD_1)) {
    if (cfg.world_size > kMaxShards || cfg.rank < 0 || cfg.rank >= cfg.world_size) return DSL_ERR_ARG;
    Comm* cm = nullptr;
    if (g_pending_host_comm) {
      cm = new HostComm(*g_pending_host_comm);
    } else {
      int rc = make_comm(cfg, &cm);
      if (rc) return rc;
    }
    *out = new BfsEngine<P>(prm, cfg, cfg.world_size, cm);
  } else if (cfg.virtual_shards > 1) {
    if (cfg.virtual_shards > kMaxShards) return DSL_ERR_ARG;
    *out = new BfsEngine<P>(prm, cfg, cfg.virtual_shards, nullptr);
  } else {
    *out = new BfsEngine<P>(prm, cfg, 1, nullptr);
  }
  return DSL_OK;
}

static int create_any(const dsl_protocol_desc& d, const dsl_engine_config& cfg, EngineBase** out) {
  switch (d.protocol) {
#ifdef DSL_ONLY_MULTIPAXOS  // measurement variants (tools/build_variant.sh): C5's protocol (hand-written, IR), fast builds
    case DSL_PROTO_MULTIPAXOS: return make_engine<MultiPaxos>(d, cfg, out);
    case DSL_PROTO_MULTIPAXOS_IR: return make_engine<MultiPaxosIR>(d, cfg, out);
#elif defined(DSL_ONLY_SYNTHETIC)  // measurement variants: C3's protocol only
    case DSL_PROTO_SYNTHETIC: return make_engine<Synthetic>(d, cfg, out);
#else
    case DSL_PROTO_PINGPONG: return make_engine<PingPong>(d, cfg, out);
    case DSL_PROTO_SIPAXOS: return make_engine<SIPaxos>(d, cfg, out);
    case DSL_PROTO_MULTIPAXOS: return make_engine<MultiPaxos>(d, cfg, out);
    case DSL_PROTO_SYNTHETIC: return make_engine<Synthetic>(d, cfg, out);
    case DSL_PROTO_AMOKV: return make_engine<AmoKV>(d, cfg, out);
    case DSL_PROTO_PB: return make_engine<PB>(d, cfg, out);
    case DSL_PROTO_MINITEST: return make_engine<MiniTest>(d, cfg, out);
    case DSL_PROTO_PINGPONG_IR: return make_engine<PingPongIR>(d, cfg, out);
    case DSL_PROTO_AMOKV_IR: return make_engine<AmoKVIR>(d, cfg, out);
    case DSL_PROTO_MULTIPAXOS_IR: return make_engine<MultiPaxosIR>(d, cfg, out);
    case DSL_PROTO_PB_IR: return make_engine<PBIR>(d, cfg, out);
#endif
    default:
      set_error("unknown protocol id " + std::to_string(d.protocol));
      return DSL_ERR_UNKNOWN_PROTOCOL;
  }
}

// dsl_drop_pending_messages / dsl_undrop_messages over one protocol's packed network.
template <class P>
static int drop_pending(uint8_t* packed, size_t len, uint64_t* dropped, int32_t cap, int32_t* n) {
  using S = typename P::State;
  if (len != sizeof(S) || *n < 0 || *n > cap) return DSL_ERR_ARG;
  S st;
  std::memcpy(&st, packed, sizeof(S));
  std::vector<uint64_t> d(dropped, dropped + *n);
  for (int i = 0; i < Net<P>::size(st.w); i++) d.push_back((uint64_t)Net<P>::at(st.w, i));
  std::sort(d.begin(), d.end());
  d.erase(std::unique(d.begin(), d.end()), d.end());
  if ((int64_t)d.size() > cap) return DSL_ERR_ARG;
  for (int i = 0; i < Net<P>::size(st.w); i++) Net<P>::put(st.w, i, 0);
  st.w[Layout<P>::kNetCount] = 0;
  std::memcpy(packed, &st, sizeof(S));
  std::copy(d.begin(), d.end(), dropped);
  *n = (int32_t)d.size();
  return DSL_OK;
}
template <class P>
static int init_packed(const dsl_protocol_desc& d, uint8_t* packed, size_t len) {
  using S = typename P::State;
  const typename P::Params prm = P::from_desc(d);
  if (len != sizeof(S) || !P::valid(prm)) return DSL_ERR_ARG;
  S st;
  if (!init_state<P>(st.w, prm)) {
    set_error("initial state exceeds the protocol's network capacity");
    return DSL_ERR_STATE_OVERFLOW;
  }
  std::memcpy(packed, &st, sizeof(S));
  return DSL_OK;
}
template <class P>
static int undrop(uint8_t* packed, size_t len, const uint64_t* dropped, int32_t n, int32_t from, int32_t to) {
  using S = typename P::State;
  if (len != sizeof(S) || n < 0) return DSL_ERR_ARG;
  S st;
  std::memcpy(&st, packed, sizeof(S));
  for (int i = 0; i < n; i++) {
    const auto r = (typename P::Rec)dropped[i];
    if ((from >= 0 && P::rec_from(r) != from) || (to >= 0 && P::rec_to(r) != to)) continue;
    if (Net<P>::insert(st.w, r) < 0) {
      set_error("undropped network exceeds the protocol's network capacity");
      return DSL_ERR_STATE_OVERFLOW;
    }
  }
  std::memcpy(packed, &st, sizeof(S));
  return DSL_OK;
}

}  // namespace dsl

struct dsl_engine {
  dsl::EngineBase* impl;
};

extern "C" {

int dsl_abi_version(void) { return DSL_ABI_VERSION; }

int dsl_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* dsl_last_error(void) { return dsl::g_last_error.c_str(); }

int dsl_state_bytes(const dsl_protocol_desc* proto) {
  if (!proto) return DSL_ERR_ARG;
  switch (proto->protocol) {
    case DSL_PROTO_PINGPONG: return (int)sizeof(dsl::PingPong::State);
    case DSL_PROTO_SIPAXOS: return (int)sizeof(dsl::SIPaxos::State);
    case DSL_PROTO_MULTIPAXOS: return (int)sizeof(dsl::MultiPaxos::State);
    case DSL_PROTO_SYNTHETIC: return (int)sizeof(dsl::Synthetic::State);
    case DSL_PROTO_AMOKV: return (int)sizeof(dsl::AmoKV::State);
    case DSL_PROTO_PB: return (int)sizeof(dsl::PB::State);
    case DSL_PROTO_MINITEST: return (int)sizeof(dsl::MiniTest::State);
    case DSL_PROTO_PINGPONG_IR: return (int)sizeof(dsl::PingPongIR::State);
    case DSL_PROTO_AMOKV_IR: return (int)sizeof(dsl::AmoKVIR::State);
    case DSL_PROTO_MULTIPAXOS_IR: return (int)sizeof(dsl::MultiPaxosIR::State);
    case DSL_PROTO_PB_IR: return (int)sizeof(dsl::PBIR::State);
    default: return DSL_ERR_UNKNOWN_PROTOCOL;
  }
}

#define DSL_PROTO_DISPATCH(call)                                        \
  switch (proto->protocol) {                                            \
    case DSL_PROTO_PINGPONG: { using P = dsl::PingPong; return call; }     \
    case DSL_PROTO_SIPAXOS: { using P = dsl::SIPaxos; return call; }       \
    case DSL_PROTO_MULTIPAXOS: { using P = dsl::MultiPaxos; return call; } \
    case DSL_PROTO_SYNTHETIC: { using P = dsl::Synthetic; return call; }   \
    case DSL_PROTO_AMOKV: { using P = dsl::AmoKV; return call; }           \
    case DSL_PROTO_PB: { using P = dsl::PB; return call; }                 \
    case DSL_PROTO_MINITEST: { using P = dsl::MiniTest; return call; }     \
    case DSL_PROTO_PINGPONG_IR: { using P = dsl::PingPongIR; return call; } \
    case DSL_PROTO_AMOKV_IR: { using P = dsl::AmoKVIR; return call; }       \
    case DSL_PROTO_MULTIPAXOS_IR: { using P = dsl::MultiPaxosIR; return call; } \
    case DSL_PROTO_PB_IR: { using P = dsl::PBIR; return call; }           \
    default: return DSL_ERR_UNKNOWN_PROTOCOL;                           \
  }

int dsl_init_state(const dsl_protocol_desc* proto, uint8_t* packed, size_t len) {
  if (!proto || !packed) return DSL_ERR_ARG;
  DSL_PROTO_DISPATCH((dsl::init_packed<P>(*proto, packed, len)))
}

int dsl_drop_pending_messages(const dsl_protocol_desc* proto, uint8_t* packed, size_t len, uint64_t* dropped,
                              int32_t cap, int32_t* n_dropped) {
  if (!proto || !packed || !n_dropped || (cap > 0 && !dropped)) return DSL_ERR_ARG;
  DSL_PROTO_DISPATCH((dsl::drop_pending<P>(packed, len, dropped, cap, n_dropped)))
}

int dsl_undrop_messages(const dsl_protocol_desc* proto, uint8_t* packed, size_t len, const uint64_t* dropped,
                        int32_t n_dropped, int32_t from, int32_t to) {
  if (!proto || !packed || (n_dropped > 0 && !dropped)) return DSL_ERR_ARG;
  DSL_PROTO_DISPATCH((dsl::undrop<P>(packed, len, dropped, n_dropped, from, to)))
}

int dsl_comm_unique_id(uint8_t out[128]) {
  if (!out) return DSL_ERR_ARG;
#ifdef DSL_WITH_RCCL
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) {
    dsl::set_error("ncclGetUniqueId failed");
    return DSL_ERR_COMM;
  }
  std::memcpy(out, &id, sizeof(id));
  return DSL_OK;
#else
  dsl::set_error("built without RCCL");
  return DSL_ERR_COMM;
#endif
}

int dsl_create(const dsl_protocol_desc* proto, const dsl_engine_config* cfg, dsl_engine** out) {
  if (!proto || !out) return DSL_ERR_ARG;
  int ndev = dsl_device_count();
  if (ndev <= 0) {
    dsl::set_error("no HIP device visible: the MI355X engine has no CPU fallback");
    return DSL_ERR_NO_DEVICE;
  }
  dsl_engine_config c{};
  c.device = -1;
  c.world_size = 1;
  c.replicate_below = -1;
  if (cfg) c = *cfg;
  if (c.world_size < 1) c.world_size = 1;
  dsl::EngineBase* impl = nullptr;
  int rc = dsl::create_any(*proto, c, &impl);
  if (rc) return rc;
  *out = new dsl_engine{impl};
  return DSL_OK;
}

int dsl_create_with_host_comm(const dsl_protocol_desc* proto, const dsl_engine_config* cfg,
                              const dsl_host_comm* comm, dsl_engine** out) {
  if (!proto || !cfg || !comm || !out || comm->size != cfg->world_size || comm->rank != cfg->rank ||
      !comm->allgather_u64 || !comm->allreduce_u64 || !comm->bcast_u64 || !comm->alltoallv)
    return DSL_ERR_ARG;
  dsl::g_pending_host_comm = comm;
  int rc = dsl_create(proto, cfg, out);
  dsl::g_pending_host_comm = nullptr;
  return rc;
}

int dsl_set_settings(dsl_engine* e, const dsl_settings* s) {
  if (!e || !s) return DSL_ERR_ARG;
  return e->impl->set_settings(*s);
}

int dsl_set_initial(dsl_engine* e, const uint8_t* packed, size_t len, int32_t depth) {
  if (!e || !packed) return DSL_ERR_ARG;
  return e->impl->set_initial(packed, len, depth);
}

int dsl_set_dropped(dsl_engine* e, const uint64_t* dropped, int32_t n_dropped) {
  if (!e) return DSL_ERR_ARG;
  return e->impl->set_dropped(dropped, n_dropped);
}

int dsl_get_initial(dsl_engine* e, uint8_t* packed, size_t len) {
  if (!e || !packed) return DSL_ERR_ARG;
  return e->impl->get_initial(packed, len);
}

int dsl_run(dsl_engine* e, dsl_result** out) {
  if (!e || !out) return DSL_ERR_ARG;
  *out = nullptr;
  return e->impl->run(out);
}

int dsl_run_dfs(dsl_engine* e, const dsl_dfs_config* cfg, dsl_result** out) {
  if (!e || !out) return DSL_ERR_ARG;
  *out = nullptr;
  dsl_dfs_config c{};
  if (cfg) c = *cfg;
  return e->impl->run_dfs(c, out);
}

int dsl_replay(dsl_engine* e, const dsl_event* trace, int32_t n, int32_t minimize, dsl_result** out) {
  if (!e || !out || n < 0 || (n > 0 && !trace)) return DSL_ERR_ARG;
  *out = nullptr;
  return e->impl->replay(trace, n, minimize, out);
}

int dsl_human_readable_trace(dsl_engine* e, const dsl_event* trace, int32_t n, dsl_result** out) {
  if (!e || !out || n < 0 || (n > 0 && !trace)) return DSL_ERR_ARG;
  *out = nullptr;
  return e->impl->human_readable(trace, n, out);
}

int dsl_progress(dsl_engine* e, uint64_t* states, int32_t* depth) {
  if (!e) return DSL_ERR_ARG;
  if (states) *states = e->impl->progress_states;
  if (depth) *depth = e->impl->progress_depth;
  return DSL_OK;
}

int dsl_kernel_stats(dsl_engine* e, dsl_stats* out) {
  if (!e || !out) return DSL_ERR_ARG;
  *out = e->impl->stats;
  return DSL_OK;
}

void dsl_result_free(dsl_result* r) {
  if (!r) return;
  free(r->per_depth);
  free(r->trace);
  free(r->terminal_state);
  free(r);
}

void dsl_destroy(dsl_engine* e) {
  if (!e) return;
  delete e->impl;
  delete e;
}

}  // extern "C"
