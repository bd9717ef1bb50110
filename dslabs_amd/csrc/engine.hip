// engine.hip -- libdslabs_hip.so: C ABI (include/dslabs_hip.h) over the templated engine.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>
#include <mutex>
#include <string>

#include "engine.hpp"
#include "protocols/all.hpp"

namespace dsl {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// TestSettings.shouldDeliver precedence (TestSettings.java:224-245): self-send always; then
// link override, sender override, receiver override, global networkActive.
// TestSettings.deliverTimers(a): per-address override else the global flag (:87-89).
int resolve_settings(const dsl_settings& in, int num_nodes, bool (*known)(int), DevSettings* out) {
  DevSettings d{};
  if (num_nodes > DSL_MAX_NODES) return DSL_ERR_ARG;
  for (int f = 0; f < num_nodes; f++) {
    uint32_t row = 0;
    for (int t = 0; t < num_nodes; t++) {
      bool ok;
      if (f == t) ok = true;
      else if (in.link_active[f][t] >= 0) ok = in.link_active[f][t] != 0;
      else if (in.sender_active[f] >= 0) ok = in.sender_active[f] != 0;
      else if (in.receiver_active[t] >= 0) ok = in.receiver_active[t] != 0;
      else ok = in.network_active != 0;
      if (ok) row |= 1u << t;
    }
    d.deliver[f] = row;
  }
  for (int a = 0; a < num_nodes; a++) {
    bool ok = in.timers_active[a] >= 0 ? in.timers_active[a] != 0 : in.deliver_timers != 0;
    if (ok) d.timer_mask |= 1u << a;
  }
  d.max_depth = in.max_depth;
  if (in.n_invariants < 0 || in.n_invariants > DSL_MAX_PREDICATES || in.n_goals < 0 ||
      in.n_goals > DSL_MAX_PREDICATES || in.n_prunes < 0 || in.n_prunes > DSL_MAX_PREDICATES)
    return DSL_ERR_ARG;
  d.n_inv = in.n_invariants;
  d.n_goal = in.n_goals;
  d.n_prune = in.n_prunes;
  auto copy = [&](const dsl_predicate* src, int n, DevPred* dst) {
    for (int i = 0; i < n; i++) {
      if (!known(src[i].pred_id)) return false;
      dst[i] = DevPred{src[i].pred_id, src[i].negate, src[i].arg0, src[i].arg1};
    }
    return true;
  };
  if (!copy(in.invariants, d.n_inv, d.inv) || !copy(in.goals, d.n_goal, d.goal) ||
      !copy(in.prunes, d.n_prune, d.prune)) {
    set_error("predicate not supported by this protocol's device predicates");
    return DSL_ERR_UNKNOWN_PREDICATE;
  }
  *out = d;
  return DSL_OK;
}

template <class P>
hipError_t Engine<P>::scan_bytes(uint64_t n, size_t* bytes) {
  return hipcub::DeviceScan::ExclusiveSum(nullptr, *bytes, d_counts, d_offsets, n, stream);
}
template <class P>
hipError_t Engine<P>::scan(uint64_t n) {
  return hipcub::DeviceScan::ExclusiveSum(d_scan_tmp, scan_tmp_bytes, d_counts, d_offsets, n, stream);
}

template <class P>
static int make_engine(const dsl_protocol_desc& d, const dsl_engine_config& cfg, EngineBase** out) {
  typename P::Params prm = P::from_desc(d);
  if (!P::valid(prm)) {
    set_error("invalid protocol parameters");
    return DSL_ERR_ARG;
  }
  *out = new Engine<P>(prm, cfg);
  return DSL_OK;
}

static int create_any(const dsl_protocol_desc& d, const dsl_engine_config& cfg, EngineBase** out) {
  switch (d.protocol) {
    case DSL_PROTO_PINGPONG: return make_engine<PingPong>(d, cfg, out);
    case DSL_PROTO_SIPAXOS: return make_engine<SIPaxos>(d, cfg, out);
    default:
      set_error("unknown protocol id " + std::to_string(d.protocol));
      return DSL_ERR_UNKNOWN_PROTOCOL;
  }
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
    default: return DSL_ERR_UNKNOWN_PROTOCOL;
  }
}

int dsl_comm_unique_id(uint8_t out[128]) {
  (void)out;
  dsl::set_error("multi-GPU communicator not built in this library version");
  return DSL_ERR_COMM;
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
  if (cfg) c = *cfg;
  if (c.world_size < 1) c.world_size = 1;
  dsl::EngineBase* impl = nullptr;
  int rc = dsl::create_any(*proto, c, &impl);
  if (rc) return rc;
  *out = new dsl_engine{impl};
  return DSL_OK;
}

int dsl_set_settings(dsl_engine* e, const dsl_settings* s) {
  if (!e || !s) return DSL_ERR_ARG;
  return e->impl->set_settings(*s);
}

int dsl_set_initial(dsl_engine* e, const uint8_t* packed, size_t len, int32_t depth) {
  if (!e || !packed) return DSL_ERR_ARG;
  return e->impl->set_initial(packed, len, depth);
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
