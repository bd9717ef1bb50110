// PingPongIR -- GENERATED from the protocol IR (dslabs_amd/ir/specs/pingpong.py) by dslabs_amd/ir/gen_device.py; do not edit.
// lab0 PingPong in the protocol IR (the same protocol as csrc/protocols/pingpong.hpp, restated):
// labs/lab0-pingpong/src/dslabs/pingpong/PingServer.java:29-32 (handlePingRequest),
// PingClient.java:41-87 (sendCommand / handlePongReply / onPingTimer), Timers.java:7-11
// (PingTimer, RETRY_MILLIS = 10 ms), inside ClientWorker with PingTest's repeatedPings workload
// (tst/dslabs/pingpong/PingTest.java:44-51): command k is Ping(k), its expected result Pong(k). The
// README mutants are parameters (README.md:299-306 no timer re-set, :342-347 no value check).
#pragma once
#include "../../nodestate.hpp"

namespace dsl {

struct PingPongIR {
  static constexpr int kNodes = 5, kNodeWords = 6, kNetCap = 120, kMaxSends = 2;
  using Self = PingPongIR;
  static constexpr int kMsgClasses = 2;
  using Rec = uint32_t;
  using State = StateOf<PingPongIR>;
  struct Params {
    int32_t clients;
    int32_t pings;
    int32_t check_value;
    int32_t reset_timer;
  };
  static DSL_HD int get(const uint32_t* w, int bit, int width) { return field_get<kNodeWords>(w, bit, width); }
  static DSL_HD void put(uint32_t* w, int bit, int width, int v) { field_put<kNodeWords>(w, bit, width, v); }
  static DSL_HD int arr_client__timers(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[1] | ((uint64_t)w[2] << 32)) >> (0 + 4 * (j))) & 15u);
  }
  static DSL_HD void arr_put_client__timers(uint32_t* w, int j, int v) {
    const int sh = 0 + 4 * (j);
    const uint64_t x = (((uint64_t)w[1] | ((uint64_t)w[2] << 32)) & ~((uint64_t)15u << sh)) | ((uint64_t)((uint32_t)v & 15u) << sh);
    w[1] = (uint32_t)x;
    w[2] = (uint32_t)(x >> 32);
  }
  static DSL_HD int arr_client__results(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[4] | ((uint64_t)w[5] << 32)) >> (0 + 4 * (j))) & 15u);
  }
  static DSL_HD void arr_put_client__results(uint32_t* w, int j, int v) {
    const int sh = 0 + 4 * (j);
    const uint64_t x = (((uint64_t)w[4] | ((uint64_t)w[5] << 32)) & ~((uint64_t)15u << sh)) | ((uint64_t)((uint32_t)v & 15u) << sh);
    w[4] = (uint32_t)x;
    w[5] = (uint32_t)(x >> 32);
  }
  static DSL_HD int rec_type(Rec r) { return (int)(r >> 31); }
  static DSL_HD int rec_from(Rec r) { return (int)((r >> 28) & 7); }
  static DSL_HD int rec_to(Rec r) { return (int)((r >> 25) & 7); }
  static DSL_HD int msg_class(Rec r) { return rec_type(r); }
  // node index -> kind: kinds are laid out in declaration order, instances consecutive
  static DSL_HD int num_nodes(const Params& p) { return 1 + p.clients; }
  static DSL_HD int first_pingserver(const Params& p) { (void)p; return 0; }
  static DSL_HD bool is_pingserver(int i, const Params& p) { return i >= first_pingserver(p) && i < first_pingserver(p) + 1; }
  static DSL_HD int first_client(const Params& p) { (void)p; return 0 + 1; }
  static DSL_HD bool is_client(int i, const Params& p) { return i >= first_client(p) && i < first_client(p) + p.clients; }
  static DSL_HD int wsize(int c, const Params& p) { (void)c; (void)p; return p.pings; }
  // timer entries: fields from bit 0 in declaration order, the type above them
  static DSL_HD void tbounds(int type, int& mn, int& mx) {
    if (type == 0) { mn = 10; mx = 10; }
  }
  static DSL_HD int ttype(int e) { return 0; }
  static DSL_HD bool push_timer_client(uint32_t* w, int e) {
    const int n = get(w, 8, 4);
    if (n >= 15) return false;
    arr_put_client__timers(w, n, e);
    put(w, 8, 4, n + 1);
    return true;
  }
  // TimerQueue.deliverable(): the index of deliverable entry j (-1: none), or their count (j < 0)
  static DSL_HD int deliverable_client(const uint32_t* w, int j) {
    const int n = get(w, 8, 4);
    return j < 0 ? (n > 0 ? 1 : 0) : (j == 0 && n > 0 ? 0 : -1);  // only the head (equal fixed durations)
  }
  static DSL_HD int deliverable_general_client(const uint32_t* w, int j) {
    const int n = get(w, 8, 4);
    int mm = 0x7fffffff, c = 0;
    for (int q = 0; q < n; q++) {
      int mn = 0, mx = 0;
      tbounds(ttype(arr_client__timers(w, q)), mn, mx);
      if (q > 0 && mn >= mm) continue;
      if (c == j) return q;
      c++;
      if (mx < mm) mm = mx;
    }
    return j < 0 ? c : -1;
  }
  static DSL_HD void remove_timer_client(uint32_t* w, int e) {  // the first equal entry
    const int n = get(w, 8, 4);
    int q0 = n;
    for (int q = n - 1; q >= 0; q--)
      if (arr_client__timers(w, q) == e) q0 = q;
    if (q0 >= n) return;
    for (int q = q0; q + 1 < n; q++) arr_put_client__timers(w, q, arr_client__timers(w, q + 1));
    arr_put_client__timers(w, n - 1, 0);
    put(w, 8, 4, n - 1);
  }
  template <class O>
  static DSL_HD int send_command_client(int i, uint32_t* w, int cmd, O& out, const Params& p) {
    (void)p;
    put(w, 0, 4, cmd);
    put(w, 4, 4, 0);
    out.send(((Rec)0 << 31) | ((Rec)(i) << 28) | ((Rec)((first_pingserver(p) + 1 - 1)) << 25) | ((Rec)((cmd) & 15) << 0));
    if (!push_timer_client(w, (((cmd) & 15) << 0))) return STEP_OVERFLOW;
    return STEP_OK;
  }
  // ClientWorker.sendNextCommandWhilePossible (waitingOnResult == |results| < workload size)
  template <class O>
  static DSL_HD void client_worker_client(int i, uint32_t* w, O& out, const Params& p) {
    int n = get(w, 96, 4);
    const int res = get(w, 4, 4);
    const int ws = wsize(i - first_client(p), p);
    if (n < ws && res != 0) {
      if (n >= 15) { out.overflow = true; return; }
      arr_put_client__results(w, n, res);
      n++;
      put(w, 96, 4, n);
      if (n < ws && send_command_client(i, w, n + 1, out, p) != STEP_OK) out.overflow = true;
    }
  }
  template <class O>
  static DSL_HD void init_node(int i, uint32_t* w, O& out, const Params& p) {
    if (is_pingserver(i, p)) {
      return;
    }
    if (is_client(i, p)) {
      if (wsize(i - first_client(p), p) > 0 && send_command_client(i, w, 1, out, p) != STEP_OK) out.overflow = true;
      return;
    }
  }
  static DSL_HD int num_timer_events(int i, const uint32_t* w, const Params& p) {
    if (is_client(i, p)) return deliverable_client(w, -1);
    (void)i; (void)w; (void)p;
    return 0;
  }
  template <class O>
  static DSL_HD int hm_pingserver_PingRequest(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    out.send(((Rec)1 << 31) | ((Rec)(i) << 28) | ((Rec)(rec_from(r)) << 25) | ((Rec)(((int)((r >> 0) & 15u)) & 15) << 0));
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_client_PongReply(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    if (((p.check_value == 0) || (get(w, 0, 4) == (int)((r >> 0) & 15u)))) {
      put(w, 4, 4, (int)((r >> 0) & 15u));
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int ht_client_PingTimer(int i, uint32_t* w, int e, O& out, const Params& p) {
    (void)i; (void)w; (void)out; (void)p;
    const int tf_value = (e >> 0) & 15;
    if (((get(w, 0, 4) == tf_value) && (get(w, 4, 4) == 0))) {
      out.send(((Rec)0 << 31) | ((Rec)(i) << 28) | ((Rec)((first_pingserver(p) + 1 - 1)) << 25) | ((Rec)((tf_value) & 15) << 0));
      if ((p.reset_timer != 0)) {
        if (!push_timer_client(w, (((tf_value) & 15) << 0))) return STEP_OVERFLOW;
      }
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int on_message(int i, uint32_t* w, Rec r, O& out, const Params& p) {
    (void)w; (void)out;
    if (is_pingserver(i, p)) {
      int fl = 0, rc;
      if (rec_type(r) == 0) rc = hm_pingserver_PingRequest(i, w, r, out, p, fl);  // PingRequest
      else return STEP_EXCEPTION;  // no handler for this message (Node.handleMessage throws)
      return rc;
    }
    if (is_client(i, p)) {
      int fl = 0, rc;
      if (rec_type(r) == 1) rc = hm_client_PongReply(i, w, r, out, p, fl);  // PongReply
      else return STEP_EXCEPTION;  // no handler for this message (Node.handleMessage throws)
      if (rc == STEP_OK) client_worker_client(i, w, out, p);
      return rc;
    }
    return STEP_EXCEPTION;
  }
  template <class O>
  static DSL_HD int on_timer(int i, uint32_t* w, int j, O& out, const Params& p) {
    (void)w; (void)j; (void)out;
    if (is_client(i, p)) {
      const int q = deliverable_client(w, j);
      if (q < 0) return STEP_NULL;
      const int e = arr_client__timers(w, q);
      if (ttype(e) == 0) {  // PingTimer
        const int rc = ht_client_PingTimer(i, w, e, out, p);
        if (rc != STEP_OK) return rc;
        client_worker_client(i, w, out, p);
        remove_timer_client(w, e);  // SearchState.stepTimer: the first equal entry
        return STEP_OK;
      }
      return STEP_EXCEPTION;  // no handler for this timer
    }
    return STEP_EXCEPTION;
  }
  static DSL_HD int eval(const DevPred& pr, const NodeView& v, const Params& p) {
    const int c0 = first_client(p), nc = p.clients;
    switch (pr.id) {
      case DSL_PRED_RESULTS_OK:  // every result equals the workload's expected result
        for (int c = c0; c < c0 + nc; c++) {
          const uint32_t* w = v.node(c);
          const int n = get(w, 96, 4);
          for (int j = 0; j < n; j++) {
            const int x = (j + 1);
            if (x >= 0 && arr_client__results(w, j) != x) return PV_FALSE;
          }
        }
        return PV_TRUE;
      case DSL_PRED_CLIENTS_DONE:
        for (int c = c0; c < c0 + nc; c++)
          if (get(v.node(c), 96, 4) < wsize(c - c0, p)) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_DONE:
        if (pr.arg0 < c0 || pr.arg0 >= c0 + nc) return PV_THREW;
        return get(v.node((int)pr.arg0), 96, 4) >= wsize((int)pr.arg0 - c0, p) ? PV_TRUE : PV_FALSE;
      case DSL_PRED_NONE_DECIDED:
        for (int c = c0; c < c0 + nc; c++)
          if (get(v.node(c), 96, 4) > 0) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_HAS_RESULTS:
        if (pr.arg0 < c0 || pr.arg0 >= c0 + nc) return PV_THREW;
        return get(v.node((int)pr.arg0), 96, 4) == pr.arg1 ? PV_TRUE : PV_FALSE;
      default:
        return PV_THREW;
    }
  }
  static uint32_t pred_reads(const DevPred& pr, const Params& p) {
    (void)pr; (void)p;
    const uint32_t clients = (((1u << (p.clients)) - 1u) << first_client(p));
    return (pr.id >= DSL_PRED_RESULTS_OK && pr.id <= DSL_PRED_CLIENT_HAS_RESULTS) ? clients : kReadsAll;
  }
  static DSL_HD bool pred_same(const DevPred& pr, const uint32_t* a, const uint32_t* b) {
    if (pr.id >= DSL_PRED_RESULTS_OK && pr.id <= DSL_PRED_CLIENT_HAS_RESULTS) return (((a[3] ^ b[3]) & 0xfu) | (a[4] ^ b[4]) | ((a[5] ^ b[5]) & 0xfffffffu)) == 0;
    return same_words<kNodeWords>(a, b);
  }
  static bool known_predicate(int id) { return (id >= DSL_PRED_RESULTS_OK && id <= DSL_PRED_CLIENT_HAS_RESULTS); }
  static bool valid(const Params& p) {
    return p.clients >= 1 && p.clients <= 4 &&
           p.pings >= 1 && p.pings <= 15 &&
           p.check_value >= 0 && p.check_value <= 1 &&
           p.reset_timer >= 0 && p.reset_timer <= 1 &&
           p.clients >= 1 && p.clients <= 4;
  }
  static Params from_desc(const dsl_protocol_desc& d) {
    Params p{};
    p.clients = d.n_params > 0 ? (int32_t)d.params[0] : 1;
    p.pings = d.n_params > 1 ? (int32_t)d.params[1] : 10;
    p.check_value = d.n_params > 2 ? (int32_t)d.params[2] : 1;
    p.reset_timer = d.n_params > 3 ? (int32_t)d.params[3] : 1;
    return p;
  }
  static void describe_message(Rec r, dsl_event* e) {
    e->from = rec_from(r);
    e->to = rec_to(r);
    e->type = rec_type(r);
    e->n_fields = 0;
    if (e->type == 0) {
      e->n_fields = 1;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
    }
    if (e->type == 1) {
      e->n_fields = 1;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
    }
  }
  static void describe_timer(int i, const uint32_t* w, int j, const Params& p, dsl_event* e) {
    e->is_timer = 1;
    e->from = e->to = i;
    (void)w; (void)j; (void)p;
    if (is_client(i, p)) {
      const int q = deliverable_client(w, j);
      if (q < 0) return;
      const int x = arr_client__timers(w, q);
      e->type = 2 + ttype(x);
      int mn = 0, mx = 0;
      tbounds(ttype(x), mn, mx);
      e->timer_min = mn;
      e->timer_max = mx;
      if (ttype(x) == 0) {
        e->n_fields = 1;
        e->fields[0] = (x >> 0) & 15;
      }
    }
  }
};

}  // namespace dsl
