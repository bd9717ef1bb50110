// pingpong.hpp -- lab0 PingPong as node-local device handlers.
//
// Re-expresses (not translates) labs/lab0-pingpong/src/dslabs/pingpong/PingServer.java:29-32,
// PingClient.java:41-87 (sendCommand / handlePongReply / onPingTimer), Timers.java:7-11
// (PingTimer, 10 ms), wrapped in the ClientWorker command loop
// (framework/tst/dslabs/framework/testing/ClientWorker.java:174-251) with the repeatedPings
// workload (labs/lab0-pingpong/tst/dslabs/pingpong/PingTest.java:44-51). README mutants:
// no pong-value check (README.md:342-347), no timer re-set (README.md:299-306).
//
// Nodes: 0 = pingserver (no fields: PingApplication has none), 1..C = client1..clientC.
// Ping values are interned as 1..N ("ping-i" -> i); 0 encodes null.
// Client node words (5):
//   w0: ping:4 | pong:4 | nres:4 | ntim:4     (PingClient.ping/pong, |results|, |timer queue|)
//   w1-w2: results[15] as nibbles            (ClientWorker.results, in order)
//   w3-w4: timer queue[15] as nibbles        (PingTimer(ping) values, insertion order)
// ClientWorker bookkeeping (waitingOnResult, workload index, resultsOk) is a function of nres
// (its equality is {client, results}: ClientWorker.java:49-51), so it is not stored.
// Records (32 bit): type:1 @31 | client:3 @28 | value:4 @24
//   type 0 PingRequest(ping-v) client -> server, type 1 PongReply(ping-v) server -> client.
#pragma once
#include "../nodestate.hpp"

namespace dsl {

struct PingPong {
  static constexpr int kMaxClients = 4, kMaxPings = 15, kRetryMillis = 10;
  static constexpr int kNodes = 1 + kMaxClients, kNodeWords = 5;
  static constexpr int kMsgClasses = 2;  // handler classes of messages (PingRequest, PongReply); timers: class 2
  static constexpr int kNetCap = 2 * kMaxClients * kMaxPings, kMaxSends = 2;
  using Rec = uint32_t;
  using State = StateOf<PingPong>;

  struct Params {
    int32_t clients, pings, check_value, reset_timer;
  };
  enum { T_PING_REQUEST = 0, T_PONG_REPLY = 1, T_PING_TIMER = 2 };

  static DSL_HD Rec rec(int type, int c, int v) { return ((Rec)type << 31) | ((Rec)c << 28) | ((Rec)v << 24); }
  static DSL_HD int rec_type(Rec r) { return (int)(r >> 31); }
  static DSL_HD int rec_client(Rec r) { return (int)((r >> 28) & 7); }
  static DSL_HD int rec_value(Rec r) { return (int)((r >> 24) & 15); }
  static DSL_HD int rec_from(Rec r) { return rec_type(r) ? 0 : rec_client(r); }
  static DSL_HD int rec_to(Rec r) { return rec_type(r) ? rec_client(r) : 0; }

  // Handler class of a message (< kMsgClasses; timers are class kMsgClasses): k_level groups a chunk's work items
  // by class so that the lanes of a wavefront run the same handler.
  static DSL_HD int msg_class(Rec r) { return rec_type(r); }
  static DSL_HD int get(const uint32_t* w, int bit, int width) { return field_get<kNodeWords>(w, bit, width); }
  static DSL_HD void put(uint32_t* w, int bit, int width, int v) { field_put<kNodeWords>(w, bit, width, v); }
  static DSL_HD int ping(const uint32_t* w) { return get(w, 0, 4); }
  static DSL_HD int pong(const uint32_t* w) { return get(w, 4, 4); }
  static DSL_HD int nres(const uint32_t* w) { return get(w, 8, 4); }
  static DSL_HD int ntim(const uint32_t* w) { return get(w, 12, 4); }
  static DSL_HD int result(const uint32_t* w, int j) { return get(w, 32 + 4 * j, 4); }
  static DSL_HD int timer(const uint32_t* w, int j) { return get(w, 96 + 4 * j, 4); }

  template <class O>
  static DSL_HD void push_timer(uint32_t* w, int v, O& out) {
    const int n = ntim(w);
    if (n >= kMaxPings) {
      out.overflow = true;
      return;
    }
    put(w, 96 + 4 * n, 4, v);
    put(w, 12, 4, n + 1);
  }
  // PingClient.sendCommand: ping = p, pong = null, send PingRequest, set PingTimer(10 ms).
  template <class O>
  static DSL_HD void send_command(int c, uint32_t* w, int v, O& out) {
    put(w, 0, 4, v);
    put(w, 4, 4, 0);
    out.send(rec(0, c, v));
    push_timer(w, v, out);
  }
  // ClientWorker.sendNextCommandWhilePossible; waitingOnResult == (nres < pings).
  template <class O>
  static DSL_HD void client_worker_continue(int c, uint32_t* w, const Params& p, O& out) {
    int n = nres(w);
    if (n < p.pings && pong(w) != 0) {
      put(w, 32 + 4 * n, 4, pong(w));
      n++;
      put(w, 8, 4, n);
      if (n < p.pings) send_command(c, w, n + 1, out);
    }
  }

  static DSL_HD int num_nodes(const Params& p) { return 1 + p.clients; }
  template <class O>
  static DSL_HD void init_node(int i, uint32_t* w, O& out, const Params& p) {
    if (i > 0) send_command(i, w, 1, out);  // ClientWorker.init -> first command
  }
  // TimerQueue.deliverable(): all PingTimers are (10,10): only the head is deliverable.
  static DSL_HD int num_timer_events(int i, const uint32_t* w, const Params&) { return i > 0 && ntim(w) > 0; }

  template <class O>
  static DSL_HD int on_message(int i, uint32_t* w, Rec r, O& out, const Params& p) {
    if (i == 0) {  // PingServer.handlePingRequest: reply Pong(value) to the sender
      if (rec_type(r) != 0) return STEP_EXCEPTION;
      out.send(rec(1, rec_client(r), rec_value(r)));
      return STEP_OK;
    }
    if (rec_type(r) != 1) return STEP_EXCEPTION;
    const int v = rec_value(r);
    if (!p.check_value || ping(w) == v) put(w, 4, 4, v);  // PingClient.handlePongReply
    client_worker_continue(i, w, p, out);
    return STEP_OK;
  }
  // PingClient.onPingTimer, the ClientWorker loop, then remove the first equal timer (the head).
  template <class O>
  static DSL_HD int on_timer(int i, uint32_t* w, int, O& out, const Params& p) {
    const int v = timer(w, 0);
    if (ping(w) == v && pong(w) == 0) {
      out.send(rec(0, i, v));
      if (p.reset_timer) push_timer(w, v, out);
    }
    client_worker_continue(i, w, p, out);
    const int n = ntim(w);
    for (int j = 0; j + 1 < n; j++) put(w, 96 + 4 * j, 4, timer(w, j + 1));
    put(w, 96 + 4 * (n - 1), 4, 0);
    put(w, 12, 4, n - 1);
    return STEP_OK;
  }

  static DSL_HD int eval(const DevPred& pr, const NodeView& v, const Params& p) {
    switch (pr.id) {
      case DSL_PRED_RESULTS_OK:
        for (int c = 1; c <= p.clients; c++) {
          const uint32_t* w = v.node(c);
          for (int j = 0; j < nres(w); j++)
            if (result(w, j) != j + 1) return PV_FALSE;
        }
        return PV_TRUE;
      case DSL_PRED_CLIENTS_DONE:
        for (int c = 1; c <= p.clients; c++)
          if (nres(v.node(c)) < p.pings) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_DONE:
        if (pr.arg0 < 1 || pr.arg0 > p.clients) return PV_THREW;
        return nres(v.node((int)pr.arg0)) >= p.pings ? PV_TRUE : PV_FALSE;
      case DSL_PRED_NONE_DECIDED:
        for (int c = 1; c <= p.clients; c++)
          if (nres(v.node(c)) > 0) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_HAS_RESULTS:
        if (pr.arg0 < 1 || pr.arg0 > p.clients) return PV_THREW;
        return nres(v.node((int)pr.arg0)) == pr.arg1 ? PV_TRUE : PV_FALSE;
      default:
        return PV_THREW;
    }
  }

  // Read sets (judge_view's incremental check): every predicate reads client nodes only.
  static uint32_t pred_reads(const DevPred& pr, const Params& p) {
    return (pr.id >= DSL_PRED_RESULTS_OK && pr.id <= DSL_PRED_CLIENT_HAS_RESULTS) ? (((1u << p.clients) - 1u) << 1)
                                                                                   : kReadsAll;
  }
  static bool known_predicate(int id) { return id >= DSL_PRED_RESULTS_OK && id <= DSL_PRED_CLIENT_HAS_RESULTS; }
  static bool valid(const Params& p) {
    return p.clients >= 1 && p.clients <= kMaxClients && p.pings >= 1 && p.pings <= kMaxPings;
  }
  static Params from_desc(const dsl_protocol_desc& d) {
    Params p{};
    p.clients = (int32_t)d.params[0];
    p.pings = (int32_t)d.params[1];
    p.check_value = d.n_params > 2 ? (int32_t)d.params[2] : 1;
    p.reset_timer = d.n_params > 3 ? (int32_t)d.params[3] : 1;
    return p;
  }
  static void describe_message(Rec r, dsl_event* e) {
    e->from = rec_from(r);
    e->to = rec_to(r);
    e->type = rec_type(r) ? T_PONG_REPLY : T_PING_REQUEST;
    e->n_fields = 1;
    e->fields[0] = rec_value(r);
  }
  static void describe_timer(int i, const uint32_t* w, int, const Params&, dsl_event* e) {
    e->is_timer = 1;
    e->from = e->to = i;
    e->type = T_PING_TIMER;
    e->timer_min = e->timer_max = kRetryMillis;
    e->n_fields = 1;
    e->fields[0] = timer(w, 0);
  }
};

}  // namespace dsl
