// pingpong.hpp -- lab0 PingPong as device transition functions over a packed state.
//
// Re-expresses (not translates) labs/lab0-pingpong/src/dslabs/pingpong/PingServer.java:29-32,
// PingClient.java:41-87 (sendCommand / handlePongReply / onPingTimer), Timers.java:7-11
// (PingTimer, 10 ms), wrapped in the ClientWorker command loop
// (framework/tst/dslabs/framework/testing/ClientWorker.java:174-251) with the
// repeatedPings workload (labs/lab0-pingpong/tst/dslabs/pingpong/PingTest.java:44-51).
//
// Nodes: 0 = pingserver, 1..C = client1..clientC. Ping values are interned as 1..N
// ("ping-i" -> i); 0 encodes null.
//
// Packed state (24 words = 96 B):
//   w[0..1]  network bitmap, PingRequest(client c, value v): bit (c-1)*N + (v-1)   (<= 60 bits)
//   w[2..3]  network bitmap, PongReply(to client c, value v): bit 64 + (c-1)*N + (v-1)
//   per client c (5 words at w[4 + 5(c-1)]):
//     word 0: ping:4 | pong:4 | nres:4 | ntim:4     (PingClient.ping/pong, |results|, |timers|)
//     words 1-2: results[15] as nibbles            (ClientWorker.results, in order)
//     words 3-4: timer queue[15] as nibbles        (PingTimer(ping) values, insertion order)
// Canonical by construction: the network is a set bitmap; lists keep order; unused nibbles 0.
// The ClientWorker bookkeeping (waitingOnResult, workload index, resultsOk) is a function of
// nres (ClientWorker equality is {client, results}: ClientWorker.java:49-51), so it is not stored.
#pragma once
#include "../common.hpp"

namespace dsl {

struct PingPong {
  static constexpr int kWords = 24;
  static constexpr int kMaxClients = 4;
  static constexpr int kMaxPings = 15;
  static constexpr int kRetryMillis = 10;
  using State = Packed<kWords>;

  struct Params {
    int32_t clients;      // 1..4
    int32_t pings;        // workload length per client, 1..15
    int32_t check_value;  // 0 = README mutant (no pong value check)
    int32_t reset_timer;  // 0 = README mutant (no PingTimer re-set)
  };

  // message / timer type ids for decoded events
  enum { T_PING_REQUEST = 0, T_PONG_REPLY = 1, T_PING_TIMER = 2 };

  static DSL_HD int cbase(int c) { return (4 + 5 * (c - 1)) * 32; }  // bit offset of client c
  static DSL_HD int ping(const State& s, int c) { return s.get(cbase(c), 4); }
  static DSL_HD int pong(const State& s, int c) { return s.get(cbase(c) + 4, 4); }
  static DSL_HD int nres(const State& s, int c) { return s.get(cbase(c) + 8, 4); }
  static DSL_HD int ntim(const State& s, int c) { return s.get(cbase(c) + 12, 4); }
  static DSL_HD int result(const State& s, int c, int j) { return s.get(cbase(c) + 32 + 4 * j, 4); }
  static DSL_HD int timer(const State& s, int c, int j) { return s.get(cbase(c) + 96 + 4 * j, 4); }
  static DSL_HD int req_bit(const Params& p, int c, int v) { return (c - 1) * p.pings + (v - 1); }
  static DSL_HD int rep_bit(const Params& p, int c, int v) { return 64 + (c - 1) * p.pings + (v - 1); }

  // PingClient.sendCommand: ping = p, pong = null, send PingRequest, set PingTimer(10ms).
  static DSL_HD bool send_command(State& s, const Params& p, int c, int v) {
    const int b = cbase(c);
    s.set(b, 4, v);
    s.set(b + 4, 4, 0);
    s.setbit(req_bit(p, c, v));
    int n = ntim(s, c);
    if (n >= kMaxPings) return false;
    s.set(b + 96 + 4 * n, 4, v);
    s.set(b + 12, 4, n + 1);
    return true;
  }

  // ClientWorker.sendNextCommandWhilePossible: harvest a result, then send the next command.
  // waitingOnResult == (nres < pings) for this workload (one command in flight until done).
  static DSL_HD bool client_worker_continue(State& s, const Params& p, int c) {
    const int b = cbase(c);
    int n = nres(s, c);
    if (n < p.pings && pong(s, c) != 0) {
      s.set(b + 32 + 4 * n, 4, pong(s, c));
      n++;
      s.set(b + 8, 4, n);
      if (n < p.pings) return send_command(s, p, c, n + 1);
    }
    return true;
  }

  static DSL_HD void init(State& s, const Params& p) {
    for (int i = 0; i < kWords; i++) s.w[i] = 0;
    for (int c = 1; c <= p.clients; c++) send_command(s, p, c, 1);  // ClientWorker.init
  }

  // Number of enabled events (SearchState.events): deliverable messages, then timers.
  static DSL_HD int num_events(const State& s, const Params& p, const DevSettings& set) {
    int n = 0;
    for (int c = 1; c <= p.clients; c++) {
      bool to_srv = should_deliver(set, c, 0), to_cli = should_deliver(set, 0, c);
      for (int v = 1; v <= p.pings; v++) {
        n += (to_srv && s.bit(req_bit(p, c, v)));
        n += (to_cli && s.bit(rep_bit(p, c, v)));
      }
      // TimerQueue.deliverable(): every PingTimer is (10,10), so only the head is deliverable.
      n += (deliver_timers(set, c) && ntim(s, c) > 0);
    }
    return n;
  }

  // Locates the k-th enabled event. kind: 0 request, 1 reply, 2 timer.
  static DSL_HD bool locate(const State& s, const Params& p, const DevSettings& set, int k, int* kind, int* c_out,
                            int* v_out) {
    for (int c = 1; c <= p.clients; c++) {
      bool to_srv = should_deliver(set, c, 0), to_cli = should_deliver(set, 0, c);
      for (int v = 1; v <= p.pings; v++) {
        if (to_srv && s.bit(req_bit(p, c, v)) && k-- == 0) {
          *kind = 0, *c_out = c, *v_out = v;
          return true;
        }
        if (to_cli && s.bit(rep_bit(p, c, v)) && k-- == 0) {
          *kind = 1, *c_out = c, *v_out = v;
          return true;
        }
      }
      if (deliver_timers(set, c) && ntim(s, c) > 0 && k-- == 0) {
        *kind = 2, *c_out = c, *v_out = timer(s, c, 0);
        return true;
      }
    }
    return false;
  }

  static DSL_HD int step(const State& in, int k, State& s, const Params& p, const DevSettings& set) {
    int kind, c, v;
    s = in;
    if (!locate(in, p, set, k, &kind, &c, &v)) return STEP_NULL;
    if (kind == 0) {
      // PingServer.handlePingRequest: reply Pong(value) to the sender.
      s.setbit(rep_bit(p, c, v));
      return STEP_OK;
    }
    const int b = cbase(c);
    if (kind == 1) {
      // PingClient.handlePongReply (value check unless mutant), then the ClientWorker loop.
      if (!p.check_value || ping(s, c) == v) s.set(b + 4, 4, v);
      return client_worker_continue(s, p, c) ? STEP_OK : STEP_OVERFLOW;
    }
    // PingClient.onPingTimer, ClientWorker loop, then remove the first equal timer (the head).
    bool ok = true;
    if (ping(s, c) == v && pong(s, c) == 0) {
      s.setbit(req_bit(p, c, v));
      if (p.reset_timer) {
        int n = ntim(s, c);
        if (n >= kMaxPings) return STEP_OVERFLOW;
        s.set(b + 96 + 4 * n, 4, v);
        s.set(b + 12, 4, n + 1);
      }
    }
    ok = client_worker_continue(s, p, c);
    int n = ntim(s, c);
    for (int j = 0; j + 1 < n; j++) s.set(b + 96 + 4 * j, 4, timer(s, c, j + 1));
    s.set(b + 96 + 4 * (n - 1), 4, 0);
    s.set(b + 12, 4, n - 1);
    return ok ? STEP_OK : STEP_OVERFLOW;
  }

  static DSL_HD int eval(const DevPred& pr, const State& s, const Params& p) {
    switch (pr.id) {
      case DSL_PRED_RESULTS_OK:
        for (int c = 1; c <= p.clients; c++)
          for (int j = 0; j < nres(s, c); j++)
            if (result(s, c, j) != j + 1) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENTS_DONE:
        for (int c = 1; c <= p.clients; c++)
          if (nres(s, c) < p.pings) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_DONE:
        if (pr.arg0 < 1 || pr.arg0 > p.clients) return PV_THREW;
        return nres(s, (int)pr.arg0) >= p.pings ? PV_TRUE : PV_FALSE;
      case DSL_PRED_NONE_DECIDED:
        for (int c = 1; c <= p.clients; c++)
          if (nres(s, c) > 0) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_HAS_RESULTS:
        if (pr.arg0 < 1 || pr.arg0 > p.clients) return PV_THREW;
        return nres(s, (int)pr.arg0) == pr.arg1 ? PV_TRUE : PV_FALSE;
      default:
        return PV_THREW;
    }
  }

  static bool known_predicate(int id) { return id >= DSL_PRED_RESULTS_OK && id <= DSL_PRED_CLIENT_HAS_RESULTS; }
  static int num_nodes(const Params& p) { return 1 + p.clients; }
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

  static void describe(const State& s, const Params& p, const DevSettings& set, int k, dsl_event* e) {
    int kind = 0, c = 0, v = 0;
    locate(s, p, set, k, &kind, &c, &v);
    *e = dsl_event{};
    e->n_fields = 1;
    e->fields[0] = v;
    if (kind == 0) {
      e->from = c, e->to = 0, e->type = T_PING_REQUEST;
    } else if (kind == 1) {
      e->from = 0, e->to = c, e->type = T_PONG_REPLY;
    } else {
      e->is_timer = 1, e->from = c, e->to = c, e->type = T_PING_TIMER;
      e->timer_min = e->timer_max = kRetryMillis;
    }
  }
};

}  // namespace dsl
