// amokv.hpp -- lab1 at-most-once client/server KV store (BASELINE config C2) as node-local device
// handlers. The reference's lab1 classes are stubs (labs/lab1-clientserver/src/dslabs/...); this
// is the builder-authored solution of DESIGN.md §11, restated object-style in
// oracle/proto_amokv.hpp.
//
// Nodes: 0 = "server" (SimpleServer over AMOApplication(KVStore)), 1..c = "client1.." (ClientWorker
// around a SimpleClient). A workload is a per-client table of commands (op, key id, value
// symbol) with optional expected results; KV values are symbol sequences (equal-length tokens,
// so string suffix/prefix tests are sequence tests). A result is 24 bits: type:2 | len:4 @2 |
// symbols 9 x 2 bits @6 (types: 0 AppendResult, 1 GetResult, 2 KeyNotFound, 3 PutOk).
//
// Node words (6):
//   server: w0..w2 = value of key 0..2 (len:4 | symbols @4);  w3..w5 = AMO[client]: seq:2 | result:24 @2
//   client: w0 = seq:2 | hasResult:1 @2 | nres:2 @3 | ntimers:3 @5 | timer seqs 4 x 2 @8
//           w1 = current result;  w2..w4 = results[0..2]
// Records (64 bit): type:1 @63 (0 Request, 1 Reply) | from:3 @60 | to:3 @57 | seq:2 @55 | result:24
// (a Request's command is the workload's command `seq` of its sender).
#pragma once
#include "../nodestate.hpp"

namespace dsl {

struct AmoKV {
  static constexpr int kMaxClients = 3, kMaxCmds = 3, kMaxKeys = 3, kMaxLen = 9, kTimerCap = 4;
  static constexpr int kNodes = 1 + kMaxClients, kNodeWords = 6, kNetCap = 24, kMaxSends = 1;
  static constexpr int kMsgClasses = 2;  // handler classes of messages (message types 0..1); timers: class 2
  static constexpr int kRetry = 100;
  using Rec = uint64_t;
  using State = StateOf<AmoKV>;
  enum { OP_GET = 0, OP_PUT = 1, OP_APPEND = 2 };
  enum { R_APPEND = 0, R_GET = 1, R_NOTFOUND = 2, R_PUTOK = 3 };
  enum { M_REQUEST = 0, M_REPLY = 1, T_CLIENT = 2 };

  struct Params {
    int32_t clients, ncmds;
    int32_t op[kMaxClients][kMaxCmds], key[kMaxClients][kMaxCmds], sym[kMaxClients][kMaxCmds];
    int32_t expected[kMaxClients][kMaxCmds];  // result encoding, -1 = no expected result
  };

  static DSL_HD int get(const uint32_t* w, int bit, int width) { return field_get<kNodeWords>(w, bit, width); }
  static DSL_HD void put(uint32_t* w, int bit, int width, int v) { field_put<kNodeWords>(w, bit, width, v); }

  static DSL_HD Rec msg(int type, int from, int to, int seq, uint32_t res) {
    return ((Rec)type << 63) | ((Rec)from << 60) | ((Rec)to << 57) | ((Rec)seq << 55) | (Rec)res;
  }
  static DSL_HD int m_type(Rec m) { return (int)(m >> 63); }
  static DSL_HD int rec_from(Rec m) { return (int)((m >> 60) & 7); }
  static DSL_HD int rec_to(Rec m) { return (int)((m >> 57) & 7); }
  static DSL_HD int m_seq(Rec m) { return (int)((m >> 55) & 3); }
  static DSL_HD uint32_t m_res(Rec m) { return (uint32_t)(m & 0xffffff); }
  static DSL_HD int msg_class(Rec r) { return m_type(r); }

  // values: len:4 | symbols from bit 4; results: type:2 | value << 2
  static DSL_HD uint32_t v_len(uint32_t v) { return v & 15; }
  static DSL_HD uint32_t v_append(uint32_t v, int sym, bool* overflow) {
    const uint32_t n = v_len(v);
    if (n >= (uint32_t)kMaxLen) {
      *overflow = true;
      return v;
    }
    return (v & ~15u) | (n + 1) | ((uint32_t)sym << (4 + 2 * n));
  }
  static DSL_HD uint32_t res(int type, uint32_t value) { return (uint32_t)type | (value << 2); }
  static DSL_HD int r_type(uint32_t r) { return (int)(r & 3); }
  static DSL_HD uint32_t r_value(uint32_t r) { return r >> 2; }

  // ---- server --------------------------------------------------------------------------------
  template <class O>
  static DSL_HD int server_request(uint32_t* w, Rec m, O& out, const Params& p) {
    const int c = rec_from(m) - 1, seq = m_seq(m);
    if (c < 0 || c >= p.clients || seq < 1 || seq > p.ncmds) return STEP_EXCEPTION;
    const uint32_t amo = sel_word<kNodeWords>(w, 3 + c);
    const int last = (int)(amo & 3);
    if (seq < last) return STEP_OK;  // superseded command: no reply
    uint32_t r;
    if (seq == last) {
      r = amo >> 2;
    } else {  // KVStore.execute
      const int k = seq - 1, op = sel_param(p.op, c, k), key = sel_param(p.key, c, k), sym = sel_param(p.sym, c, k);
      uint32_t v = sel_word<kNodeWords>(w, key);
      if (op == OP_GET) {
        r = v_len(v) ? res(R_GET, v) : res(R_NOTFOUND, 0);
      } else if (op == OP_PUT) {
        sel_put<kNodeWords>(w, key, 1u | ((uint32_t)sym << 4));
        r = res(R_PUTOK, 0);
      } else {
        bool ovf = false;
        v = v_append(v, sym, &ovf);
        if (ovf) return STEP_OVERFLOW;
        sel_put<kNodeWords>(w, key, v);
        r = res(R_APPEND, v);
      }
      sel_put<kNodeWords>(w, 3 + c, (uint32_t)seq | (r << 2));
    }
    out.send(msg(M_REPLY, 0, c + 1, seq, r));
    return STEP_OK;
  }

  // ---- client (SimpleClient inside a ClientWorker) ---------------------------------------------
  static DSL_HD int seq_of(const uint32_t* w) { return get(w, 0, 2); }
  static DSL_HD int has_result(const uint32_t* w) { return get(w, 2, 1); }
  static DSL_HD int nres(const uint32_t* w) { return get(w, 3, 2); }
  static DSL_HD int ntim(const uint32_t* w) { return get(w, 5, 3); }
  static DSL_HD int timer(const uint32_t* w, int j) { return get(w, 8 + 2 * j, 2); }
  static DSL_HD bool push_timer(uint32_t* w, int seq) {
    const int n = ntim(w);
    if (n >= kTimerCap) return false;
    put(w, 8 + 2 * n, 2, seq);
    put(w, 5, 3, n + 1);
    return true;
  }
  // SimpleClient.sendCommand: seq++, Request(cmd, seq) to the server, ClientTimer(seq)
  template <class O>
  static DSL_HD bool send_command(int i, uint32_t* w, O& out) {
    const int seq = seq_of(w) + 1;
    put(w, 0, 2, seq);
    put(w, 2, 1, 0);
    w[1] = 0;
    out.send(msg(M_REQUEST, i, 0, seq, 0));
    return push_timer(w, seq);
  }
  // ClientWorker.sendNextCommandWhilePossible: harvest the result, then the next command
  template <class O>
  static DSL_HD bool worker_continue(int i, uint32_t* w, O& out, const Params& p) {
    int n = nres(w);
    if (n < seq_of(w) && has_result(w)) {  // waiting on a result and the client has one
      sel_put<kNodeWords>(w, 2 + n, w[1]);
      n++;
      put(w, 3, 2, n);
    }
    if (n == seq_of(w) && seq_of(w) < p.ncmds) return send_command(i, w, out);
    return true;
  }

  // ---- protocol interface -------------------------------------------------------------------------
  static DSL_HD int num_nodes(const Params& p) { return 1 + p.clients; }
  template <class O>
  static DSL_HD void init_node(int i, uint32_t* w, O& out, const Params& p) {
    if (i > 0 && !worker_continue(i, w, out, p)) out.overflow = true;
  }
  // ClientTimers are all (100, 100): only the head of the queue is deliverable
  static DSL_HD int num_timer_events(int i, const uint32_t* w, const Params&) { return i > 0 && ntim(w) > 0; }

  // Deliveries that surely change nothing (nodestate.hpp NoopFilter), read off on_message below:
  // a superseded Request at the server (seq below the client's last: no reply, no state), and a
  // Reply the client neither takes (handleReply) nor lets the worker loop act on. The server's
  // cached re-reply (seq == last) is not claimed: its Reply may or may not be in the network.
  static DSL_HD bool surely_noop(int i, const uint32_t* row, Rec m, const Params& p) {
    const uint32_t* w = row + i * kNodeWords;
    if (i == 0) {
      if (m_type(m) != M_REQUEST) return false;
      const int c = rec_from(m) - 1, seq = m_seq(m);
      if (c < 0 || c >= p.clients || seq < 1 || seq > p.ncmds) return false;  // throws
      return seq < (int)(sel_word<kNodeWords>(w, 3 + c) & 3);
    }
    if (m_type(m) != M_REPLY) return false;
    const int n = nres(w), s = seq_of(w);
    if (n < s && !has_result(w) && m_seq(m) == s) return false;  // handleReply takes it
    return !(n < s && has_result(w)) && !(n == s && s < p.ncmds);  // worker_continue idle
  }

  template <class O>
  static DSL_HD int on_message(int i, uint32_t* w, Rec m, O& out, const Params& p) {
    if (i == 0) {
      if (m_type(m) != M_REQUEST) return STEP_EXCEPTION;
      return server_request(w, m, out, p);
    }
    if (m_type(m) != M_REPLY) return STEP_EXCEPTION;
    if (nres(w) < seq_of(w) && !has_result(w) && m_seq(m) == seq_of(w)) {  // handleReply
      w[1] = m_res(m);
      put(w, 2, 1, 1);
    }
    return worker_continue(i, w, out, p) ? STEP_OK : STEP_OVERFLOW;
  }
  template <class O>
  static DSL_HD int on_timer(int i, uint32_t* w, int, O& out, const Params& p) {
    const int t = timer(w, 0);
    if (nres(w) < seq_of(w) && !has_result(w) && t == seq_of(w)) {  // onClientTimer: re-send, re-set
      out.send(msg(M_REQUEST, i, 0, t, 0));
      if (!push_timer(w, t)) return STEP_OVERFLOW;
    }
    if (!worker_continue(i, w, out, p)) return STEP_OVERFLOW;
    const int n = ntim(w);  // remove the first equal timer: the head
    for (int j = 0; j + 1 < kTimerCap; j++) put(w, 8 + 2 * j, 2, j + 1 < n ? timer(w, j + 1) : 0);
    put(w, 8 + 2 * (kTimerCap - 1), 2, 0);
    put(w, 5, 3, n - 1);
    return STEP_OK;
  }

  // ---- predicates ---------------------------------------------------------------------------------
  static DSL_HD int eval(const DevPred& pr, const NodeView& v, const Params& p) {
    switch (pr.id) {
      case DSL_PRED_RESULTS_OK:
        for (int c = 0; c < p.clients; c++) {
          const uint32_t* w = v.node(1 + c);
          const int n = nres(w);
          for (int k = 0; k < n; k++)
            if (sel_param(p.expected, c, k) >= 0 && sel_word<kNodeWords>(w, 2 + k) != (uint32_t)sel_param(p.expected, c, k)) return PV_FALSE;
        }
        return PV_TRUE;
      case DSL_PRED_CLIENTS_DONE:
        for (int c = 0; c < p.clients; c++)
          if (nres(v.node(1 + c)) < p.ncmds) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_DONE:
        if (pr.arg0 < 1 || pr.arg0 > p.clients) return PV_THREW;
        return nres(v.node((int)pr.arg0)) >= p.ncmds ? PV_TRUE : PV_FALSE;
      case DSL_PRED_NONE_DECIDED:
        for (int c = 0; c < p.clients; c++)
          if (nres(v.node(1 + c)) > 0) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_HAS_RESULTS:
        if (pr.arg0 < 1 || pr.arg0 > p.clients) return PV_THREW;
        return nres(v.node((int)pr.arg0)) == pr.arg1 ? PV_TRUE : PV_FALSE;
      case DSL_PRED_APPENDS_LINEARIZABLE: {  // KVStoreWorkload.java:282-340
        uint32_t all[kMaxClients * kMaxCmds];
        int n = 0;
        for (int c = 0; c < p.clients; c++) {
          const uint32_t* w = v.node(1 + c);
          const int nr = nres(w);
          for (int k = 0; k < nr; k++) {
            if (sel_param(p.op, c, k) != OP_APPEND) return PV_THREW;  // "Client workers have non-Append Commands"
            const uint32_t r = sel_word<kNodeWords>(w, 2 + k);
            if (r_type(r) != R_APPEND) return PV_FALSE;
            const uint32_t val = r_value(r), len = v_len(val);
            if (len == 0 || (int)((val >> (4 + 2 * (len - 1))) & 3) != sel_param(p.sym, c, k)) return PV_FALSE;  // endsWith
            all[n++] = val;
          }
        }
        for (int a = 1; a < n; a++)  // stable sort by length
          for (int j = a; j > 0 && v_len(all[j]) < v_len(all[j - 1]); j--) {
            const uint32_t t = all[j];
            all[j] = all[j - 1];
            all[j - 1] = t;
          }
        for (int a = 0; a + 1 < n; a++) {
          const uint32_t la = v_len(all[a]), lb = v_len(all[a + 1]);
          if (la == lb) return PV_FALSE;  // equal length: equal strings or not prefixes
          const uint32_t mask = (1u << (2 * la)) - 1u;
          if (((all[a] >> 4) & mask) != ((all[a + 1] >> 4) & mask)) return PV_FALSE;
        }
        return PV_TRUE;
      }
      default:
        return PV_THREW;
    }
  }
  static uint32_t pred_reads(const DevPred& pr, const Params& p) {
    const uint32_t clients = ((1u << p.clients) - 1u) << 1;
    switch (pr.id) {
      case DSL_PRED_RESULTS_OK: case DSL_PRED_CLIENTS_DONE: case DSL_PRED_CLIENT_DONE: case DSL_PRED_NONE_DECIDED:
      case DSL_PRED_CLIENT_HAS_RESULTS: case DSL_PRED_APPENDS_LINEARIZABLE: return clients;
      default: return kReadsAll;
    }
  }
  static bool known_predicate(int id) {
    return (id >= DSL_PRED_RESULTS_OK && id <= DSL_PRED_CLIENT_HAS_RESULTS) || id == DSL_PRED_APPENDS_LINEARIZABLE;
  }
  static bool valid(const Params& p) {
    if (p.clients < 1 || p.clients > kMaxClients || p.ncmds < 1 || p.ncmds > kMaxCmds) return false;
    for (int c = 0; c < p.clients; c++)
      for (int k = 0; k < p.ncmds; k++)
        if (p.op[c][k] < 0 || p.op[c][k] > 2 || p.key[c][k] < 0 || p.key[c][k] >= kMaxKeys || p.sym[c][k] < 0 ||
            p.sym[c][k] > 3)
          return false;
    return true;
  }
  // params: clients, ncmds, then per client c < 3, command k < 3: op, key, sym, expected
  static Params from_desc(const dsl_protocol_desc& d) {
    Params p{};
    p.clients = (int32_t)d.params[0];
    p.ncmds = (int32_t)d.params[1];
    for (int c = 0; c < kMaxClients; c++)
      for (int k = 0; k < kMaxCmds; k++) {
        const int b = 2 + 4 * (c * kMaxCmds + k);
        p.op[c][k] = (int32_t)d.params[b];
        p.key[c][k] = (int32_t)d.params[b + 1];
        p.sym[c][k] = (int32_t)d.params[b + 2];
        p.expected[c][k] = (int32_t)d.params[b + 3];
      }
    return p;
  }
  static void describe_message(Rec m, dsl_event* e) {
    e->from = rec_from(m);
    e->to = rec_to(m);
    e->type = m_type(m);
    e->n_fields = 2;
    e->fields[0] = m_seq(m);
    e->fields[1] = m_res(m);
  }
  static void describe_timer(int i, const uint32_t* w, int, const Params&, dsl_event* e) {
    e->is_timer = 1;
    e->from = e->to = i;
    e->timer_min = e->timer_max = kRetry;
    e->type = T_CLIENT;
    e->n_fields = 1;
    e->fields[0] = timer(w, 0);
  }
};

}  // namespace dsl
