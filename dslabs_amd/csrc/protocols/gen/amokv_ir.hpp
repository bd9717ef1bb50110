// AmoKVIR -- GENERATED from the protocol IR (dslabs_amd/ir/specs/amokv.py) by dslabs_amd/ir/gen_device.py; do not edit.
// lab1 at-most-once KV store in the protocol IR (the same protocol as csrc/protocols/amokv.hpp,
// restated): SimpleServer over AMOApplication(KVStore) (lab1 README; KVStore.java:
// 59-78 as lab1 specifies it) and SimpleClient inside ClientWorker with a per-client command table
// (KVStoreWorkload.java:40-66, :76-133). A Request carries its sequence number; its command is the
// sender's workload command of that number. KV values are token sequences len:4 | tokens 2 bits
// each from bit 4 (at most 9); a result is type:2 | value << 2 (0 AppendResult, 1 GetResult,
// 2 KeyNotFound, 3 PutOk), never 0 once set.
#pragma once
#include "../../nodestate.hpp"

namespace dsl {

struct AmoKVIR {
  static constexpr int kNodes = 4, kNodeWords = 6, kNetCap = 24, kMaxSends = 1;
  using Self = AmoKVIR;
  static constexpr int kMsgClasses = 2;
  using Rec = uint32_t;
  using State = StateOf<AmoKVIR>;
  struct Params {
    int32_t clients;
    int32_t ncmds;
    int32_t op[3][3];
    int32_t key[3][3];
    int32_t sym[3][3];
    int32_t expected[3][3];
    uint64_t op_pk;  // op[r][c] at bit 2 * (r * 3 + c) (from_desc)
    uint64_t key_pk;  // key[r][c] at bit 2 * (r * 3 + c) (from_desc)
    uint64_t sym_pk;  // sym[r][c] at bit 2 * (r * 3 + c) (from_desc)
  };
  static DSL_HD int get(const uint32_t* w, int bit, int width) { return field_get<kNodeWords>(w, bit, width); }
  static DSL_HD void put(uint32_t* w, int bit, int width, int v) { field_put<kNodeWords>(w, bit, width, v); }
  static DSL_HD int arr_client__timers(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[1]) >> (0 + 2 * (j))) & 3u);
  }
  static DSL_HD void arr_put_client__timers(uint32_t* w, int j, int v) {
    const int sh = 0 + 2 * (j);
    const uint64_t x = (((uint64_t)w[1]) & ~((uint64_t)3u << sh)) | ((uint64_t)((uint32_t)v & 3u) << sh);
    w[1] = (uint32_t)x;
  }
  static DSL_HD int rec_type(Rec r) { return (int)(r >> 31); }
  static DSL_HD int rec_from(Rec r) { return (int)((r >> 29) & 3); }
  static DSL_HD int rec_to(Rec r) { return (int)((r >> 27) & 3); }
  static DSL_HD int msg_class(Rec r) { return rec_type(r); }
  // node index -> kind: kinds are laid out in declaration order, instances consecutive
  static DSL_HD int num_nodes(const Params& p) { return 1 + p.clients; }
  static DSL_HD int first_server(const Params& p) { (void)p; return 0; }
  static DSL_HD bool is_server(int i, const Params& p) { return i >= first_server(p) && i < first_server(p) + 1; }
  static DSL_HD int first_client(const Params& p) { (void)p; return 0 + 1; }
  static DSL_HD bool is_client(int i, const Params& p) { return i >= first_client(p) && i < first_client(p) + p.clients; }
  static DSL_HD int wsize(int c, const Params& p) { (void)c; (void)p; return p.ncmds; }
  // timer entries: fields from bit 0 in declaration order, the type above them
  static DSL_HD void tbounds(int type, int& mn, int& mx) {
    if (type == 0) { mn = 100; mx = 100; }
  }
  static DSL_HD int ttype(int e) { return 0; }
  static DSL_HD bool push_timer_client(uint32_t* w, int e) {
    const int n = get(w, 26, 3);
    if (n >= 4) return false;
    arr_put_client__timers(w, n, e);
    put(w, 26, 3, n + 1);
    return true;
  }
  // TimerQueue.deliverable(): the index of deliverable entry j (-1: none), or their count (j < 0)
  static DSL_HD int deliverable_client(const uint32_t* w, int j) {
    const int n = get(w, 26, 3);
    return j < 0 ? (n > 0 ? 1 : 0) : (j == 0 && n > 0 ? 0 : -1);  // only the head (equal fixed durations)
  }
  static DSL_HD int deliverable_general_client(const uint32_t* w, int j) {
    const int n = get(w, 26, 3);
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
    const int n = get(w, 26, 3);
    int q0 = n;
    for (int q = n - 1; q >= 0; q--)
      if (arr_client__timers(w, q) == e) q0 = q;
    if (q0 >= n) return;
    for (int q = q0; q + 1 < n; q++) arr_put_client__timers(w, q, arr_client__timers(w, q + 1));
    arr_put_client__timers(w, n - 1, 0);
    put(w, 26, 3, n - 1);
  }
  template <class O>
  static DSL_HD int send_command_client(int i, uint32_t* w, int cmd, O& out, const Params& p) {
    (void)p;
    put(w, 0, 2, cmd);
    put(w, 2, 24, 0);
    out.send(((Rec)0 << 31) | ((Rec)(i) << 29) | ((Rec)((first_server(p) + 1 - 1)) << 27) | ((Rec)((cmd) & 3) << 0));
    if (!push_timer_client(w, (((cmd) & 3) << 0))) return STEP_OVERFLOW;
    return STEP_OK;
  }
  // ClientWorker.sendNextCommandWhilePossible (waitingOnResult == |results| < workload size)
  template <class O>
  static DSL_HD void client_worker_client(int i, uint32_t* w, O& out, const Params& p) {
    int n = get(w, 64, 2);
    const int res = get(w, 2, 24);
    const int ws = wsize(i - first_client(p), p);
    if (n < ws && res != 0) {
      if (n >= 3) { out.overflow = true; return; }
      put(w, 96 + 32 * (n), 24, res);
      n++;
      put(w, 64, 2, n);
      if (n < ws && send_command_client(i, w, n + 1, out, p) != STEP_OK) out.overflow = true;
    }
  }
  template <class O>
  static DSL_HD void init_node(int i, uint32_t* w, O& out, const Params& p) {
    if (is_server(i, p)) {
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
  static DSL_HD int hm_server_Request(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_c = (rec_from(r) - 1);
    const int l_seq = (int)((r >> 0) & 3u);
    if (((((l_c < 0) || (l_c >= p.clients)) || (l_seq < 1)) || (l_seq > p.ncmds))) {
      return STEP_EXCEPTION;  // request from an unknown client or command
    }
    const int l_amo = get(w, 96 + 32 * (l_c), 26);
    const int l_last = (l_amo & 3);
    if ((l_seq < l_last)) {
      return STEP_OK;
    }
    int l_r = (l_amo >> 2);
    if ((l_seq > l_last)) {
      const int l_k = (l_seq - 1);
      const int l_op = (int)((p.op_pk >> ((2 * ((l_c) * 3 + (l_k))) & 63)) & 3u);
      const int l_key = (int)((p.key_pk >> ((2 * ((l_c) * 3 + (l_k))) & 63)) & 3u);
      const int l_sym = (int)((p.sym_pk >> ((2 * ((l_c) * 3 + (l_k))) & 63)) & 3u);
      const int l_v = get(w, 0 + 32 * (l_key), 22);
      if ((l_op == 0)) {
        if (((l_v & 15) != 0)) {
          l_r = ((l_v << 2) | 1);
        } else {
          l_r = 2;
        }
      }
      if ((l_op == 1)) {
        put(w, 0 + 32 * (l_key), 22, ((l_sym << 4) | 1));
        l_r = 3;
      }
      if ((l_op == 2)) {
        const int l_n = (l_v & 15);
        if ((l_n >= 9)) {
          return STEP_OVERFLOW;  // value longer than 9 tokens
        }
        const int l_v2 = (((l_v - l_n) | (l_n + 1)) | (l_sym << ((l_n * 2) + 4)));
        put(w, 0 + 32 * (l_key), 22, l_v2);
        l_r = (l_v2 << 2);
      }
      put(w, 96 + 32 * (l_c), 26, (l_seq | (l_r << 2)));
    }
    out.send(((Rec)1 << 31) | ((Rec)(i) << 29) | ((Rec)(rec_from(r)) << 27) | ((Rec)((l_seq) & 3) << 0) | ((Rec)((l_r) & 16777215) << 2));
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_client_Reply(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    if (((get(w, 2, 24) == 0) && ((int)((r >> 0) & 3u) == get(w, 0, 2)))) {
      put(w, 2, 24, (int)((r >> 2) & 16777215u));
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int ht_client_ClientTimer(int i, uint32_t* w, int e, O& out, const Params& p) {
    (void)i; (void)w; (void)out; (void)p;
    const int tf_seq = (e >> 0) & 3;
    if (((get(w, 2, 24) == 0) && (tf_seq == get(w, 0, 2)))) {
      out.send(((Rec)0 << 31) | ((Rec)(i) << 29) | ((Rec)((first_server(p) + 1 - 1)) << 27) | ((Rec)((tf_seq) & 3) << 0));
      if (!push_timer_client(w, (((tf_seq) & 3) << 0))) return STEP_OVERFLOW;
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int on_message(int i, uint32_t* w, Rec r, O& out, const Params& p) {
    (void)w; (void)out;
    if (is_server(i, p)) {
      int fl = 0, rc;
      if (rec_type(r) == 0) rc = hm_server_Request(i, w, r, out, p, fl);  // Request
      else return STEP_EXCEPTION;  // no handler for this message (Node.handleMessage throws)
      return rc;
    }
    if (is_client(i, p)) {
      int fl = 0, rc;
      if (rec_type(r) == 1) rc = hm_client_Reply(i, w, r, out, p, fl);  // Reply
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
      if (ttype(e) == 0) {  // ClientTimer
        const int rc = ht_client_ClientTimer(i, w, e, out, p);
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
          const int n = get(w, 64, 2);
          for (int j = 0; j < n; j++) {
            const int x = sel_param(p.expected, (c - c0), (j + 1) - 1);
            if (x >= 0 && get(w, 96 + 32 * (j), 24) != x) return PV_FALSE;
          }
        }
        return PV_TRUE;
      case DSL_PRED_CLIENTS_DONE:
        for (int c = c0; c < c0 + nc; c++)
          if (get(v.node(c), 64, 2) < wsize(c - c0, p)) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_DONE:
        if (pr.arg0 < c0 || pr.arg0 >= c0 + nc) return PV_THREW;
        return get(v.node((int)pr.arg0), 64, 2) >= wsize((int)pr.arg0 - c0, p) ? PV_TRUE : PV_FALSE;
      case DSL_PRED_NONE_DECIDED:
        for (int c = c0; c < c0 + nc; c++)
          if (get(v.node(c), 64, 2) > 0) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_HAS_RESULTS:
        if (pr.arg0 < c0 || pr.arg0 >= c0 + nc) return PV_THREW;
        return get(v.node((int)pr.arg0), 64, 2) == pr.arg1 ? PV_TRUE : PV_FALSE;
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
    if (pr.id >= DSL_PRED_RESULTS_OK && pr.id <= DSL_PRED_CLIENT_HAS_RESULTS) return (((a[2] ^ b[2]) & 0x3u) | ((a[3] ^ b[3]) & 0xffffffu) | ((a[4] ^ b[4]) & 0xffffffu) | ((a[5] ^ b[5]) & 0xffffffu)) == 0;
    return same_words<kNodeWords>(a, b);
  }
  static bool known_predicate(int id) { return (id >= DSL_PRED_RESULTS_OK && id <= DSL_PRED_CLIENT_HAS_RESULTS); }
  static bool valid(const Params& p) {
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        if (p.op[r][c] < 0 || p.op[r][c] > 2) return false;
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        if (p.key[r][c] < 0 || p.key[r][c] > 2) return false;
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        if (p.sym[r][c] < 0 || p.sym[r][c] > 3) return false;
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        if (p.expected[r][c] < -1 || p.expected[r][c] > 16777215) return false;
    return p.clients >= 1 && p.clients <= 3 &&
           p.ncmds >= 1 && p.ncmds <= 3 &&
           p.clients >= 1 && p.clients <= 3;
  }
  static Params from_desc(const dsl_protocol_desc& d) {
    Params p{};
    p.clients = d.n_params > 0 ? (int32_t)d.params[0] : 2;
    p.ncmds = d.n_params > 1 ? (int32_t)d.params[1] : 3;
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        const int q = 2 + r * 3 + c;
        p.op[r][c] = d.n_params > q ? (int32_t)d.params[q] : 0;
      }
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        const int q = 11 + r * 3 + c;
        p.key[r][c] = d.n_params > q ? (int32_t)d.params[q] : 0;
      }
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        const int q = 20 + r * 3 + c;
        p.sym[r][c] = d.n_params > q ? (int32_t)d.params[q] : 0;
      }
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        const int q = 29 + r * 3 + c;
        p.expected[r][c] = d.n_params > q ? (int32_t)d.params[q] : -1;
      }
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        p.op_pk |= (uint64_t)((uint32_t)p.op[r][c] & 3u) << (2 * (r * 3 + c));
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        p.key_pk |= (uint64_t)((uint32_t)p.key[r][c] & 3u) << (2 * (r * 3 + c));
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        p.sym_pk |= (uint64_t)((uint32_t)p.sym[r][c] & 3u) << (2 * (r * 3 + c));
    return p;
  }
  static void describe_message(Rec r, dsl_event* e) {
    e->from = rec_from(r);
    e->to = rec_to(r);
    e->type = rec_type(r);
    e->n_fields = 0;
    if (e->type == 0) {
      e->n_fields = 1;
      e->fields[0] = (int64_t)((r >> 0) & 3u);
    }
    if (e->type == 1) {
      e->n_fields = 2;
      e->fields[0] = (int64_t)((r >> 0) & 3u);
      e->fields[1] = (int64_t)((r >> 2) & 16777215u);
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
        e->fields[0] = (x >> 0) & 3;
      }
    }
  }
};

}  // namespace dsl
