// MultiPaxosIR -- GENERATED from the protocol IR (dslabs_amd/ir/specs/multipaxos.py) by dslabs_amd/ir/gen_device.py; do not edit.
// lab3 Multi-Paxos in the protocol IR -- BASELINE config C5's protocol, the same one as
// csrc/protocols/multipaxos.hpp and oracle/proto_multipaxos.hpp, restated once here
// and generated into both forms. It follows labs/lab3-paxos/README.md:25-106 (PMMC roles in one
// server, stable leader + heartbeat-check timer, clients broadcasting requests, AMO KV store) and
// exposes what PaxosTest's predicates read (PaxosTest.java:113-346).
// 
// Servers "server1.." (node 0 .. servers-1), clients "client1.." after them. Ballot = (round,
// leader) compared as round << 2 | leader; (0, server1) is active at start. A log entry is 11 bits:
// status:2 | ballot:6 | cmd:3 (EMPTY 0, ACCEPTED 1, CHOSEN 2; a chosen entry keeps ballot 0).
// Command id 1 + 3 c + (q - 1) is client c's q-th command (0 = no-op); its KV op (1 Put, 2 Append,
// 3 Get) and value token come from the workload tables. The key's value is len:3 | tokens 2 bits
// each; a result is 7 PutOk, 6 KeyNotFound or a value. The application state is a function of the
// executed log prefix, so it is recomputed, not stored. Server Tick timers (100 ms) are re-set on
// every fire; a client's ClientTimer(seq) (100 ms) re-sends while its command is pending.
#pragma once
#include "../../nodestate.hpp"

namespace dsl {

struct MultiPaxosIR {
  static constexpr int kNodes = 5, kNodeWords = 6, kNetCap = 64, kMaxSends = 12;
  static constexpr bool kSendsDistinct = true;  // checked by tests/hostcheck (dup_sends)
  using Self = MultiPaxosIR;
  static constexpr int kMsgClasses = 8;
  using Rec = uint64_t;
  using State = StateOf<MultiPaxosIR>;
  struct Params {
    int32_t servers;
    int32_t clients;
    int32_t ncmd[2][1];
    int32_t op[2][3];
    int32_t val[2][3];
    int32_t expected[2][3];
    uint64_t ncmd_pk;  // ncmd[r][c] at bit 2 * (r * 1 + c) (from_desc)
    uint64_t op_pk;  // op[r][c] at bit 2 * (r * 3 + c) (from_desc)
    uint64_t val_pk;  // val[r][c] at bit 2 * (r * 3 + c) (from_desc)
  };
  static DSL_HD int get(const uint32_t* w, int bit, int width) { return field_get<kNodeWords>(w, bit, width); }
  static DSL_HD void put(uint32_t* w, int bit, int width, int v) { field_put<kNodeWords>(w, bit, width, v); }
  static DSL_HD int arr_server_log(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[1] | ((uint64_t)w[2] << 32)) >> (0 + (j) / 2 * 32 + (j) % 2 * 11)) & 2047u);
  }
  static DSL_HD void arr_put_server_log(uint32_t* w, int j, int v) {
    const int sh = 0 + (j) / 2 * 32 + (j) % 2 * 11;
    const uint64_t x = (((uint64_t)w[1] | ((uint64_t)w[2] << 32)) & ~((uint64_t)2047u << sh)) | ((uint64_t)((uint32_t)v & 2047u) << sh);
    w[1] = (uint32_t)x;
    w[2] = (uint32_t)(x >> 32);
  }
  static DSL_HD int arr_server_p1blog(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[3] | ((uint64_t)w[4] << 32)) >> (0 + (j) / 2 * 32 + (j) % 2 * 11)) & 2047u);
  }
  static DSL_HD void arr_put_server_p1blog(uint32_t* w, int j, int v) {
    const int sh = 0 + (j) / 2 * 32 + (j) % 2 * 11;
    const uint64_t x = (((uint64_t)w[3] | ((uint64_t)w[4] << 32)) & ~((uint64_t)2047u << sh)) | ((uint64_t)((uint32_t)v & 2047u) << sh);
    w[3] = (uint32_t)x;
    w[4] = (uint32_t)(x >> 32);
  }
  static DSL_HD int arr_server_votes(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[5]) >> (0 + (j) / 4 * 32 + (j) % 4 * 3)) & 7u);
  }
  static DSL_HD void arr_put_server_votes(uint32_t* w, int j, int v) {
    const int sh = 0 + (j) / 4 * 32 + (j) % 4 * 3;
    const uint64_t x = (((uint64_t)w[5]) & ~((uint64_t)7u << sh)) | ((uint64_t)((uint32_t)v & 7u) << sh);
    w[5] = (uint32_t)x;
  }
  static DSL_HD int arr_server__timers(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[5]) >> (14 + (j) / 2 * 32 + (j) % 2 * 3)) & 7u);
  }
  static DSL_HD void arr_put_server__timers(uint32_t* w, int j, int v) {
    const int sh = 14 + (j) / 2 * 32 + (j) % 2 * 3;
    const uint64_t x = (((uint64_t)w[5]) & ~((uint64_t)7u << sh)) | ((uint64_t)((uint32_t)v & 7u) << sh);
    w[5] = (uint32_t)x;
  }
  static DSL_HD int arr_client__timers(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[0]) >> (17 + (j) / 3 * 32 + (j) % 3 * 3)) & 7u);
  }
  static DSL_HD void arr_put_client__timers(uint32_t* w, int j, int v) {
    const int sh = 17 + (j) / 3 * 32 + (j) % 3 * 3;
    const uint64_t x = (((uint64_t)w[0]) & ~((uint64_t)7u << sh)) | ((uint64_t)((uint32_t)v & 7u) << sh);
    w[0] = (uint32_t)x;
  }
  static DSL_HD int arr_client__results(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[1] | ((uint64_t)w[2] << 32)) >> (0 + (j) / 2 * 32 + (j) % 2 * 12)) & 4095u);
  }
  static DSL_HD void arr_put_client__results(uint32_t* w, int j, int v) {
    const int sh = 0 + (j) / 2 * 32 + (j) % 2 * 12;
    const uint64_t x = (((uint64_t)w[1] | ((uint64_t)w[2] << 32)) & ~((uint64_t)4095u << sh)) | ((uint64_t)((uint32_t)v & 4095u) << sh);
    w[1] = (uint32_t)x;
    w[2] = (uint32_t)(x >> 32);
  }
  static DSL_HD int rec_type(Rec r) { return (int)(r >> 61); }
  static DSL_HD int rec_from(Rec r) { return (int)((r >> 58) & 7); }
  static DSL_HD int rec_to(Rec r) { return (int)((r >> 55) & 7); }
  static DSL_HD int msg_class(Rec r) { return rec_type(r); }
  // node index -> kind: kinds are laid out in declaration order, instances consecutive
  static DSL_HD int num_nodes(const Params& p) { return p.servers + p.clients; }
  static DSL_HD int first_server(const Params& p) { (void)p; return 0; }
  static DSL_HD bool is_server(int i, const Params& p) { return i >= first_server(p) && i < first_server(p) + p.servers; }
  static DSL_HD int first_client(const Params& p) { (void)p; return 0 + p.servers; }
  static DSL_HD bool is_client(int i, const Params& p) { return i >= first_client(p) && i < first_client(p) + p.clients; }
  static DSL_HD int wsize(int c, const Params& p) { (void)c; (void)p; return (int)((p.ncmd_pk >> ((2 * ((c) * 1 + (0))) & 63)) & 3u); }
  // timer entries: fields from bit 0 in declaration order, the type above them
  static DSL_HD void tbounds(int type, int& mn, int& mx) {
    if (type == 0) { mn = 100; mx = 100; }
    if (type == 1) { mn = 100; mx = 100; }
  }
  static DSL_HD int ttype(int e) { return e >> 2; }
  static DSL_HD bool push_timer_server(uint32_t* w, int e) {
    const int n = get(w, 172, 2);
    if (n >= 2) return false;
    arr_put_server__timers(w, n, e);
    put(w, 172, 2, n + 1);
    return true;
  }
  // TimerQueue.deliverable(): the index of deliverable entry j (-1: none), or their count (j < 0)
  static DSL_HD int deliverable_server(const uint32_t* w, int j) {
    const int n = get(w, 172, 2);
    return j < 0 ? (n > 0 ? 1 : 0) : (j == 0 && n > 0 ? 0 : -1);  // only the head (equal fixed durations)
  }
  static DSL_HD int deliverable_general_server(const uint32_t* w, int j) {
    const int n = get(w, 172, 2);
    int mm = 0x7fffffff, c = 0;
    for (int q = 0; q < n; q++) {
      int mn = 0, mx = 0;
      tbounds(ttype(arr_server__timers(w, q)), mn, mx);
      if (q > 0 && mn >= mm) continue;
      if (c == j) return q;
      c++;
      if (mx < mm) mm = mx;
    }
    return j < 0 ? c : -1;
  }
  static DSL_HD void remove_timer_server(uint32_t* w, int e) {  // the first equal entry
    const int n = get(w, 172, 2);
    int q0 = n;
    for (int q = n - 1; q >= 0; q--)
      if (arr_server__timers(w, q) == e) q0 = q;
    if (q0 >= n) return;
    for (int q = q0; q + 1 < n; q++) arr_put_server__timers(w, q, arr_server__timers(w, q + 1));
    arr_put_server__timers(w, n - 1, 0);
    put(w, 172, 2, n - 1);
  }
  static DSL_HD bool push_timer_client(uint32_t* w, int e) {
    const int n = get(w, 15, 2);
    if (n >= 3) return false;
    arr_put_client__timers(w, n, e);
    put(w, 15, 2, n + 1);
    return true;
  }
  // TimerQueue.deliverable(): the index of deliverable entry j (-1: none), or their count (j < 0)
  static DSL_HD int deliverable_client(const uint32_t* w, int j) {
    const int n = get(w, 15, 2);
    return j < 0 ? (n > 0 ? 1 : 0) : (j == 0 && n > 0 ? 0 : -1);  // only the head (equal fixed durations)
  }
  static DSL_HD int deliverable_general_client(const uint32_t* w, int j) {
    const int n = get(w, 15, 2);
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
    const int n = get(w, 15, 2);
    int q0 = n;
    for (int q = n - 1; q >= 0; q--)
      if (arr_client__timers(w, q) == e) q0 = q;
    if (q0 >= n) return;
    for (int q = q0; q + 1 < n; q++) arr_put_client__timers(w, q, arr_client__timers(w, q + 1));
    arr_put_client__timers(w, n - 1, 0);
    put(w, 15, 2, n - 1);
  }
  template <class O>
  static DSL_HD int send_command_client(int i, uint32_t* w, int cmd, O& out, const Params& p) {
    (void)p;
    put(w, 0, 2, cmd);
    put(w, 2, 1, 1);
    put(w, 3, 12, 0);
    const int l_cid0 = (((i - first_client(p)) * 3) + cmd);
    if ((0 < p.servers)) {
      out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((l_cid0) & 7) << 0));
    }
    if ((1 < p.servers)) {
      out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((l_cid0) & 7) << 0));
    }
    if ((2 < p.servers)) {
      out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((l_cid0) & 7) << 0));
    }
    if (!push_timer_client(w, (((cmd) & 3) << 0) | (1 << 2))) return STEP_OVERFLOW;
    return STEP_OK;
  }
  // ClientWorker.sendNextCommandWhilePossible (waitingOnResult == |results| < workload size)
  template <class O>
  static DSL_HD void client_worker_client(int i, uint32_t* w, O& out, const Params& p) {
    int n = get(w, 26, 2);
    const int res = get(w, 3, 12);
    const int ws = wsize(i - first_client(p), p);
    if (n < ws && res != 0) {
      if (n >= 3) { out.overflow = true; return; }
      arr_put_client__results(w, n, res);
      n++;
      put(w, 26, 2, n);
      if (n < ws && send_command_client(i, w, n + 1, out, p) != STEP_OK) out.overflow = true;
    }
  }
  template <class O>
  static DSL_HD void init_node(int i, uint32_t* w, O& out, const Params& p) {
    if (is_server(i, p)) {
      if (init_server(i, w, out, p) != STEP_OK) out.overflow = true;
      return;
    }
    if (is_client(i, p)) {
      if (wsize(i - first_client(p), p) > 0 && send_command_client(i, w, 1, out, p) != STEP_OK) out.overflow = true;
      return;
    }
  }
  static DSL_HD int num_timer_events(int i, const uint32_t* w, const Params& p) {
    if (is_server(i, p)) return deliverable_server(w, -1);
    if (is_client(i, p)) return deliverable_client(w, -1);
    (void)i; (void)w; (void)p;
    return 0;
  }
  template <class O>
  static DSL_HD int init_server(int i, uint32_t* w, O& out, const Params& p) {
    (void)i; (void)p; (void)out;
    put(w, 14, 3, 1);
    put(w, 17, 3, 1);
    if (((i - first_server(p)) == 0)) {
      put(w, 6, 1, 1);
    }
    if (!push_timer_server(w, (0 << 2))) return STEP_OVERFLOW;
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_Request(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_cmd = (int)((r >> 0) & 7u);
    const int l_c = ((l_cmd >= 4) ? 1 : 0);
    const int l_q = (l_cmd - (((l_cmd >= 4) ? 1 : 0) * 3));
    const int l_upto1 = get(w, 14, 3);
    int l_kv2 = 0;
    int l_ls03 = 0;
    int l_ls14 = 0;
    int l_r5 = 0;
    const int l_cmd6 = ((arr_server_log(w, 0) >> 8) & 7);
    const int l_c7 = ((l_cmd6 >= 4) ? 1 : 0);
    const int l_q8 = (l_cmd6 - (((l_cmd6 >= 4) ? 1 : 0) * 3));
    if ((((1 < l_upto1) && (l_cmd6 != 0)) && ((l_c7 ? l_ls14 : l_ls03) < l_q8))) {
      const int l_c9 = ((l_cmd6 >= 4) ? 1 : 0);
      const int l_op10 = (int)((p.op_pk >> ((2 * ((l_c9) * 3 + (((l_cmd6 - (((l_cmd6 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v11 = (int)((p.val_pk >> ((2 * ((l_c9) * 3 + (((l_cmd6 - (((l_cmd6 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x12 = 0;
      if ((l_op10 == 1)) {
        l_kv2 = (1 | (l_v11 << 3));
        l_x12 = 7;
      }
      if ((l_op10 == 2)) {
        const int l_len13 = (l_kv2 & 7);
        l_kv2 = (((l_len13 + 1) | (l_kv2 & -8)) | (l_v11 << (3 + (l_len13 * 2))));
        l_x12 = l_kv2;
      }
      if ((l_op10 == 3)) {
        l_x12 = (((l_kv2 & 7) != 0) ? l_kv2 : 6);
      }
      if ((l_c7 != 0)) {
        l_ls14 = l_q8;
      } else {
        l_ls03 = l_q8;
      }
      if (((l_c7 == l_c) && (l_q8 == l_q))) {
        l_r5 = l_x12;
      }
    }
    const int l_cmd14 = ((arr_server_log(w, 1) >> 8) & 7);
    const int l_c15 = ((l_cmd14 >= 4) ? 1 : 0);
    const int l_q16 = (l_cmd14 - (((l_cmd14 >= 4) ? 1 : 0) * 3));
    if ((((2 < l_upto1) && (l_cmd14 != 0)) && ((l_c15 ? l_ls14 : l_ls03) < l_q16))) {
      const int l_c17 = ((l_cmd14 >= 4) ? 1 : 0);
      const int l_op18 = (int)((p.op_pk >> ((2 * ((l_c17) * 3 + (((l_cmd14 - (((l_cmd14 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v19 = (int)((p.val_pk >> ((2 * ((l_c17) * 3 + (((l_cmd14 - (((l_cmd14 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x20 = 0;
      if ((l_op18 == 1)) {
        l_kv2 = (1 | (l_v19 << 3));
        l_x20 = 7;
      }
      if ((l_op18 == 2)) {
        const int l_len21 = (l_kv2 & 7);
        l_kv2 = (((l_len21 + 1) | (l_kv2 & -8)) | (l_v19 << (3 + (l_len21 * 2))));
        l_x20 = l_kv2;
      }
      if ((l_op18 == 3)) {
        l_x20 = (((l_kv2 & 7) != 0) ? l_kv2 : 6);
      }
      if ((l_c15 != 0)) {
        l_ls14 = l_q16;
      } else {
        l_ls03 = l_q16;
      }
      if (((l_c15 == l_c) && (l_q16 == l_q))) {
        l_r5 = l_x20;
      }
    }
    const int l_cmd22 = ((arr_server_log(w, 2) >> 8) & 7);
    const int l_c23 = ((l_cmd22 >= 4) ? 1 : 0);
    const int l_q24 = (l_cmd22 - (((l_cmd22 >= 4) ? 1 : 0) * 3));
    if ((((3 < l_upto1) && (l_cmd22 != 0)) && ((l_c23 ? l_ls14 : l_ls03) < l_q24))) {
      const int l_c25 = ((l_cmd22 >= 4) ? 1 : 0);
      const int l_op26 = (int)((p.op_pk >> ((2 * ((l_c25) * 3 + (((l_cmd22 - (((l_cmd22 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v27 = (int)((p.val_pk >> ((2 * ((l_c25) * 3 + (((l_cmd22 - (((l_cmd22 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x28 = 0;
      if ((l_op26 == 1)) {
        l_kv2 = (1 | (l_v27 << 3));
        l_x28 = 7;
      }
      if ((l_op26 == 2)) {
        const int l_len29 = (l_kv2 & 7);
        l_kv2 = (((l_len29 + 1) | (l_kv2 & -8)) | (l_v27 << (3 + (l_len29 * 2))));
        l_x28 = l_kv2;
      }
      if ((l_op26 == 3)) {
        l_x28 = (((l_kv2 & 7) != 0) ? l_kv2 : 6);
      }
      if ((l_c23 != 0)) {
        l_ls14 = l_q24;
      } else {
        l_ls03 = l_q24;
      }
      if (((l_c23 == l_c) && (l_q24 == l_q))) {
        l_r5 = l_x28;
      }
    }
    const int l_cmd30 = ((arr_server_log(w, 3) >> 8) & 7);
    const int l_c31 = ((l_cmd30 >= 4) ? 1 : 0);
    const int l_q32 = (l_cmd30 - (((l_cmd30 >= 4) ? 1 : 0) * 3));
    if ((((4 < l_upto1) && (l_cmd30 != 0)) && ((l_c31 ? l_ls14 : l_ls03) < l_q32))) {
      const int l_c33 = ((l_cmd30 >= 4) ? 1 : 0);
      const int l_op34 = (int)((p.op_pk >> ((2 * ((l_c33) * 3 + (((l_cmd30 - (((l_cmd30 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v35 = (int)((p.val_pk >> ((2 * ((l_c33) * 3 + (((l_cmd30 - (((l_cmd30 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x36 = 0;
      if ((l_op34 == 1)) {
        l_kv2 = (1 | (l_v35 << 3));
        l_x36 = 7;
      }
      if ((l_op34 == 2)) {
        const int l_len37 = (l_kv2 & 7);
        l_kv2 = (((l_len37 + 1) | (l_kv2 & -8)) | (l_v35 << (3 + (l_len37 * 2))));
        l_x36 = l_kv2;
      }
      if ((l_op34 == 3)) {
        l_x36 = (((l_kv2 & 7) != 0) ? l_kv2 : 6);
      }
      if ((l_c31 != 0)) {
        l_ls14 = l_q32;
      } else {
        l_ls03 = l_q32;
      }
      if (((l_c31 == l_c) && (l_q32 == l_q))) {
        l_r5 = l_x36;
      }
    }
    const int l_ls = (l_c ? l_ls14 : l_ls03);
    if ((l_ls >= l_q)) {
      if (((get(w, 6, 1) != 0) && (l_ls == l_q))) {
        out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c + 1) - 1)) << 55) | ((Rec)((l_q) & 3) << 0) | ((Rec)((l_r5) & 4095) << 2));
      }
      return STEP_OK;
    }
    int l_slot = get(w, 17, 3);
    int l_inlog = 0;
    const int l_e38 = arr_server_log(w, 0);
    if ((((l_e38 & 3) != 0) && (2 > l_slot))) {
      l_slot = 2;
    }
    if ((((l_e38 & 3) != 0) && (((l_e38 >> 8) & 7) == l_cmd))) {
      l_inlog = 1;
    }
    const int l_e39 = arr_server_log(w, 1);
    if ((((l_e39 & 3) != 0) && (3 > l_slot))) {
      l_slot = 3;
    }
    if ((((l_e39 & 3) != 0) && (((l_e39 >> 8) & 7) == l_cmd))) {
      l_inlog = 1;
    }
    const int l_e40 = arr_server_log(w, 2);
    if ((((l_e40 & 3) != 0) && (4 > l_slot))) {
      l_slot = 4;
    }
    if ((((l_e40 & 3) != 0) && (((l_e40 >> 8) & 7) == l_cmd))) {
      l_inlog = 1;
    }
    const int l_e41 = arr_server_log(w, 3);
    if ((((l_e41 & 3) != 0) && (5 > l_slot))) {
      l_slot = 5;
    }
    if ((((l_e41 & 3) != 0) && (((l_e41 >> 8) & 7) == l_cmd))) {
      l_inlog = 1;
    }
    if ((((get(w, 6, 1) == 0) || (l_slot > 4)) || (l_inlog != 0))) {
      return STEP_OK;
    }
    put(w, 17, 3, (l_slot + 1));
    arr_put_server_log(w, (l_slot - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | (l_cmd << 8)));
    arr_put_server_votes(w, (l_slot - 1), (1 << (i - first_server(p))));
    if (((0 < p.servers) && (0 != (i - first_server(p))))) {
      out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((l_slot) & 7) << 6) | ((Rec)((l_cmd) & 7) << 9));
    }
    if (((1 < p.servers) && (1 != (i - first_server(p))))) {
      out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((l_slot) & 7) << 6) | ((Rec)((l_cmd) & 7) << 9));
    }
    if (((2 < p.servers) && (2 != (i - first_server(p))))) {
      out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((l_slot) & 7) << 6) | ((Rec)((l_cmd) & 7) << 9));
    }
    if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
      const int l_ccmd42 = ((arr_server_log(w, (l_slot - 1)) >> 8) & 7);
      arr_put_server_log(w, (l_slot - 1), ((2 | (0 << 2)) | (l_ccmd42 << 8)));
      arr_put_server_votes(w, (l_slot - 1), 0);
      if (((0 < p.servers) && (0 != (i - first_server(p))))) {
        out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd42) & 7) << 3));
      }
      if (((1 < p.servers) && (1 != (i - first_server(p))))) {
        out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd42) & 7) << 3));
      }
      if (((2 < p.servers) && (2 != (i - first_server(p))))) {
        out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd42) & 7) << 3));
      }
    }
    if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
      fl |= 1;
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_P1a(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_b = (((int)((r >> 0) & 15u) << 2) | (int)((r >> 4) & 3u));
    if ((l_b < ((get(w, 0, 4) << 2) | get(w, 4, 2)))) {
      return STEP_OK;
    }
    if ((l_b > ((get(w, 0, 4) << 2) | get(w, 4, 2)))) {
      put(w, 0, 4, (l_b >> 2));
      put(w, 4, 2, (l_b & 3));
      put(w, 6, 1, 0);
      put(w, 7, 1, 0);
      put(w, 11, 3, 0);
      arr_put_server_votes(w, 0, 0);
      arr_put_server_p1blog(w, 0, 0);
      arr_put_server_votes(w, 1, 0);
      arr_put_server_p1blog(w, 1, 0);
      arr_put_server_votes(w, 2, 0);
      arr_put_server_p1blog(w, 2, 0);
      arr_put_server_votes(w, 3, 0);
      arr_put_server_p1blog(w, 3, 0);
    }
    put(w, 8, 1, 1);
    out.send(((Rec)3 << 61) | ((Rec)(i) << 58) | ((Rec)(rec_from(r)) << 55) | ((Rec)(((int)((r >> 0) & 15u)) & 15) << 0) | ((Rec)(((int)((r >> 4) & 3u)) & 3) << 4) | ((Rec)((arr_server_log(w, 0)) & 2047) << 6) | ((Rec)((arr_server_log(w, 1)) & 2047) << 17) | ((Rec)((arr_server_log(w, 2)) & 2047) << 28) | ((Rec)((arr_server_log(w, 3)) & 2047) << 39));
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_P1b(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_b = (((int)((r >> 0) & 15u) << 2) | (int)((r >> 4) & 3u));
    if (((get(w, 7, 1) == 0) || (l_b != ((get(w, 0, 4) << 2) | get(w, 4, 2))))) {
      return STEP_OK;
    }
    const int l_v = (get(w, 11, 3) | (1 << (rec_from(r) - (first_server(p) + 1 - 1))));
    put(w, 11, 3, l_v);
    const int l_me43 = (int)((r >> 6) & 2047u);
    const int l_mm44 = arr_server_p1blog(w, 0);
    if (((l_me43 & 3) == 2)) {
      arr_put_server_p1blog(w, 0, ((2 | (0 << 2)) | (((l_me43 >> 8) & 7) << 8)));
    } else {
      if (((((l_me43 & 3) == 1) && ((l_mm44 & 3) != 2)) && (((l_mm44 & 3) == 0) || (((l_mm44 >> 2) & 63) < ((l_me43 >> 2) & 63))))) {
        arr_put_server_p1blog(w, 0, l_me43);
      }
    }
    const int l_me45 = (int)((r >> 17) & 2047u);
    const int l_mm46 = arr_server_p1blog(w, 1);
    if (((l_me45 & 3) == 2)) {
      arr_put_server_p1blog(w, 1, ((2 | (0 << 2)) | (((l_me45 >> 8) & 7) << 8)));
    } else {
      if (((((l_me45 & 3) == 1) && ((l_mm46 & 3) != 2)) && (((l_mm46 & 3) == 0) || (((l_mm46 >> 2) & 63) < ((l_me45 >> 2) & 63))))) {
        arr_put_server_p1blog(w, 1, l_me45);
      }
    }
    const int l_me47 = (int)((r >> 28) & 2047u);
    const int l_mm48 = arr_server_p1blog(w, 2);
    if (((l_me47 & 3) == 2)) {
      arr_put_server_p1blog(w, 2, ((2 | (0 << 2)) | (((l_me47 >> 8) & 7) << 8)));
    } else {
      if (((((l_me47 & 3) == 1) && ((l_mm48 & 3) != 2)) && (((l_mm48 & 3) == 0) || (((l_mm48 >> 2) & 63) < ((l_me47 >> 2) & 63))))) {
        arr_put_server_p1blog(w, 2, l_me47);
      }
    }
    const int l_me49 = (int)((r >> 39) & 2047u);
    const int l_mm50 = arr_server_p1blog(w, 3);
    if (((l_me49 & 3) == 2)) {
      arr_put_server_p1blog(w, 3, ((2 | (0 << 2)) | (((l_me49 >> 8) & 7) << 8)));
    } else {
      if (((((l_me49 & 3) == 1) && ((l_mm50 & 3) != 2)) && (((l_mm50 & 3) == 0) || (((l_mm50 >> 2) & 63) < ((l_me49 >> 2) & 63))))) {
        arr_put_server_p1blog(w, 3, l_me49);
      }
    }
    if ((!(((((l_v & 1) + ((l_v >> 1) & 1)) + ((l_v >> 2) & 1)) * 2) > p.servers))) {
      return STEP_OK;
    }
    fl |= 2;
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_P2a(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_b = (((int)((r >> 0) & 15u) << 2) | (int)((r >> 4) & 3u));
    if ((l_b < ((get(w, 0, 4) << 2) | get(w, 4, 2)))) {
      return STEP_OK;
    }
    if ((l_b > ((get(w, 0, 4) << 2) | get(w, 4, 2)))) {
      put(w, 0, 4, (l_b >> 2));
      put(w, 4, 2, (l_b & 3));
      put(w, 6, 1, 0);
      put(w, 7, 1, 0);
      put(w, 11, 3, 0);
      arr_put_server_votes(w, 0, 0);
      arr_put_server_p1blog(w, 0, 0);
      arr_put_server_votes(w, 1, 0);
      arr_put_server_p1blog(w, 1, 0);
      arr_put_server_votes(w, 2, 0);
      arr_put_server_p1blog(w, 2, 0);
      arr_put_server_votes(w, 3, 0);
      arr_put_server_p1blog(w, 3, 0);
    }
    put(w, 8, 1, 1);
    const int l_slot = (int)((r >> 6) & 7u);
    if (((arr_server_log(w, (l_slot - 1)) & 3) != 2)) {
      arr_put_server_log(w, (l_slot - 1), ((1 | (l_b << 2)) | ((int)((r >> 9) & 7u) << 8)));
    }
    out.send(((Rec)5 << 61) | ((Rec)(i) << 58) | ((Rec)(rec_from(r)) << 55) | ((Rec)(((int)((r >> 0) & 15u)) & 15) << 0) | ((Rec)(((int)((r >> 4) & 3u)) & 3) << 4) | ((Rec)((l_slot) & 7) << 6));
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_P2b(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_b = (((int)((r >> 0) & 15u) << 2) | (int)((r >> 4) & 3u));
    const int l_slot = (int)((r >> 6) & 7u);
    if ((((get(w, 6, 1) == 0) || (l_b != ((get(w, 0, 4) << 2) | get(w, 4, 2)))) || ((arr_server_log(w, (l_slot - 1)) & 3) != 1))) {
      return STEP_OK;
    }
    const int l_v = (arr_server_votes(w, (l_slot - 1)) | (1 << (rec_from(r) - (first_server(p) + 1 - 1))));
    arr_put_server_votes(w, (l_slot - 1), l_v);
    if ((!(((((l_v & 1) + ((l_v >> 1) & 1)) + ((l_v >> 2) & 1)) * 2) > p.servers))) {
      return STEP_OK;
    }
    const int l_ccmd51 = ((arr_server_log(w, (l_slot - 1)) >> 8) & 7);
    arr_put_server_log(w, (l_slot - 1), ((2 | (0 << 2)) | (l_ccmd51 << 8)));
    arr_put_server_votes(w, (l_slot - 1), 0);
    if (((0 < p.servers) && (0 != (i - first_server(p))))) {
      out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd51) & 7) << 3));
    }
    if (((1 < p.servers) && (1 != (i - first_server(p))))) {
      out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd51) & 7) << 3));
    }
    if (((2 < p.servers) && (2 != (i - first_server(p))))) {
      out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd51) & 7) << 3));
    }
    fl |= 1;
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_Decision(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_slot = (int)((r >> 0) & 7u);
    if (((arr_server_log(w, (l_slot - 1)) & 3) == 2)) {
      return STEP_OK;
    }
    arr_put_server_log(w, (l_slot - 1), ((2 | (0 << 2)) | ((int)((r >> 3) & 7u) << 8)));
    arr_put_server_votes(w, (l_slot - 1), 0);
    fl |= 1;
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_Heartbeat(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_b = (((int)((r >> 0) & 15u) << 2) | (int)((r >> 4) & 3u));
    if ((l_b < ((get(w, 0, 4) << 2) | get(w, 4, 2)))) {
      return STEP_OK;
    }
    if ((l_b > ((get(w, 0, 4) << 2) | get(w, 4, 2)))) {
      put(w, 0, 4, (l_b >> 2));
      put(w, 4, 2, (l_b & 3));
      put(w, 6, 1, 0);
      put(w, 7, 1, 0);
      put(w, 11, 3, 0);
      arr_put_server_votes(w, 0, 0);
      arr_put_server_p1blog(w, 0, 0);
      arr_put_server_votes(w, 1, 0);
      arr_put_server_p1blog(w, 1, 0);
      arr_put_server_votes(w, 2, 0);
      arr_put_server_p1blog(w, 2, 0);
      arr_put_server_votes(w, 3, 0);
      arr_put_server_p1blog(w, 3, 0);
    }
    put(w, 8, 1, 1);
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int ht_server_Tick(int i, uint32_t* w, int e, O& out, const Params& p) {
    (void)i; (void)w; (void)out; (void)p;
    if ((get(w, 6, 1) != 0)) {
      if (((0 < p.servers) && (0 != (i - first_server(p))))) {
        out.send(((Rec)7 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4));
      }
      if (((1 < p.servers) && (1 != (i - first_server(p))))) {
        out.send(((Rec)7 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4));
      }
      if (((2 < p.servers) && (2 != (i - first_server(p))))) {
        out.send(((Rec)7 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4));
      }
    } else {
      if ((get(w, 8, 1) != 0)) {
        put(w, 8, 1, 0);
        put(w, 9, 2, 0);
      } else {
        const int l_mis = (((get(w, 9, 2) + 1) > 2) ? 2 : (get(w, 9, 2) + 1));
        put(w, 9, 2, l_mis);
        if (((l_mis >= 2) && (get(w, 0, 4) < 15))) {
          put(w, 9, 2, 0);
          put(w, 8, 1, 0);
          put(w, 0, 4, (get(w, 0, 4) + 1));
          put(w, 4, 2, (i - first_server(p)));
          put(w, 7, 1, 1);
          put(w, 6, 1, 0);
          arr_put_server_votes(w, 0, 0);
          arr_put_server_p1blog(w, 0, 0);
          arr_put_server_votes(w, 1, 0);
          arr_put_server_p1blog(w, 1, 0);
          arr_put_server_votes(w, 2, 0);
          arr_put_server_p1blog(w, 2, 0);
          arr_put_server_votes(w, 3, 0);
          arr_put_server_p1blog(w, 3, 0);
          put(w, 11, 3, (1 << (i - first_server(p))));
          const int l_me52 = arr_server_log(w, 0);
          const int l_mm53 = arr_server_p1blog(w, 0);
          if (((l_me52 & 3) == 2)) {
            arr_put_server_p1blog(w, 0, ((2 | (0 << 2)) | (((l_me52 >> 8) & 7) << 8)));
          } else {
            if (((((l_me52 & 3) == 1) && ((l_mm53 & 3) != 2)) && (((l_mm53 & 3) == 0) || (((l_mm53 >> 2) & 63) < ((l_me52 >> 2) & 63))))) {
              arr_put_server_p1blog(w, 0, l_me52);
            }
          }
          const int l_me54 = arr_server_log(w, 1);
          const int l_mm55 = arr_server_p1blog(w, 1);
          if (((l_me54 & 3) == 2)) {
            arr_put_server_p1blog(w, 1, ((2 | (0 << 2)) | (((l_me54 >> 8) & 7) << 8)));
          } else {
            if (((((l_me54 & 3) == 1) && ((l_mm55 & 3) != 2)) && (((l_mm55 & 3) == 0) || (((l_mm55 >> 2) & 63) < ((l_me54 >> 2) & 63))))) {
              arr_put_server_p1blog(w, 1, l_me54);
            }
          }
          const int l_me56 = arr_server_log(w, 2);
          const int l_mm57 = arr_server_p1blog(w, 2);
          if (((l_me56 & 3) == 2)) {
            arr_put_server_p1blog(w, 2, ((2 | (0 << 2)) | (((l_me56 >> 8) & 7) << 8)));
          } else {
            if (((((l_me56 & 3) == 1) && ((l_mm57 & 3) != 2)) && (((l_mm57 & 3) == 0) || (((l_mm57 >> 2) & 63) < ((l_me56 >> 2) & 63))))) {
              arr_put_server_p1blog(w, 2, l_me56);
            }
          }
          const int l_me58 = arr_server_log(w, 3);
          const int l_mm59 = arr_server_p1blog(w, 3);
          if (((l_me58 & 3) == 2)) {
            arr_put_server_p1blog(w, 3, ((2 | (0 << 2)) | (((l_me58 >> 8) & 7) << 8)));
          } else {
            if (((((l_me58 & 3) == 1) && ((l_mm59 & 3) != 2)) && (((l_mm59 & 3) == 0) || (((l_mm59 >> 2) & 63) < ((l_me58 >> 2) & 63))))) {
              arr_put_server_p1blog(w, 3, l_me58);
            }
          }
          if (((0 < p.servers) && (0 != (i - first_server(p))))) {
            out.send(((Rec)2 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4));
          }
          if (((1 < p.servers) && (1 != (i - first_server(p))))) {
            out.send(((Rec)2 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4));
          }
          if (((2 < p.servers) && (2 != (i - first_server(p))))) {
            out.send(((Rec)2 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4));
          }
          if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
            put(w, 6, 1, 1);
            put(w, 7, 1, 0);
            put(w, 11, 3, 0);
            const int l_mg60 = arr_server_p1blog(w, 0);
            const int l_mg61 = arr_server_p1blog(w, 1);
            const int l_mg62 = arr_server_p1blog(w, 2);
            const int l_mg63 = arr_server_p1blog(w, 3);
            int l_last64 = 0;
            if ((((l_mg60 & 3) != 0) || ((arr_server_log(w, 0) & 3) != 0))) {
              l_last64 = 1;
            }
            if ((((l_mg61 & 3) != 0) || ((arr_server_log(w, 1) & 3) != 0))) {
              l_last64 = 2;
            }
            if ((((l_mg62 & 3) != 0) || ((arr_server_log(w, 2) & 3) != 0))) {
              l_last64 = 3;
            }
            if ((((l_mg63 & 3) != 0) || ((arr_server_log(w, 3) & 3) != 0))) {
              l_last64 = 4;
            }
            arr_put_server_p1blog(w, 0, 0);
            arr_put_server_p1blog(w, 1, 0);
            arr_put_server_p1blog(w, 2, 0);
            arr_put_server_p1blog(w, 3, 0);
            if (((1 <= l_last64) && ((arr_server_log(w, 0) & 3) != 2))) {
              if (((l_mg60 & 3) == 2)) {
                arr_put_server_log(w, 0, ((2 | (0 << 2)) | (((l_mg60 >> 8) & 7) << 8)));
                arr_put_server_votes(w, 0, 0);
              } else {
                arr_put_server_log(w, (1 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg60 & 3) == 1) ? ((l_mg60 >> 8) & 7) : 0) << 8)));
                arr_put_server_votes(w, (1 - 1), (1 << (i - first_server(p))));
                if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg60 & 3) == 1) ? ((l_mg60 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg60 & 3) == 1) ? ((l_mg60 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg60 & 3) == 1) ? ((l_mg60 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
                  const int l_ccmd65 = ((arr_server_log(w, (1 - 1)) >> 8) & 7);
                  arr_put_server_log(w, (1 - 1), ((2 | (0 << 2)) | (l_ccmd65 << 8)));
                  arr_put_server_votes(w, (1 - 1), 0);
                  if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd65) & 7) << 3));
                  }
                  if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd65) & 7) << 3));
                  }
                  if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd65) & 7) << 3));
                  }
                }
              }
            }
            if (((2 <= l_last64) && ((arr_server_log(w, 1) & 3) != 2))) {
              if (((l_mg61 & 3) == 2)) {
                arr_put_server_log(w, 1, ((2 | (0 << 2)) | (((l_mg61 >> 8) & 7) << 8)));
                arr_put_server_votes(w, 1, 0);
              } else {
                arr_put_server_log(w, (2 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg61 & 3) == 1) ? ((l_mg61 >> 8) & 7) : 0) << 8)));
                arr_put_server_votes(w, (2 - 1), (1 << (i - first_server(p))));
                if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg61 & 3) == 1) ? ((l_mg61 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg61 & 3) == 1) ? ((l_mg61 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg61 & 3) == 1) ? ((l_mg61 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
                  const int l_ccmd66 = ((arr_server_log(w, (2 - 1)) >> 8) & 7);
                  arr_put_server_log(w, (2 - 1), ((2 | (0 << 2)) | (l_ccmd66 << 8)));
                  arr_put_server_votes(w, (2 - 1), 0);
                  if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd66) & 7) << 3));
                  }
                  if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd66) & 7) << 3));
                  }
                  if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd66) & 7) << 3));
                  }
                }
              }
            }
            if (((3 <= l_last64) && ((arr_server_log(w, 2) & 3) != 2))) {
              if (((l_mg62 & 3) == 2)) {
                arr_put_server_log(w, 2, ((2 | (0 << 2)) | (((l_mg62 >> 8) & 7) << 8)));
                arr_put_server_votes(w, 2, 0);
              } else {
                arr_put_server_log(w, (3 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg62 & 3) == 1) ? ((l_mg62 >> 8) & 7) : 0) << 8)));
                arr_put_server_votes(w, (3 - 1), (1 << (i - first_server(p))));
                if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg62 & 3) == 1) ? ((l_mg62 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg62 & 3) == 1) ? ((l_mg62 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg62 & 3) == 1) ? ((l_mg62 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
                  const int l_ccmd67 = ((arr_server_log(w, (3 - 1)) >> 8) & 7);
                  arr_put_server_log(w, (3 - 1), ((2 | (0 << 2)) | (l_ccmd67 << 8)));
                  arr_put_server_votes(w, (3 - 1), 0);
                  if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd67) & 7) << 3));
                  }
                  if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd67) & 7) << 3));
                  }
                  if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd67) & 7) << 3));
                  }
                }
              }
            }
            if (((4 <= l_last64) && ((arr_server_log(w, 3) & 3) != 2))) {
              if (((l_mg63 & 3) == 2)) {
                arr_put_server_log(w, 3, ((2 | (0 << 2)) | (((l_mg63 >> 8) & 7) << 8)));
                arr_put_server_votes(w, 3, 0);
              } else {
                arr_put_server_log(w, (4 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg63 & 3) == 1) ? ((l_mg63 >> 8) & 7) : 0) << 8)));
                arr_put_server_votes(w, (4 - 1), (1 << (i - first_server(p))));
                if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg63 & 3) == 1) ? ((l_mg63 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg63 & 3) == 1) ? ((l_mg63 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg63 & 3) == 1) ? ((l_mg63 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
                  const int l_ccmd68 = ((arr_server_log(w, (4 - 1)) >> 8) & 7);
                  arr_put_server_log(w, (4 - 1), ((2 | (0 << 2)) | (l_ccmd68 << 8)));
                  arr_put_server_votes(w, (4 - 1), 0);
                  if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd68) & 7) << 3));
                  }
                  if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd68) & 7) << 3));
                  }
                  if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd68) & 7) << 3));
                  }
                }
              }
            }
            put(w, 17, 3, (l_last64 + 1));
            const int l_so069 = get(w, 14, 3);
            const int l_act70 = get(w, 6, 1);
            int l_kv71 = 0;
            int l_ls072 = 0;
            int l_ls173 = 0;
            int l_so74 = l_so069;
            int l_run75 = 1;
            const int l_e76 = arr_server_log(w, 0);
            const int l_cmd77 = ((l_e76 >> 8) & 7);
            const int l_c78 = ((l_cmd77 >= 4) ? 1 : 0);
            const int l_q79 = (l_cmd77 - (((l_cmd77 >= 4) ? 1 : 0) * 3));
            const int l_before80 = (1 < l_so069);
            const int l_now81 = (((!l_before80) && (l_run75 != 0)) && ((l_e76 & 3) == 2));
            l_run75 = (((l_run75 != 0) && (l_before80 || l_now81)) ? 1 : 0);
            if ((((l_before80 || l_now81) && (l_cmd77 != 0)) && ((l_c78 ? l_ls173 : l_ls072) < l_q79))) {
              const int l_c82 = ((l_cmd77 >= 4) ? 1 : 0);
              const int l_op83 = (int)((p.op_pk >> ((2 * ((l_c82) * 3 + (((l_cmd77 - (((l_cmd77 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              const int l_v84 = (int)((p.val_pk >> ((2 * ((l_c82) * 3 + (((l_cmd77 - (((l_cmd77 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              int l_x85 = 0;
              if ((l_op83 == 1)) {
                l_kv71 = (1 | (l_v84 << 3));
                l_x85 = 7;
              }
              if ((l_op83 == 2)) {
                const int l_len86 = (l_kv71 & 7);
                l_kv71 = (((l_len86 + 1) | (l_kv71 & -8)) | (l_v84 << (3 + (l_len86 * 2))));
                l_x85 = l_kv71;
              }
              if ((l_op83 == 3)) {
                l_x85 = (((l_kv71 & 7) != 0) ? l_kv71 : 6);
              }
              if ((l_c78 != 0)) {
                l_ls173 = l_q79;
              } else {
                l_ls072 = l_q79;
              }
              if ((l_now81 && (l_act70 != 0))) {
                out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c78 + 1) - 1)) << 55) | ((Rec)((l_q79) & 3) << 0) | ((Rec)((l_x85) & 4095) << 2));
              }
            }
            if (l_now81) {
              l_so74 = 2;
            }
            const int l_e87 = arr_server_log(w, 1);
            const int l_cmd88 = ((l_e87 >> 8) & 7);
            const int l_c89 = ((l_cmd88 >= 4) ? 1 : 0);
            const int l_q90 = (l_cmd88 - (((l_cmd88 >= 4) ? 1 : 0) * 3));
            const int l_before91 = (2 < l_so069);
            const int l_now92 = (((!l_before91) && (l_run75 != 0)) && ((l_e87 & 3) == 2));
            l_run75 = (((l_run75 != 0) && (l_before91 || l_now92)) ? 1 : 0);
            if ((((l_before91 || l_now92) && (l_cmd88 != 0)) && ((l_c89 ? l_ls173 : l_ls072) < l_q90))) {
              const int l_c93 = ((l_cmd88 >= 4) ? 1 : 0);
              const int l_op94 = (int)((p.op_pk >> ((2 * ((l_c93) * 3 + (((l_cmd88 - (((l_cmd88 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              const int l_v95 = (int)((p.val_pk >> ((2 * ((l_c93) * 3 + (((l_cmd88 - (((l_cmd88 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              int l_x96 = 0;
              if ((l_op94 == 1)) {
                l_kv71 = (1 | (l_v95 << 3));
                l_x96 = 7;
              }
              if ((l_op94 == 2)) {
                const int l_len97 = (l_kv71 & 7);
                l_kv71 = (((l_len97 + 1) | (l_kv71 & -8)) | (l_v95 << (3 + (l_len97 * 2))));
                l_x96 = l_kv71;
              }
              if ((l_op94 == 3)) {
                l_x96 = (((l_kv71 & 7) != 0) ? l_kv71 : 6);
              }
              if ((l_c89 != 0)) {
                l_ls173 = l_q90;
              } else {
                l_ls072 = l_q90;
              }
              if ((l_now92 && (l_act70 != 0))) {
                out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c89 + 1) - 1)) << 55) | ((Rec)((l_q90) & 3) << 0) | ((Rec)((l_x96) & 4095) << 2));
              }
            }
            if (l_now92) {
              l_so74 = 3;
            }
            const int l_e98 = arr_server_log(w, 2);
            const int l_cmd99 = ((l_e98 >> 8) & 7);
            const int l_c100 = ((l_cmd99 >= 4) ? 1 : 0);
            const int l_q101 = (l_cmd99 - (((l_cmd99 >= 4) ? 1 : 0) * 3));
            const int l_before102 = (3 < l_so069);
            const int l_now103 = (((!l_before102) && (l_run75 != 0)) && ((l_e98 & 3) == 2));
            l_run75 = (((l_run75 != 0) && (l_before102 || l_now103)) ? 1 : 0);
            if ((((l_before102 || l_now103) && (l_cmd99 != 0)) && ((l_c100 ? l_ls173 : l_ls072) < l_q101))) {
              const int l_c104 = ((l_cmd99 >= 4) ? 1 : 0);
              const int l_op105 = (int)((p.op_pk >> ((2 * ((l_c104) * 3 + (((l_cmd99 - (((l_cmd99 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              const int l_v106 = (int)((p.val_pk >> ((2 * ((l_c104) * 3 + (((l_cmd99 - (((l_cmd99 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              int l_x107 = 0;
              if ((l_op105 == 1)) {
                l_kv71 = (1 | (l_v106 << 3));
                l_x107 = 7;
              }
              if ((l_op105 == 2)) {
                const int l_len108 = (l_kv71 & 7);
                l_kv71 = (((l_len108 + 1) | (l_kv71 & -8)) | (l_v106 << (3 + (l_len108 * 2))));
                l_x107 = l_kv71;
              }
              if ((l_op105 == 3)) {
                l_x107 = (((l_kv71 & 7) != 0) ? l_kv71 : 6);
              }
              if ((l_c100 != 0)) {
                l_ls173 = l_q101;
              } else {
                l_ls072 = l_q101;
              }
              if ((l_now103 && (l_act70 != 0))) {
                out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c100 + 1) - 1)) << 55) | ((Rec)((l_q101) & 3) << 0) | ((Rec)((l_x107) & 4095) << 2));
              }
            }
            if (l_now103) {
              l_so74 = 4;
            }
            const int l_e109 = arr_server_log(w, 3);
            const int l_cmd110 = ((l_e109 >> 8) & 7);
            const int l_c111 = ((l_cmd110 >= 4) ? 1 : 0);
            const int l_q112 = (l_cmd110 - (((l_cmd110 >= 4) ? 1 : 0) * 3));
            const int l_before113 = (4 < l_so069);
            const int l_now114 = (((!l_before113) && (l_run75 != 0)) && ((l_e109 & 3) == 2));
            l_run75 = (((l_run75 != 0) && (l_before113 || l_now114)) ? 1 : 0);
            if ((((l_before113 || l_now114) && (l_cmd110 != 0)) && ((l_c111 ? l_ls173 : l_ls072) < l_q112))) {
              const int l_c115 = ((l_cmd110 >= 4) ? 1 : 0);
              const int l_op116 = (int)((p.op_pk >> ((2 * ((l_c115) * 3 + (((l_cmd110 - (((l_cmd110 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              const int l_v117 = (int)((p.val_pk >> ((2 * ((l_c115) * 3 + (((l_cmd110 - (((l_cmd110 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              int l_x118 = 0;
              if ((l_op116 == 1)) {
                l_kv71 = (1 | (l_v117 << 3));
                l_x118 = 7;
              }
              if ((l_op116 == 2)) {
                const int l_len119 = (l_kv71 & 7);
                l_kv71 = (((l_len119 + 1) | (l_kv71 & -8)) | (l_v117 << (3 + (l_len119 * 2))));
                l_x118 = l_kv71;
              }
              if ((l_op116 == 3)) {
                l_x118 = (((l_kv71 & 7) != 0) ? l_kv71 : 6);
              }
              if ((l_c111 != 0)) {
                l_ls173 = l_q112;
              } else {
                l_ls072 = l_q112;
              }
              if ((l_now114 && (l_act70 != 0))) {
                out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c111 + 1) - 1)) << 55) | ((Rec)((l_q112) & 3) << 0) | ((Rec)((l_x118) & 4095) << 2));
              }
            }
            if (l_now114) {
              l_so74 = 5;
            }
            put(w, 14, 3, l_so74);
          }
        }
      }
    }
    if (!push_timer_server(w, (0 << 2))) return STEP_OVERFLOW;
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int tail_server(int i, uint32_t* w, int fl, O& out, const Params& p) {
    (void)i; (void)w; (void)out; (void)p;
    if (((fl >> 1) & 1)) {
      put(w, 6, 1, 1);
      put(w, 7, 1, 0);
      put(w, 11, 3, 0);
      const int l_mg120 = arr_server_p1blog(w, 0);
      const int l_mg121 = arr_server_p1blog(w, 1);
      const int l_mg122 = arr_server_p1blog(w, 2);
      const int l_mg123 = arr_server_p1blog(w, 3);
      int l_last124 = 0;
      if ((((l_mg120 & 3) != 0) || ((arr_server_log(w, 0) & 3) != 0))) {
        l_last124 = 1;
      }
      if ((((l_mg121 & 3) != 0) || ((arr_server_log(w, 1) & 3) != 0))) {
        l_last124 = 2;
      }
      if ((((l_mg122 & 3) != 0) || ((arr_server_log(w, 2) & 3) != 0))) {
        l_last124 = 3;
      }
      if ((((l_mg123 & 3) != 0) || ((arr_server_log(w, 3) & 3) != 0))) {
        l_last124 = 4;
      }
      arr_put_server_p1blog(w, 0, 0);
      arr_put_server_p1blog(w, 1, 0);
      arr_put_server_p1blog(w, 2, 0);
      arr_put_server_p1blog(w, 3, 0);
      if (((1 <= l_last124) && ((arr_server_log(w, 0) & 3) != 2))) {
        if (((l_mg120 & 3) == 2)) {
          arr_put_server_log(w, 0, ((2 | (0 << 2)) | (((l_mg120 >> 8) & 7) << 8)));
          arr_put_server_votes(w, 0, 0);
        } else {
          arr_put_server_log(w, (1 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg120 & 3) == 1) ? ((l_mg120 >> 8) & 7) : 0) << 8)));
          arr_put_server_votes(w, (1 - 1), (1 << (i - first_server(p))));
          if (((0 < p.servers) && (0 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg120 & 3) == 1) ? ((l_mg120 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((1 < p.servers) && (1 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg120 & 3) == 1) ? ((l_mg120 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((2 < p.servers) && (2 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg120 & 3) == 1) ? ((l_mg120 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
            const int l_ccmd125 = ((arr_server_log(w, (1 - 1)) >> 8) & 7);
            arr_put_server_log(w, (1 - 1), ((2 | (0 << 2)) | (l_ccmd125 << 8)));
            arr_put_server_votes(w, (1 - 1), 0);
            if (((0 < p.servers) && (0 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd125) & 7) << 3));
            }
            if (((1 < p.servers) && (1 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd125) & 7) << 3));
            }
            if (((2 < p.servers) && (2 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd125) & 7) << 3));
            }
          }
        }
      }
      if (((2 <= l_last124) && ((arr_server_log(w, 1) & 3) != 2))) {
        if (((l_mg121 & 3) == 2)) {
          arr_put_server_log(w, 1, ((2 | (0 << 2)) | (((l_mg121 >> 8) & 7) << 8)));
          arr_put_server_votes(w, 1, 0);
        } else {
          arr_put_server_log(w, (2 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg121 & 3) == 1) ? ((l_mg121 >> 8) & 7) : 0) << 8)));
          arr_put_server_votes(w, (2 - 1), (1 << (i - first_server(p))));
          if (((0 < p.servers) && (0 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg121 & 3) == 1) ? ((l_mg121 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((1 < p.servers) && (1 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg121 & 3) == 1) ? ((l_mg121 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((2 < p.servers) && (2 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg121 & 3) == 1) ? ((l_mg121 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
            const int l_ccmd126 = ((arr_server_log(w, (2 - 1)) >> 8) & 7);
            arr_put_server_log(w, (2 - 1), ((2 | (0 << 2)) | (l_ccmd126 << 8)));
            arr_put_server_votes(w, (2 - 1), 0);
            if (((0 < p.servers) && (0 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd126) & 7) << 3));
            }
            if (((1 < p.servers) && (1 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd126) & 7) << 3));
            }
            if (((2 < p.servers) && (2 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd126) & 7) << 3));
            }
          }
        }
      }
      if (((3 <= l_last124) && ((arr_server_log(w, 2) & 3) != 2))) {
        if (((l_mg122 & 3) == 2)) {
          arr_put_server_log(w, 2, ((2 | (0 << 2)) | (((l_mg122 >> 8) & 7) << 8)));
          arr_put_server_votes(w, 2, 0);
        } else {
          arr_put_server_log(w, (3 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg122 & 3) == 1) ? ((l_mg122 >> 8) & 7) : 0) << 8)));
          arr_put_server_votes(w, (3 - 1), (1 << (i - first_server(p))));
          if (((0 < p.servers) && (0 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg122 & 3) == 1) ? ((l_mg122 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((1 < p.servers) && (1 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg122 & 3) == 1) ? ((l_mg122 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((2 < p.servers) && (2 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg122 & 3) == 1) ? ((l_mg122 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
            const int l_ccmd127 = ((arr_server_log(w, (3 - 1)) >> 8) & 7);
            arr_put_server_log(w, (3 - 1), ((2 | (0 << 2)) | (l_ccmd127 << 8)));
            arr_put_server_votes(w, (3 - 1), 0);
            if (((0 < p.servers) && (0 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd127) & 7) << 3));
            }
            if (((1 < p.servers) && (1 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd127) & 7) << 3));
            }
            if (((2 < p.servers) && (2 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd127) & 7) << 3));
            }
          }
        }
      }
      if (((4 <= l_last124) && ((arr_server_log(w, 3) & 3) != 2))) {
        if (((l_mg123 & 3) == 2)) {
          arr_put_server_log(w, 3, ((2 | (0 << 2)) | (((l_mg123 >> 8) & 7) << 8)));
          arr_put_server_votes(w, 3, 0);
        } else {
          arr_put_server_log(w, (4 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg123 & 3) == 1) ? ((l_mg123 >> 8) & 7) : 0) << 8)));
          arr_put_server_votes(w, (4 - 1), (1 << (i - first_server(p))));
          if (((0 < p.servers) && (0 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg123 & 3) == 1) ? ((l_mg123 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((1 < p.servers) && (1 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg123 & 3) == 1) ? ((l_mg123 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((2 < p.servers) && (2 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg123 & 3) == 1) ? ((l_mg123 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
            const int l_ccmd128 = ((arr_server_log(w, (4 - 1)) >> 8) & 7);
            arr_put_server_log(w, (4 - 1), ((2 | (0 << 2)) | (l_ccmd128 << 8)));
            arr_put_server_votes(w, (4 - 1), 0);
            if (((0 < p.servers) && (0 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd128) & 7) << 3));
            }
            if (((1 < p.servers) && (1 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd128) & 7) << 3));
            }
            if (((2 < p.servers) && (2 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd128) & 7) << 3));
            }
          }
        }
      }
      put(w, 17, 3, (l_last124 + 1));
    }
    const int l_so0129 = get(w, 14, 3);
    const int l_act130 = get(w, 6, 1);
    int l_kv131 = 0;
    int l_ls0132 = 0;
    int l_ls1133 = 0;
    int l_so134 = l_so0129;
    int l_run135 = 1;
    const int l_e136 = arr_server_log(w, 0);
    const int l_cmd137 = ((l_e136 >> 8) & 7);
    const int l_c138 = ((l_cmd137 >= 4) ? 1 : 0);
    const int l_q139 = (l_cmd137 - (((l_cmd137 >= 4) ? 1 : 0) * 3));
    const int l_before140 = (1 < l_so0129);
    const int l_now141 = (((!l_before140) && (l_run135 != 0)) && ((l_e136 & 3) == 2));
    l_run135 = (((l_run135 != 0) && (l_before140 || l_now141)) ? 1 : 0);
    if ((((l_before140 || l_now141) && (l_cmd137 != 0)) && ((l_c138 ? l_ls1133 : l_ls0132) < l_q139))) {
      const int l_c142 = ((l_cmd137 >= 4) ? 1 : 0);
      const int l_op143 = (int)((p.op_pk >> ((2 * ((l_c142) * 3 + (((l_cmd137 - (((l_cmd137 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v144 = (int)((p.val_pk >> ((2 * ((l_c142) * 3 + (((l_cmd137 - (((l_cmd137 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x145 = 0;
      if ((l_op143 == 1)) {
        l_kv131 = (1 | (l_v144 << 3));
        l_x145 = 7;
      }
      if ((l_op143 == 2)) {
        const int l_len146 = (l_kv131 & 7);
        l_kv131 = (((l_len146 + 1) | (l_kv131 & -8)) | (l_v144 << (3 + (l_len146 * 2))));
        l_x145 = l_kv131;
      }
      if ((l_op143 == 3)) {
        l_x145 = (((l_kv131 & 7) != 0) ? l_kv131 : 6);
      }
      if ((l_c138 != 0)) {
        l_ls1133 = l_q139;
      } else {
        l_ls0132 = l_q139;
      }
      if ((l_now141 && (l_act130 != 0))) {
        out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c138 + 1) - 1)) << 55) | ((Rec)((l_q139) & 3) << 0) | ((Rec)((l_x145) & 4095) << 2));
      }
    }
    if (l_now141) {
      l_so134 = 2;
    }
    const int l_e147 = arr_server_log(w, 1);
    const int l_cmd148 = ((l_e147 >> 8) & 7);
    const int l_c149 = ((l_cmd148 >= 4) ? 1 : 0);
    const int l_q150 = (l_cmd148 - (((l_cmd148 >= 4) ? 1 : 0) * 3));
    const int l_before151 = (2 < l_so0129);
    const int l_now152 = (((!l_before151) && (l_run135 != 0)) && ((l_e147 & 3) == 2));
    l_run135 = (((l_run135 != 0) && (l_before151 || l_now152)) ? 1 : 0);
    if ((((l_before151 || l_now152) && (l_cmd148 != 0)) && ((l_c149 ? l_ls1133 : l_ls0132) < l_q150))) {
      const int l_c153 = ((l_cmd148 >= 4) ? 1 : 0);
      const int l_op154 = (int)((p.op_pk >> ((2 * ((l_c153) * 3 + (((l_cmd148 - (((l_cmd148 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v155 = (int)((p.val_pk >> ((2 * ((l_c153) * 3 + (((l_cmd148 - (((l_cmd148 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x156 = 0;
      if ((l_op154 == 1)) {
        l_kv131 = (1 | (l_v155 << 3));
        l_x156 = 7;
      }
      if ((l_op154 == 2)) {
        const int l_len157 = (l_kv131 & 7);
        l_kv131 = (((l_len157 + 1) | (l_kv131 & -8)) | (l_v155 << (3 + (l_len157 * 2))));
        l_x156 = l_kv131;
      }
      if ((l_op154 == 3)) {
        l_x156 = (((l_kv131 & 7) != 0) ? l_kv131 : 6);
      }
      if ((l_c149 != 0)) {
        l_ls1133 = l_q150;
      } else {
        l_ls0132 = l_q150;
      }
      if ((l_now152 && (l_act130 != 0))) {
        out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c149 + 1) - 1)) << 55) | ((Rec)((l_q150) & 3) << 0) | ((Rec)((l_x156) & 4095) << 2));
      }
    }
    if (l_now152) {
      l_so134 = 3;
    }
    const int l_e158 = arr_server_log(w, 2);
    const int l_cmd159 = ((l_e158 >> 8) & 7);
    const int l_c160 = ((l_cmd159 >= 4) ? 1 : 0);
    const int l_q161 = (l_cmd159 - (((l_cmd159 >= 4) ? 1 : 0) * 3));
    const int l_before162 = (3 < l_so0129);
    const int l_now163 = (((!l_before162) && (l_run135 != 0)) && ((l_e158 & 3) == 2));
    l_run135 = (((l_run135 != 0) && (l_before162 || l_now163)) ? 1 : 0);
    if ((((l_before162 || l_now163) && (l_cmd159 != 0)) && ((l_c160 ? l_ls1133 : l_ls0132) < l_q161))) {
      const int l_c164 = ((l_cmd159 >= 4) ? 1 : 0);
      const int l_op165 = (int)((p.op_pk >> ((2 * ((l_c164) * 3 + (((l_cmd159 - (((l_cmd159 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v166 = (int)((p.val_pk >> ((2 * ((l_c164) * 3 + (((l_cmd159 - (((l_cmd159 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x167 = 0;
      if ((l_op165 == 1)) {
        l_kv131 = (1 | (l_v166 << 3));
        l_x167 = 7;
      }
      if ((l_op165 == 2)) {
        const int l_len168 = (l_kv131 & 7);
        l_kv131 = (((l_len168 + 1) | (l_kv131 & -8)) | (l_v166 << (3 + (l_len168 * 2))));
        l_x167 = l_kv131;
      }
      if ((l_op165 == 3)) {
        l_x167 = (((l_kv131 & 7) != 0) ? l_kv131 : 6);
      }
      if ((l_c160 != 0)) {
        l_ls1133 = l_q161;
      } else {
        l_ls0132 = l_q161;
      }
      if ((l_now163 && (l_act130 != 0))) {
        out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c160 + 1) - 1)) << 55) | ((Rec)((l_q161) & 3) << 0) | ((Rec)((l_x167) & 4095) << 2));
      }
    }
    if (l_now163) {
      l_so134 = 4;
    }
    const int l_e169 = arr_server_log(w, 3);
    const int l_cmd170 = ((l_e169 >> 8) & 7);
    const int l_c171 = ((l_cmd170 >= 4) ? 1 : 0);
    const int l_q172 = (l_cmd170 - (((l_cmd170 >= 4) ? 1 : 0) * 3));
    const int l_before173 = (4 < l_so0129);
    const int l_now174 = (((!l_before173) && (l_run135 != 0)) && ((l_e169 & 3) == 2));
    l_run135 = (((l_run135 != 0) && (l_before173 || l_now174)) ? 1 : 0);
    if ((((l_before173 || l_now174) && (l_cmd170 != 0)) && ((l_c171 ? l_ls1133 : l_ls0132) < l_q172))) {
      const int l_c175 = ((l_cmd170 >= 4) ? 1 : 0);
      const int l_op176 = (int)((p.op_pk >> ((2 * ((l_c175) * 3 + (((l_cmd170 - (((l_cmd170 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v177 = (int)((p.val_pk >> ((2 * ((l_c175) * 3 + (((l_cmd170 - (((l_cmd170 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x178 = 0;
      if ((l_op176 == 1)) {
        l_kv131 = (1 | (l_v177 << 3));
        l_x178 = 7;
      }
      if ((l_op176 == 2)) {
        const int l_len179 = (l_kv131 & 7);
        l_kv131 = (((l_len179 + 1) | (l_kv131 & -8)) | (l_v177 << (3 + (l_len179 * 2))));
        l_x178 = l_kv131;
      }
      if ((l_op176 == 3)) {
        l_x178 = (((l_kv131 & 7) != 0) ? l_kv131 : 6);
      }
      if ((l_c171 != 0)) {
        l_ls1133 = l_q172;
      } else {
        l_ls0132 = l_q172;
      }
      if ((l_now174 && (l_act130 != 0))) {
        out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c171 + 1) - 1)) << 55) | ((Rec)((l_q172) & 3) << 0) | ((Rec)((l_x178) & 4095) << 2));
      }
    }
    if (l_now174) {
      l_so134 = 5;
    }
    put(w, 14, 3, l_so134);
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_client_Reply(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    if (((get(w, 2, 1) != 0) && ((int)((r >> 0) & 3u) == get(w, 0, 2)))) {
      put(w, 3, 12, (int)((r >> 2) & 4095u));
      put(w, 2, 1, 0);
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int ht_client_ClientTimer(int i, uint32_t* w, int e, O& out, const Params& p) {
    (void)i; (void)w; (void)out; (void)p;
    const int tf_seq = (e >> 0) & 3;
    if (((get(w, 2, 1) != 0) && (tf_seq == get(w, 0, 2)))) {
      const int l_cid180 = (((i - first_client(p)) * 3) + tf_seq);
      if ((0 < p.servers)) {
        out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((l_cid180) & 7) << 0));
      }
      if ((1 < p.servers)) {
        out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((l_cid180) & 7) << 0));
      }
      if ((2 < p.servers)) {
        out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((l_cid180) & 7) << 0));
      }
      if (!push_timer_client(w, (((tf_seq) & 3) << 0) | (1 << 2))) return STEP_OVERFLOW;
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int on_message(int i, uint32_t* w, Rec r, O& out, const Params& p) {
    (void)w; (void)out;
    if (is_server(i, p)) {
      int fl = 0, rc;
      if (rec_type(r) == 0) rc = hm_server_Request(i, w, r, out, p, fl);  // Request
      else if (rec_type(r) == 2) rc = hm_server_P1a(i, w, r, out, p, fl);  // P1a
      else if (rec_type(r) == 3) rc = hm_server_P1b(i, w, r, out, p, fl);  // P1b
      else if (rec_type(r) == 4) rc = hm_server_P2a(i, w, r, out, p, fl);  // P2a
      else if (rec_type(r) == 5) rc = hm_server_P2b(i, w, r, out, p, fl);  // P2b
      else if (rec_type(r) == 6) rc = hm_server_Decision(i, w, r, out, p, fl);  // Decision
      else if (rec_type(r) == 7) rc = hm_server_Heartbeat(i, w, r, out, p, fl);  // Heartbeat
      else return STEP_EXCEPTION;  // no handler for this message (Node.handleMessage throws)
      if (rc == STEP_OK && fl) rc = tail_server(i, w, fl, out, p);  // the handlers' common tail
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
    if (is_server(i, p)) {
      const int q = deliverable_server(w, j);
      if (q < 0) return STEP_NULL;
      const int e = arr_server__timers(w, q);
      if (ttype(e) == 0) {  // Tick
        const int rc = ht_server_Tick(i, w, e, out, p);
        if (rc != STEP_OK) return rc;
        remove_timer_server(w, e);  // SearchState.stepTimer: the first equal entry
        return STEP_OK;
      }
      return STEP_EXCEPTION;  // no handler for this timer
    }
    if (is_client(i, p)) {
      const int q = deliverable_client(w, j);
      if (q < 0) return STEP_NULL;
      const int e = arr_client__timers(w, q);
      if (ttype(e) == 1) {  // ClientTimer
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
          const int n = get(w, 26, 2);
          for (int j = 0; j < n; j++) {
            const int x = sel_param(p.expected, (c - c0), (j + 1) - 1);
            if (x >= 0 && arr_client__results(w, j) != x) return PV_FALSE;
          }
        }
        return PV_TRUE;
      case DSL_PRED_CLIENTS_DONE:
        for (int c = c0; c < c0 + nc; c++)
          if (get(v.node(c), 26, 2) < wsize(c - c0, p)) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_DONE:
        if (pr.arg0 < c0 || pr.arg0 >= c0 + nc) return PV_THREW;
        return get(v.node((int)pr.arg0), 26, 2) >= wsize((int)pr.arg0 - c0, p) ? PV_TRUE : PV_FALSE;
      case DSL_PRED_NONE_DECIDED:
        for (int c = c0; c < c0 + nc; c++)
          if (get(v.node(c), 26, 2) > 0) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_HAS_RESULTS:
        if (pr.arg0 < c0 || pr.arg0 >= c0 + nc) return PV_THREW;
        return get(v.node((int)pr.arg0), 26, 2) == pr.arg1 ? PV_TRUE : PV_FALSE;
      case 400:  // LOGS_CONSISTENT_ALL_SLOTS / LOGS_CONSISTENT
      case 401:  // LOGS_CONSISTENT_ALL_SLOTS / LOGS_CONSISTENT
      {
        int l_isch181 = 0;
        int l_confl182 = 0;
        int l_chosen183 = 0;
        int l_count184 = 0;
        if ((0 < p.servers)) {
          const int l_e185 = arr_server_log(v.node(first_server(p) + 0), 0);
          if (((l_e185 & 3) == 2)) {
            const int l_x186 = ((((l_e185 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e185 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e185 >> 8) & 7) - (((((l_e185 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e185 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e185 >> 8) & 7) - (((((l_e185 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch181 != 0) && (l_x186 != l_chosen183))) {
              l_confl182 = 1;
            }
            l_chosen183 = l_x186;
            l_isch181 = 1;
          }
        }
        if ((1 < p.servers)) {
          const int l_e187 = arr_server_log(v.node(first_server(p) + 1), 0);
          if (((l_e187 & 3) == 2)) {
            const int l_x188 = ((((l_e187 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e187 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e187 >> 8) & 7) - (((((l_e187 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e187 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e187 >> 8) & 7) - (((((l_e187 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch181 != 0) && (l_x188 != l_chosen183))) {
              l_confl182 = 1;
            }
            l_chosen183 = l_x188;
            l_isch181 = 1;
          }
        }
        if ((2 < p.servers)) {
          const int l_e189 = arr_server_log(v.node(first_server(p) + 2), 0);
          if (((l_e189 & 3) == 2)) {
            const int l_x190 = ((((l_e189 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e189 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e189 >> 8) & 7) - (((((l_e189 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e189 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e189 >> 8) & 7) - (((((l_e189 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch181 != 0) && (l_x190 != l_chosen183))) {
              l_confl182 = 1;
            }
            l_chosen183 = l_x190;
            l_isch181 = 1;
          }
        }
        if ((0 < p.servers)) {
          const int l_e191 = arr_server_log(v.node(first_server(p) + 0), 0);
          if ((((l_e191 & 3) != 0) && (((l_e191 & 3) != 1) || (((((l_e191 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e191 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e191 >> 8) & 7) - (((((l_e191 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e191 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e191 >> 8) & 7) - (((((l_e191 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen183)))) {
            l_count184 = (l_count184 + 1);
          }
        }
        if ((1 < p.servers)) {
          const int l_e192 = arr_server_log(v.node(first_server(p) + 1), 0);
          if ((((l_e192 & 3) != 0) && (((l_e192 & 3) != 1) || (((((l_e192 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e192 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e192 >> 8) & 7) - (((((l_e192 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e192 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e192 >> 8) & 7) - (((((l_e192 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen183)))) {
            l_count184 = (l_count184 + 1);
          }
        }
        if ((2 < p.servers)) {
          const int l_e193 = arr_server_log(v.node(first_server(p) + 2), 0);
          if ((((l_e193 & 3) != 0) && (((l_e193 & 3) != 1) || (((((l_e193 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e193 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e193 >> 8) & 7) - (((((l_e193 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e193 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e193 >> 8) & 7) - (((((l_e193 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen183)))) {
            l_count184 = (l_count184 + 1);
          }
        }
        if (((l_isch181 != 0) && ((l_confl182 != 0) || ((l_count184 * 2) <= p.servers)))) {
          return PV_FALSE;
        }
        int l_isch194 = 0;
        int l_confl195 = 0;
        int l_chosen196 = 0;
        int l_count197 = 0;
        if ((0 < p.servers)) {
          const int l_e198 = arr_server_log(v.node(first_server(p) + 0), 1);
          if (((l_e198 & 3) == 2)) {
            const int l_x199 = ((((l_e198 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e198 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e198 >> 8) & 7) - (((((l_e198 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e198 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e198 >> 8) & 7) - (((((l_e198 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch194 != 0) && (l_x199 != l_chosen196))) {
              l_confl195 = 1;
            }
            l_chosen196 = l_x199;
            l_isch194 = 1;
          }
        }
        if ((1 < p.servers)) {
          const int l_e200 = arr_server_log(v.node(first_server(p) + 1), 1);
          if (((l_e200 & 3) == 2)) {
            const int l_x201 = ((((l_e200 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e200 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e200 >> 8) & 7) - (((((l_e200 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e200 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e200 >> 8) & 7) - (((((l_e200 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch194 != 0) && (l_x201 != l_chosen196))) {
              l_confl195 = 1;
            }
            l_chosen196 = l_x201;
            l_isch194 = 1;
          }
        }
        if ((2 < p.servers)) {
          const int l_e202 = arr_server_log(v.node(first_server(p) + 2), 1);
          if (((l_e202 & 3) == 2)) {
            const int l_x203 = ((((l_e202 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e202 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e202 >> 8) & 7) - (((((l_e202 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e202 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e202 >> 8) & 7) - (((((l_e202 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch194 != 0) && (l_x203 != l_chosen196))) {
              l_confl195 = 1;
            }
            l_chosen196 = l_x203;
            l_isch194 = 1;
          }
        }
        if ((0 < p.servers)) {
          const int l_e204 = arr_server_log(v.node(first_server(p) + 0), 1);
          if ((((l_e204 & 3) != 0) && (((l_e204 & 3) != 1) || (((((l_e204 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e204 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e204 >> 8) & 7) - (((((l_e204 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e204 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e204 >> 8) & 7) - (((((l_e204 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen196)))) {
            l_count197 = (l_count197 + 1);
          }
        }
        if ((1 < p.servers)) {
          const int l_e205 = arr_server_log(v.node(first_server(p) + 1), 1);
          if ((((l_e205 & 3) != 0) && (((l_e205 & 3) != 1) || (((((l_e205 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e205 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e205 >> 8) & 7) - (((((l_e205 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e205 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e205 >> 8) & 7) - (((((l_e205 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen196)))) {
            l_count197 = (l_count197 + 1);
          }
        }
        if ((2 < p.servers)) {
          const int l_e206 = arr_server_log(v.node(first_server(p) + 2), 1);
          if ((((l_e206 & 3) != 0) && (((l_e206 & 3) != 1) || (((((l_e206 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e206 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e206 >> 8) & 7) - (((((l_e206 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e206 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e206 >> 8) & 7) - (((((l_e206 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen196)))) {
            l_count197 = (l_count197 + 1);
          }
        }
        if (((l_isch194 != 0) && ((l_confl195 != 0) || ((l_count197 * 2) <= p.servers)))) {
          return PV_FALSE;
        }
        int l_isch207 = 0;
        int l_confl208 = 0;
        int l_chosen209 = 0;
        int l_count210 = 0;
        if ((0 < p.servers)) {
          const int l_e211 = arr_server_log(v.node(first_server(p) + 0), 2);
          if (((l_e211 & 3) == 2)) {
            const int l_x212 = ((((l_e211 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e211 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e211 >> 8) & 7) - (((((l_e211 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e211 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e211 >> 8) & 7) - (((((l_e211 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch207 != 0) && (l_x212 != l_chosen209))) {
              l_confl208 = 1;
            }
            l_chosen209 = l_x212;
            l_isch207 = 1;
          }
        }
        if ((1 < p.servers)) {
          const int l_e213 = arr_server_log(v.node(first_server(p) + 1), 2);
          if (((l_e213 & 3) == 2)) {
            const int l_x214 = ((((l_e213 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e213 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e213 >> 8) & 7) - (((((l_e213 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e213 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e213 >> 8) & 7) - (((((l_e213 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch207 != 0) && (l_x214 != l_chosen209))) {
              l_confl208 = 1;
            }
            l_chosen209 = l_x214;
            l_isch207 = 1;
          }
        }
        if ((2 < p.servers)) {
          const int l_e215 = arr_server_log(v.node(first_server(p) + 2), 2);
          if (((l_e215 & 3) == 2)) {
            const int l_x216 = ((((l_e215 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e215 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e215 >> 8) & 7) - (((((l_e215 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e215 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e215 >> 8) & 7) - (((((l_e215 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch207 != 0) && (l_x216 != l_chosen209))) {
              l_confl208 = 1;
            }
            l_chosen209 = l_x216;
            l_isch207 = 1;
          }
        }
        if ((0 < p.servers)) {
          const int l_e217 = arr_server_log(v.node(first_server(p) + 0), 2);
          if ((((l_e217 & 3) != 0) && (((l_e217 & 3) != 1) || (((((l_e217 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e217 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e217 >> 8) & 7) - (((((l_e217 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e217 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e217 >> 8) & 7) - (((((l_e217 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen209)))) {
            l_count210 = (l_count210 + 1);
          }
        }
        if ((1 < p.servers)) {
          const int l_e218 = arr_server_log(v.node(first_server(p) + 1), 2);
          if ((((l_e218 & 3) != 0) && (((l_e218 & 3) != 1) || (((((l_e218 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e218 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e218 >> 8) & 7) - (((((l_e218 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e218 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e218 >> 8) & 7) - (((((l_e218 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen209)))) {
            l_count210 = (l_count210 + 1);
          }
        }
        if ((2 < p.servers)) {
          const int l_e219 = arr_server_log(v.node(first_server(p) + 2), 2);
          if ((((l_e219 & 3) != 0) && (((l_e219 & 3) != 1) || (((((l_e219 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e219 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e219 >> 8) & 7) - (((((l_e219 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e219 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e219 >> 8) & 7) - (((((l_e219 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen209)))) {
            l_count210 = (l_count210 + 1);
          }
        }
        if (((l_isch207 != 0) && ((l_confl208 != 0) || ((l_count210 * 2) <= p.servers)))) {
          return PV_FALSE;
        }
        int l_isch220 = 0;
        int l_confl221 = 0;
        int l_chosen222 = 0;
        int l_count223 = 0;
        if ((0 < p.servers)) {
          const int l_e224 = arr_server_log(v.node(first_server(p) + 0), 3);
          if (((l_e224 & 3) == 2)) {
            const int l_x225 = ((((l_e224 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e224 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e224 >> 8) & 7) - (((((l_e224 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e224 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e224 >> 8) & 7) - (((((l_e224 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch220 != 0) && (l_x225 != l_chosen222))) {
              l_confl221 = 1;
            }
            l_chosen222 = l_x225;
            l_isch220 = 1;
          }
        }
        if ((1 < p.servers)) {
          const int l_e226 = arr_server_log(v.node(first_server(p) + 1), 3);
          if (((l_e226 & 3) == 2)) {
            const int l_x227 = ((((l_e226 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e226 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e226 >> 8) & 7) - (((((l_e226 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e226 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e226 >> 8) & 7) - (((((l_e226 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch220 != 0) && (l_x227 != l_chosen222))) {
              l_confl221 = 1;
            }
            l_chosen222 = l_x227;
            l_isch220 = 1;
          }
        }
        if ((2 < p.servers)) {
          const int l_e228 = arr_server_log(v.node(first_server(p) + 2), 3);
          if (((l_e228 & 3) == 2)) {
            const int l_x229 = ((((l_e228 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e228 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e228 >> 8) & 7) - (((((l_e228 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e228 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e228 >> 8) & 7) - (((((l_e228 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch220 != 0) && (l_x229 != l_chosen222))) {
              l_confl221 = 1;
            }
            l_chosen222 = l_x229;
            l_isch220 = 1;
          }
        }
        if ((0 < p.servers)) {
          const int l_e230 = arr_server_log(v.node(first_server(p) + 0), 3);
          if ((((l_e230 & 3) != 0) && (((l_e230 & 3) != 1) || (((((l_e230 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e230 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e230 >> 8) & 7) - (((((l_e230 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e230 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e230 >> 8) & 7) - (((((l_e230 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen222)))) {
            l_count223 = (l_count223 + 1);
          }
        }
        if ((1 < p.servers)) {
          const int l_e231 = arr_server_log(v.node(first_server(p) + 1), 3);
          if ((((l_e231 & 3) != 0) && (((l_e231 & 3) != 1) || (((((l_e231 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e231 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e231 >> 8) & 7) - (((((l_e231 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e231 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e231 >> 8) & 7) - (((((l_e231 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen222)))) {
            l_count223 = (l_count223 + 1);
          }
        }
        if ((2 < p.servers)) {
          const int l_e232 = arr_server_log(v.node(first_server(p) + 2), 3);
          if ((((l_e232 & 3) != 0) && (((l_e232 & 3) != 1) || (((((l_e232 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e232 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e232 >> 8) & 7) - (((((l_e232 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e232 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e232 >> 8) & 7) - (((((l_e232 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen222)))) {
            l_count223 = (l_count223 + 1);
          }
        }
        if (((l_isch220 != 0) && ((l_confl221 != 0) || ((l_count223 * 2) <= p.servers)))) {
          return PV_FALSE;
        }
        return PV_TRUE;
        return PV_TRUE;
      }
      case 402:  // slotValid
      {
        const int l_i = (int)pr.arg0;
        if ((l_i < 1)) {
          return PV_FALSE;
        }
        if ((l_i > 4)) {
          return PV_TRUE;
        }
        int l_isch = 0;
        int l_confl = 0;
        int l_chosen = 0;
        int l_count = 0;
        if ((0 < p.servers)) {
          const int l_e233 = arr_server_log(v.node(first_server(p) + 0), (l_i - 1));
          if (((l_e233 & 3) == 2)) {
            const int l_x234 = ((((l_e233 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e233 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e233 >> 8) & 7) - (((((l_e233 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e233 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e233 >> 8) & 7) - (((((l_e233 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch != 0) && (l_x234 != l_chosen))) {
              l_confl = 1;
            }
            l_chosen = l_x234;
            l_isch = 1;
          }
        }
        if ((1 < p.servers)) {
          const int l_e235 = arr_server_log(v.node(first_server(p) + 1), (l_i - 1));
          if (((l_e235 & 3) == 2)) {
            const int l_x236 = ((((l_e235 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e235 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e235 >> 8) & 7) - (((((l_e235 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e235 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e235 >> 8) & 7) - (((((l_e235 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch != 0) && (l_x236 != l_chosen))) {
              l_confl = 1;
            }
            l_chosen = l_x236;
            l_isch = 1;
          }
        }
        if ((2 < p.servers)) {
          const int l_e237 = arr_server_log(v.node(first_server(p) + 2), (l_i - 1));
          if (((l_e237 & 3) == 2)) {
            const int l_x238 = ((((l_e237 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e237 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e237 >> 8) & 7) - (((((l_e237 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e237 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e237 >> 8) & 7) - (((((l_e237 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch != 0) && (l_x238 != l_chosen))) {
              l_confl = 1;
            }
            l_chosen = l_x238;
            l_isch = 1;
          }
        }
        if ((0 < p.servers)) {
          const int l_e239 = arr_server_log(v.node(first_server(p) + 0), (l_i - 1));
          if ((((l_e239 & 3) != 0) && (((l_e239 & 3) != 1) || (((((l_e239 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e239 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e239 >> 8) & 7) - (((((l_e239 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e239 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e239 >> 8) & 7) - (((((l_e239 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen)))) {
            l_count = (l_count + 1);
          }
        }
        if ((1 < p.servers)) {
          const int l_e240 = arr_server_log(v.node(first_server(p) + 1), (l_i - 1));
          if ((((l_e240 & 3) != 0) && (((l_e240 & 3) != 1) || (((((l_e240 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e240 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e240 >> 8) & 7) - (((((l_e240 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e240 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e240 >> 8) & 7) - (((((l_e240 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen)))) {
            l_count = (l_count + 1);
          }
        }
        if ((2 < p.servers)) {
          const int l_e241 = arr_server_log(v.node(first_server(p) + 2), (l_i - 1));
          if ((((l_e241 & 3) != 0) && (((l_e241 & 3) != 1) || (((((l_e241 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e241 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e241 >> 8) & 7) - (((((l_e241 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e241 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e241 >> 8) & 7) - (((((l_e241 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen)))) {
            l_count = (l_count + 1);
          }
        }
        if (((l_isch != 0) && ((l_confl != 0) || ((l_count * 2) <= p.servers)))) {
          return PV_FALSE;
        }
        return PV_TRUE;
        return PV_TRUE;
      }
      case 403:  // hasStatus
      {
        const int l_k242 = ((int)pr.arg0 - (first_server(p) + 1 - 1));
        if (((l_k242 < 0) || (l_k242 >= p.servers))) {
          return PV_THREW;
        }
        const int l_slot243 = ((int)pr.arg1 >> 4);
        int l_se244 = 0;
        if (((l_slot243 >= 1) && (l_slot243 <= 4))) {
          l_se244 = arr_server_log(v.node(first_server(p) + l_k242), (l_slot243 - 1));
        }
        if (((l_se244 & 3) == ((int)pr.arg1 & 15))) {
          return PV_TRUE;
        }
        return PV_FALSE;
        return PV_TRUE;
      }
      case 404:  // hasCommand
      {
        const int l_k245 = ((int)pr.arg0 - (first_server(p) + 1 - 1));
        if (((l_k245 < 0) || (l_k245 >= p.servers))) {
          return PV_THREW;
        }
        const int l_slot246 = ((int)pr.arg1 >> 8);
        int l_se247 = 0;
        if (((l_slot246 >= 1) && (l_slot246 <= 4))) {
          l_se247 = arr_server_log(v.node(first_server(p) + l_k245), (l_slot246 - 1));
        }
        const int l_cc = (((l_se247 & 3) == 0) ? 0 : ((((l_se247 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_se247 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_se247 >> 8) & 7) - (((((l_se247 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_se247 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_se247 >> 8) & 7) - (((((l_se247 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0));
        if ((l_cc == ((int)pr.arg1 & 255))) {
          return PV_TRUE;
        }
        return PV_FALSE;
        return PV_TRUE;
      }
      case 300:  // APPENDS_LINEARIZABLE
      {
        const int l_pres248 = ((0 < p.clients) && (0 < get(v.node(first_client(p) + 0), 26, 2)));
        if ((l_pres248 && ((int)((p.op_pk >> ((2 * ((0) * 3 + (0))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res249 = (l_pres248 ? arr_client__results(v.node(first_client(p) + 0), 0) : 0);
        const int l_rlen250 = (l_res249 & 7);
        if ((l_pres248 && (((l_rlen250 == 0) || (l_rlen250 > 4)) || (((l_res249 >> (1 + (l_rlen250 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((0) * 3 + (0))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        const int l_pres251 = ((0 < p.clients) && (1 < get(v.node(first_client(p) + 0), 26, 2)));
        if ((l_pres251 && ((int)((p.op_pk >> ((2 * ((0) * 3 + (1))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res252 = (l_pres251 ? arr_client__results(v.node(first_client(p) + 0), 1) : 0);
        const int l_rlen253 = (l_res252 & 7);
        if ((l_pres251 && (((l_rlen253 == 0) || (l_rlen253 > 4)) || (((l_res252 >> (1 + (l_rlen253 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((0) * 3 + (1))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        const int l_pres254 = ((0 < p.clients) && (2 < get(v.node(first_client(p) + 0), 26, 2)));
        if ((l_pres254 && ((int)((p.op_pk >> ((2 * ((0) * 3 + (2))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res255 = (l_pres254 ? arr_client__results(v.node(first_client(p) + 0), 2) : 0);
        const int l_rlen256 = (l_res255 & 7);
        if ((l_pres254 && (((l_rlen256 == 0) || (l_rlen256 > 4)) || (((l_res255 >> (1 + (l_rlen256 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((0) * 3 + (2))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        const int l_pres257 = ((1 < p.clients) && (0 < get(v.node(first_client(p) + 1), 26, 2)));
        if ((l_pres257 && ((int)((p.op_pk >> ((2 * ((1) * 3 + (0))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res258 = (l_pres257 ? arr_client__results(v.node(first_client(p) + 1), 0) : 0);
        const int l_rlen259 = (l_res258 & 7);
        if ((l_pres257 && (((l_rlen259 == 0) || (l_rlen259 > 4)) || (((l_res258 >> (1 + (l_rlen259 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((1) * 3 + (0))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        const int l_pres260 = ((1 < p.clients) && (1 < get(v.node(first_client(p) + 1), 26, 2)));
        if ((l_pres260 && ((int)((p.op_pk >> ((2 * ((1) * 3 + (1))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res261 = (l_pres260 ? arr_client__results(v.node(first_client(p) + 1), 1) : 0);
        const int l_rlen262 = (l_res261 & 7);
        if ((l_pres260 && (((l_rlen262 == 0) || (l_rlen262 > 4)) || (((l_res261 >> (1 + (l_rlen262 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((1) * 3 + (1))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        const int l_pres263 = ((1 < p.clients) && (2 < get(v.node(first_client(p) + 1), 26, 2)));
        if ((l_pres263 && ((int)((p.op_pk >> ((2 * ((1) * 3 + (2))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res264 = (l_pres263 ? arr_client__results(v.node(first_client(p) + 1), 2) : 0);
        const int l_rlen265 = (l_res264 & 7);
        if ((l_pres263 && (((l_rlen265 == 0) || (l_rlen265 > 4)) || (((l_res264 >> (1 + (l_rlen265 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((1) * 3 + (2))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        if ((l_pres248 && l_pres251)) {
          if ((l_rlen250 == l_rlen253)) {
            return PV_FALSE;
          }
          if ((((l_res249 >> 3) & ((1 << (((l_rlen250 < l_rlen253) ? l_rlen250 : l_rlen253) * 2)) - 1)) != ((l_res252 >> 3) & ((1 << (((l_rlen250 < l_rlen253) ? l_rlen250 : l_rlen253) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres248 && l_pres254)) {
          if ((l_rlen250 == l_rlen256)) {
            return PV_FALSE;
          }
          if ((((l_res249 >> 3) & ((1 << (((l_rlen250 < l_rlen256) ? l_rlen250 : l_rlen256) * 2)) - 1)) != ((l_res255 >> 3) & ((1 << (((l_rlen250 < l_rlen256) ? l_rlen250 : l_rlen256) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres248 && l_pres257)) {
          if ((l_rlen250 == l_rlen259)) {
            return PV_FALSE;
          }
          if ((((l_res249 >> 3) & ((1 << (((l_rlen250 < l_rlen259) ? l_rlen250 : l_rlen259) * 2)) - 1)) != ((l_res258 >> 3) & ((1 << (((l_rlen250 < l_rlen259) ? l_rlen250 : l_rlen259) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres248 && l_pres260)) {
          if ((l_rlen250 == l_rlen262)) {
            return PV_FALSE;
          }
          if ((((l_res249 >> 3) & ((1 << (((l_rlen250 < l_rlen262) ? l_rlen250 : l_rlen262) * 2)) - 1)) != ((l_res261 >> 3) & ((1 << (((l_rlen250 < l_rlen262) ? l_rlen250 : l_rlen262) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres248 && l_pres263)) {
          if ((l_rlen250 == l_rlen265)) {
            return PV_FALSE;
          }
          if ((((l_res249 >> 3) & ((1 << (((l_rlen250 < l_rlen265) ? l_rlen250 : l_rlen265) * 2)) - 1)) != ((l_res264 >> 3) & ((1 << (((l_rlen250 < l_rlen265) ? l_rlen250 : l_rlen265) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres251 && l_pres254)) {
          if ((l_rlen253 == l_rlen256)) {
            return PV_FALSE;
          }
          if ((((l_res252 >> 3) & ((1 << (((l_rlen253 < l_rlen256) ? l_rlen253 : l_rlen256) * 2)) - 1)) != ((l_res255 >> 3) & ((1 << (((l_rlen253 < l_rlen256) ? l_rlen253 : l_rlen256) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres251 && l_pres257)) {
          if ((l_rlen253 == l_rlen259)) {
            return PV_FALSE;
          }
          if ((((l_res252 >> 3) & ((1 << (((l_rlen253 < l_rlen259) ? l_rlen253 : l_rlen259) * 2)) - 1)) != ((l_res258 >> 3) & ((1 << (((l_rlen253 < l_rlen259) ? l_rlen253 : l_rlen259) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres251 && l_pres260)) {
          if ((l_rlen253 == l_rlen262)) {
            return PV_FALSE;
          }
          if ((((l_res252 >> 3) & ((1 << (((l_rlen253 < l_rlen262) ? l_rlen253 : l_rlen262) * 2)) - 1)) != ((l_res261 >> 3) & ((1 << (((l_rlen253 < l_rlen262) ? l_rlen253 : l_rlen262) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres251 && l_pres263)) {
          if ((l_rlen253 == l_rlen265)) {
            return PV_FALSE;
          }
          if ((((l_res252 >> 3) & ((1 << (((l_rlen253 < l_rlen265) ? l_rlen253 : l_rlen265) * 2)) - 1)) != ((l_res264 >> 3) & ((1 << (((l_rlen253 < l_rlen265) ? l_rlen253 : l_rlen265) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres254 && l_pres257)) {
          if ((l_rlen256 == l_rlen259)) {
            return PV_FALSE;
          }
          if ((((l_res255 >> 3) & ((1 << (((l_rlen256 < l_rlen259) ? l_rlen256 : l_rlen259) * 2)) - 1)) != ((l_res258 >> 3) & ((1 << (((l_rlen256 < l_rlen259) ? l_rlen256 : l_rlen259) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres254 && l_pres260)) {
          if ((l_rlen256 == l_rlen262)) {
            return PV_FALSE;
          }
          if ((((l_res255 >> 3) & ((1 << (((l_rlen256 < l_rlen262) ? l_rlen256 : l_rlen262) * 2)) - 1)) != ((l_res261 >> 3) & ((1 << (((l_rlen256 < l_rlen262) ? l_rlen256 : l_rlen262) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres254 && l_pres263)) {
          if ((l_rlen256 == l_rlen265)) {
            return PV_FALSE;
          }
          if ((((l_res255 >> 3) & ((1 << (((l_rlen256 < l_rlen265) ? l_rlen256 : l_rlen265) * 2)) - 1)) != ((l_res264 >> 3) & ((1 << (((l_rlen256 < l_rlen265) ? l_rlen256 : l_rlen265) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres257 && l_pres260)) {
          if ((l_rlen259 == l_rlen262)) {
            return PV_FALSE;
          }
          if ((((l_res258 >> 3) & ((1 << (((l_rlen259 < l_rlen262) ? l_rlen259 : l_rlen262) * 2)) - 1)) != ((l_res261 >> 3) & ((1 << (((l_rlen259 < l_rlen262) ? l_rlen259 : l_rlen262) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres257 && l_pres263)) {
          if ((l_rlen259 == l_rlen265)) {
            return PV_FALSE;
          }
          if ((((l_res258 >> 3) & ((1 << (((l_rlen259 < l_rlen265) ? l_rlen259 : l_rlen265) * 2)) - 1)) != ((l_res264 >> 3) & ((1 << (((l_rlen259 < l_rlen265) ? l_rlen259 : l_rlen265) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres260 && l_pres263)) {
          if ((l_rlen262 == l_rlen265)) {
            return PV_FALSE;
          }
          if ((((l_res261 >> 3) & ((1 << (((l_rlen262 < l_rlen265) ? l_rlen262 : l_rlen265) * 2)) - 1)) != ((l_res264 >> 3) & ((1 << (((l_rlen262 < l_rlen265) ? l_rlen262 : l_rlen265) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        return PV_TRUE;
        return PV_TRUE;
      }
      default:
        return PV_THREW;
    }
  }
  static uint32_t pred_reads(const DevPred& pr, const Params& p) {
    (void)pr; (void)p;
    if (pr.id == 400 || pr.id == 401) return (((1u << (p.servers)) - 1u) << first_server(p));
    if (pr.id == 402) return (((1u << (p.servers)) - 1u) << first_server(p));
    if (pr.id == 403) return (((1u << (p.servers)) - 1u) << first_server(p));
    if (pr.id == 404) return (((1u << (p.servers)) - 1u) << first_server(p));
    if (pr.id == 300) return (((1u << (p.clients)) - 1u) << first_client(p));
    const uint32_t clients = (((1u << (p.clients)) - 1u) << first_client(p));
    return (pr.id >= DSL_PRED_RESULTS_OK && pr.id <= DSL_PRED_CLIENT_HAS_RESULTS) ? clients : kReadsAll;
  }
  static DSL_HD bool pred_same(const DevPred& pr, const uint32_t* a, const uint32_t* b) {
    if (pr.id == 400 || pr.id == 401) return (((a[1] ^ b[1]) & 0x3fffffu) | ((a[2] ^ b[2]) & 0x3fffffu)) == 0;
    if (pr.id == 402) return (((a[1] ^ b[1]) & 0x3fffffu) | ((a[2] ^ b[2]) & 0x3fffffu)) == 0;
    if (pr.id == 403) return (((a[1] ^ b[1]) & 0x3fffffu) | ((a[2] ^ b[2]) & 0x3fffffu)) == 0;
    if (pr.id == 404) return (((a[1] ^ b[1]) & 0x3fffffu) | ((a[2] ^ b[2]) & 0x3fffffu)) == 0;
    if (pr.id == 300) return (((a[0] ^ b[0]) & 0xc000000u) | ((a[1] ^ b[1]) & 0xffffffu) | ((a[2] ^ b[2]) & 0xfffu)) == 0;
    if (pr.id >= DSL_PRED_RESULTS_OK && pr.id <= DSL_PRED_CLIENT_HAS_RESULTS) return (((a[0] ^ b[0]) & 0xc000000u) | ((a[1] ^ b[1]) & 0xffffffu) | ((a[2] ^ b[2]) & 0xfffu)) == 0;
    return same_words<kNodeWords>(a, b);
  }
  static bool known_predicate(int id) { return (id >= DSL_PRED_RESULTS_OK && id <= DSL_PRED_CLIENT_HAS_RESULTS) || id == 400 || id == 401 || id == 402 || id == 403 || id == 404 || id == 300; }
  static DSL_HD bool surely_noop(int i, const uint32_t* row, Rec r, const Params& p) {
    const uint32_t* w = row + i * kNodeWords;
    bool x = false;
    x = (is_server(i, p) && rec_type(r) == 0) ? (bool)((get(w, 6, 1) == 0)) : x;  // server <- Request
    x = (is_server(i, p) && rec_type(r) == 2) ? (bool)(((((int)((r >> 0) & 15u) << 2) | (int)((r >> 4) & 3u)) < ((get(w, 0, 4) << 2) | get(w, 4, 2)))) : x;  // server <- P1a
    x = (is_server(i, p) && rec_type(r) == 3) ? (bool)(((get(w, 7, 1) == 0) || ((((int)((r >> 0) & 15u) << 2) | (int)((r >> 4) & 3u)) != ((get(w, 0, 4) << 2) | get(w, 4, 2))))) : x;  // server <- P1b
    x = (is_server(i, p) && rec_type(r) == 4) ? (bool)(((((int)((r >> 0) & 15u) << 2) | (int)((r >> 4) & 3u)) < ((get(w, 0, 4) << 2) | get(w, 4, 2)))) : x;  // server <- P2a
    x = (is_server(i, p) && rec_type(r) == 5) ? (bool)(((((get(w, 6, 1) == 0) || ((((int)((r >> 0) & 15u) << 2) | (int)((r >> 4) & 3u)) != ((get(w, 0, 4) << 2) | get(w, 4, 2)))) || ((arr_server_log(w, ((int)((r >> 6) & 7u) - 1)) & 3) != 1)) || ((((arr_server_votes(w, ((int)((r >> 6) & 7u) - 1)) >> (rec_from(r) - (first_server(p) + 1 - 1))) & 1) != 0) && (!(((((arr_server_votes(w, ((int)((r >> 6) & 7u) - 1)) & 1) + ((arr_server_votes(w, ((int)((r >> 6) & 7u) - 1)) >> 1) & 1)) + ((arr_server_votes(w, ((int)((r >> 6) & 7u) - 1)) >> 2) & 1)) * 2) > p.servers))))) : x;  // server <- P2b
    x = (is_server(i, p) && rec_type(r) == 6) ? (bool)(((arr_server_log(w, ((int)((r >> 0) & 7u) - 1)) & 3) == 2)) : x;  // server <- Decision
    x = (is_server(i, p) && rec_type(r) == 7) ? (bool)((((((int)((r >> 0) & 15u) << 2) | (int)((r >> 4) & 3u)) < ((get(w, 0, 4) << 2) | get(w, 4, 2))) || (((((int)((r >> 0) & 15u) << 2) | (int)((r >> 4) & 3u)) == ((get(w, 0, 4) << 2) | get(w, 4, 2))) && (get(w, 8, 1) != 0)))) : x;  // server <- Heartbeat
    x = (is_client(i, p) && rec_type(r) == 1) ? (bool)(((!((get(w, 2, 1) != 0) && ((int)((r >> 0) & 3u) == get(w, 0, 2)))) && (!((get(w, 26, 2) < wsize(i - first_client(p), p)) && (get(w, 3, 12) != 0))))) : x;  // client <- Reply
    return x;
  }
  static bool valid(const Params& p) {
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 1; c++)
        if (p.ncmd[r][c] < 0 || p.ncmd[r][c] > 3) return false;
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        if (p.op[r][c] < 0 || p.op[r][c] > 3) return false;
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        if (p.val[r][c] < 0 || p.val[r][c] > 3) return false;
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        if (p.expected[r][c] < -1 || p.expected[r][c] > 4095) return false;
    return p.servers >= 1 && p.servers <= 3 &&
           p.clients >= 1 && p.clients <= 2 &&
           p.servers >= 1 && p.servers <= 3 &&
           p.clients >= 1 && p.clients <= 2;
  }
  static Params from_desc(const dsl_protocol_desc& d) {
    Params p{};
    p.servers = d.n_params > 0 ? (int32_t)d.params[0] : 3;
    p.clients = d.n_params > 1 ? (int32_t)d.params[1] : 2;
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 1; c++) {
        const int q = 2 + r * 1 + c;
        p.ncmd[r][c] = d.n_params > q ? (int32_t)d.params[q] : 0;
      }
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++) {
        const int q = 4 + r * 3 + c;
        p.op[r][c] = d.n_params > q ? (int32_t)d.params[q] : 0;
      }
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++) {
        const int q = 10 + r * 3 + c;
        p.val[r][c] = d.n_params > q ? (int32_t)d.params[q] : 0;
      }
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++) {
        const int q = 16 + r * 3 + c;
        p.expected[r][c] = d.n_params > q ? (int32_t)d.params[q] : -1;
      }
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 1; c++)
        p.ncmd_pk |= (uint64_t)((uint32_t)p.ncmd[r][c] & 3u) << (2 * (r * 1 + c));
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        p.op_pk |= (uint64_t)((uint32_t)p.op[r][c] & 3u) << (2 * (r * 3 + c));
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        p.val_pk |= (uint64_t)((uint32_t)p.val[r][c] & 3u) << (2 * (r * 3 + c));
    return p;
  }
  static void describe_message(Rec r, dsl_event* e) {
    e->from = rec_from(r);
    e->to = rec_to(r);
    e->type = rec_type(r);
    e->n_fields = 0;
    if (e->type == 0) {
      e->n_fields = 1;
      e->fields[0] = (int64_t)((r >> 0) & 7u);
    }
    if (e->type == 1) {
      e->n_fields = 2;
      e->fields[0] = (int64_t)((r >> 0) & 3u);
      e->fields[1] = (int64_t)((r >> 2) & 4095u);
    }
    if (e->type == 2) {
      e->n_fields = 2;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
      e->fields[1] = (int64_t)((r >> 4) & 3u);
    }
    if (e->type == 3) {
      e->n_fields = 6;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
      e->fields[1] = (int64_t)((r >> 4) & 3u);
      e->fields[2] = (int64_t)((r >> 6) & 2047u);
      e->fields[3] = (int64_t)((r >> 17) & 2047u);
      e->fields[4] = (int64_t)((r >> 28) & 2047u);
      e->fields[5] = (int64_t)((r >> 39) & 2047u);
    }
    if (e->type == 4) {
      e->n_fields = 4;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
      e->fields[1] = (int64_t)((r >> 4) & 3u);
      e->fields[2] = (int64_t)((r >> 6) & 7u);
      e->fields[3] = (int64_t)((r >> 9) & 7u);
    }
    if (e->type == 5) {
      e->n_fields = 3;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
      e->fields[1] = (int64_t)((r >> 4) & 3u);
      e->fields[2] = (int64_t)((r >> 6) & 7u);
    }
    if (e->type == 6) {
      e->n_fields = 2;
      e->fields[0] = (int64_t)((r >> 0) & 7u);
      e->fields[1] = (int64_t)((r >> 3) & 7u);
    }
    if (e->type == 7) {
      e->n_fields = 2;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
      e->fields[1] = (int64_t)((r >> 4) & 3u);
    }
  }
  static void describe_timer(int i, const uint32_t* w, int j, const Params& p, dsl_event* e) {
    e->is_timer = 1;
    e->from = e->to = i;
    (void)w; (void)j; (void)p;
    if (is_server(i, p)) {
      const int q = deliverable_server(w, j);
      if (q < 0) return;
      const int x = arr_server__timers(w, q);
      e->type = 8 + ttype(x);
      int mn = 0, mx = 0;
      tbounds(ttype(x), mn, mx);
      e->timer_min = mn;
      e->timer_max = mx;
      if (ttype(x) == 0) {
        e->n_fields = 0;
      }
      if (ttype(x) == 1) {
        e->n_fields = 1;
        e->fields[0] = (x >> 0) & 3;
      }
    }
    if (is_client(i, p)) {
      const int q = deliverable_client(w, j);
      if (q < 0) return;
      const int x = arr_client__timers(w, q);
      e->type = 8 + ttype(x);
      int mn = 0, mx = 0;
      tbounds(ttype(x), mn, mx);
      e->timer_min = mn;
      e->timer_max = mx;
      if (ttype(x) == 0) {
        e->n_fields = 0;
      }
      if (ttype(x) == 1) {
        e->n_fields = 1;
        e->fields[0] = (x >> 0) & 3;
      }
    }
  }
};

}  // namespace dsl
