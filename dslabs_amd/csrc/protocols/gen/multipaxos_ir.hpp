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
    const int l_cid179 = (((i - first_client(p)) * 3) + cmd);
    if ((0 < p.servers)) {
      out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((l_cid179) & 7) << 0));
    }
    if ((1 < p.servers)) {
      out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((l_cid179) & 7) << 0));
    }
    if ((2 < p.servers)) {
      out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((l_cid179) & 7) << 0));
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
    if (is_server(i, p)) return 1;  // [Tick] in every state
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
    // set Tick: the queue stays [Tick]
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_Request(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_cmd = (int)((r >> 0) & 7u);
    const int l_c = ((l_cmd >= 4) ? 1 : 0);
    const int l_q = (l_cmd - (((l_cmd >= 4) ? 1 : 0) * 3));
    const int l_upto180 = get(w, 14, 3);
    int l_kv181 = 0;
    int l_ls0182 = 0;
    int l_ls1183 = 0;
    int l_r184 = 0;
    const int l_cmd185 = ((arr_server_log(w, 0) >> 8) & 7);
    const int l_c186 = ((l_cmd185 >= 4) ? 1 : 0);
    const int l_q187 = (l_cmd185 - (((l_cmd185 >= 4) ? 1 : 0) * 3));
    if ((((1 < l_upto180) && (l_cmd185 != 0)) && ((l_c186 ? l_ls1183 : l_ls0182) < l_q187))) {
      const int l_c188 = ((l_cmd185 >= 4) ? 1 : 0);
      const int l_op189 = (int)((p.op_pk >> ((2 * ((l_c188) * 3 + (((l_cmd185 - (((l_cmd185 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v190 = (int)((p.val_pk >> ((2 * ((l_c188) * 3 + (((l_cmd185 - (((l_cmd185 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x191 = 0;
      if ((l_op189 == 1)) {
        l_kv181 = (1 | (l_v190 << 3));
        l_x191 = 7;
      }
      if ((l_op189 == 2)) {
        const int l_len192 = (l_kv181 & 7);
        l_kv181 = (((l_len192 + 1) | (l_kv181 & -8)) | (l_v190 << (3 + (l_len192 * 2))));
        l_x191 = l_kv181;
      }
      if ((l_op189 == 3)) {
        l_x191 = (((l_kv181 & 7) != 0) ? l_kv181 : 6);
      }
      if ((l_c186 != 0)) {
        l_ls1183 = l_q187;
      } else {
        l_ls0182 = l_q187;
      }
      if (((l_c186 == l_c) && (l_q187 == l_q))) {
        l_r184 = l_x191;
      }
    }
    const int l_cmd193 = ((arr_server_log(w, 1) >> 8) & 7);
    const int l_c194 = ((l_cmd193 >= 4) ? 1 : 0);
    const int l_q195 = (l_cmd193 - (((l_cmd193 >= 4) ? 1 : 0) * 3));
    if ((((2 < l_upto180) && (l_cmd193 != 0)) && ((l_c194 ? l_ls1183 : l_ls0182) < l_q195))) {
      const int l_c196 = ((l_cmd193 >= 4) ? 1 : 0);
      const int l_op197 = (int)((p.op_pk >> ((2 * ((l_c196) * 3 + (((l_cmd193 - (((l_cmd193 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v198 = (int)((p.val_pk >> ((2 * ((l_c196) * 3 + (((l_cmd193 - (((l_cmd193 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x199 = 0;
      if ((l_op197 == 1)) {
        l_kv181 = (1 | (l_v198 << 3));
        l_x199 = 7;
      }
      if ((l_op197 == 2)) {
        const int l_len200 = (l_kv181 & 7);
        l_kv181 = (((l_len200 + 1) | (l_kv181 & -8)) | (l_v198 << (3 + (l_len200 * 2))));
        l_x199 = l_kv181;
      }
      if ((l_op197 == 3)) {
        l_x199 = (((l_kv181 & 7) != 0) ? l_kv181 : 6);
      }
      if ((l_c194 != 0)) {
        l_ls1183 = l_q195;
      } else {
        l_ls0182 = l_q195;
      }
      if (((l_c194 == l_c) && (l_q195 == l_q))) {
        l_r184 = l_x199;
      }
    }
    const int l_cmd201 = ((arr_server_log(w, 2) >> 8) & 7);
    const int l_c202 = ((l_cmd201 >= 4) ? 1 : 0);
    const int l_q203 = (l_cmd201 - (((l_cmd201 >= 4) ? 1 : 0) * 3));
    if ((((3 < l_upto180) && (l_cmd201 != 0)) && ((l_c202 ? l_ls1183 : l_ls0182) < l_q203))) {
      const int l_c204 = ((l_cmd201 >= 4) ? 1 : 0);
      const int l_op205 = (int)((p.op_pk >> ((2 * ((l_c204) * 3 + (((l_cmd201 - (((l_cmd201 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v206 = (int)((p.val_pk >> ((2 * ((l_c204) * 3 + (((l_cmd201 - (((l_cmd201 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x207 = 0;
      if ((l_op205 == 1)) {
        l_kv181 = (1 | (l_v206 << 3));
        l_x207 = 7;
      }
      if ((l_op205 == 2)) {
        const int l_len208 = (l_kv181 & 7);
        l_kv181 = (((l_len208 + 1) | (l_kv181 & -8)) | (l_v206 << (3 + (l_len208 * 2))));
        l_x207 = l_kv181;
      }
      if ((l_op205 == 3)) {
        l_x207 = (((l_kv181 & 7) != 0) ? l_kv181 : 6);
      }
      if ((l_c202 != 0)) {
        l_ls1183 = l_q203;
      } else {
        l_ls0182 = l_q203;
      }
      if (((l_c202 == l_c) && (l_q203 == l_q))) {
        l_r184 = l_x207;
      }
    }
    const int l_cmd209 = ((arr_server_log(w, 3) >> 8) & 7);
    const int l_c210 = ((l_cmd209 >= 4) ? 1 : 0);
    const int l_q211 = (l_cmd209 - (((l_cmd209 >= 4) ? 1 : 0) * 3));
    if ((((4 < l_upto180) && (l_cmd209 != 0)) && ((l_c210 ? l_ls1183 : l_ls0182) < l_q211))) {
      const int l_c212 = ((l_cmd209 >= 4) ? 1 : 0);
      const int l_op213 = (int)((p.op_pk >> ((2 * ((l_c212) * 3 + (((l_cmd209 - (((l_cmd209 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v214 = (int)((p.val_pk >> ((2 * ((l_c212) * 3 + (((l_cmd209 - (((l_cmd209 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x215 = 0;
      if ((l_op213 == 1)) {
        l_kv181 = (1 | (l_v214 << 3));
        l_x215 = 7;
      }
      if ((l_op213 == 2)) {
        const int l_len216 = (l_kv181 & 7);
        l_kv181 = (((l_len216 + 1) | (l_kv181 & -8)) | (l_v214 << (3 + (l_len216 * 2))));
        l_x215 = l_kv181;
      }
      if ((l_op213 == 3)) {
        l_x215 = (((l_kv181 & 7) != 0) ? l_kv181 : 6);
      }
      if ((l_c210 != 0)) {
        l_ls1183 = l_q211;
      } else {
        l_ls0182 = l_q211;
      }
      if (((l_c210 == l_c) && (l_q211 == l_q))) {
        l_r184 = l_x215;
      }
    }
    const int l_ls = (l_c ? l_ls1183 : l_ls0182);
    if ((l_ls >= l_q)) {
      if (((get(w, 6, 1) != 0) && (l_ls == l_q))) {
        out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c + 1) - 1)) << 55) | ((Rec)((l_q) & 3) << 0) | ((Rec)((l_r184) & 4095) << 2));
      }
      return STEP_OK;
    }
    int l_slot = get(w, 17, 3);
    int l_inlog = 0;
    const int l_e217 = arr_server_log(w, 0);
    if ((((l_e217 & 3) != 0) && (2 > l_slot))) {
      l_slot = 2;
    }
    if ((((l_e217 & 3) != 0) && (((l_e217 >> 8) & 7) == l_cmd))) {
      l_inlog = 1;
    }
    const int l_e218 = arr_server_log(w, 1);
    if ((((l_e218 & 3) != 0) && (3 > l_slot))) {
      l_slot = 3;
    }
    if ((((l_e218 & 3) != 0) && (((l_e218 >> 8) & 7) == l_cmd))) {
      l_inlog = 1;
    }
    const int l_e219 = arr_server_log(w, 2);
    if ((((l_e219 & 3) != 0) && (4 > l_slot))) {
      l_slot = 4;
    }
    if ((((l_e219 & 3) != 0) && (((l_e219 >> 8) & 7) == l_cmd))) {
      l_inlog = 1;
    }
    const int l_e220 = arr_server_log(w, 3);
    if ((((l_e220 & 3) != 0) && (5 > l_slot))) {
      l_slot = 5;
    }
    if ((((l_e220 & 3) != 0) && (((l_e220 >> 8) & 7) == l_cmd))) {
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
      const int l_ccmd221 = ((arr_server_log(w, (l_slot - 1)) >> 8) & 7);
      arr_put_server_log(w, (l_slot - 1), ((2 | (0 << 2)) | (l_ccmd221 << 8)));
      arr_put_server_votes(w, (l_slot - 1), 0);
      if (((0 < p.servers) && (0 != (i - first_server(p))))) {
        out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd221) & 7) << 3));
      }
      if (((1 < p.servers) && (1 != (i - first_server(p))))) {
        out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd221) & 7) << 3));
      }
      if (((2 < p.servers) && (2 != (i - first_server(p))))) {
        out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd221) & 7) << 3));
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
    const int l_me222 = (int)((r >> 6) & 2047u);
    const int l_mm223 = arr_server_p1blog(w, 0);
    if (((l_me222 & 3) == 2)) {
      arr_put_server_p1blog(w, 0, ((2 | (0 << 2)) | (((l_me222 >> 8) & 7) << 8)));
    } else {
      if (((((l_me222 & 3) == 1) && ((l_mm223 & 3) != 2)) && (((l_mm223 & 3) == 0) || (((l_mm223 >> 2) & 63) < ((l_me222 >> 2) & 63))))) {
        arr_put_server_p1blog(w, 0, l_me222);
      }
    }
    const int l_me224 = (int)((r >> 17) & 2047u);
    const int l_mm225 = arr_server_p1blog(w, 1);
    if (((l_me224 & 3) == 2)) {
      arr_put_server_p1blog(w, 1, ((2 | (0 << 2)) | (((l_me224 >> 8) & 7) << 8)));
    } else {
      if (((((l_me224 & 3) == 1) && ((l_mm225 & 3) != 2)) && (((l_mm225 & 3) == 0) || (((l_mm225 >> 2) & 63) < ((l_me224 >> 2) & 63))))) {
        arr_put_server_p1blog(w, 1, l_me224);
      }
    }
    const int l_me226 = (int)((r >> 28) & 2047u);
    const int l_mm227 = arr_server_p1blog(w, 2);
    if (((l_me226 & 3) == 2)) {
      arr_put_server_p1blog(w, 2, ((2 | (0 << 2)) | (((l_me226 >> 8) & 7) << 8)));
    } else {
      if (((((l_me226 & 3) == 1) && ((l_mm227 & 3) != 2)) && (((l_mm227 & 3) == 0) || (((l_mm227 >> 2) & 63) < ((l_me226 >> 2) & 63))))) {
        arr_put_server_p1blog(w, 2, l_me226);
      }
    }
    const int l_me228 = (int)((r >> 39) & 2047u);
    const int l_mm229 = arr_server_p1blog(w, 3);
    if (((l_me228 & 3) == 2)) {
      arr_put_server_p1blog(w, 3, ((2 | (0 << 2)) | (((l_me228 >> 8) & 7) << 8)));
    } else {
      if (((((l_me228 & 3) == 1) && ((l_mm229 & 3) != 2)) && (((l_mm229 & 3) == 0) || (((l_mm229 >> 2) & 63) < ((l_me228 >> 2) & 63))))) {
        arr_put_server_p1blog(w, 3, l_me228);
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
    const int l_ccmd230 = ((arr_server_log(w, (l_slot - 1)) >> 8) & 7);
    arr_put_server_log(w, (l_slot - 1), ((2 | (0 << 2)) | (l_ccmd230 << 8)));
    arr_put_server_votes(w, (l_slot - 1), 0);
    if (((0 < p.servers) && (0 != (i - first_server(p))))) {
      out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd230) & 7) << 3));
    }
    if (((1 < p.servers) && (1 != (i - first_server(p))))) {
      out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd230) & 7) << 3));
    }
    if (((2 < p.servers) && (2 != (i - first_server(p))))) {
      out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((l_slot) & 7) << 0) | ((Rec)((l_ccmd230) & 7) << 3));
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
          const int l_me231 = arr_server_log(w, 0);
          const int l_mm232 = arr_server_p1blog(w, 0);
          if (((l_me231 & 3) == 2)) {
            arr_put_server_p1blog(w, 0, ((2 | (0 << 2)) | (((l_me231 >> 8) & 7) << 8)));
          } else {
            if (((((l_me231 & 3) == 1) && ((l_mm232 & 3) != 2)) && (((l_mm232 & 3) == 0) || (((l_mm232 >> 2) & 63) < ((l_me231 >> 2) & 63))))) {
              arr_put_server_p1blog(w, 0, l_me231);
            }
          }
          const int l_me233 = arr_server_log(w, 1);
          const int l_mm234 = arr_server_p1blog(w, 1);
          if (((l_me233 & 3) == 2)) {
            arr_put_server_p1blog(w, 1, ((2 | (0 << 2)) | (((l_me233 >> 8) & 7) << 8)));
          } else {
            if (((((l_me233 & 3) == 1) && ((l_mm234 & 3) != 2)) && (((l_mm234 & 3) == 0) || (((l_mm234 >> 2) & 63) < ((l_me233 >> 2) & 63))))) {
              arr_put_server_p1blog(w, 1, l_me233);
            }
          }
          const int l_me235 = arr_server_log(w, 2);
          const int l_mm236 = arr_server_p1blog(w, 2);
          if (((l_me235 & 3) == 2)) {
            arr_put_server_p1blog(w, 2, ((2 | (0 << 2)) | (((l_me235 >> 8) & 7) << 8)));
          } else {
            if (((((l_me235 & 3) == 1) && ((l_mm236 & 3) != 2)) && (((l_mm236 & 3) == 0) || (((l_mm236 >> 2) & 63) < ((l_me235 >> 2) & 63))))) {
              arr_put_server_p1blog(w, 2, l_me235);
            }
          }
          const int l_me237 = arr_server_log(w, 3);
          const int l_mm238 = arr_server_p1blog(w, 3);
          if (((l_me237 & 3) == 2)) {
            arr_put_server_p1blog(w, 3, ((2 | (0 << 2)) | (((l_me237 >> 8) & 7) << 8)));
          } else {
            if (((((l_me237 & 3) == 1) && ((l_mm238 & 3) != 2)) && (((l_mm238 & 3) == 0) || (((l_mm238 >> 2) & 63) < ((l_me237 >> 2) & 63))))) {
              arr_put_server_p1blog(w, 3, l_me237);
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
            const int l_mg239 = arr_server_p1blog(w, 0);
            const int l_mg240 = arr_server_p1blog(w, 1);
            const int l_mg241 = arr_server_p1blog(w, 2);
            const int l_mg242 = arr_server_p1blog(w, 3);
            int l_last243 = 0;
            if ((((l_mg239 & 3) != 0) || ((arr_server_log(w, 0) & 3) != 0))) {
              l_last243 = 1;
            }
            if ((((l_mg240 & 3) != 0) || ((arr_server_log(w, 1) & 3) != 0))) {
              l_last243 = 2;
            }
            if ((((l_mg241 & 3) != 0) || ((arr_server_log(w, 2) & 3) != 0))) {
              l_last243 = 3;
            }
            if ((((l_mg242 & 3) != 0) || ((arr_server_log(w, 3) & 3) != 0))) {
              l_last243 = 4;
            }
            arr_put_server_p1blog(w, 0, 0);
            arr_put_server_p1blog(w, 1, 0);
            arr_put_server_p1blog(w, 2, 0);
            arr_put_server_p1blog(w, 3, 0);
            if (((1 <= l_last243) && ((arr_server_log(w, 0) & 3) != 2))) {
              if (((l_mg239 & 3) == 2)) {
                arr_put_server_log(w, 0, ((2 | (0 << 2)) | (((l_mg239 >> 8) & 7) << 8)));
                arr_put_server_votes(w, 0, 0);
              } else {
                arr_put_server_log(w, (1 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg239 & 3) == 1) ? ((l_mg239 >> 8) & 7) : 0) << 8)));
                arr_put_server_votes(w, (1 - 1), (1 << (i - first_server(p))));
                if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg239 & 3) == 1) ? ((l_mg239 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg239 & 3) == 1) ? ((l_mg239 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg239 & 3) == 1) ? ((l_mg239 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
                  const int l_ccmd244 = ((arr_server_log(w, (1 - 1)) >> 8) & 7);
                  arr_put_server_log(w, (1 - 1), ((2 | (0 << 2)) | (l_ccmd244 << 8)));
                  arr_put_server_votes(w, (1 - 1), 0);
                  if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd244) & 7) << 3));
                  }
                  if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd244) & 7) << 3));
                  }
                  if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd244) & 7) << 3));
                  }
                }
              }
            }
            if (((2 <= l_last243) && ((arr_server_log(w, 1) & 3) != 2))) {
              if (((l_mg240 & 3) == 2)) {
                arr_put_server_log(w, 1, ((2 | (0 << 2)) | (((l_mg240 >> 8) & 7) << 8)));
                arr_put_server_votes(w, 1, 0);
              } else {
                arr_put_server_log(w, (2 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg240 & 3) == 1) ? ((l_mg240 >> 8) & 7) : 0) << 8)));
                arr_put_server_votes(w, (2 - 1), (1 << (i - first_server(p))));
                if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg240 & 3) == 1) ? ((l_mg240 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg240 & 3) == 1) ? ((l_mg240 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg240 & 3) == 1) ? ((l_mg240 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
                  const int l_ccmd245 = ((arr_server_log(w, (2 - 1)) >> 8) & 7);
                  arr_put_server_log(w, (2 - 1), ((2 | (0 << 2)) | (l_ccmd245 << 8)));
                  arr_put_server_votes(w, (2 - 1), 0);
                  if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd245) & 7) << 3));
                  }
                  if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd245) & 7) << 3));
                  }
                  if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd245) & 7) << 3));
                  }
                }
              }
            }
            if (((3 <= l_last243) && ((arr_server_log(w, 2) & 3) != 2))) {
              if (((l_mg241 & 3) == 2)) {
                arr_put_server_log(w, 2, ((2 | (0 << 2)) | (((l_mg241 >> 8) & 7) << 8)));
                arr_put_server_votes(w, 2, 0);
              } else {
                arr_put_server_log(w, (3 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg241 & 3) == 1) ? ((l_mg241 >> 8) & 7) : 0) << 8)));
                arr_put_server_votes(w, (3 - 1), (1 << (i - first_server(p))));
                if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg241 & 3) == 1) ? ((l_mg241 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg241 & 3) == 1) ? ((l_mg241 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg241 & 3) == 1) ? ((l_mg241 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
                  const int l_ccmd246 = ((arr_server_log(w, (3 - 1)) >> 8) & 7);
                  arr_put_server_log(w, (3 - 1), ((2 | (0 << 2)) | (l_ccmd246 << 8)));
                  arr_put_server_votes(w, (3 - 1), 0);
                  if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd246) & 7) << 3));
                  }
                  if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd246) & 7) << 3));
                  }
                  if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd246) & 7) << 3));
                  }
                }
              }
            }
            if (((4 <= l_last243) && ((arr_server_log(w, 3) & 3) != 2))) {
              if (((l_mg242 & 3) == 2)) {
                arr_put_server_log(w, 3, ((2 | (0 << 2)) | (((l_mg242 >> 8) & 7) << 8)));
                arr_put_server_votes(w, 3, 0);
              } else {
                arr_put_server_log(w, (4 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg242 & 3) == 1) ? ((l_mg242 >> 8) & 7) : 0) << 8)));
                arr_put_server_votes(w, (4 - 1), (1 << (i - first_server(p))));
                if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg242 & 3) == 1) ? ((l_mg242 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg242 & 3) == 1) ? ((l_mg242 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                  out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg242 & 3) == 1) ? ((l_mg242 >> 8) & 7) : 0)) & 7) << 9));
                }
                if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
                  const int l_ccmd247 = ((arr_server_log(w, (4 - 1)) >> 8) & 7);
                  arr_put_server_log(w, (4 - 1), ((2 | (0 << 2)) | (l_ccmd247 << 8)));
                  arr_put_server_votes(w, (4 - 1), 0);
                  if (((0 < p.servers) && (0 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd247) & 7) << 3));
                  }
                  if (((1 < p.servers) && (1 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd247) & 7) << 3));
                  }
                  if (((2 < p.servers) && (2 != (i - first_server(p))))) {
                    out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd247) & 7) << 3));
                  }
                }
              }
            }
            put(w, 17, 3, (l_last243 + 1));
            const int l_so0248 = get(w, 14, 3);
            const int l_act249 = get(w, 6, 1);
            int l_kv250 = 0;
            int l_ls0251 = 0;
            int l_ls1252 = 0;
            int l_so253 = l_so0248;
            int l_run254 = 1;
            const int l_e255 = arr_server_log(w, 0);
            const int l_cmd256 = ((l_e255 >> 8) & 7);
            const int l_c257 = ((l_cmd256 >= 4) ? 1 : 0);
            const int l_q258 = (l_cmd256 - (((l_cmd256 >= 4) ? 1 : 0) * 3));
            const int l_before259 = (1 < l_so0248);
            const int l_now260 = (((!l_before259) && (l_run254 != 0)) && ((l_e255 & 3) == 2));
            l_run254 = (((l_run254 != 0) && (l_before259 || l_now260)) ? 1 : 0);
            if ((((l_before259 || l_now260) && (l_cmd256 != 0)) && ((l_c257 ? l_ls1252 : l_ls0251) < l_q258))) {
              const int l_c261 = ((l_cmd256 >= 4) ? 1 : 0);
              const int l_op262 = (int)((p.op_pk >> ((2 * ((l_c261) * 3 + (((l_cmd256 - (((l_cmd256 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              const int l_v263 = (int)((p.val_pk >> ((2 * ((l_c261) * 3 + (((l_cmd256 - (((l_cmd256 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              int l_x264 = 0;
              if ((l_op262 == 1)) {
                l_kv250 = (1 | (l_v263 << 3));
                l_x264 = 7;
              }
              if ((l_op262 == 2)) {
                const int l_len265 = (l_kv250 & 7);
                l_kv250 = (((l_len265 + 1) | (l_kv250 & -8)) | (l_v263 << (3 + (l_len265 * 2))));
                l_x264 = l_kv250;
              }
              if ((l_op262 == 3)) {
                l_x264 = (((l_kv250 & 7) != 0) ? l_kv250 : 6);
              }
              if ((l_c257 != 0)) {
                l_ls1252 = l_q258;
              } else {
                l_ls0251 = l_q258;
              }
              if ((l_now260 && (l_act249 != 0))) {
                out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c257 + 1) - 1)) << 55) | ((Rec)((l_q258) & 3) << 0) | ((Rec)((l_x264) & 4095) << 2));
              }
            }
            if (l_now260) {
              l_so253 = 2;
            }
            const int l_e266 = arr_server_log(w, 1);
            const int l_cmd267 = ((l_e266 >> 8) & 7);
            const int l_c268 = ((l_cmd267 >= 4) ? 1 : 0);
            const int l_q269 = (l_cmd267 - (((l_cmd267 >= 4) ? 1 : 0) * 3));
            const int l_before270 = (2 < l_so0248);
            const int l_now271 = (((!l_before270) && (l_run254 != 0)) && ((l_e266 & 3) == 2));
            l_run254 = (((l_run254 != 0) && (l_before270 || l_now271)) ? 1 : 0);
            if ((((l_before270 || l_now271) && (l_cmd267 != 0)) && ((l_c268 ? l_ls1252 : l_ls0251) < l_q269))) {
              const int l_c272 = ((l_cmd267 >= 4) ? 1 : 0);
              const int l_op273 = (int)((p.op_pk >> ((2 * ((l_c272) * 3 + (((l_cmd267 - (((l_cmd267 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              const int l_v274 = (int)((p.val_pk >> ((2 * ((l_c272) * 3 + (((l_cmd267 - (((l_cmd267 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              int l_x275 = 0;
              if ((l_op273 == 1)) {
                l_kv250 = (1 | (l_v274 << 3));
                l_x275 = 7;
              }
              if ((l_op273 == 2)) {
                const int l_len276 = (l_kv250 & 7);
                l_kv250 = (((l_len276 + 1) | (l_kv250 & -8)) | (l_v274 << (3 + (l_len276 * 2))));
                l_x275 = l_kv250;
              }
              if ((l_op273 == 3)) {
                l_x275 = (((l_kv250 & 7) != 0) ? l_kv250 : 6);
              }
              if ((l_c268 != 0)) {
                l_ls1252 = l_q269;
              } else {
                l_ls0251 = l_q269;
              }
              if ((l_now271 && (l_act249 != 0))) {
                out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c268 + 1) - 1)) << 55) | ((Rec)((l_q269) & 3) << 0) | ((Rec)((l_x275) & 4095) << 2));
              }
            }
            if (l_now271) {
              l_so253 = 3;
            }
            const int l_e277 = arr_server_log(w, 2);
            const int l_cmd278 = ((l_e277 >> 8) & 7);
            const int l_c279 = ((l_cmd278 >= 4) ? 1 : 0);
            const int l_q280 = (l_cmd278 - (((l_cmd278 >= 4) ? 1 : 0) * 3));
            const int l_before281 = (3 < l_so0248);
            const int l_now282 = (((!l_before281) && (l_run254 != 0)) && ((l_e277 & 3) == 2));
            l_run254 = (((l_run254 != 0) && (l_before281 || l_now282)) ? 1 : 0);
            if ((((l_before281 || l_now282) && (l_cmd278 != 0)) && ((l_c279 ? l_ls1252 : l_ls0251) < l_q280))) {
              const int l_c283 = ((l_cmd278 >= 4) ? 1 : 0);
              const int l_op284 = (int)((p.op_pk >> ((2 * ((l_c283) * 3 + (((l_cmd278 - (((l_cmd278 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              const int l_v285 = (int)((p.val_pk >> ((2 * ((l_c283) * 3 + (((l_cmd278 - (((l_cmd278 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              int l_x286 = 0;
              if ((l_op284 == 1)) {
                l_kv250 = (1 | (l_v285 << 3));
                l_x286 = 7;
              }
              if ((l_op284 == 2)) {
                const int l_len287 = (l_kv250 & 7);
                l_kv250 = (((l_len287 + 1) | (l_kv250 & -8)) | (l_v285 << (3 + (l_len287 * 2))));
                l_x286 = l_kv250;
              }
              if ((l_op284 == 3)) {
                l_x286 = (((l_kv250 & 7) != 0) ? l_kv250 : 6);
              }
              if ((l_c279 != 0)) {
                l_ls1252 = l_q280;
              } else {
                l_ls0251 = l_q280;
              }
              if ((l_now282 && (l_act249 != 0))) {
                out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c279 + 1) - 1)) << 55) | ((Rec)((l_q280) & 3) << 0) | ((Rec)((l_x286) & 4095) << 2));
              }
            }
            if (l_now282) {
              l_so253 = 4;
            }
            const int l_e288 = arr_server_log(w, 3);
            const int l_cmd289 = ((l_e288 >> 8) & 7);
            const int l_c290 = ((l_cmd289 >= 4) ? 1 : 0);
            const int l_q291 = (l_cmd289 - (((l_cmd289 >= 4) ? 1 : 0) * 3));
            const int l_before292 = (4 < l_so0248);
            const int l_now293 = (((!l_before292) && (l_run254 != 0)) && ((l_e288 & 3) == 2));
            l_run254 = (((l_run254 != 0) && (l_before292 || l_now293)) ? 1 : 0);
            if ((((l_before292 || l_now293) && (l_cmd289 != 0)) && ((l_c290 ? l_ls1252 : l_ls0251) < l_q291))) {
              const int l_c294 = ((l_cmd289 >= 4) ? 1 : 0);
              const int l_op295 = (int)((p.op_pk >> ((2 * ((l_c294) * 3 + (((l_cmd289 - (((l_cmd289 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              const int l_v296 = (int)((p.val_pk >> ((2 * ((l_c294) * 3 + (((l_cmd289 - (((l_cmd289 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
              int l_x297 = 0;
              if ((l_op295 == 1)) {
                l_kv250 = (1 | (l_v296 << 3));
                l_x297 = 7;
              }
              if ((l_op295 == 2)) {
                const int l_len298 = (l_kv250 & 7);
                l_kv250 = (((l_len298 + 1) | (l_kv250 & -8)) | (l_v296 << (3 + (l_len298 * 2))));
                l_x297 = l_kv250;
              }
              if ((l_op295 == 3)) {
                l_x297 = (((l_kv250 & 7) != 0) ? l_kv250 : 6);
              }
              if ((l_c290 != 0)) {
                l_ls1252 = l_q291;
              } else {
                l_ls0251 = l_q291;
              }
              if ((l_now293 && (l_act249 != 0))) {
                out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c290 + 1) - 1)) << 55) | ((Rec)((l_q291) & 3) << 0) | ((Rec)((l_x297) & 4095) << 2));
              }
            }
            if (l_now293) {
              l_so253 = 5;
            }
            put(w, 14, 3, l_so253);
          }
        }
      }
    }
    // set Tick: the queue stays [Tick]
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int tail_server(int i, uint32_t* w, int fl, O& out, const Params& p) {
    (void)i; (void)w; (void)out; (void)p;
    if (((fl >> 1) & 1)) {
      put(w, 6, 1, 1);
      put(w, 7, 1, 0);
      put(w, 11, 3, 0);
      const int l_mg299 = arr_server_p1blog(w, 0);
      const int l_mg300 = arr_server_p1blog(w, 1);
      const int l_mg301 = arr_server_p1blog(w, 2);
      const int l_mg302 = arr_server_p1blog(w, 3);
      int l_last303 = 0;
      if ((((l_mg299 & 3) != 0) || ((arr_server_log(w, 0) & 3) != 0))) {
        l_last303 = 1;
      }
      if ((((l_mg300 & 3) != 0) || ((arr_server_log(w, 1) & 3) != 0))) {
        l_last303 = 2;
      }
      if ((((l_mg301 & 3) != 0) || ((arr_server_log(w, 2) & 3) != 0))) {
        l_last303 = 3;
      }
      if ((((l_mg302 & 3) != 0) || ((arr_server_log(w, 3) & 3) != 0))) {
        l_last303 = 4;
      }
      arr_put_server_p1blog(w, 0, 0);
      arr_put_server_p1blog(w, 1, 0);
      arr_put_server_p1blog(w, 2, 0);
      arr_put_server_p1blog(w, 3, 0);
      if (((1 <= l_last303) && ((arr_server_log(w, 0) & 3) != 2))) {
        if (((l_mg299 & 3) == 2)) {
          arr_put_server_log(w, 0, ((2 | (0 << 2)) | (((l_mg299 >> 8) & 7) << 8)));
          arr_put_server_votes(w, 0, 0);
        } else {
          arr_put_server_log(w, (1 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg299 & 3) == 1) ? ((l_mg299 >> 8) & 7) : 0) << 8)));
          arr_put_server_votes(w, (1 - 1), (1 << (i - first_server(p))));
          if (((0 < p.servers) && (0 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg299 & 3) == 1) ? ((l_mg299 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((1 < p.servers) && (1 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg299 & 3) == 1) ? ((l_mg299 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((2 < p.servers) && (2 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((1) & 7) << 6) | ((Rec)(((((l_mg299 & 3) == 1) ? ((l_mg299 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
            const int l_ccmd304 = ((arr_server_log(w, (1 - 1)) >> 8) & 7);
            arr_put_server_log(w, (1 - 1), ((2 | (0 << 2)) | (l_ccmd304 << 8)));
            arr_put_server_votes(w, (1 - 1), 0);
            if (((0 < p.servers) && (0 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd304) & 7) << 3));
            }
            if (((1 < p.servers) && (1 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd304) & 7) << 3));
            }
            if (((2 < p.servers) && (2 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((1) & 7) << 0) | ((Rec)((l_ccmd304) & 7) << 3));
            }
          }
        }
      }
      if (((2 <= l_last303) && ((arr_server_log(w, 1) & 3) != 2))) {
        if (((l_mg300 & 3) == 2)) {
          arr_put_server_log(w, 1, ((2 | (0 << 2)) | (((l_mg300 >> 8) & 7) << 8)));
          arr_put_server_votes(w, 1, 0);
        } else {
          arr_put_server_log(w, (2 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg300 & 3) == 1) ? ((l_mg300 >> 8) & 7) : 0) << 8)));
          arr_put_server_votes(w, (2 - 1), (1 << (i - first_server(p))));
          if (((0 < p.servers) && (0 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg300 & 3) == 1) ? ((l_mg300 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((1 < p.servers) && (1 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg300 & 3) == 1) ? ((l_mg300 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((2 < p.servers) && (2 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((2) & 7) << 6) | ((Rec)(((((l_mg300 & 3) == 1) ? ((l_mg300 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
            const int l_ccmd305 = ((arr_server_log(w, (2 - 1)) >> 8) & 7);
            arr_put_server_log(w, (2 - 1), ((2 | (0 << 2)) | (l_ccmd305 << 8)));
            arr_put_server_votes(w, (2 - 1), 0);
            if (((0 < p.servers) && (0 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd305) & 7) << 3));
            }
            if (((1 < p.servers) && (1 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd305) & 7) << 3));
            }
            if (((2 < p.servers) && (2 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((2) & 7) << 0) | ((Rec)((l_ccmd305) & 7) << 3));
            }
          }
        }
      }
      if (((3 <= l_last303) && ((arr_server_log(w, 2) & 3) != 2))) {
        if (((l_mg301 & 3) == 2)) {
          arr_put_server_log(w, 2, ((2 | (0 << 2)) | (((l_mg301 >> 8) & 7) << 8)));
          arr_put_server_votes(w, 2, 0);
        } else {
          arr_put_server_log(w, (3 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg301 & 3) == 1) ? ((l_mg301 >> 8) & 7) : 0) << 8)));
          arr_put_server_votes(w, (3 - 1), (1 << (i - first_server(p))));
          if (((0 < p.servers) && (0 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg301 & 3) == 1) ? ((l_mg301 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((1 < p.servers) && (1 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg301 & 3) == 1) ? ((l_mg301 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((2 < p.servers) && (2 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((3) & 7) << 6) | ((Rec)(((((l_mg301 & 3) == 1) ? ((l_mg301 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
            const int l_ccmd306 = ((arr_server_log(w, (3 - 1)) >> 8) & 7);
            arr_put_server_log(w, (3 - 1), ((2 | (0 << 2)) | (l_ccmd306 << 8)));
            arr_put_server_votes(w, (3 - 1), 0);
            if (((0 < p.servers) && (0 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd306) & 7) << 3));
            }
            if (((1 < p.servers) && (1 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd306) & 7) << 3));
            }
            if (((2 < p.servers) && (2 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((3) & 7) << 0) | ((Rec)((l_ccmd306) & 7) << 3));
            }
          }
        }
      }
      if (((4 <= l_last303) && ((arr_server_log(w, 3) & 3) != 2))) {
        if (((l_mg302 & 3) == 2)) {
          arr_put_server_log(w, 3, ((2 | (0 << 2)) | (((l_mg302 >> 8) & 7) << 8)));
          arr_put_server_votes(w, 3, 0);
        } else {
          arr_put_server_log(w, (4 - 1), ((1 | (((get(w, 0, 4) << 2) | get(w, 4, 2)) << 2)) | ((((l_mg302 & 3) == 1) ? ((l_mg302 >> 8) & 7) : 0) << 8)));
          arr_put_server_votes(w, (4 - 1), (1 << (i - first_server(p))));
          if (((0 < p.servers) && (0 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg302 & 3) == 1) ? ((l_mg302 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((1 < p.servers) && (1 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg302 & 3) == 1) ? ((l_mg302 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((2 < p.servers) && (2 != (i - first_server(p))))) {
            out.send(((Rec)4 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((4) & 7) << 6) | ((Rec)(((((l_mg302 & 3) == 1) ? ((l_mg302 >> 8) & 7) : 0)) & 7) << 9));
          }
          if (((((((1 << (i - first_server(p))) & 1) + (((1 << (i - first_server(p))) >> 1) & 1)) + (((1 << (i - first_server(p))) >> 2) & 1)) * 2) > p.servers)) {
            const int l_ccmd307 = ((arr_server_log(w, (4 - 1)) >> 8) & 7);
            arr_put_server_log(w, (4 - 1), ((2 | (0 << 2)) | (l_ccmd307 << 8)));
            arr_put_server_votes(w, (4 - 1), 0);
            if (((0 < p.servers) && (0 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd307) & 7) << 3));
            }
            if (((1 < p.servers) && (1 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd307) & 7) << 3));
            }
            if (((2 < p.servers) && (2 != (i - first_server(p))))) {
              out.send(((Rec)6 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((4) & 7) << 0) | ((Rec)((l_ccmd307) & 7) << 3));
            }
          }
        }
      }
      put(w, 17, 3, (l_last303 + 1));
    }
    const int l_so0308 = get(w, 14, 3);
    const int l_act309 = get(w, 6, 1);
    int l_kv310 = 0;
    int l_ls0311 = 0;
    int l_ls1312 = 0;
    int l_so313 = l_so0308;
    int l_run314 = 1;
    const int l_e315 = arr_server_log(w, 0);
    const int l_cmd316 = ((l_e315 >> 8) & 7);
    const int l_c317 = ((l_cmd316 >= 4) ? 1 : 0);
    const int l_q318 = (l_cmd316 - (((l_cmd316 >= 4) ? 1 : 0) * 3));
    const int l_before319 = (1 < l_so0308);
    const int l_now320 = (((!l_before319) && (l_run314 != 0)) && ((l_e315 & 3) == 2));
    l_run314 = (((l_run314 != 0) && (l_before319 || l_now320)) ? 1 : 0);
    if ((((l_before319 || l_now320) && (l_cmd316 != 0)) && ((l_c317 ? l_ls1312 : l_ls0311) < l_q318))) {
      const int l_c321 = ((l_cmd316 >= 4) ? 1 : 0);
      const int l_op322 = (int)((p.op_pk >> ((2 * ((l_c321) * 3 + (((l_cmd316 - (((l_cmd316 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v323 = (int)((p.val_pk >> ((2 * ((l_c321) * 3 + (((l_cmd316 - (((l_cmd316 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x324 = 0;
      if ((l_op322 == 1)) {
        l_kv310 = (1 | (l_v323 << 3));
        l_x324 = 7;
      }
      if ((l_op322 == 2)) {
        const int l_len325 = (l_kv310 & 7);
        l_kv310 = (((l_len325 + 1) | (l_kv310 & -8)) | (l_v323 << (3 + (l_len325 * 2))));
        l_x324 = l_kv310;
      }
      if ((l_op322 == 3)) {
        l_x324 = (((l_kv310 & 7) != 0) ? l_kv310 : 6);
      }
      if ((l_c317 != 0)) {
        l_ls1312 = l_q318;
      } else {
        l_ls0311 = l_q318;
      }
      if ((l_now320 && (l_act309 != 0))) {
        out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c317 + 1) - 1)) << 55) | ((Rec)((l_q318) & 3) << 0) | ((Rec)((l_x324) & 4095) << 2));
      }
    }
    if (l_now320) {
      l_so313 = 2;
    }
    const int l_e326 = arr_server_log(w, 1);
    const int l_cmd327 = ((l_e326 >> 8) & 7);
    const int l_c328 = ((l_cmd327 >= 4) ? 1 : 0);
    const int l_q329 = (l_cmd327 - (((l_cmd327 >= 4) ? 1 : 0) * 3));
    const int l_before330 = (2 < l_so0308);
    const int l_now331 = (((!l_before330) && (l_run314 != 0)) && ((l_e326 & 3) == 2));
    l_run314 = (((l_run314 != 0) && (l_before330 || l_now331)) ? 1 : 0);
    if ((((l_before330 || l_now331) && (l_cmd327 != 0)) && ((l_c328 ? l_ls1312 : l_ls0311) < l_q329))) {
      const int l_c332 = ((l_cmd327 >= 4) ? 1 : 0);
      const int l_op333 = (int)((p.op_pk >> ((2 * ((l_c332) * 3 + (((l_cmd327 - (((l_cmd327 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v334 = (int)((p.val_pk >> ((2 * ((l_c332) * 3 + (((l_cmd327 - (((l_cmd327 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x335 = 0;
      if ((l_op333 == 1)) {
        l_kv310 = (1 | (l_v334 << 3));
        l_x335 = 7;
      }
      if ((l_op333 == 2)) {
        const int l_len336 = (l_kv310 & 7);
        l_kv310 = (((l_len336 + 1) | (l_kv310 & -8)) | (l_v334 << (3 + (l_len336 * 2))));
        l_x335 = l_kv310;
      }
      if ((l_op333 == 3)) {
        l_x335 = (((l_kv310 & 7) != 0) ? l_kv310 : 6);
      }
      if ((l_c328 != 0)) {
        l_ls1312 = l_q329;
      } else {
        l_ls0311 = l_q329;
      }
      if ((l_now331 && (l_act309 != 0))) {
        out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c328 + 1) - 1)) << 55) | ((Rec)((l_q329) & 3) << 0) | ((Rec)((l_x335) & 4095) << 2));
      }
    }
    if (l_now331) {
      l_so313 = 3;
    }
    const int l_e337 = arr_server_log(w, 2);
    const int l_cmd338 = ((l_e337 >> 8) & 7);
    const int l_c339 = ((l_cmd338 >= 4) ? 1 : 0);
    const int l_q340 = (l_cmd338 - (((l_cmd338 >= 4) ? 1 : 0) * 3));
    const int l_before341 = (3 < l_so0308);
    const int l_now342 = (((!l_before341) && (l_run314 != 0)) && ((l_e337 & 3) == 2));
    l_run314 = (((l_run314 != 0) && (l_before341 || l_now342)) ? 1 : 0);
    if ((((l_before341 || l_now342) && (l_cmd338 != 0)) && ((l_c339 ? l_ls1312 : l_ls0311) < l_q340))) {
      const int l_c343 = ((l_cmd338 >= 4) ? 1 : 0);
      const int l_op344 = (int)((p.op_pk >> ((2 * ((l_c343) * 3 + (((l_cmd338 - (((l_cmd338 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v345 = (int)((p.val_pk >> ((2 * ((l_c343) * 3 + (((l_cmd338 - (((l_cmd338 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x346 = 0;
      if ((l_op344 == 1)) {
        l_kv310 = (1 | (l_v345 << 3));
        l_x346 = 7;
      }
      if ((l_op344 == 2)) {
        const int l_len347 = (l_kv310 & 7);
        l_kv310 = (((l_len347 + 1) | (l_kv310 & -8)) | (l_v345 << (3 + (l_len347 * 2))));
        l_x346 = l_kv310;
      }
      if ((l_op344 == 3)) {
        l_x346 = (((l_kv310 & 7) != 0) ? l_kv310 : 6);
      }
      if ((l_c339 != 0)) {
        l_ls1312 = l_q340;
      } else {
        l_ls0311 = l_q340;
      }
      if ((l_now342 && (l_act309 != 0))) {
        out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c339 + 1) - 1)) << 55) | ((Rec)((l_q340) & 3) << 0) | ((Rec)((l_x346) & 4095) << 2));
      }
    }
    if (l_now342) {
      l_so313 = 4;
    }
    const int l_e348 = arr_server_log(w, 3);
    const int l_cmd349 = ((l_e348 >> 8) & 7);
    const int l_c350 = ((l_cmd349 >= 4) ? 1 : 0);
    const int l_q351 = (l_cmd349 - (((l_cmd349 >= 4) ? 1 : 0) * 3));
    const int l_before352 = (4 < l_so0308);
    const int l_now353 = (((!l_before352) && (l_run314 != 0)) && ((l_e348 & 3) == 2));
    l_run314 = (((l_run314 != 0) && (l_before352 || l_now353)) ? 1 : 0);
    if ((((l_before352 || l_now353) && (l_cmd349 != 0)) && ((l_c350 ? l_ls1312 : l_ls0311) < l_q351))) {
      const int l_c354 = ((l_cmd349 >= 4) ? 1 : 0);
      const int l_op355 = (int)((p.op_pk >> ((2 * ((l_c354) * 3 + (((l_cmd349 - (((l_cmd349 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      const int l_v356 = (int)((p.val_pk >> ((2 * ((l_c354) * 3 + (((l_cmd349 - (((l_cmd349 >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u);
      int l_x357 = 0;
      if ((l_op355 == 1)) {
        l_kv310 = (1 | (l_v356 << 3));
        l_x357 = 7;
      }
      if ((l_op355 == 2)) {
        const int l_len358 = (l_kv310 & 7);
        l_kv310 = (((l_len358 + 1) | (l_kv310 & -8)) | (l_v356 << (3 + (l_len358 * 2))));
        l_x357 = l_kv310;
      }
      if ((l_op355 == 3)) {
        l_x357 = (((l_kv310 & 7) != 0) ? l_kv310 : 6);
      }
      if ((l_c350 != 0)) {
        l_ls1312 = l_q351;
      } else {
        l_ls0311 = l_q351;
      }
      if ((l_now353 && (l_act309 != 0))) {
        out.send(((Rec)1 << 61) | ((Rec)(i) << 58) | ((Rec)((first_client(p) + (l_c350 + 1) - 1)) << 55) | ((Rec)((l_q351) & 3) << 0) | ((Rec)((l_x357) & 4095) << 2));
      }
    }
    if (l_now353) {
      l_so313 = 5;
    }
    put(w, 14, 3, l_so313);
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
      const int l_cid359 = (((i - first_client(p)) * 3) + tf_seq);
      if ((0 < p.servers)) {
        out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 1 - 1)) << 55) | ((Rec)((l_cid359) & 7) << 0));
      }
      if ((1 < p.servers)) {
        out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 2 - 1)) << 55) | ((Rec)((l_cid359) & 7) << 0));
      }
      if ((2 < p.servers)) {
        out.send(((Rec)0 << 61) | ((Rec)(i) << 58) | ((Rec)((first_server(p) + 3 - 1)) << 55) | ((Rec)((l_cid359) & 7) << 0));
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
      if (j != 0) return STEP_NULL;
      return ht_server_Tick(i, w, (0 << 2), out, p);  // Tick
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
        uint32_t pn_server_0[kNodeWords];
        { const uint32_t* q_ = v.node(first_server(p) + 0);  // < kNodes: in bounds for any run
          for (int w_ = 0; w_ < kNodeWords; w_++) pn_server_0[w_] = q_[w_]; }
        uint32_t pn_server_1[kNodeWords];
        { const uint32_t* q_ = v.node(first_server(p) + 1);  // < kNodes: in bounds for any run
          for (int w_ = 0; w_ < kNodeWords; w_++) pn_server_1[w_] = q_[w_]; }
        uint32_t pn_server_2[kNodeWords];
        { const uint32_t* q_ = v.node(first_server(p) + 2);  // < kNodes: in bounds for any run
          for (int w_ = 0; w_ < kNodeWords; w_++) pn_server_2[w_] = q_[w_]; }
        int l_isch360 = 0;
        int l_confl361 = 0;
        int l_chosen362 = 0;
        int l_count363 = 0;
        if ((0 < p.servers)) {
          const int l_e364 = arr_server_log(pn_server_0, 0);
          if (((l_e364 & 3) == 2)) {
            const int l_x365 = ((((l_e364 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e364 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e364 >> 8) & 7) - (((((l_e364 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e364 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e364 >> 8) & 7) - (((((l_e364 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch360 != 0) && (l_x365 != l_chosen362))) {
              l_confl361 = 1;
            }
            l_chosen362 = l_x365;
            l_isch360 = 1;
          }
        }
        if ((1 < p.servers)) {
          const int l_e366 = arr_server_log(pn_server_1, 0);
          if (((l_e366 & 3) == 2)) {
            const int l_x367 = ((((l_e366 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e366 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e366 >> 8) & 7) - (((((l_e366 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e366 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e366 >> 8) & 7) - (((((l_e366 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch360 != 0) && (l_x367 != l_chosen362))) {
              l_confl361 = 1;
            }
            l_chosen362 = l_x367;
            l_isch360 = 1;
          }
        }
        if ((2 < p.servers)) {
          const int l_e368 = arr_server_log(pn_server_2, 0);
          if (((l_e368 & 3) == 2)) {
            const int l_x369 = ((((l_e368 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e368 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e368 >> 8) & 7) - (((((l_e368 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e368 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e368 >> 8) & 7) - (((((l_e368 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch360 != 0) && (l_x369 != l_chosen362))) {
              l_confl361 = 1;
            }
            l_chosen362 = l_x369;
            l_isch360 = 1;
          }
        }
        if ((0 < p.servers)) {
          const int l_e370 = arr_server_log(pn_server_0, 0);
          if ((((l_e370 & 3) != 0) && (((l_e370 & 3) != 1) || (((((l_e370 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e370 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e370 >> 8) & 7) - (((((l_e370 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e370 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e370 >> 8) & 7) - (((((l_e370 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen362)))) {
            l_count363 = (l_count363 + 1);
          }
        }
        if ((1 < p.servers)) {
          const int l_e371 = arr_server_log(pn_server_1, 0);
          if ((((l_e371 & 3) != 0) && (((l_e371 & 3) != 1) || (((((l_e371 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e371 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e371 >> 8) & 7) - (((((l_e371 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e371 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e371 >> 8) & 7) - (((((l_e371 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen362)))) {
            l_count363 = (l_count363 + 1);
          }
        }
        if ((2 < p.servers)) {
          const int l_e372 = arr_server_log(pn_server_2, 0);
          if ((((l_e372 & 3) != 0) && (((l_e372 & 3) != 1) || (((((l_e372 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e372 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e372 >> 8) & 7) - (((((l_e372 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e372 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e372 >> 8) & 7) - (((((l_e372 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen362)))) {
            l_count363 = (l_count363 + 1);
          }
        }
        if (((l_isch360 != 0) && ((l_confl361 != 0) || ((l_count363 * 2) <= p.servers)))) {
          return PV_FALSE;
        }
        int l_isch373 = 0;
        int l_confl374 = 0;
        int l_chosen375 = 0;
        int l_count376 = 0;
        if ((0 < p.servers)) {
          const int l_e377 = arr_server_log(pn_server_0, 1);
          if (((l_e377 & 3) == 2)) {
            const int l_x378 = ((((l_e377 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e377 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e377 >> 8) & 7) - (((((l_e377 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e377 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e377 >> 8) & 7) - (((((l_e377 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch373 != 0) && (l_x378 != l_chosen375))) {
              l_confl374 = 1;
            }
            l_chosen375 = l_x378;
            l_isch373 = 1;
          }
        }
        if ((1 < p.servers)) {
          const int l_e379 = arr_server_log(pn_server_1, 1);
          if (((l_e379 & 3) == 2)) {
            const int l_x380 = ((((l_e379 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e379 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e379 >> 8) & 7) - (((((l_e379 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e379 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e379 >> 8) & 7) - (((((l_e379 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch373 != 0) && (l_x380 != l_chosen375))) {
              l_confl374 = 1;
            }
            l_chosen375 = l_x380;
            l_isch373 = 1;
          }
        }
        if ((2 < p.servers)) {
          const int l_e381 = arr_server_log(pn_server_2, 1);
          if (((l_e381 & 3) == 2)) {
            const int l_x382 = ((((l_e381 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e381 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e381 >> 8) & 7) - (((((l_e381 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e381 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e381 >> 8) & 7) - (((((l_e381 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch373 != 0) && (l_x382 != l_chosen375))) {
              l_confl374 = 1;
            }
            l_chosen375 = l_x382;
            l_isch373 = 1;
          }
        }
        if ((0 < p.servers)) {
          const int l_e383 = arr_server_log(pn_server_0, 1);
          if ((((l_e383 & 3) != 0) && (((l_e383 & 3) != 1) || (((((l_e383 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e383 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e383 >> 8) & 7) - (((((l_e383 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e383 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e383 >> 8) & 7) - (((((l_e383 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen375)))) {
            l_count376 = (l_count376 + 1);
          }
        }
        if ((1 < p.servers)) {
          const int l_e384 = arr_server_log(pn_server_1, 1);
          if ((((l_e384 & 3) != 0) && (((l_e384 & 3) != 1) || (((((l_e384 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e384 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e384 >> 8) & 7) - (((((l_e384 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e384 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e384 >> 8) & 7) - (((((l_e384 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen375)))) {
            l_count376 = (l_count376 + 1);
          }
        }
        if ((2 < p.servers)) {
          const int l_e385 = arr_server_log(pn_server_2, 1);
          if ((((l_e385 & 3) != 0) && (((l_e385 & 3) != 1) || (((((l_e385 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e385 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e385 >> 8) & 7) - (((((l_e385 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e385 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e385 >> 8) & 7) - (((((l_e385 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen375)))) {
            l_count376 = (l_count376 + 1);
          }
        }
        if (((l_isch373 != 0) && ((l_confl374 != 0) || ((l_count376 * 2) <= p.servers)))) {
          return PV_FALSE;
        }
        int l_isch386 = 0;
        int l_confl387 = 0;
        int l_chosen388 = 0;
        int l_count389 = 0;
        if ((0 < p.servers)) {
          const int l_e390 = arr_server_log(pn_server_0, 2);
          if (((l_e390 & 3) == 2)) {
            const int l_x391 = ((((l_e390 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e390 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e390 >> 8) & 7) - (((((l_e390 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e390 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e390 >> 8) & 7) - (((((l_e390 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch386 != 0) && (l_x391 != l_chosen388))) {
              l_confl387 = 1;
            }
            l_chosen388 = l_x391;
            l_isch386 = 1;
          }
        }
        if ((1 < p.servers)) {
          const int l_e392 = arr_server_log(pn_server_1, 2);
          if (((l_e392 & 3) == 2)) {
            const int l_x393 = ((((l_e392 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e392 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e392 >> 8) & 7) - (((((l_e392 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e392 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e392 >> 8) & 7) - (((((l_e392 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch386 != 0) && (l_x393 != l_chosen388))) {
              l_confl387 = 1;
            }
            l_chosen388 = l_x393;
            l_isch386 = 1;
          }
        }
        if ((2 < p.servers)) {
          const int l_e394 = arr_server_log(pn_server_2, 2);
          if (((l_e394 & 3) == 2)) {
            const int l_x395 = ((((l_e394 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e394 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e394 >> 8) & 7) - (((((l_e394 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e394 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e394 >> 8) & 7) - (((((l_e394 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch386 != 0) && (l_x395 != l_chosen388))) {
              l_confl387 = 1;
            }
            l_chosen388 = l_x395;
            l_isch386 = 1;
          }
        }
        if ((0 < p.servers)) {
          const int l_e396 = arr_server_log(pn_server_0, 2);
          if ((((l_e396 & 3) != 0) && (((l_e396 & 3) != 1) || (((((l_e396 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e396 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e396 >> 8) & 7) - (((((l_e396 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e396 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e396 >> 8) & 7) - (((((l_e396 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen388)))) {
            l_count389 = (l_count389 + 1);
          }
        }
        if ((1 < p.servers)) {
          const int l_e397 = arr_server_log(pn_server_1, 2);
          if ((((l_e397 & 3) != 0) && (((l_e397 & 3) != 1) || (((((l_e397 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e397 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e397 >> 8) & 7) - (((((l_e397 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e397 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e397 >> 8) & 7) - (((((l_e397 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen388)))) {
            l_count389 = (l_count389 + 1);
          }
        }
        if ((2 < p.servers)) {
          const int l_e398 = arr_server_log(pn_server_2, 2);
          if ((((l_e398 & 3) != 0) && (((l_e398 & 3) != 1) || (((((l_e398 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e398 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e398 >> 8) & 7) - (((((l_e398 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e398 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e398 >> 8) & 7) - (((((l_e398 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen388)))) {
            l_count389 = (l_count389 + 1);
          }
        }
        if (((l_isch386 != 0) && ((l_confl387 != 0) || ((l_count389 * 2) <= p.servers)))) {
          return PV_FALSE;
        }
        int l_isch399 = 0;
        int l_confl400 = 0;
        int l_chosen401 = 0;
        int l_count402 = 0;
        if ((0 < p.servers)) {
          const int l_e403 = arr_server_log(pn_server_0, 3);
          if (((l_e403 & 3) == 2)) {
            const int l_x404 = ((((l_e403 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e403 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e403 >> 8) & 7) - (((((l_e403 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e403 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e403 >> 8) & 7) - (((((l_e403 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch399 != 0) && (l_x404 != l_chosen401))) {
              l_confl400 = 1;
            }
            l_chosen401 = l_x404;
            l_isch399 = 1;
          }
        }
        if ((1 < p.servers)) {
          const int l_e405 = arr_server_log(pn_server_1, 3);
          if (((l_e405 & 3) == 2)) {
            const int l_x406 = ((((l_e405 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e405 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e405 >> 8) & 7) - (((((l_e405 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e405 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e405 >> 8) & 7) - (((((l_e405 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch399 != 0) && (l_x406 != l_chosen401))) {
              l_confl400 = 1;
            }
            l_chosen401 = l_x406;
            l_isch399 = 1;
          }
        }
        if ((2 < p.servers)) {
          const int l_e407 = arr_server_log(pn_server_2, 3);
          if (((l_e407 & 3) == 2)) {
            const int l_x408 = ((((l_e407 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e407 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e407 >> 8) & 7) - (((((l_e407 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e407 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e407 >> 8) & 7) - (((((l_e407 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch399 != 0) && (l_x408 != l_chosen401))) {
              l_confl400 = 1;
            }
            l_chosen401 = l_x408;
            l_isch399 = 1;
          }
        }
        if ((0 < p.servers)) {
          const int l_e409 = arr_server_log(pn_server_0, 3);
          if ((((l_e409 & 3) != 0) && (((l_e409 & 3) != 1) || (((((l_e409 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e409 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e409 >> 8) & 7) - (((((l_e409 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e409 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e409 >> 8) & 7) - (((((l_e409 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen401)))) {
            l_count402 = (l_count402 + 1);
          }
        }
        if ((1 < p.servers)) {
          const int l_e410 = arr_server_log(pn_server_1, 3);
          if ((((l_e410 & 3) != 0) && (((l_e410 & 3) != 1) || (((((l_e410 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e410 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e410 >> 8) & 7) - (((((l_e410 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e410 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e410 >> 8) & 7) - (((((l_e410 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen401)))) {
            l_count402 = (l_count402 + 1);
          }
        }
        if ((2 < p.servers)) {
          const int l_e411 = arr_server_log(pn_server_2, 3);
          if ((((l_e411 & 3) != 0) && (((l_e411 & 3) != 1) || (((((l_e411 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e411 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e411 >> 8) & 7) - (((((l_e411 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e411 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e411 >> 8) & 7) - (((((l_e411 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen401)))) {
            l_count402 = (l_count402 + 1);
          }
        }
        if (((l_isch399 != 0) && ((l_confl400 != 0) || ((l_count402 * 2) <= p.servers)))) {
          return PV_FALSE;
        }
        return PV_TRUE;
        return PV_TRUE;
      }
      case 402:  // slotValid
      {
        uint32_t pn_server_0[kNodeWords];
        { const uint32_t* q_ = v.node(first_server(p) + 0);  // < kNodes: in bounds for any run
          for (int w_ = 0; w_ < kNodeWords; w_++) pn_server_0[w_] = q_[w_]; }
        uint32_t pn_server_1[kNodeWords];
        { const uint32_t* q_ = v.node(first_server(p) + 1);  // < kNodes: in bounds for any run
          for (int w_ = 0; w_ < kNodeWords; w_++) pn_server_1[w_] = q_[w_]; }
        uint32_t pn_server_2[kNodeWords];
        { const uint32_t* q_ = v.node(first_server(p) + 2);  // < kNodes: in bounds for any run
          for (int w_ = 0; w_ < kNodeWords; w_++) pn_server_2[w_] = q_[w_]; }
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
          const int l_e412 = arr_server_log(pn_server_0, (l_i - 1));
          if (((l_e412 & 3) == 2)) {
            const int l_x413 = ((((l_e412 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e412 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e412 >> 8) & 7) - (((((l_e412 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e412 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e412 >> 8) & 7) - (((((l_e412 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch != 0) && (l_x413 != l_chosen))) {
              l_confl = 1;
            }
            l_chosen = l_x413;
            l_isch = 1;
          }
        }
        if ((1 < p.servers)) {
          const int l_e414 = arr_server_log(pn_server_1, (l_i - 1));
          if (((l_e414 & 3) == 2)) {
            const int l_x415 = ((((l_e414 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e414 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e414 >> 8) & 7) - (((((l_e414 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e414 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e414 >> 8) & 7) - (((((l_e414 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch != 0) && (l_x415 != l_chosen))) {
              l_confl = 1;
            }
            l_chosen = l_x415;
            l_isch = 1;
          }
        }
        if ((2 < p.servers)) {
          const int l_e416 = arr_server_log(pn_server_2, (l_i - 1));
          if (((l_e416 & 3) == 2)) {
            const int l_x417 = ((((l_e416 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e416 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e416 >> 8) & 7) - (((((l_e416 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e416 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e416 >> 8) & 7) - (((((l_e416 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0);
            if (((l_isch != 0) && (l_x417 != l_chosen))) {
              l_confl = 1;
            }
            l_chosen = l_x417;
            l_isch = 1;
          }
        }
        if ((0 < p.servers)) {
          const int l_e418 = arr_server_log(pn_server_0, (l_i - 1));
          if ((((l_e418 & 3) != 0) && (((l_e418 & 3) != 1) || (((((l_e418 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e418 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e418 >> 8) & 7) - (((((l_e418 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e418 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e418 >> 8) & 7) - (((((l_e418 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen)))) {
            l_count = (l_count + 1);
          }
        }
        if ((1 < p.servers)) {
          const int l_e419 = arr_server_log(pn_server_1, (l_i - 1));
          if ((((l_e419 & 3) != 0) && (((l_e419 & 3) != 1) || (((((l_e419 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e419 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e419 >> 8) & 7) - (((((l_e419 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e419 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e419 >> 8) & 7) - (((((l_e419 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen)))) {
            l_count = (l_count + 1);
          }
        }
        if ((2 < p.servers)) {
          const int l_e420 = arr_server_log(pn_server_2, (l_i - 1));
          if ((((l_e420 & 3) != 0) && (((l_e420 & 3) != 1) || (((((l_e420 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_e420 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e420 >> 8) & 7) - (((((l_e420 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_e420 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_e420 >> 8) & 7) - (((((l_e420 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0) == l_chosen)))) {
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
        const int l_k421 = ((int)pr.arg0 - (first_server(p) + 1 - 1));
        if (((l_k421 < 0) || (l_k421 >= p.servers))) {
          return PV_THREW;
        }
        const int l_slot422 = ((int)pr.arg1 >> 4);
        int l_se423 = 0;
        if (((l_slot422 >= 1) && (l_slot422 <= 4))) {
          l_se423 = arr_server_log(v.node(first_server(p) + l_k421), (l_slot422 - 1));
        }
        if (((l_se423 & 3) == ((int)pr.arg1 & 15))) {
          return PV_TRUE;
        }
        return PV_FALSE;
        return PV_TRUE;
      }
      case 404:  // hasCommand
      {
        const int l_k424 = ((int)pr.arg0 - (first_server(p) + 1 - 1));
        if (((l_k424 < 0) || (l_k424 >= p.servers))) {
          return PV_THREW;
        }
        const int l_slot425 = ((int)pr.arg1 >> 8);
        int l_se426 = 0;
        if (((l_slot425 >= 1) && (l_slot425 <= 4))) {
          l_se426 = arr_server_log(v.node(first_server(p) + l_k424), (l_slot425 - 1));
        }
        const int l_cc = (((l_se426 & 3) == 0) ? 0 : ((((l_se426 >> 8) & 7) != 0) ? (((int)((p.op_pk >> ((2 * ((((((l_se426 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_se426 >> 8) & 7) - (((((l_se426 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u) << 2) | (int)((p.val_pk >> ((2 * ((((((l_se426 >> 8) & 7) >= 4) ? 1 : 0)) * 3 + (((((l_se426 >> 8) & 7) - (((((l_se426 >> 8) & 7) >= 4) ? 1 : 0) * 3)) - 1)))) & 63)) & 3u)) : 0));
        if ((l_cc == ((int)pr.arg1 & 255))) {
          return PV_TRUE;
        }
        return PV_FALSE;
        return PV_TRUE;
      }
      case 300:  // APPENDS_LINEARIZABLE
      {
        uint32_t pn_client_0[kNodeWords];
        { const uint32_t* q_ = v.node(first_client(p) + 0);  // < kNodes: in bounds for any run
          for (int w_ = 0; w_ < kNodeWords; w_++) pn_client_0[w_] = q_[w_]; }
        uint32_t pn_client_1[kNodeWords];
        { const uint32_t* q_ = v.node(first_client(p) + 1);  // < kNodes: in bounds for any run
          for (int w_ = 0; w_ < kNodeWords; w_++) pn_client_1[w_] = q_[w_]; }
        const int l_pres427 = ((0 < p.clients) && (0 < get(pn_client_0, 26, 2)));
        if ((l_pres427 && ((int)((p.op_pk >> ((2 * ((0) * 3 + (0))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res428 = (l_pres427 ? arr_client__results(pn_client_0, 0) : 0);
        const int l_rlen429 = (l_res428 & 7);
        if ((l_pres427 && (((l_rlen429 == 0) || (l_rlen429 > 4)) || (((l_res428 >> (1 + (l_rlen429 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((0) * 3 + (0))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        const int l_pres430 = ((0 < p.clients) && (1 < get(pn_client_0, 26, 2)));
        if ((l_pres430 && ((int)((p.op_pk >> ((2 * ((0) * 3 + (1))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res431 = (l_pres430 ? arr_client__results(pn_client_0, 1) : 0);
        const int l_rlen432 = (l_res431 & 7);
        if ((l_pres430 && (((l_rlen432 == 0) || (l_rlen432 > 4)) || (((l_res431 >> (1 + (l_rlen432 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((0) * 3 + (1))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        const int l_pres433 = ((0 < p.clients) && (2 < get(pn_client_0, 26, 2)));
        if ((l_pres433 && ((int)((p.op_pk >> ((2 * ((0) * 3 + (2))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res434 = (l_pres433 ? arr_client__results(pn_client_0, 2) : 0);
        const int l_rlen435 = (l_res434 & 7);
        if ((l_pres433 && (((l_rlen435 == 0) || (l_rlen435 > 4)) || (((l_res434 >> (1 + (l_rlen435 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((0) * 3 + (2))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        const int l_pres436 = ((1 < p.clients) && (0 < get(pn_client_1, 26, 2)));
        if ((l_pres436 && ((int)((p.op_pk >> ((2 * ((1) * 3 + (0))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res437 = (l_pres436 ? arr_client__results(pn_client_1, 0) : 0);
        const int l_rlen438 = (l_res437 & 7);
        if ((l_pres436 && (((l_rlen438 == 0) || (l_rlen438 > 4)) || (((l_res437 >> (1 + (l_rlen438 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((1) * 3 + (0))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        const int l_pres439 = ((1 < p.clients) && (1 < get(pn_client_1, 26, 2)));
        if ((l_pres439 && ((int)((p.op_pk >> ((2 * ((1) * 3 + (1))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res440 = (l_pres439 ? arr_client__results(pn_client_1, 1) : 0);
        const int l_rlen441 = (l_res440 & 7);
        if ((l_pres439 && (((l_rlen441 == 0) || (l_rlen441 > 4)) || (((l_res440 >> (1 + (l_rlen441 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((1) * 3 + (1))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        const int l_pres442 = ((1 < p.clients) && (2 < get(pn_client_1, 26, 2)));
        if ((l_pres442 && ((int)((p.op_pk >> ((2 * ((1) * 3 + (2))) & 63)) & 3u) != 2))) {
          return PV_THREW;
        }
        const int l_res443 = (l_pres442 ? arr_client__results(pn_client_1, 2) : 0);
        const int l_rlen444 = (l_res443 & 7);
        if ((l_pres442 && (((l_rlen444 == 0) || (l_rlen444 > 4)) || (((l_res443 >> (1 + (l_rlen444 * 2))) & 3) != (int)((p.val_pk >> ((2 * ((1) * 3 + (2))) & 63)) & 3u))))) {
          return PV_FALSE;
        }
        if ((l_pres427 && l_pres430)) {
          if ((l_rlen429 == l_rlen432)) {
            return PV_FALSE;
          }
          if ((((l_res428 >> 3) & ((1 << (((l_rlen429 < l_rlen432) ? l_rlen429 : l_rlen432) * 2)) - 1)) != ((l_res431 >> 3) & ((1 << (((l_rlen429 < l_rlen432) ? l_rlen429 : l_rlen432) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres427 && l_pres433)) {
          if ((l_rlen429 == l_rlen435)) {
            return PV_FALSE;
          }
          if ((((l_res428 >> 3) & ((1 << (((l_rlen429 < l_rlen435) ? l_rlen429 : l_rlen435) * 2)) - 1)) != ((l_res434 >> 3) & ((1 << (((l_rlen429 < l_rlen435) ? l_rlen429 : l_rlen435) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres427 && l_pres436)) {
          if ((l_rlen429 == l_rlen438)) {
            return PV_FALSE;
          }
          if ((((l_res428 >> 3) & ((1 << (((l_rlen429 < l_rlen438) ? l_rlen429 : l_rlen438) * 2)) - 1)) != ((l_res437 >> 3) & ((1 << (((l_rlen429 < l_rlen438) ? l_rlen429 : l_rlen438) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres427 && l_pres439)) {
          if ((l_rlen429 == l_rlen441)) {
            return PV_FALSE;
          }
          if ((((l_res428 >> 3) & ((1 << (((l_rlen429 < l_rlen441) ? l_rlen429 : l_rlen441) * 2)) - 1)) != ((l_res440 >> 3) & ((1 << (((l_rlen429 < l_rlen441) ? l_rlen429 : l_rlen441) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres427 && l_pres442)) {
          if ((l_rlen429 == l_rlen444)) {
            return PV_FALSE;
          }
          if ((((l_res428 >> 3) & ((1 << (((l_rlen429 < l_rlen444) ? l_rlen429 : l_rlen444) * 2)) - 1)) != ((l_res443 >> 3) & ((1 << (((l_rlen429 < l_rlen444) ? l_rlen429 : l_rlen444) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres430 && l_pres433)) {
          if ((l_rlen432 == l_rlen435)) {
            return PV_FALSE;
          }
          if ((((l_res431 >> 3) & ((1 << (((l_rlen432 < l_rlen435) ? l_rlen432 : l_rlen435) * 2)) - 1)) != ((l_res434 >> 3) & ((1 << (((l_rlen432 < l_rlen435) ? l_rlen432 : l_rlen435) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres430 && l_pres436)) {
          if ((l_rlen432 == l_rlen438)) {
            return PV_FALSE;
          }
          if ((((l_res431 >> 3) & ((1 << (((l_rlen432 < l_rlen438) ? l_rlen432 : l_rlen438) * 2)) - 1)) != ((l_res437 >> 3) & ((1 << (((l_rlen432 < l_rlen438) ? l_rlen432 : l_rlen438) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres430 && l_pres439)) {
          if ((l_rlen432 == l_rlen441)) {
            return PV_FALSE;
          }
          if ((((l_res431 >> 3) & ((1 << (((l_rlen432 < l_rlen441) ? l_rlen432 : l_rlen441) * 2)) - 1)) != ((l_res440 >> 3) & ((1 << (((l_rlen432 < l_rlen441) ? l_rlen432 : l_rlen441) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres430 && l_pres442)) {
          if ((l_rlen432 == l_rlen444)) {
            return PV_FALSE;
          }
          if ((((l_res431 >> 3) & ((1 << (((l_rlen432 < l_rlen444) ? l_rlen432 : l_rlen444) * 2)) - 1)) != ((l_res443 >> 3) & ((1 << (((l_rlen432 < l_rlen444) ? l_rlen432 : l_rlen444) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres433 && l_pres436)) {
          if ((l_rlen435 == l_rlen438)) {
            return PV_FALSE;
          }
          if ((((l_res434 >> 3) & ((1 << (((l_rlen435 < l_rlen438) ? l_rlen435 : l_rlen438) * 2)) - 1)) != ((l_res437 >> 3) & ((1 << (((l_rlen435 < l_rlen438) ? l_rlen435 : l_rlen438) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres433 && l_pres439)) {
          if ((l_rlen435 == l_rlen441)) {
            return PV_FALSE;
          }
          if ((((l_res434 >> 3) & ((1 << (((l_rlen435 < l_rlen441) ? l_rlen435 : l_rlen441) * 2)) - 1)) != ((l_res440 >> 3) & ((1 << (((l_rlen435 < l_rlen441) ? l_rlen435 : l_rlen441) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres433 && l_pres442)) {
          if ((l_rlen435 == l_rlen444)) {
            return PV_FALSE;
          }
          if ((((l_res434 >> 3) & ((1 << (((l_rlen435 < l_rlen444) ? l_rlen435 : l_rlen444) * 2)) - 1)) != ((l_res443 >> 3) & ((1 << (((l_rlen435 < l_rlen444) ? l_rlen435 : l_rlen444) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres436 && l_pres439)) {
          if ((l_rlen438 == l_rlen441)) {
            return PV_FALSE;
          }
          if ((((l_res437 >> 3) & ((1 << (((l_rlen438 < l_rlen441) ? l_rlen438 : l_rlen441) * 2)) - 1)) != ((l_res440 >> 3) & ((1 << (((l_rlen438 < l_rlen441) ? l_rlen438 : l_rlen441) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres436 && l_pres442)) {
          if ((l_rlen438 == l_rlen444)) {
            return PV_FALSE;
          }
          if ((((l_res437 >> 3) & ((1 << (((l_rlen438 < l_rlen444) ? l_rlen438 : l_rlen444) * 2)) - 1)) != ((l_res443 >> 3) & ((1 << (((l_rlen438 < l_rlen444) ? l_rlen438 : l_rlen444) * 2)) - 1)))) {
            return PV_FALSE;
          }
        }
        if ((l_pres439 && l_pres442)) {
          if ((l_rlen441 == l_rlen444)) {
            return PV_FALSE;
          }
          if ((((l_res440 >> 3) & ((1 << (((l_rlen441 < l_rlen444) ? l_rlen441 : l_rlen444) * 2)) - 1)) != ((l_res443 >> 3) & ((1 << (((l_rlen441 < l_rlen444) ? l_rlen441 : l_rlen444) * 2)) - 1)))) {
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
      if (j != 0) return;
      const int x = (0 << 2);
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
