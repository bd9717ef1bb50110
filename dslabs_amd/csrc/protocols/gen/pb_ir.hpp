// PBIR -- GENERATED from the protocol IR (dslabs_amd/ir/specs/pb.py) by dslabs_amd/ir/gen_device.py; do not edit.
// lab2 primary-backup with a ViewServer in the protocol IR -- BASELINE config C4's protocol, the
// same one as csrc/protocols/pb.hpp and oracle/proto_pb.hpp, restated once here and
// generated into both forms. It follows labs/lab2-primarybackup/README.md:154-330.
// 
// Nodes: "viewserver" (node 0), "server1..S" (nodes 1..S: a server's id in a view is its node index,
// 0 = null), "client1..c" after them (ClientWorkers around PBClients). ViewServer: the first pinging
// server is primary of view 1; a server is dead when it did not ping between the last two
// PingCheckTimers; a view changes only after its primary acknowledged it (Ping(current viewNum)); a
// check replaces a dead primary by a live backup (stuck otherwise), drops a dead backup and fills a
// missing backup from the lowest live idle server; a ping also fills a missing backup. PBServer: pings
// every 25 ms with its latest view number (the last started one while it is the primary of a view whose
// backup has not acknowledged the state transfer); a new view with it as primary and a backup sends
// StateTransfer (the application: two key values, two AMO entries); the backup installs it once and
// acknowledges; the primary serves requests once started, forwarding each to its backup and executing
// it when the backup has. PBClient: lab1's client plus a cached view. KV values are len:2 | tokens 2 bits
// each (at most 3); a result is type:2 | value << 2 (0 AppendResult, 1 GetResult, 2 KeyNotFound,
// 3 PutOk); an AMO entry is seq:2 | result:10.
// 
// Unlike the hand-written form, which keeps the ViewServer's highest ViewReply number as a field for
// hasViewReply(n), the predicates here read the network (q.any_msg), as PrimaryBackupTest's do
// (PrimaryBackupTest.java:104-156); the two forms have equal per-depth counts (the field is a
// function of the network).
#pragma once
#include "../../nodestate.hpp"

namespace dsl {

struct PBIR {
  static constexpr int kNodes = 6, kNodeWords = 3, kNetCap = 64, kMaxSends = 3;
  static constexpr bool kNetPreds = true;  // a predicate reads the network (view_any_record)
  using Self = PBIR;
  static constexpr int kMsgClasses = 9;
  using Rec = uint64_t;
  using State = StateOf<PBIR>;
  struct Params {
    int32_t servers;
    int32_t clients;
    int32_t ncmds;
    int32_t op[2][3];
    int32_t key[2][3];
    int32_t sym[2][3];
    int32_t expected[2][3];
    uint64_t op_pk;  // op[r][c] at bit 2 * (r * 3 + c) (from_desc)
    uint64_t key_pk;  // key[r][c] at bit 1 * (r * 3 + c) (from_desc)
    uint64_t sym_pk;  // sym[r][c] at bit 2 * (r * 3 + c) (from_desc)
  };
  static DSL_HD int get(const uint32_t* w, int bit, int width) { return field_get<kNodeWords>(w, bit, width); }
  static DSL_HD void put(uint32_t* w, int bit, int width, int v) { field_put<kNodeWords>(w, bit, width, v); }
  static DSL_HD int arr_server_kv(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[0]) >> (13 + 8 * (j))) & 255u);
  }
  static DSL_HD void arr_put_server_kv(uint32_t* w, int j, int v) {
    const int sh = 13 + 8 * (j);
    const uint64_t x = (((uint64_t)w[0]) & ~((uint64_t)255u << sh)) | ((uint64_t)((uint32_t)v & 255u) << sh);
    w[0] = (uint32_t)x;
  }
  static DSL_HD int arr_server_amo(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[1]) >> (0 + (j) / 2 * 32 + (j) % 2 * 12)) & 4095u);
  }
  static DSL_HD void arr_put_server_amo(uint32_t* w, int j, int v) {
    const int sh = 0 + (j) / 2 * 32 + (j) % 2 * 12;
    const uint64_t x = (((uint64_t)w[1]) & ~((uint64_t)4095u << sh)) | ((uint64_t)((uint32_t)v & 4095u) << sh);
    w[1] = (uint32_t)x;
  }
  static DSL_HD int arr_client__timers(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[1]) >> (0 + 4 * (j))) & 15u);
  }
  static DSL_HD void arr_put_client__timers(uint32_t* w, int j, int v) {
    const int sh = 0 + 4 * (j);
    const uint64_t x = (((uint64_t)w[1]) & ~((uint64_t)15u << sh)) | ((uint64_t)((uint32_t)v & 15u) << sh);
    w[1] = (uint32_t)x;
  }
  static DSL_HD int arr_client__results(const uint32_t* w, int j) {
    return (int)((((uint64_t)w[2]) >> (2 + (j) / 3 * 32 + (j) % 3 * 10)) & 1023u);
  }
  static DSL_HD void arr_put_client__results(uint32_t* w, int j, int v) {
    const int sh = 2 + (j) / 3 * 32 + (j) % 3 * 10;
    const uint64_t x = (((uint64_t)w[2]) & ~((uint64_t)1023u << sh)) | ((uint64_t)((uint32_t)v & 1023u) << sh);
    w[2] = (uint32_t)x;
  }
  static DSL_HD int rec_type(Rec r) { return (int)(r >> 60); }
  static DSL_HD int rec_from(Rec r) { return (int)((r >> 57) & 7); }
  static DSL_HD int rec_to(Rec r) { return (int)((r >> 54) & 7); }
  static DSL_HD int msg_class(Rec r) { return rec_type(r); }
  // node index -> kind: kinds are laid out in declaration order, instances consecutive
  static DSL_HD int num_nodes(const Params& p) { return 1 + p.servers + p.clients; }
  static DSL_HD int first_viewserver(const Params& p) { (void)p; return 0; }
  static DSL_HD bool is_viewserver(int i, const Params& p) { return i >= first_viewserver(p) && i < first_viewserver(p) + 1; }
  static DSL_HD int first_server(const Params& p) { (void)p; return 0 + 1; }
  static DSL_HD bool is_server(int i, const Params& p) { return i >= first_server(p) && i < first_server(p) + p.servers; }
  static DSL_HD int first_client(const Params& p) { (void)p; return 0 + 1 + p.servers; }
  static DSL_HD bool is_client(int i, const Params& p) { return i >= first_client(p) && i < first_client(p) + p.clients; }
  static DSL_HD int wsize(int c, const Params& p) { (void)c; (void)p; return p.ncmds; }
  // timer entries: fields from bit 0 in declaration order, the type above them
  static DSL_HD void tbounds(int type, int& mn, int& mx) {
    if (type == 0) { mn = 100; mx = 100; }
    if (type == 1) { mn = 25; mx = 25; }
    if (type == 2) { mn = 100; mx = 100; }
  }
  static DSL_HD int ttype(int e) { return e >> 2; }
  static DSL_HD bool push_timer_client(uint32_t* w, int e) {
    const int n = get(w, 18, 3);
    if (n >= 4) return false;
    arr_put_client__timers(w, n, e);
    put(w, 18, 3, n + 1);
    return true;
  }
  // TimerQueue.deliverable(): the index of deliverable entry j (-1: none), or their count (j < 0)
  static DSL_HD int deliverable_client(const uint32_t* w, int j) {
    const int n = get(w, 18, 3);
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
    const int n = get(w, 18, 3);
    int q0 = n;
    for (int q = n - 1; q >= 0; q--)
      if (arr_client__timers(w, q) == e) q0 = q;
    if (q0 >= n) return;
    for (int q = q0; q + 1 < n; q++) arr_put_client__timers(w, q, arr_client__timers(w, q + 1));
    arr_put_client__timers(w, n - 1, 0);
    put(w, 18, 3, n - 1);
  }
  template <class O>
  static DSL_HD int send_command_client(int i, uint32_t* w, int cmd, O& out, const Params& p) {
    (void)p;
    put(w, 6, 2, cmd);
    put(w, 8, 10, 0);
    if ((get(w, 4, 2) != 0)) {
      out.send(((Rec)3 << 60) | ((Rec)(i) << 57) | ((Rec)(get(w, 4, 2)) << 54) | ((Rec)((cmd) & 3) << 0));
    } else {
      out.send(((Rec)1 << 60) | ((Rec)(i) << 57) | ((Rec)((first_viewserver(p) + 1 - 1)) << 54));
    }
    if (!push_timer_client(w, (((cmd) & 3) << 0) | (2 << 2))) return STEP_OVERFLOW;
    return STEP_OK;
  }
  // ClientWorker.sendNextCommandWhilePossible (waitingOnResult == |results| < workload size)
  template <class O>
  static DSL_HD void client_worker_client(int i, uint32_t* w, O& out, const Params& p) {
    int n = get(w, 64, 2);
    const int res = get(w, 8, 10);
    const int ws = wsize(i - first_client(p), p);
    if (n < ws && res != 0) {
      if (n >= 3) { out.overflow = true; return; }
      arr_put_client__results(w, n, res);
      n++;
      put(w, 64, 2, n);
      if (n < ws && send_command_client(i, w, n + 1, out, p) != STEP_OK) out.overflow = true;
    }
  }
  template <class O>
  static DSL_HD void init_node(int i, uint32_t* w, O& out, const Params& p) {
    if (is_viewserver(i, p)) {
      if (init_viewserver(i, w, out, p) != STEP_OK) out.overflow = true;
      return;
    }
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
    if (is_viewserver(i, p)) return 1;  // [PingCheckTimer] in every state
    if (is_server(i, p)) return 1;  // [PingTimer] in every state
    if (is_client(i, p)) return deliverable_client(w, -1);
    (void)i; (void)w; (void)p;
    return 0;
  }
  template <class O>
  static DSL_HD int init_viewserver(int i, uint32_t* w, O& out, const Params& p) {
    (void)i; (void)p; (void)out;
    // set PingCheckTimer: the queue stays [PingCheckTimer]
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_viewserver_Ping(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_frm = rec_from(r);
    if (((l_frm < 1) || (l_frm > p.servers))) {
      return STEP_EXCEPTION;  // Ping from a node that is not a server
    }
    put(w, 9, 3, (get(w, 9, 3) | (1 << (l_frm - 1))));
    if ((get(w, 0, 4) == 0)) {
      put(w, 0, 4, 1);
      put(w, 4, 2, l_frm);
      put(w, 6, 2, 0);
      put(w, 8, 1, 0);
    }
    if (((l_frm == get(w, 4, 2)) && ((int)((r >> 0) & 15u) == get(w, 0, 4)))) {
      put(w, 8, 1, 1);
    }
    if (((get(w, 8, 1) == 1) && (get(w, 6, 2) == 0))) {
      const int l_live = (get(w, 9, 3) | get(w, 12, 3));
      int l_pidle = 0;
      if (((((3 <= p.servers) && (((l_live >> 2) & 1) == 1)) && (3 != get(w, 4, 2))) && (3 != 0))) {
        l_pidle = 3;
      }
      if (((((2 <= p.servers) && (((l_live >> 1) & 1) == 1)) && (2 != get(w, 4, 2))) && (2 != 0))) {
        l_pidle = 2;
      }
      if (((((1 <= p.servers) && (((l_live >> 0) & 1) == 1)) && (1 != get(w, 4, 2))) && (1 != 0))) {
        l_pidle = 1;
      }
      if ((l_pidle != 0)) {
        if (((get(w, 0, 4) + 1) > 15)) {
          return STEP_OVERFLOW;  // view number past 15
        }
        put(w, 0, 4, (get(w, 0, 4) + 1));
        put(w, 4, 2, get(w, 4, 2));
        put(w, 6, 2, l_pidle);
        put(w, 8, 1, 0);
      }
    }
    out.send(((Rec)2 << 60) | ((Rec)(i) << 57) | ((Rec)(l_frm) << 54) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((get(w, 6, 2)) & 3) << 6));
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_viewserver_GetView(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    out.send(((Rec)2 << 60) | ((Rec)(i) << 57) | ((Rec)(rec_from(r)) << 54) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((get(w, 4, 2)) & 3) << 4) | ((Rec)((get(w, 6, 2)) & 3) << 6));
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int ht_viewserver_PingCheckTimer(int i, uint32_t* w, int e, O& out, const Params& p) {
    (void)i; (void)w; (void)out; (void)p;
    const int l_alv = get(w, 9, 3);
    put(w, 12, 3, l_alv);
    put(w, 9, 3, 0);
    if (((get(w, 8, 1) == 1) && (get(w, 0, 4) != 0))) {
      const int l_pp = get(w, 4, 2);
      const int l_bb = get(w, 6, 2);
      const int l_palive = ((l_alv >> (l_pp - 1)) & 1);
      const int l_balive = ((l_bb != 0) && (((l_alv >> (l_bb - 1)) & 1) == 1));
      if ((l_palive == 0)) {
        if (l_balive) {
          int l_cidle1 = 0;
          if (((((3 <= p.servers) && (((l_alv >> 2) & 1) == 1)) && (3 != l_bb)) && (3 != 0))) {
            l_cidle1 = 3;
          }
          if (((((2 <= p.servers) && (((l_alv >> 1) & 1) == 1)) && (2 != l_bb)) && (2 != 0))) {
            l_cidle1 = 2;
          }
          if (((((1 <= p.servers) && (((l_alv >> 0) & 1) == 1)) && (1 != l_bb)) && (1 != 0))) {
            l_cidle1 = 1;
          }
          if (((get(w, 0, 4) + 1) > 15)) {
            return STEP_OVERFLOW;  // view number past 15
          }
          put(w, 0, 4, (get(w, 0, 4) + 1));
          put(w, 4, 2, l_bb);
          put(w, 6, 2, l_cidle1);
          put(w, 8, 1, 0);
        }
      }
      if ((((l_palive == 1) && (l_bb != 0)) && (!l_balive))) {
        int l_cidle2 = 0;
        if (((((3 <= p.servers) && (((l_alv >> 2) & 1) == 1)) && (3 != l_pp)) && (3 != 0))) {
          l_cidle2 = 3;
        }
        if (((((2 <= p.servers) && (((l_alv >> 1) & 1) == 1)) && (2 != l_pp)) && (2 != 0))) {
          l_cidle2 = 2;
        }
        if (((((1 <= p.servers) && (((l_alv >> 0) & 1) == 1)) && (1 != l_pp)) && (1 != 0))) {
          l_cidle2 = 1;
        }
        if (((get(w, 0, 4) + 1) > 15)) {
          return STEP_OVERFLOW;  // view number past 15
        }
        put(w, 0, 4, (get(w, 0, 4) + 1));
        put(w, 4, 2, l_pp);
        put(w, 6, 2, l_cidle2);
        put(w, 8, 1, 0);
      }
      if (((l_palive == 1) && (l_bb == 0))) {
        int l_cidle3 = 0;
        if (((((3 <= p.servers) && (((l_alv >> 2) & 1) == 1)) && (3 != l_pp)) && (3 != 0))) {
          l_cidle3 = 3;
        }
        if (((((2 <= p.servers) && (((l_alv >> 1) & 1) == 1)) && (2 != l_pp)) && (2 != 0))) {
          l_cidle3 = 2;
        }
        if (((((1 <= p.servers) && (((l_alv >> 0) & 1) == 1)) && (1 != l_pp)) && (1 != 0))) {
          l_cidle3 = 1;
        }
        if ((l_cidle3 != 0)) {
          if (((get(w, 0, 4) + 1) > 15)) {
            return STEP_OVERFLOW;  // view number past 15
          }
          put(w, 0, 4, (get(w, 0, 4) + 1));
          put(w, 4, 2, l_pp);
          put(w, 6, 2, l_cidle3);
          put(w, 8, 1, 0);
        }
      }
    }
    // set PingCheckTimer: the queue stays [PingCheckTimer]
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int init_server(int i, uint32_t* w, O& out, const Params& p) {
    (void)i; (void)p; (void)out;
    out.send(((Rec)0 << 60) | ((Rec)(i) << 57) | ((Rec)((first_viewserver(p) + 1 - 1)) << 54) | ((Rec)((0) & 15) << 0));
    // set PingTimer: the queue stays [PingTimer]
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_ViewReply(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    if (((int)((r >> 0) & 15u) <= get(w, 0, 4))) {
      return STEP_OK;
    }
    put(w, 0, 4, (int)((r >> 0) & 15u));
    put(w, 4, 2, (int)((r >> 4) & 3u));
    put(w, 6, 2, (int)((r >> 6) & 3u));
    put(w, 8, 1, 0);
    if (((int)((r >> 4) & 3u) == i)) {
      if (((int)((r >> 6) & 3u) == 0)) {
        put(w, 8, 1, 1);
        put(w, 9, 4, (int)((r >> 0) & 15u));
      } else {
        out.send(((Rec)5 << 60) | ((Rec)(i) << 57) | ((Rec)((int)((r >> 6) & 3u)) << 54) | ((Rec)(((int)((r >> 0) & 15u)) & 15) << 0) | ((Rec)(((int)((r >> 4) & 3u)) & 3) << 4) | ((Rec)(((int)((r >> 6) & 3u)) & 3) << 6) | ((Rec)((arr_server_kv(w, 0)) & 255) << 8) | ((Rec)((arr_server_kv(w, 1)) & 255) << 16) | ((Rec)((arr_server_amo(w, 0)) & 4095) << 24) | ((Rec)((arr_server_amo(w, 1)) & 4095) << 36));
      }
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_Request(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_seq = (int)((r >> 0) & 3u);
    const int l_c = (rec_from(r) - (first_client(p) + 1 - 1));
    if (((((l_c < 0) || (l_c >= p.clients)) || (l_seq < 1)) || (l_seq > p.ncmds))) {
      return STEP_EXCEPTION;  // request from an unknown client or command
    }
    if (((get(w, 4, 2) != i) || (get(w, 8, 1) == 0))) {
      return STEP_OK;
    }
    if ((get(w, 6, 2) == 0)) {
      int l_r = -1;
      const int l_amo = arr_server_amo(w, l_c);
      const int l_lastseq = (l_amo & 3);
      l_r = -1;
      if ((l_seq == l_lastseq)) {
        l_r = (l_amo >> 2);
      }
      if ((l_seq > l_lastseq)) {
        const int l_k = (l_seq - 1);
        const int l_op = (int)((p.op_pk >> ((2 * ((l_c) * 3 + (l_k))) & 63)) & 3u);
        const int l_key = (int)((p.key_pk >> ((1 * ((l_c) * 3 + (l_k))) & 63)) & 1u);
        const int l_sym = (int)((p.sym_pk >> ((2 * ((l_c) * 3 + (l_k))) & 63)) & 3u);
        const int l_v = arr_server_kv(w, l_key);
        if ((l_op == 0)) {
          if (((l_v & 3) != 0)) {
            l_r = ((l_v << 2) | 1);
          } else {
            l_r = 2;
          }
        }
        if ((l_op == 1)) {
          arr_put_server_kv(w, l_key, ((l_sym << 2) | 1));
          l_r = 3;
        }
        if ((l_op == 2)) {
          const int l_n = (l_v & 3);
          if ((l_n >= 3)) {
            return STEP_OVERFLOW;  // value longer than 3 tokens
          }
          const int l_v2 = (((l_v - l_n) | (l_n + 1)) | (l_sym << ((l_n * 2) + 2)));
          arr_put_server_kv(w, l_key, l_v2);
          l_r = (l_v2 << 2);
        }
        arr_put_server_amo(w, l_c, (l_seq | (l_r << 2)));
      }
      if ((l_r >= 0)) {
        out.send(((Rec)4 << 60) | ((Rec)(i) << 57) | ((Rec)(rec_from(r)) << 54) | ((Rec)((l_seq) & 3) << 0) | ((Rec)((l_r) & 1023) << 2));
      }
    } else {
      out.send(((Rec)7 << 60) | ((Rec)(i) << 57) | ((Rec)(get(w, 6, 2)) << 54) | ((Rec)((get(w, 0, 4)) & 15) << 0) | ((Rec)((rec_from(r)) & 7) << 4) | ((Rec)((l_seq) & 3) << 7));
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_StateTransfer(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    if (((((int)((r >> 0) & 15u) < get(w, 0, 4)) || ((int)((r >> 6) & 3u) != i)) || ((int)((r >> 4) & 3u) != rec_from(r)))) {
      return STEP_OK;
    }
    if ((((int)((r >> 0) & 15u) == get(w, 0, 4)) && (get(w, 8, 1) == 1))) {
      return STEP_OK;
    }
    put(w, 0, 4, (int)((r >> 0) & 15u));
    put(w, 4, 2, (int)((r >> 4) & 3u));
    put(w, 6, 2, (int)((r >> 6) & 3u));
    put(w, 8, 1, 1);
    arr_put_server_kv(w, 0, (int)((r >> 8) & 255u));
    arr_put_server_kv(w, 1, (int)((r >> 16) & 255u));
    arr_put_server_amo(w, 0, (int)((r >> 24) & 4095u));
    arr_put_server_amo(w, 1, (int)((r >> 36) & 4095u));
    out.send(((Rec)6 << 60) | ((Rec)(i) << 57) | ((Rec)(rec_from(r)) << 54) | ((Rec)(((int)((r >> 0) & 15u)) & 15) << 0));
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_StateTransferAck(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    if ((((get(w, 4, 2) == i) && (get(w, 8, 1) == 0)) && ((int)((r >> 0) & 15u) == get(w, 0, 4)))) {
      put(w, 8, 1, 1);
      put(w, 9, 4, get(w, 0, 4));
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_Forward(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_seq = (int)((r >> 7) & 3u);
    const int l_ca = (int)((r >> 4) & 7u);
    const int l_c = (l_ca - (first_client(p) + 1 - 1));
    if (((((l_c < 0) || (l_c >= p.clients)) || (l_seq < 1)) || (l_seq > p.ncmds))) {
      return STEP_EXCEPTION;  // forward of an unknown client or command
    }
    if ((((get(w, 0, 4) != (int)((r >> 0) & 15u)) || (get(w, 6, 2) != i)) || (get(w, 4, 2) != rec_from(r)))) {
      return STEP_OK;
    }
    int l_r = -1;
    const int l_amo = arr_server_amo(w, l_c);
    const int l_lastseq = (l_amo & 3);
    l_r = -1;
    if ((l_seq == l_lastseq)) {
      l_r = (l_amo >> 2);
    }
    if ((l_seq > l_lastseq)) {
      const int l_k = (l_seq - 1);
      const int l_op = (int)((p.op_pk >> ((2 * ((l_c) * 3 + (l_k))) & 63)) & 3u);
      const int l_key = (int)((p.key_pk >> ((1 * ((l_c) * 3 + (l_k))) & 63)) & 1u);
      const int l_sym = (int)((p.sym_pk >> ((2 * ((l_c) * 3 + (l_k))) & 63)) & 3u);
      const int l_v = arr_server_kv(w, l_key);
      if ((l_op == 0)) {
        if (((l_v & 3) != 0)) {
          l_r = ((l_v << 2) | 1);
        } else {
          l_r = 2;
        }
      }
      if ((l_op == 1)) {
        arr_put_server_kv(w, l_key, ((l_sym << 2) | 1));
        l_r = 3;
      }
      if ((l_op == 2)) {
        const int l_n = (l_v & 3);
        if ((l_n >= 3)) {
          return STEP_OVERFLOW;  // value longer than 3 tokens
        }
        const int l_v2 = (((l_v - l_n) | (l_n + 1)) | (l_sym << ((l_n * 2) + 2)));
        arr_put_server_kv(w, l_key, l_v2);
        l_r = (l_v2 << 2);
      }
      arr_put_server_amo(w, l_c, (l_seq | (l_r << 2)));
    }
    out.send(((Rec)8 << 60) | ((Rec)(i) << 57) | ((Rec)(rec_from(r)) << 54) | ((Rec)(((int)((r >> 0) & 15u)) & 15) << 0) | ((Rec)((l_ca) & 7) << 4) | ((Rec)((l_seq) & 3) << 7));
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_server_ForwardAck(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    const int l_seq = (int)((r >> 7) & 3u);
    const int l_ca = (int)((r >> 4) & 7u);
    const int l_c = (l_ca - (first_client(p) + 1 - 1));
    if (((((l_c < 0) || (l_c >= p.clients)) || (l_seq < 1)) || (l_seq > p.ncmds))) {
      return STEP_EXCEPTION;  // forward of an unknown client or command
    }
    if ((((get(w, 4, 2) != i) || (get(w, 8, 1) == 0)) || (get(w, 0, 4) != (int)((r >> 0) & 15u)))) {
      return STEP_OK;
    }
    int l_r = -1;
    const int l_amo = arr_server_amo(w, l_c);
    const int l_lastseq = (l_amo & 3);
    l_r = -1;
    if ((l_seq == l_lastseq)) {
      l_r = (l_amo >> 2);
    }
    if ((l_seq > l_lastseq)) {
      const int l_k = (l_seq - 1);
      const int l_op = (int)((p.op_pk >> ((2 * ((l_c) * 3 + (l_k))) & 63)) & 3u);
      const int l_key = (int)((p.key_pk >> ((1 * ((l_c) * 3 + (l_k))) & 63)) & 1u);
      const int l_sym = (int)((p.sym_pk >> ((2 * ((l_c) * 3 + (l_k))) & 63)) & 3u);
      const int l_v = arr_server_kv(w, l_key);
      if ((l_op == 0)) {
        if (((l_v & 3) != 0)) {
          l_r = ((l_v << 2) | 1);
        } else {
          l_r = 2;
        }
      }
      if ((l_op == 1)) {
        arr_put_server_kv(w, l_key, ((l_sym << 2) | 1));
        l_r = 3;
      }
      if ((l_op == 2)) {
        const int l_n = (l_v & 3);
        if ((l_n >= 3)) {
          return STEP_OVERFLOW;  // value longer than 3 tokens
        }
        const int l_v2 = (((l_v - l_n) | (l_n + 1)) | (l_sym << ((l_n * 2) + 2)));
        arr_put_server_kv(w, l_key, l_v2);
        l_r = (l_v2 << 2);
      }
      arr_put_server_amo(w, l_c, (l_seq | (l_r << 2)));
    }
    if ((l_r >= 0)) {
      out.send(((Rec)4 << 60) | ((Rec)(i) << 57) | ((Rec)(l_ca) << 54) | ((Rec)((l_seq) & 3) << 0) | ((Rec)((l_r) & 1023) << 2));
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int ht_server_PingTimer(int i, uint32_t* w, int e, O& out, const Params& p) {
    (void)i; (void)w; (void)out; (void)p;
    const int l_n = get(w, 0, 4);
    if (((get(w, 4, 2) == i) && (get(w, 8, 1) == 0))) {
      out.send(((Rec)0 << 60) | ((Rec)(i) << 57) | ((Rec)((first_viewserver(p) + 1 - 1)) << 54) | ((Rec)((get(w, 9, 4)) & 15) << 0));
    } else {
      out.send(((Rec)0 << 60) | ((Rec)(i) << 57) | ((Rec)((first_viewserver(p) + 1 - 1)) << 54) | ((Rec)((l_n) & 15) << 0));
    }
    // set PingTimer: the queue stays [PingTimer]
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_client_ViewReply(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    if (((int)((r >> 0) & 15u) > get(w, 0, 4))) {
      put(w, 0, 4, (int)((r >> 0) & 15u));
      put(w, 4, 2, (int)((r >> 4) & 3u));
      if (((get(w, 6, 2) > 0) && (get(w, 8, 10) == 0))) {
        if ((get(w, 4, 2) != 0)) {
          out.send(((Rec)3 << 60) | ((Rec)(i) << 57) | ((Rec)(get(w, 4, 2)) << 54) | ((Rec)((get(w, 6, 2)) & 3) << 0));
        } else {
          out.send(((Rec)1 << 60) | ((Rec)(i) << 57) | ((Rec)((first_viewserver(p) + 1 - 1)) << 54));
        }
      }
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int hm_client_Reply(int i, uint32_t* w, Rec r, O& out, const Params& p, int& fl) {
    (void)i; (void)w; (void)r; (void)out; (void)p; (void)fl;
    if ((((get(w, 6, 2) > 0) && (get(w, 8, 10) == 0)) && ((int)((r >> 0) & 3u) == get(w, 6, 2)))) {
      put(w, 8, 10, (int)((r >> 2) & 1023u));
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int ht_client_ClientTimer(int i, uint32_t* w, int e, O& out, const Params& p) {
    (void)i; (void)w; (void)out; (void)p;
    const int tf_seq = (e >> 0) & 3;
    if ((((get(w, 6, 2) > 0) && (get(w, 8, 10) == 0)) && (tf_seq == get(w, 6, 2)))) {
      out.send(((Rec)1 << 60) | ((Rec)(i) << 57) | ((Rec)((first_viewserver(p) + 1 - 1)) << 54));
      if ((get(w, 4, 2) != 0)) {
        out.send(((Rec)3 << 60) | ((Rec)(i) << 57) | ((Rec)(get(w, 4, 2)) << 54) | ((Rec)((tf_seq) & 3) << 0));
      }
      if (!push_timer_client(w, (((tf_seq) & 3) << 0) | (2 << 2))) return STEP_OVERFLOW;
    }
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int on_message(int i, uint32_t* w, Rec r, O& out, const Params& p) {
    (void)w; (void)out;
    if (is_viewserver(i, p)) {
      int fl = 0, rc;
      if (rec_type(r) == 0) rc = hm_viewserver_Ping(i, w, r, out, p, fl);  // Ping
      else if (rec_type(r) == 1) rc = hm_viewserver_GetView(i, w, r, out, p, fl);  // GetView
      else return STEP_EXCEPTION;  // no handler for this message (Node.handleMessage throws)
      return rc;
    }
    if (is_server(i, p)) {
      int fl = 0, rc;
      if (rec_type(r) == 2) rc = hm_server_ViewReply(i, w, r, out, p, fl);  // ViewReply
      else if (rec_type(r) == 3) rc = hm_server_Request(i, w, r, out, p, fl);  // Request
      else if (rec_type(r) == 5) rc = hm_server_StateTransfer(i, w, r, out, p, fl);  // StateTransfer
      else if (rec_type(r) == 6) rc = hm_server_StateTransferAck(i, w, r, out, p, fl);  // StateTransferAck
      else if (rec_type(r) == 7) rc = hm_server_Forward(i, w, r, out, p, fl);  // Forward
      else if (rec_type(r) == 8) rc = hm_server_ForwardAck(i, w, r, out, p, fl);  // ForwardAck
      else return STEP_EXCEPTION;  // no handler for this message (Node.handleMessage throws)
      return rc;
    }
    if (is_client(i, p)) {
      int fl = 0, rc;
      if (rec_type(r) == 2) rc = hm_client_ViewReply(i, w, r, out, p, fl);  // ViewReply
      else if (rec_type(r) == 4) rc = hm_client_Reply(i, w, r, out, p, fl);  // Reply
      else return STEP_EXCEPTION;  // no handler for this message (Node.handleMessage throws)
      if (rc == STEP_OK) client_worker_client(i, w, out, p);
      return rc;
    }
    return STEP_EXCEPTION;
  }
  template <class O>
  static DSL_HD int on_timer(int i, uint32_t* w, int j, O& out, const Params& p) {
    (void)w; (void)j; (void)out;
    if (is_viewserver(i, p)) {
      if (j != 0) return STEP_NULL;
      return ht_viewserver_PingCheckTimer(i, w, (0 << 2), out, p);  // PingCheckTimer
    }
    if (is_server(i, p)) {
      if (j != 0) return STEP_NULL;
      return ht_server_PingTimer(i, w, (1 << 2), out, p);  // PingTimer
    }
    if (is_client(i, p)) {
      const int q = deliverable_client(w, j);
      if (q < 0) return STEP_NULL;
      const int e = arr_client__timers(w, q);
      if (ttype(e) == 2) {  // ClientTimer
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
            if (x >= 0 && arr_client__results(w, j) != x) return PV_FALSE;
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
      case 500:  // hasViewReply
      {
        if (view_any_record<Self>(v, [&](Rec r) { return rec_type(r) == 2 && (((int)((r >> 0) & 15u) >= (int)pr.arg0)); })) {
          return PV_TRUE;
        }
        return PV_FALSE;
        return PV_TRUE;
      }
      case 501:  // hasViewReplyExact
      {
        if (view_any_record<Self>(v, [&](Rec r) { return rec_type(r) == 2 && (((((int)((r >> 0) & 15u) | ((int)((r >> 4) & 3u) << 4)) | ((int)((r >> 6) & 3u) << 6)) == (int)pr.arg0)); })) {
          return PV_TRUE;
        }
        return PV_FALSE;
        return PV_TRUE;
      }
      case 502:  // viewRepliesSent
      {
        const int l_view = (int)pr.arg0;
        const int l_prim = ((l_view >> 4) & 3);
        const int l_num = (l_view & 15);
        if ((!view_any_record<Self>(v, [&](Rec r) { return rec_type(r) == 0 && ((((rec_from(r) == l_prim) && (rec_to(r) == 0)) && ((int)((r >> 0) & 15u) == l_num))); }))) {
          return PV_FALSE;
        }
        if ((((((int)pr.arg1 >> 0) & 1) == 1) && (!view_any_record<Self>(v, [&](Rec r) { return rec_type(r) == 2 && (((rec_to(r) == 0) && ((((int)((r >> 0) & 15u) | ((int)((r >> 4) & 3u) << 4)) | ((int)((r >> 6) & 3u) << 6)) == l_view))); })))) {
          return PV_FALSE;
        }
        if ((((((int)pr.arg1 >> 1) & 1) == 1) && (!view_any_record<Self>(v, [&](Rec r) { return rec_type(r) == 2 && (((rec_to(r) == 1) && ((((int)((r >> 0) & 15u) | ((int)((r >> 4) & 3u) << 4)) | ((int)((r >> 6) & 3u) << 6)) == l_view))); })))) {
          return PV_FALSE;
        }
        if ((((((int)pr.arg1 >> 2) & 1) == 1) && (!view_any_record<Self>(v, [&](Rec r) { return rec_type(r) == 2 && (((rec_to(r) == 2) && ((((int)((r >> 0) & 15u) | ((int)((r >> 4) & 3u) << 4)) | ((int)((r >> 6) & 3u) << 6)) == l_view))); })))) {
          return PV_FALSE;
        }
        if ((((((int)pr.arg1 >> 3) & 1) == 1) && (!view_any_record<Self>(v, [&](Rec r) { return rec_type(r) == 2 && (((rec_to(r) == 3) && ((((int)((r >> 0) & 15u) | ((int)((r >> 4) & 3u) << 4)) | ((int)((r >> 6) & 3u) << 6)) == l_view))); })))) {
          return PV_FALSE;
        }
        if ((((((int)pr.arg1 >> 4) & 1) == 1) && (!view_any_record<Self>(v, [&](Rec r) { return rec_type(r) == 2 && (((rec_to(r) == 4) && ((((int)((r >> 0) & 15u) | ((int)((r >> 4) & 3u) << 4)) | ((int)((r >> 6) & 3u) << 6)) == l_view))); })))) {
          return PV_FALSE;
        }
        if ((((((int)pr.arg1 >> 5) & 1) == 1) && (!view_any_record<Self>(v, [&](Rec r) { return rec_type(r) == 2 && (((rec_to(r) == 5) && ((((int)((r >> 0) & 15u) | ((int)((r >> 4) & 3u) << 4)) | ((int)((r >> 6) & 3u) << 6)) == l_view))); })))) {
          return PV_FALSE;
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
    if (pr.id == 500) return kReadsAll;
    if (pr.id == 501) return kReadsAll;
    if (pr.id == 502) return kReadsAll;
    const uint32_t clients = (((1u << (p.clients)) - 1u) << first_client(p));
    return (pr.id >= DSL_PRED_RESULTS_OK && pr.id <= DSL_PRED_CLIENT_HAS_RESULTS) ? clients : kReadsAll;
  }
  static DSL_HD bool pred_same(const DevPred& pr, const uint32_t* a, const uint32_t* b) {
    if (pr.id == 500) return (0u) == 0;
    if (pr.id == 501) return (0u) == 0;
    if (pr.id == 502) return (0u) == 0;
    if (pr.id >= DSL_PRED_RESULTS_OK && pr.id <= DSL_PRED_CLIENT_HAS_RESULTS) return ((a[2] ^ b[2])) == 0;
    return same_words<kNodeWords>(a, b);
  }
  static bool known_predicate(int id) { return (id >= DSL_PRED_RESULTS_OK && id <= DSL_PRED_CLIENT_HAS_RESULTS) || id == 500 || id == 501 || id == 502; }
  static bool valid(const Params& p) {
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        if (p.op[r][c] < 0 || p.op[r][c] > 2) return false;
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        if (p.key[r][c] < 0 || p.key[r][c] > 1) return false;
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        if (p.sym[r][c] < 0 || p.sym[r][c] > 3) return false;
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        if (p.expected[r][c] < -1 || p.expected[r][c] > 1023) return false;
    return p.servers >= 1 && p.servers <= 3 &&
           p.clients >= 1 && p.clients <= 2 &&
           p.ncmds >= 1 && p.ncmds <= 3 &&
           p.servers >= 1 && p.servers <= 3 &&
           p.clients >= 1 && p.clients <= 2;
  }
  static Params from_desc(const dsl_protocol_desc& d) {
    Params p{};
    p.servers = d.n_params > 0 ? (int32_t)d.params[0] : 2;
    p.clients = d.n_params > 1 ? (int32_t)d.params[1] : 1;
    p.ncmds = d.n_params > 2 ? (int32_t)d.params[2] : 2;
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++) {
        const int q = 3 + r * 3 + c;
        p.op[r][c] = d.n_params > q ? (int32_t)d.params[q] : 0;
      }
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++) {
        const int q = 9 + r * 3 + c;
        p.key[r][c] = d.n_params > q ? (int32_t)d.params[q] : 0;
      }
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++) {
        const int q = 15 + r * 3 + c;
        p.sym[r][c] = d.n_params > q ? (int32_t)d.params[q] : 0;
      }
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++) {
        const int q = 21 + r * 3 + c;
        p.expected[r][c] = d.n_params > q ? (int32_t)d.params[q] : -1;
      }
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        p.op_pk |= (uint64_t)((uint32_t)p.op[r][c] & 3u) << (2 * (r * 3 + c));
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        p.key_pk |= (uint64_t)((uint32_t)p.key[r][c] & 1u) << (1 * (r * 3 + c));
    for (int r = 0; r < 2; r++)
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
      e->fields[0] = (int64_t)((r >> 0) & 15u);
    }
    if (e->type == 1) {
      e->n_fields = 0;
    }
    if (e->type == 2) {
      e->n_fields = 3;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
      e->fields[1] = (int64_t)((r >> 4) & 3u);
      e->fields[2] = (int64_t)((r >> 6) & 3u);
    }
    if (e->type == 3) {
      e->n_fields = 1;
      e->fields[0] = (int64_t)((r >> 0) & 3u);
    }
    if (e->type == 4) {
      e->n_fields = 2;
      e->fields[0] = (int64_t)((r >> 0) & 3u);
      e->fields[1] = (int64_t)((r >> 2) & 1023u);
    }
    if (e->type == 5) {
      e->n_fields = 7;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
      e->fields[1] = (int64_t)((r >> 4) & 3u);
      e->fields[2] = (int64_t)((r >> 6) & 3u);
      e->fields[3] = (int64_t)((r >> 8) & 255u);
      e->fields[4] = (int64_t)((r >> 16) & 255u);
      e->fields[5] = (int64_t)((r >> 24) & 4095u);
      e->fields[6] = (int64_t)((r >> 36) & 4095u);
    }
    if (e->type == 6) {
      e->n_fields = 1;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
    }
    if (e->type == 7) {
      e->n_fields = 3;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
      e->fields[1] = (int64_t)((r >> 4) & 7u);
      e->fields[2] = (int64_t)((r >> 7) & 3u);
    }
    if (e->type == 8) {
      e->n_fields = 3;
      e->fields[0] = (int64_t)((r >> 0) & 15u);
      e->fields[1] = (int64_t)((r >> 4) & 7u);
      e->fields[2] = (int64_t)((r >> 7) & 3u);
    }
  }
  static void describe_timer(int i, const uint32_t* w, int j, const Params& p, dsl_event* e) {
    e->is_timer = 1;
    e->from = e->to = i;
    (void)w; (void)j; (void)p;
    if (is_viewserver(i, p)) {
      if (j != 0) return;
      const int x = (0 << 2);
      e->type = 9 + ttype(x);
      int mn = 0, mx = 0;
      tbounds(ttype(x), mn, mx);
      e->timer_min = mn;
      e->timer_max = mx;
      if (ttype(x) == 0) {
        e->n_fields = 0;
      }
      if (ttype(x) == 1) {
        e->n_fields = 0;
      }
      if (ttype(x) == 2) {
        e->n_fields = 1;
        e->fields[0] = (x >> 0) & 3;
      }
    }
    if (is_server(i, p)) {
      if (j != 0) return;
      const int x = (1 << 2);
      e->type = 9 + ttype(x);
      int mn = 0, mx = 0;
      tbounds(ttype(x), mn, mx);
      e->timer_min = mn;
      e->timer_max = mx;
      if (ttype(x) == 0) {
        e->n_fields = 0;
      }
      if (ttype(x) == 1) {
        e->n_fields = 0;
      }
      if (ttype(x) == 2) {
        e->n_fields = 1;
        e->fields[0] = (x >> 0) & 3;
      }
    }
    if (is_client(i, p)) {
      const int q = deliverable_client(w, j);
      if (q < 0) return;
      const int x = arr_client__timers(w, q);
      e->type = 9 + ttype(x);
      int mn = 0, mx = 0;
      tbounds(ttype(x), mn, mx);
      e->timer_min = mn;
      e->timer_max = mx;
      if (ttype(x) == 0) {
        e->n_fields = 0;
      }
      if (ttype(x) == 1) {
        e->n_fields = 0;
      }
      if (ttype(x) == 2) {
        e->n_fields = 1;
        e->fields[0] = (x >> 0) & 3;
      }
    }
  }
};

}  // namespace dsl
