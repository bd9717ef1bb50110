// multipaxos.hpp -- lab3 Multi-Paxos (3 servers, 2 clients; BASELINE config C5) as node-local
// device handlers.
//
// The reference's lab3 is a stub (labs/lab3-paxos/src/dslabs/paxos/PaxosServer.java:16-127); this
// is the builder-authored protocol specified in DESIGN.md §9 and restated object-style in
// oracle/proto_multipaxos.hpp. It follows labs/lab3-paxos/README.md:25-106 (PMMC roles in one
// server, stable leader + heartbeat-check timer, clients broadcasting requests, AMO KV store) and
// exposes what PaxosTest's predicates read (status / command / lastNonEmpty, PaxosTest.java:113-346).
//
// Nodes: servers 0..n-1 ("server1.."), clients n..n+c-1 ("client1.."). Ballot = (round, leader),
// compared as (round << 2) | leader. Commands: id 1 + 3*client + (seq-1) (0 = no-op); command
// (c, q) is ops[c][q-1] in {Put, Append, Get} on the single key "foo" with value token
// vals[c][q-1] (KVStoreWorkload put / append / get, KVStoreWorkload.java:40-66). The key's value is
// a sequence of <= 4 value tokens, 11 bits = len:3 | tokens 2 bits each. A KV result (12 bits) is
// PutOk (7), KeyNotFound (6), or AppendResult / GetResult of a value (its len is 1..4; which of
// the two is fixed by the command). Application state (the key's value, the AMO last-seq table) is
// a function of the log's executed prefix (slots < slotOut), so it is recomputed, not stored.
//
// Node words (6):
//   server: w0 = round:4 | leader:2 @4 | active:1 @6 | electing:1 @7 | heard:1 @8 | missed:2 @9 |
//                p1bVotes:3 @11 | slotOut:3 @14 | slotIn:3 @17
//           w1-w2 = log[1..4], 16 bits each: status:2 | ballot:6 @2 | cmd:3 @8
//           w3 = p2bVotes[1..4], 3 bits each;  w4-w5 = p1bLog[1..4] (merged phase-1 log)
//   client: w0 = seq:2 | pending:1 @2 | result:12 @3 | nres:2 @15 | ntim:2 @17 | timers[3] @19, 21, 23
//           w1 = results[0..1], 12 bits each; w2 = results[2]
// Records (64 bit): type:3 @61 | from:3 @58 | to:3 @55 | payload
//   0 Request  cmd:3                    4 P2a       round:4 leader:2 slot:3 @6 cmd:3 @9
//   1 Reply    seq:2 result:12 @2       5 P2b       round:4 leader:2 slot:3 @6
//   2 P1a      round:4 leader:2 @4      6 Decision  slot:3 cmd:3 @3
//   3 P1b      round:4 leader:2 log 4x11 bits @6   7 Heartbeat round:4 leader:2
// Server Tick timers (100 ms, re-set on every fire) are a constant queue [Tick] and not stored;
// client queues hold ClientTimer(seq) entries (100 ms), only the head is deliverable.
#pragma once
#include "../nodestate.hpp"


namespace dsl {

struct MultiPaxos {
  static constexpr int kMaxServers = 3, kMaxClients = 2, kMaxCmds = 3, kSlots = 4, kMaxRound = 15;
  static constexpr int kMaxTokens = 4;  // value tokens of the key's value
  // kMaxSends: the most records one handler sends is 12 (P1b completing phase 1: a P2a to both
  // other servers for each of the 4 slots, plus up to 4 replies from execute); a larger send
  // list would be a hard STEP_OVERFLOW error, never a truncation.
  static constexpr int kNodes = kMaxServers + kMaxClients, kNodeWords = 6, kNetCap = 64, kMaxSends = 12;
  static constexpr int kMsgClasses = 8;  // handler classes of messages (message types 0..7); timers: 8 (Tick), 9 (ClientTimer)
  // No handler sends one record twice in one step (broadcasts go to distinct servers, execute
  // replies once per newly executed command, become_leader proposes each slot once), so Sender
  // skips its duplicate check; tests/hostcheck checks distinctness on every explored step.
  static constexpr bool kSendsDistinct = true;
  static constexpr int kTick = 100, kClientRetry = 100;
  using Rec = uint64_t;
  using State = StateOf<MultiPaxos>;

  struct Params {
    int32_t servers, clients;
    int32_t ncmds[kMaxClients];
    int32_t ops[kMaxClients][kMaxCmds];       // OP_PUT / OP_APPEND / OP_GET
    int32_t vals[kMaxClients][kMaxCmds];      // value token 1..3 (0 for a Get)
    int32_t expected[kMaxClients][kMaxCmds];  // expected result code, -1 = the workload checks none
    // Derived by from_desc, read by the device code (a shift and a mask per lookup instead of a
    // select chain over the arrays above): cmdtab bits 4*cmd .. +3 = op << 2 | value token of
    // command id cmd (1..6); exptab[c] bits 16*k .. +15 = 0x8000 | expected[c][k] (0 = no check).
    uint32_t cmdtab;
    uint32_t pad;
    uint64_t exptab[kMaxClients];
  };
  enum { OP_PUT = 1, OP_APPEND = 2, OP_GET = 3 };
  static constexpr uint32_t kPutOk = 7, kKeyNotFound = 6;  // result codes beside values (len 1..4)
  enum { M_REQUEST = 0, M_REPLY, M_P1A, M_P1B, M_P2A, M_P2B, M_DECISION, M_HEARTBEAT, T_TICK = 8, T_CLIENT = 9 };
  enum { EMPTY = 0, ACCEPTED = 1, CHOSEN = 2 };

  // Handler class of a message (< kMsgClasses; timers are class kMsgClasses): k_level groups a chunk's work items
  // by class so that the lanes of a wavefront run the same handler.
  static DSL_HD int msg_class(Rec r) { return m_type(r); }
  // Timer handler classes: a server's Tick and a client's ClientTimer (nodestate.hpp TimerClasses)
  static constexpr int kTimerClasses = 2;
  static DSL_HD int timer_class(int node, const Params& p) { return node >= p.servers ? 1 : 0; }
  static DSL_HD int get(const uint32_t* w, int bit, int width) { return field_get<kNodeWords>(w, bit, width); }
  static DSL_HD void put(uint32_t* w, int bit, int width, int v) { field_put<kNodeWords>(w, bit, width, v); }
  // ---- server fields ------------------------------------------------------------------------------
  // The log (w1-w2) and the merged phase-1 log (w4-w5) as 64-bit words, 16 bits per slot: a
  // run-time slot is a 64-bit shift (no select chain over the node words); a constant one folds.
  static DSL_HD uint64_t log64(const uint32_t* w, int wi) { return (uint64_t)w[wi] | ((uint64_t)w[wi + 1] << 32); }
  static DSL_HD void set16(uint32_t* w, int wi, int slot, uint32_t e) {
    const int sh = 16 * (slot - 1);
    const uint64_t lg = (log64(w, wi) & ~(0xffffull << sh)) | ((uint64_t)(e & 0xffffu) << sh);
    w[wi] = (uint32_t)lg;
    w[wi + 1] = (uint32_t)(lg >> 32);
  }
  static DSL_HD uint32_t entry(const uint32_t* w, int slot) { return (uint32_t)(log64(w, 1) >> (16 * (slot - 1))) & 0xffffu; }
  static DSL_HD void set_entry(uint32_t* w, int slot, uint32_t e) { set16(w, 1, slot, e); }
  static DSL_HD uint32_t p1entry(const uint32_t* w, int slot) { return (uint32_t)(log64(w, 4) >> (16 * (slot - 1))) & 0xffffu; }
  static DSL_HD void set_p1entry(uint32_t* w, int slot, uint32_t e) { set16(w, 4, slot, e); }
  static DSL_HD uint32_t mk_entry(int status, int ballot, int cmd) {
    return (uint32_t)status | ((uint32_t)ballot << 2) | ((uint32_t)cmd << 8);
  }
  static DSL_HD int e_status(uint32_t e) { return e & 3; }
  static DSL_HD int e_ballot(uint32_t e) { return (e >> 2) & 0x3f; }
  static DSL_HD int e_cmd(uint32_t e) { return (e >> 8) & 7; }
  static DSL_HD int votes2(const uint32_t* w, int slot) { return (int)((w[3] >> (3 * (slot - 1))) & 7u); }
  static DSL_HD void set_votes2(uint32_t* w, int slot, int v) {
    const int sh = 3 * (slot - 1);
    w[3] = (w[3] & ~(7u << sh)) | (((uint32_t)v & 7u) << sh);
  }
  static DSL_HD int cmp_ballot(const uint32_t* w) { return (get(w, 0, 4) << 2) | get(w, 4, 2); }
  static DSL_HD void set_ballot(uint32_t* w, int b) {
    put(w, 0, 4, b >> 2);
    put(w, 4, 2, b & 3);
  }
  static DSL_HD int active(const uint32_t* w) { return get(w, 6, 1); }
  static DSL_HD int electing(const uint32_t* w) { return get(w, 7, 1); }
  static DSL_HD int heard(const uint32_t* w) { return get(w, 8, 1); }
  static DSL_HD int missed(const uint32_t* w) { return get(w, 9, 2); }
  static DSL_HD int p1votes(const uint32_t* w) { return get(w, 11, 3); }
  static DSL_HD int slot_out(const uint32_t* w) { return get(w, 14, 3); }
  static DSL_HD int slot_in(const uint32_t* w) { return get(w, 17, 3); }

  // ---- records -------------------------------------------------------------------------------------
  static DSL_HD Rec msg(int type, int from, int to, uint64_t payload) {
    return ((Rec)type << 61) | ((Rec)from << 58) | ((Rec)to << 55) | payload;
  }
  static DSL_HD int m_type(Rec m) { return (int)(m >> 61); }
  static DSL_HD int rec_from(Rec m) { return (int)((m >> 58) & 7); }
  static DSL_HD int rec_to(Rec m) { return (int)((m >> 55) & 7); }
  static DSL_HD uint64_t ballot_field(int b) { return (uint64_t)(b >> 2) | ((uint64_t)(b & 3) << 4); }
  static DSL_HD int m_ballot(Rec m) { return (int)(((m & 0xf) << 2) | ((m >> 4) & 3)); }

  template <class O>
  static DSL_HD void bcast_servers(int from, const Params& p, int type, uint64_t payload, O& out) {
    for (int s = 0; s < p.servers; s++)
      if (s != from) out.send(msg(type, from, s, payload));
  }

  // Workload parameters by client / command index, from the packed tables (Params::cmdtab,
  // exptab): a shift and a mask, no run-time index into the kernel-argument arrays (which the
  // compiler would copy to scratch memory) and no select chain.
  static DSL_HD int cmd_id(int c, int q) { return 1 + 3 * c + (q - 1); }
  static DSL_HD int cmd_client(int cmd) { return cmd >= 4 ? 1 : 0; }  // cmd in 1..6
  static DSL_HD int cmd_seq(int cmd) { return cmd - 3 * cmd_client(cmd); }
  static DSL_HD int cmd_op(const Params& p, int cmd) { return (int)((p.cmdtab >> (4 * cmd + 2)) & 3u); }
  static DSL_HD int cmd_val(const Params& p, int cmd) { return (int)((p.cmdtab >> (4 * cmd)) & 3u); }
  static DSL_HD int val(const Params& p, int c, int k) { return cmd_val(p, cmd_id(c, k + 1)); }
  static DSL_HD int op_of(const Params& p, int c, int k) { return cmd_op(p, cmd_id(c, k + 1)); }
  static DSL_HD int expect(const Params& p, int c, int k) {
    const uint32_t x = (uint32_t)((c ? p.exptab[1] : p.exptab[0]) >> (16 * k)) & 0xffffu;
    return x ? (int)(x & 0xfffu) : -1;
  }
  static DSL_HD int ncmd(const Params& p, int c) { return c ? p.ncmds[1] : p.ncmds[0]; }

  // ---- application: the executed prefix ----------------------------------------------------------
  static DSL_HD uint32_t res_push(uint32_t r, int v) {
    int len = r & 7;
    return (uint32_t)(len + 1) | (r & ~7u) | ((uint32_t)v << (3 + 2 * len));
  }
  // KVStore.execute of command id cmd on the key's value `kv`: the new value in *kv, the result
  // code returned (KVStore.java:59-78 as lab1 specifies it: Put -> PutOk, Append -> the new value,
  // Get -> the value or KeyNotFound).
  static DSL_HD uint32_t kv_apply(const Params& p, int cmd, uint32_t* kv) {
    const int op = cmd_op(p, cmd), v = cmd_val(p, cmd);
    if (op == OP_PUT) {
      *kv = 1u | ((uint32_t)v << 3);
      return kPutOk;
    }
    if (op == OP_APPEND) {
      *kv = res_push(*kv, v);
      return *kv;
    }
    return (*kv & 7) ? *kv : kKeyNotFound;
  }
  // Bit offset of a client's result k (never straddling a word).
  static DSL_HD int res_bit(int k) { return k < 2 ? 32 + 12 * k : 64; }
  // The executed prefix (slots [1, upto)): client c0's last executed sequence number, and the
  // result command (c0, q0) had when it executed (the AMO cache's entry). Fixed trip counts over
  // the kSlots slots: the loop unrolls and every log access has a constant bit offset.
  static DSL_HD uint32_t executed(const uint32_t* w, const Params& p, int upto, int c0, int q0, int* last_seq) {
    uint32_t kv = 0, r = 0;
    int ls0 = 0, ls1 = 0;
#pragma unroll
    for (int slot = 1; slot <= kSlots; slot++) {
      const int cmd = e_cmd(entry(w, slot));
      const int c = cmd_client(cmd), q = cmd_seq(cmd);
      if (slot < upto && cmd && (c ? ls1 : ls0) < q) {
        const uint32_t x = kv_apply(p, cmd, &kv);
        if (c) ls1 = q;
        else ls0 = q;
        if (c == c0 && q == q0) r = x;
      }
    }
    *last_seq = c0 ? ls1 : ls0;
    return r;
  }
  // Executes the chosen slots from slotOut on, in order (replies from an active leader). The
  // server handlers run it ONCE, as their common tail (on_message / on_timer): every slot a
  // handler chooses is executed there, which is what executing right after each choice does
  // (execution only reads the log, chosen entries never change, and the send list is a set).
  template <class O>
  static DSL_HD void execute(int s, uint32_t* w, const Params& p, O& out) {
    const int so0 = slot_out(w);
    const bool act = active(w);
    uint32_t kv = 0;
    int ls0 = 0, ls1 = 0, so = so0;
    bool run = true;  // every slot from slotOut to here is chosen
#pragma unroll
    for (int slot = 1; slot <= kSlots; slot++) {
      const uint32_t e = entry(w, slot);
      const int cmd = e_cmd(e);
      const int c = cmd_client(cmd), q = cmd_seq(cmd);
      const bool before = slot < so0;
      const bool now = !before && run && e_status(e) == CHOSEN;
      run = run && (before || now);
      if ((before || now) && cmd && (c ? ls1 : ls0) < q) {
        const uint32_t x = kv_apply(p, cmd, &kv);
        if (c) ls1 = q;
        else ls0 = q;
        if (now && act) out.send(msg(M_REPLY, s, p.servers + c, (uint64_t)q | ((uint64_t)x << 2)));
      }
      if (now) so = slot + 1;
    }
    put(w, 14, 3, so);
  }
  static DSL_HD void adopt(uint32_t* w, int b) {  // a higher ballot steps this server down
    if (b > cmp_ballot(w)) {
      set_ballot(w, b);
      put(w, 6, 2, 0);   // active, electing
      put(w, 11, 3, 0);  // p1bVotes
      w[3] = 0;          // p2bVotes
      w[4] = 0;          // p1bLog
      w[5] = 0;
    }
  }
  static DSL_HD bool majority(const Params& p, int votes) { return __builtin_popcount(votes) * 2 > p.servers; }
  // Marks the slot chosen and broadcasts the Decision; the caller's tail executes it.
  template <class O>
  static DSL_HD void choose(int s, uint32_t* w, const Params& p, int slot, O& out) {
    const int cmd = e_cmd(entry(w, slot));
    set_entry(w, slot, mk_entry(CHOSEN, 0, cmd));
    set_votes2(w, slot, 0);
    bcast_servers(s, p, M_DECISION, (uint64_t)slot | ((uint64_t)cmd << 3), out);
  }
  template <class O>
  static DSL_HD void propose(int s, uint32_t* w, const Params& p, int slot, int cmd, O& out) {
    const int b = cmp_ballot(w);
    set_entry(w, slot, mk_entry(ACCEPTED, b, cmd));
    set_votes2(w, slot, 1 << s);
    bcast_servers(s, p, M_P2A, ballot_field(b) | ((uint64_t)slot << 6) | ((uint64_t)cmd << 9), out);
    if (majority(p, 1 << s)) choose(s, w, p, slot, out);  // a one-server group
  }
  static DSL_HD void merge(uint32_t* w, int slot, uint32_t e) {
    const uint32_t m = p1entry(w, slot);
    if (e_status(e) == CHOSEN) {
      set_p1entry(w, slot, mk_entry(CHOSEN, 0, e_cmd(e)));
    } else if (e_status(e) == ACCEPTED && e_status(m) != CHOSEN && (e_status(m) == EMPTY || e_ballot(m) < e_ballot(e))) {
      set_p1entry(w, slot, e);
    }
  }
  // Phase 1 complete: re-propose the merged log (chosen entries adopted, holes become no-ops),
  // slotIn after the last used slot. The caller's tail executes. A rolled loop over the slots
  // (the merged log and the log are 64-bit words shifted by 16 per slot): one copy of propose.
  template <class O>
  static DSL_HD void become_leader(int s, uint32_t* w, const Params& p, O& out) {
    put(w, 6, 1, 1);   // active
    put(w, 7, 1, 0);   // electing
    put(w, 11, 3, 0);  // p1bVotes
    const uint64_t merged = (uint64_t)w[4] | ((uint64_t)w[5] << 32);
    int last = 0;
#pragma unroll
    for (int i = 1; i <= kSlots; i++)
      if (e_status((uint32_t)(merged >> (16 * (i - 1)))) != EMPTY || e_status(entry(w, i)) != EMPTY) last = i;
    w[4] = 0;
    w[5] = 0;
#pragma unroll 1
    for (int i = 1; i <= last; i++) {
      if (e_status(entry(w, i)) == CHOSEN) continue;
      const uint32_t m = (uint32_t)(merged >> (16 * (i - 1))) & 0xffffu;
      if (e_status(m) == CHOSEN) {
        set_entry(w, i, mk_entry(CHOSEN, 0, e_cmd(m)));
        set_votes2(w, i, 0);
      } else {
        propose(s, w, p, i, e_status(m) == ACCEPTED ? e_cmd(m) : 0, out);
      }
    }
    put(w, 17, 3, last + 1);
  }

  // ---- clients (PaxosClient inside a ClientWorker) ------------------------------------------------
  template <class O>
  static DSL_HD void client_send(int c, uint32_t* w, const Params& p, int q, O& out) {
    put(w, 0, 2, q);
    put(w, 2, 1, 1);
    put(w, 3, 12, 0);
    const int cmd = cmd_id(c, q);
    for (int s = 0; s < p.servers; s++) out.send(msg(M_REQUEST, p.servers + c, s, (uint64_t)cmd));
    const int n = get(w, 17, 2);
    if (n >= kMaxCmds) {
      out.overflow = true;
      return;
    }
    put(w, 19 + 2 * n, 2, q);
    put(w, 17, 2, n + 1);
  }
  template <class O>
  static DSL_HD void client_worker_continue(int c, uint32_t* w, const Params& p, O& out) {
    int nres = get(w, 15, 2);
    const int res = get(w, 3, 12);
    if (nres < ncmd(p, c) && res != 0) {
      put(w, res_bit(nres), 12, res);
      nres++;
      put(w, 15, 2, nres);
      if (nres < ncmd(p, c)) client_send(c, w, p, nres + 1, out);
    }
  }

  // ---- protocol interface -------------------------------------------------------------------------
  static DSL_HD int num_nodes(const Params& p) { return p.servers + p.clients; }
  template <class O>
  static DSL_HD void init_node(int i, uint32_t* w, O& out, const Params& p) {
    if (i < p.servers) {
      put(w, 14, 3, 1);
      put(w, 17, 3, 1);
      if (i == 0) put(w, 6, 1, 1);  // server1 leads ballot (0, server1)
    } else {
      client_send(i - p.servers, w, p, 1, out);
    }
  }
  static DSL_HD int num_timer_events(int i, const uint32_t* w, const Params& p) {
    return i < p.servers ? 1 : (get(w, 17, 2) > 0);
  }

  template <class O>
  static DSL_HD int on_timer(int i, uint32_t* w, int, O& out, const Params& p) {
    if (i >= p.servers) {  // ClientTimer at the head: onClientTimer, ClientWorker loop, remove head
      const int c = i - p.servers;
      const int t = get(w, 19, 2);
      if (get(w, 2, 1) && t == get(w, 0, 2)) {
        const int cmd = cmd_id(c, t);
        for (int s = 0; s < p.servers; s++) out.send(msg(M_REQUEST, i, s, (uint64_t)cmd));
        const int n = get(w, 17, 2);
        if (n >= kMaxCmds) return STEP_OVERFLOW;
        put(w, 19 + 2 * n, 2, t);
        put(w, 17, 2, n + 1);
      }
      client_worker_continue(c, w, p, out);
      const int n = get(w, 17, 2);
      // remove the head (the queue's entries move up one; the last slot empties)
      put(w, 19, 2, n > 1 ? get(w, 21, 2) : 0);
      put(w, 21, 2, n > 2 ? get(w, 23, 2) : 0);
      put(w, 23, 2, 0);
      put(w, 17, 2, n - 1);
      return STEP_OK;
    }
    // server Tick (the queue stays [Tick])
    const int s = i;
    if (active(w)) {
      bcast_servers(s, p, M_HEARTBEAT, ballot_field(cmp_ballot(w)), out);
    } else if (heard(w)) {
      put(w, 8, 1, 0);
      put(w, 9, 2, 0);
    } else {
      const int mis = missed(w) + 1 > 2 ? 2 : missed(w) + 1;
      put(w, 9, 2, mis);
      const int b = cmp_ballot(w);
      if (mis >= 2 && (b >> 2) < kMaxRound) {  // two ticks without the leader: phase 1
        put(w, 9, 2, 0);
        put(w, 8, 1, 0);
        set_ballot(w, (((b >> 2) + 1) << 2) | s);
        put(w, 7, 1, 1);  // electing
        put(w, 6, 1, 0);  // active
        w[3] = 0;         // p2bVotes
        put(w, 11, 3, 1 << s);
        w[4] = 0;
        w[5] = 0;
#pragma unroll
        for (int k = 1; k <= kSlots; k++) merge(w, k, entry(w, k));
        bcast_servers(s, p, M_P1A, ballot_field(cmp_ballot(w)), out);
        if (majority(p, 1 << s)) {  // a one-server group leads at once
          become_leader(s, w, p, out);
          execute(s, w, p, out);
        }
      }
    }
    return STEP_OK;
  }

  // Deliveries that surely change nothing (nodestate.hpp NoopFilter), read off on_message below: a
  // stale ballot, a P2b / P1b / Decision that no longer applies, a vote already counted, a
  // Heartbeat of the current ballot already heard, a Request at a server that is not the active
  // leader (it neither replies nor proposes), a Reply the client does not take. False otherwise:
  // the cases that re-send an answer already in the network would need a search of the record
  // array here, which cost more in k_level's classification than the skipped handlers saved
  // (measured: a P2a / P1a / Tick check by Net::contains, +7 % of the events skipped, C5 d12 and
  // d14 2-10 % slower). w = the state row.
  // Branch-free: every lane evaluates every case and selects by the message type (the lanes of a
  // classification pass hold different types; a switch compiled to one exec-masked block per type).
  static DSL_HD bool surely_noop(int i, const uint32_t* row, Rec m, const Params& p) {
    const uint32_t* w = row + i * kNodeWords;
    const uint32_t w0 = w[0], w3 = w[3];
    const uint64_t lg = log64(w, 1);
    const int type = m_type(m);
    // client: a Reply it does not take, with the ClientWorker loop idle
    const int c = i - p.servers, q = (int)(m & 3);
    const bool takes = ((w0 >> 2) & 1u) && q == (int)(w0 & 3u);
    const bool cont = (int)((w0 >> 15) & 3u) < ncmd(p, c > 0 ? 1 : 0) && ((w0 >> 3) & 0xfffu) != 0;
    const bool client = type == M_REPLY && !takes && !cont;  // a non-Reply throws: never skipped
    // server
    const int b = m_ballot(m), cur = (int)(((w0 & 0xfu) << 2) | ((w0 >> 4) & 3u)), from = rec_from(m);
    const bool act = (w0 >> 6) & 1u, elect = (w0 >> 7) & 1u, hrd = (w0 >> 8) & 1u;
    const int slot = type == M_DECISION ? (int)(m & 7) : (int)((m >> 6) & 7);
    const int si = (slot - 1) & 3;
    const uint32_t e = (uint32_t)(lg >> (16 * si)) & 0xffffu;
    const int v = (int)((w3 >> (3 * si)) & 7u);
    const bool p2b = !act || b != cur || e_status(e) != ACCEPTED || (((v >> from) & 1) && !majority(p, v));
    bool server = false;
    server = type == M_REQUEST ? !act : server;
    server = (type == M_P2A || type == M_P1A) ? b < cur : server;
    server = type == M_HEARTBEAT ? (b < cur || (b == cur && hrd)) : server;
    server = type == M_P2B ? p2b : server;
    server = type == M_DECISION ? e_status(e) == CHOSEN : server;
    server = type == M_P1B ? (!elect || b != cur) : server;
    return i >= p.servers ? client : server;
  }

  template <class O>
  static DSL_HD int on_message(int i, uint32_t* w, Rec m, O& out, const Params& p) {
    const int type = m_type(m), from = rec_from(m);
    if (i >= p.servers) {  // PaxosClient.handlePaxosReply, then the ClientWorker loop
      if (type != M_REPLY) return STEP_EXCEPTION;
      const int c = i - p.servers, q = (int)(m & 3);
      if (get(w, 2, 1) && q == get(w, 0, 2)) {
        put(w, 3, 12, (int)((m >> 2) & 0xfff));
        put(w, 2, 1, 0);
      }
      client_worker_continue(c, w, p, out);
      return STEP_OK;
    }
    const int s = i;
    bool ex = false;    // a slot became chosen: execute (the common tail)
    bool lead = false;  // phase 1 completed: become_leader, then execute
    if (type == M_REQUEST) {
      const int cmd = (int)(m & 7), c = cmd_client(cmd), q = cmd_seq(cmd);
      int ls;
      const uint32_t r = executed(w, p, slot_out(w), c, q, &ls);
      if (ls >= q) {  // AMO: already executed; an active leader replies from the cache
        if (active(w) && ls == q) out.send(msg(M_REPLY, s, p.servers + c, (uint64_t)q | ((uint64_t)r << 2)));
        return STEP_OK;
      }
      // a new proposal goes after every slot this server knows to be in use; no free slot ->
      // ignore (clients retry)
      int slot = slot_in(w);
      bool inlog = false;
#pragma unroll
      for (int k = 1; k <= kSlots; k++) {
        const uint32_t e = entry(w, k);
        if (e_status(e) != EMPTY && k + 1 > slot) slot = k + 1;
        inlog |= e_status(e) != EMPTY && e_cmd(e) == cmd;
      }
      if (!active(w) || slot > kSlots || inlog) return STEP_OK;  // inlog: already in the log
      put(w, 17, 3, slot + 1);
      propose(s, w, p, slot, cmd, out);
      ex = majority(p, 1 << s);
    } else {
      const int b = m_ballot(m);
      switch (type) {
        case M_P2A: {
          if (b < cmp_ballot(w)) return STEP_OK;
          adopt(w, b);
          put(w, 8, 1, 1);
          const int slot = (int)((m >> 6) & 7), cmd = (int)((m >> 9) & 7);
          if (e_status(entry(w, slot)) != CHOSEN) set_entry(w, slot, mk_entry(ACCEPTED, b, cmd));
          out.send(msg(M_P2B, s, from, ballot_field(b) | ((uint64_t)slot << 6)));
          return STEP_OK;
        }
        case M_P2B: {
          const int slot = (int)((m >> 6) & 7);
          if (!active(w) || b != cmp_ballot(w) || e_status(entry(w, slot)) != ACCEPTED) return STEP_OK;
          const int v = votes2(w, slot) | (1 << from);
          set_votes2(w, slot, v);
          if (!majority(p, v)) return STEP_OK;
          choose(s, w, p, slot, out);
          ex = true;
          break;
        }
        case M_DECISION: {
          const int slot = (int)(m & 7), cmd = (int)((m >> 3) & 7);
          if (e_status(entry(w, slot)) == CHOSEN) return STEP_OK;
          set_entry(w, slot, mk_entry(CHOSEN, 0, cmd));
          set_votes2(w, slot, 0);
          ex = true;
          break;
        }
        case M_HEARTBEAT:
          if (b < cmp_ballot(w)) return STEP_OK;
          adopt(w, b);
          put(w, 8, 1, 1);
          return STEP_OK;
        case M_P1A: {
          if (b < cmp_ballot(w)) return STEP_OK;
          adopt(w, b);
          put(w, 8, 1, 1);
          const uint64_t lg = log64(w, 1);
          uint64_t logbits = 0;
#pragma unroll
          for (int k = 0; k < kSlots; k++) logbits |= ((lg >> (16 * k)) & 0x7ffull) << (11 * k);
          out.send(msg(M_P1B, s, from, ballot_field(b) | (logbits << 6)));
          return STEP_OK;
        }
        case M_P1B: {
          if (!electing(w) || b != cmp_ballot(w)) return STEP_OK;
          const int v = p1votes(w) | (1 << from);
          put(w, 11, 3, v);
#pragma unroll
          for (int k = 1; k <= kSlots; k++) merge(w, k, (uint32_t)((m >> (6 + 11 * (k - 1))) & 0x7ff));
          if (!majority(p, v)) return STEP_OK;
          lead = true;
          break;
        }
        default:
          return STEP_EXCEPTION;
      }
    }
    if (lead) become_leader(s, w, p, out);
    if (ex || lead) execute(s, w, p, out);
    return STEP_OK;
  }

  // ---- predicates -----------------------------------------------------------------------------------
  // Predicates read node words that live in LDS (parent rows, the changed node's copy) or in host
  // memory, never in a per-lane array: direct indexing (the select chain of get() would load every
  // word of a node for a run-time field index).
  static DSL_HD int getd(const uint32_t* w, int bit, int width) {
    return (int)((w[bit >> 5] >> (bit & 31)) & ((1u << width) - 1u));
  }
  static DSL_HD uint32_t entryd(const uint32_t* w, int slot) { return (uint32_t)getd(w, 32 + 16 * (slot - 1), 16); }
  // PaxosServer.command(i) as a KV command code: op << 2 | value token (0 = null: an empty slot or a
  // no-op). Commands compare as KV commands (Lombok equals of Put / Append / Get), not as AMO
  // commands: PaxosTest's slotValid requires command(i) to return the unwrapped command.
  static DSL_HD int kv_cmd(const Params& p, int cmd) { return cmd ? (int)((p.cmdtab >> (4 * cmd)) & 15u) : 0; }

  // PaxosTest.slotValid(st, i) (PaxosTest.java:215-279) over the servers' log words lw; with no
  // garbage collection firstNonCleared() == 1 and no slot is CLEARED, lastNonEmpty() is the last
  // non-EMPTY slot, and command(i) is null exactly for EMPTY slots and no-ops.
  static DSL_HD bool slot_valid(const uint32_t (&lw)[kMaxServers][2], const Params& p, int slot) {
    if (slot < 1) return false;  // i < firstNonCleared but the status is not CLEARED
    if (slot > kSlots) return true;  // EMPTY everywhere: never chosen
    bool is_chosen = false, conflict = false;
    int chosen = 0, count = 0;
#pragma unroll
    for (int s = 0; s < kMaxServers; s++) {
      const uint32_t e = (sel2(lw[s], (slot - 1) >> 1) >> (16 * ((slot - 1) & 1))) & 0xffffu;
      if (s < p.servers && e_status(e) == CHOSEN) {
        const int x = kv_cmd(p, e_cmd(e));
        conflict |= is_chosen && x != chosen;
        chosen = x;
        is_chosen = true;
      }
    }
#pragma unroll
    for (int s = 0; s < kMaxServers; s++) {
      const uint32_t e = (sel2(lw[s], (slot - 1) >> 1) >> (16 * ((slot - 1) & 1))) & 0xffffu;
      if (s < p.servers && e_status(e) != EMPTY && (e_status(e) != ACCEPTED || kv_cmd(p, e_cmd(e)) == chosen)) count++;
    }
    return !is_chosen || (!conflict && 2 * count > p.servers);
  }
  static DSL_HD uint32_t sel2(const uint32_t (&a)[2], int i) { return i ? a[1] : a[0]; }
  static DSL_HD void load_logs(const NodeView& v, const Params& p, uint32_t (&lw)[kMaxServers][2]) {
#pragma unroll
    for (int s = 0; s < kMaxServers; s++) {
      const uint32_t* w = v.node(s < p.servers ? s : 0);
      lw[s][0] = s < p.servers ? w[1] : 0u;
      lw[s][1] = s < p.servers ? w[2] : 0u;
    }
  }
  // PaxosTest.LOGS_CONSISTENT_ALL_SLOTS (:302-322): every slot up to the last non-empty one; and
  // LOGS_CONSISTENT (:282-300): slots from the smallest firstNonCleared() -- 1 here -- on, so the
  // two coincide. MARKERS_VALID (:128-193) holds by construction. The servers' log words are
  // read once (independent LDS reads), then everything is register arithmetic; slots past the
  // last non-empty one are EMPTY everywhere and valid.
  static DSL_HD int logs_consistent(const NodeView& v, const Params& p) {
    uint32_t lw[kMaxServers][2];
    load_logs(v, p, lw);
    bool ok = true;
#pragma unroll
    for (int slot = 1; slot <= kSlots; slot++) ok &= slot_valid(lw, p, slot);
    return ok ? PV_TRUE : PV_FALSE;
  }

  // KVStoreWorkload.APPENDS_LINEARIZABLE (KVStoreWorkload.java:282-340): clients in address order,
  // their (command, result) pairs in order; a non-Append command throws.
  static DSL_HD int appends_linearizable(const NodeView& v, const Params& p) {
    uint32_t all[kMaxClients * kMaxCmds];
    int n = 0;
    for (int c = 0; c < p.clients; c++) {
      const uint32_t* w = v.node(p.servers + c);
      const int nres = getd(w, 15, 2);
      for (int k = 0; k < nres; k++) {
        if (op_of(p, c, k) != OP_APPEND) return PV_THREW;  // "Client workers have non-Append Commands"
        const uint32_t r = (uint32_t)getd(w, res_bit(k), 12);
        const int len = r & 7;
        if (len == 0 || len > kMaxTokens || (int)((r >> (3 + 2 * (len - 1))) & 3) != val(p, c, k)) return PV_FALSE;
        all[n++] = r;
      }
    }
    for (int a = 1; a < n; a++)
      for (int j = a; j > 0 && (all[j] & 7) < (all[j - 1] & 7); j--) {
        const uint32_t t = all[j];
        all[j] = all[j - 1];
        all[j - 1] = t;
      }
    for (int a = 0; a + 1 < n; a++) {
      const int la = all[a] & 7, lb = all[a + 1] & 7;
      if (la == lb) return PV_FALSE;
      const uint32_t mask = (1u << (2 * la)) - 1;
      if (((all[a] >> 3) & mask) != ((all[a + 1] >> 3) & mask)) return PV_FALSE;
    }
    return PV_TRUE;
  }

  // LOGS_CONSISTENT on a successor whose parent held it (nodestate.hpp EvalHeld): a slot's validity
  // reads only the servers' entries of that slot, so only the slots whose entry the changed server
  // changed can have become invalid; each lane checks those (usually one: a uniform loop over the
  // wave's changed slots instead of all four slots of the full check).
  static DSL_HD int logs_consistent_held(const NodeView& v, const Params& p) {
    if (v.changed < 0 || v.changed >= p.servers) return logs_consistent(v, p);
    const uint32_t* o = v.base + v.changed * v.nw;
    const uint32_t* n = v.over;
    const uint32_t d1 = o[1] ^ n[1], d2 = o[2] ^ n[2];
    uint32_t m = (d1 & 0xffffu ? 1u : 0u) | (d1 >> 16 ? 2u : 0u) | (d2 & 0xffffu ? 4u : 0u) | (d2 >> 16 ? 8u : 0u);
    uint32_t lw[kMaxServers][2];
    load_logs(v, p, lw);
    bool ok = true;
    while (!wave_none(m != 0u)) {
      if (m) {
        const int slot = __builtin_ctz(m) + 1;
        m &= m - 1u;
        ok &= slot_valid(lw, p, slot);
      }
    }
    return ok ? PV_TRUE : PV_FALSE;
  }
  static DSL_HD int eval_held(const DevPred& pr, const NodeView& v, const Params& p, bool held) {
    if (held && (pr.id == DSL_PRED_LOGS_CONSISTENT || pr.id == DSL_PRED_LOGS_CONSISTENT_ACTIVE))
      return logs_consistent_held(v, p);
    return eval(pr, v, p);
  }
  static DSL_HD int eval(const DevPred& pr, const NodeView& v, const Params& p) {
    switch (pr.id) {
      case DSL_PRED_RESULTS_OK:
        for (int c = 0; c < p.clients; c++) {
          const uint32_t* w = v.node(p.servers + c);
          const int nres = getd(w, 15, 2);
          for (int k = 0; k < nres; k++)
            if (expect(p, c, k) >= 0 && getd(w, res_bit(k), 12) != expect(p, c, k)) return PV_FALSE;
        }
        return PV_TRUE;
      case DSL_PRED_CLIENTS_DONE:
        for (int c = 0; c < p.clients; c++)
          if (getd(v.node(p.servers + c), 15, 2) < ncmd(p, c)) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_DONE: {
        const int c = pr.arg0 - p.servers;
        if (c < 0 || c >= p.clients) return PV_THREW;
        return getd(v.node(p.servers + c), 15, 2) >= ncmd(p, c) ? PV_TRUE : PV_FALSE;
      }
      case DSL_PRED_NONE_DECIDED:
        for (int c = 0; c < p.clients; c++)
          if (getd(v.node(p.servers + c), 15, 2) > 0) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_HAS_RESULTS: {
        const int c = pr.arg0 - p.servers;
        if (c < 0 || c >= p.clients) return PV_THREW;
        return getd(v.node(p.servers + c), 15, 2) == pr.arg1 ? PV_TRUE : PV_FALSE;
      }
      case DSL_PRED_LOGS_CONSISTENT:
      case DSL_PRED_LOGS_CONSISTENT_ACTIVE:
        return logs_consistent(v, p);
      case DSL_PRED_SLOT_VALID: {
        uint32_t lw[kMaxServers][2];
        load_logs(v, p, lw);
        return slot_valid(lw, p, pr.arg0) ? PV_TRUE : PV_FALSE;
      }
      case DSL_PRED_HAS_STATUS:
      case DSL_PRED_HAS_COMMAND: {  // (PaxosServer) st.server(a): a non-server address throws
        if (pr.arg0 < 0 || pr.arg0 >= p.servers) return PV_THREW;
        const int slot = pr.id == DSL_PRED_HAS_STATUS ? pr.arg1 >> 4 : pr.arg1 >> 8;
        const uint32_t e = slot >= 1 && slot <= kSlots ? entryd(v.node(pr.arg0), slot) : 0u;
        if (pr.id == DSL_PRED_HAS_STATUS) return e_status(e) == (pr.arg1 & 15) ? PV_TRUE : PV_FALSE;
        const int c = e_status(e) == EMPTY ? 0 : kv_cmd(p, e_cmd(e));
        return c == (pr.arg1 & 0xff) ? PV_TRUE : PV_FALSE;
      }
      case DSL_PRED_APPENDS_LINEARIZABLE:
        return appends_linearizable(v, p);
      default:
        return PV_THREW;
    }
  }

  static DSL_HD bool server_log_pred(int id) {
    return id == DSL_PRED_LOGS_CONSISTENT || id == DSL_PRED_LOGS_CONSISTENT_ACTIVE || id == DSL_PRED_SLOT_VALID ||
           id == DSL_PRED_HAS_STATUS || id == DSL_PRED_HAS_COMMAND;
  }
  // Word-level read sets for the incremental check: a client predicate reads the client's
  // result count (w0 bits 15-16) and results (w1-w2); a log predicate a server's log (w1-w2).
  static DSL_HD bool pred_same(const DevPred& pr, const uint32_t* a, const uint32_t* b) {
    if (server_log_pred(pr.id)) return ((a[1] ^ b[1]) | (a[2] ^ b[2])) == 0;
    if ((pr.id >= DSL_PRED_RESULTS_OK && pr.id <= DSL_PRED_CLIENT_HAS_RESULTS) || pr.id == DSL_PRED_APPENDS_LINEARIZABLE)
      return (((a[0] ^ b[0]) & (3u << 15)) | (a[1] ^ b[1]) | (a[2] ^ b[2])) == 0;
    return same_words<kNodeWords>(a, b);
  }
  // Read sets (judge_view's incremental check): client predicates read client nodes only, log
  // predicates the servers (hasStatus / hasCommand: their one server).
  static uint32_t pred_reads(const DevPred& pr, const Params& p) {
    const uint32_t servers = (1u << p.servers) - 1u, clients = ((1u << p.clients) - 1u) << p.servers;
    switch (pr.id) {
      case DSL_PRED_LOGS_CONSISTENT: case DSL_PRED_LOGS_CONSISTENT_ACTIVE: case DSL_PRED_SLOT_VALID: return servers;
      case DSL_PRED_HAS_STATUS: case DSL_PRED_HAS_COMMAND:
        return pr.arg0 >= 0 && pr.arg0 < p.servers ? 1u << pr.arg0 : kReadsAll;
      case DSL_PRED_RESULTS_OK: case DSL_PRED_CLIENTS_DONE: case DSL_PRED_CLIENT_DONE: case DSL_PRED_NONE_DECIDED:
      case DSL_PRED_CLIENT_HAS_RESULTS: case DSL_PRED_APPENDS_LINEARIZABLE: return clients;
      default: return kReadsAll;
    }
  }
  static bool known_predicate(int id) {
    return (id >= DSL_PRED_RESULTS_OK && id <= DSL_PRED_CLIENT_HAS_RESULTS) || server_log_pred(id) ||
           id == DSL_PRED_APPENDS_LINEARIZABLE;
  }
  static bool valid(const Params& p) {
    if (p.servers < 1 || p.servers > kMaxServers || p.clients < 1 || p.clients > kMaxClients) return false;
    int tokens = 0;  // the key's value never exceeds kMaxTokens (every Put / Append adds at most one)
    for (int c = 0; c < p.clients; c++) {
      if (p.ncmds[c] < 1 || p.ncmds[c] > kMaxCmds) return false;
      for (int k = 0; k < p.ncmds[c]; k++) {
        const int op = p.ops[c][k];
        if (op != OP_PUT && op != OP_APPEND && op != OP_GET) return false;
        if (op != OP_GET && (p.vals[c][k] < 1 || p.vals[c][k] > 3)) return false;
        tokens += op != OP_GET;
      }
    }
    return tokens <= kMaxTokens;
  }
  // params: servers, clients, then per client: ncmds, ops[3], vals[3], expected[3]
  static Params from_desc(const dsl_protocol_desc& d) {
    Params p{};
    p.servers = (int32_t)d.params[0];
    p.clients = (int32_t)d.params[1];
    for (int c = 0; c < kMaxClients; c++) {
      const int b = 2 + (1 + 3 * kMaxCmds) * c;
      p.ncmds[c] = (int32_t)d.params[b];
      for (int k = 0; k < kMaxCmds; k++) {
        p.ops[c][k] = (int32_t)d.params[b + 1 + k];
        p.vals[c][k] = (int32_t)d.params[b + 1 + kMaxCmds + k];
        p.expected[c][k] = (int32_t)d.params[b + 1 + 2 * kMaxCmds + k];
      }
    }
    for (int c = 0; c < kMaxClients; c++)
      for (int k = 0; k < kMaxCmds; k++) {
        const int cmd = cmd_id(c, k + 1);
        p.cmdtab |= ((((uint32_t)p.ops[c][k] & 3u) << 2) | ((uint32_t)p.vals[c][k] & 3u)) << (4 * cmd);
        if (p.expected[c][k] >= 0)
          p.exptab[c] |= (uint64_t)(0x8000u | ((uint32_t)p.expected[c][k] & 0xfffu)) << (16 * k);
      }
    return p;
  }
  static void describe_message(Rec m, dsl_event* e) {
    e->from = rec_from(m);
    e->to = rec_to(m);
    e->type = m_type(m);
    e->n_fields = 1;
    e->fields[0] = (int64_t)(m & ((1ull << 55) - 1));
  }
  static void describe_timer(int i, const uint32_t* w, int, const Params& p, dsl_event* e) {
    e->is_timer = 1;
    e->from = e->to = i;
    e->timer_min = e->timer_max = 100;
    e->type = i < p.servers ? T_TICK : T_CLIENT;  // TickTimer / ClientTimer(seq at the head)
    e->n_fields = 1;
    e->fields[0] = i < p.servers ? 0 : get(w, 19, 2);
  }
};

}  // namespace dsl
