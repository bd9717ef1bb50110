// multipaxos.hpp -- lab3 Multi-Paxos (3 servers, 2 clients; BASELINE config C5) as packed
// device transitions.
//
// The reference's lab3 is a stub (labs/lab3-paxos/src/dslabs/paxos/PaxosServer.java:16-127); this
// is the builder-authored protocol specified in DESIGN.md §9 and restated object-style in
// oracle/proto_multipaxos.hpp. It follows labs/lab3-paxos/README.md:25-106 (PMMC roles in one
// server, stable leader + heartbeat-check timer, clients broadcasting requests, AMO KV store) and
// exposes what PaxosTest's predicates read (status / command / lastNonEmpty, PaxosTest.java:113-346).
//
// Nodes: servers 0..n-1 ("server1.."), clients n..n+c-1 ("client1.."). Ballot = (round, leader).
// Commands: id 1 + 2*client + (seq-1) (0 = no-op); a command appends value id vals[client][seq-1].
// KV results: the executed append sequence, 12 bits = len:3 | value ids 2 bits each.
// Application state (the "foo" value, AMO last-seq table) is a function of the log's executed
// prefix (slots < slotOut), so it is recomputed, not stored.
//
// Packed state (152 words = 608 B):
//   server s, 6 words at w[6s]:
//     w0: round:4 | leader:2 @4 | active:1 @6 | electing:1 @7 | heard:1 @8 | missed:2 @9 |
//         p1bVotes:3 @11 | slotOut:3 @14 | slotIn:3 @17
//     w1-w2: log[1..4], 16 bits each: entry = status:2 | round:4 @2 | leader:2 @6 | cmd:3 @8
//     w3: p2bVotes[1..4], 3 bits each
//     w4-w5: p1bLog[1..4] (merged phase-1 log), entries as the log
//   client c, 2 words at w[18 + 2c]:
//     w0: seq:2 | pending:1 @2 | result:12 @3 | nres:2 @15 | ntim:2 @17 | timers[2] seq:2 @19, @21
//     w1: results[0..1], 12 bits each
//   network: w[22] = count, w[24..151] = up to 64 sorted 64-bit records
//     record = type:3 @61 | from:3 @58 | to:3 @55 | payload
//       0 Request  cmd:3                    4 P2a       round:4 leader:2 slot:3 @6 cmd:3 @9
//       1 Reply    seq:2 result:12 @2       5 P2b       round:4 leader:2 slot:3 @6
//       2 P1a      round:4 leader:2 @4      6 Decision  slot:3 cmd:3 @3
//       3 P1b      round:4 leader:2 log 4x11 bits @6   7 Heartbeat round:4 leader:2
// Server Tick timers (100 ms, re-set on every fire) are a constant queue [Tick] and not stored;
// client queues hold ClientTimer(seq) entries (100 ms), only the head is deliverable.
#pragma once
#include "../common.hpp"

namespace dsl {

struct MultiPaxos {
  static constexpr int kWords = 152;
  static constexpr int kMaxServers = 3, kMaxClients = 2, kMaxCmds = 2, kSlots = 4, kMaxRound = 15;
  static constexpr int kNetCount = 22, kNetBase = 24, kNetCap = 64;
  static constexpr int kTick = 100, kClientRetry = 100;
  using State = Packed<kWords>;

  struct Params {
    int32_t servers, clients;
    int32_t ncmds[kMaxClients];
    int32_t vals[kMaxClients][kMaxCmds];      // value id 1..3 of each command
    int32_t expected[kMaxClients][kMaxCmds];  // expected result encoding, -1 = workload has no results
  };
  enum { M_REQUEST = 0, M_REPLY, M_P1A, M_P1B, M_P2A, M_P2B, M_DECISION, M_HEARTBEAT, T_TICK = 8, T_CLIENT = 9 };
  enum { EMPTY = 0, ACCEPTED = 1, CHOSEN = 2 };

  // ---- field access --------------------------------------------------------------------------
  static DSL_HD int sb(int s) { return 6 * s * 32; }
  static DSL_HD int cb(int c) { return (18 + 2 * c) * 32; }
  static DSL_HD uint32_t entry(const State& st, int s, int slot) { return st.get(sb(s) + 32 + 16 * (slot - 1), 16); }
  static DSL_HD void set_entry(State& st, int s, int slot, uint32_t e) { st.set(sb(s) + 32 + 16 * (slot - 1), 16, e); }
  static DSL_HD uint32_t p1entry(const State& st, int s, int slot) {
    return st.get(sb(s) + 128 + 16 * (slot - 1), 16);
  }
  static DSL_HD void set_p1entry(State& st, int s, int slot, uint32_t e) {
    st.set(sb(s) + 128 + 16 * (slot - 1), 16, e);
  }
  static DSL_HD uint32_t mk_entry(int status, int ballot, int cmd) {
    return (uint32_t)status | ((uint32_t)ballot << 2) | ((uint32_t)cmd << 8);
  }
  static DSL_HD int e_status(uint32_t e) { return e & 3; }
  static DSL_HD int e_ballot(uint32_t e) { return (e >> 2) & 0x3f; }  // round:4 | leader:2 (orders as ballot)
  static DSL_HD int e_cmd(uint32_t e) { return (e >> 8) & 7; }
  static DSL_HD int ballot(const State& st, int s) { return st.get(sb(s), 6); }  // round:4 low? see b_of
  static DSL_HD int votes2(const State& st, int s, int slot) { return st.get(sb(s) + 96 + 3 * (slot - 1), 3); }
  static DSL_HD void set_votes2(State& st, int s, int slot, int v) { st.set(sb(s) + 96 + 3 * (slot - 1), 3, v); }

  // A ballot is packed as round:4 (low) | leader:2 (high) in the server word; the comparable form
  // (used in log entries and messages) is (round << 2) | leader.
  static DSL_HD int cmp_ballot(const State& st, int s) { return (st.get(sb(s), 4) << 2) | st.get(sb(s) + 4, 2); }
  static DSL_HD void set_ballot(State& st, int s, int cb_) {
    st.set(sb(s), 4, cb_ >> 2);
    st.set(sb(s) + 4, 2, cb_ & 3);
  }
  static DSL_HD int active(const State& st, int s) { return st.get(sb(s) + 6, 1); }
  static DSL_HD int electing(const State& st, int s) { return st.get(sb(s) + 7, 1); }
  static DSL_HD int heard(const State& st, int s) { return st.get(sb(s) + 8, 1); }
  static DSL_HD int missed(const State& st, int s) { return st.get(sb(s) + 9, 2); }
  static DSL_HD int p1votes(const State& st, int s) { return st.get(sb(s) + 11, 3); }
  static DSL_HD int slot_out(const State& st, int s) { return st.get(sb(s) + 14, 3); }
  static DSL_HD int slot_in(const State& st, int s) { return st.get(sb(s) + 17, 3); }

  // messages
  static DSL_HD uint64_t msg(int type, int from, int to, uint64_t payload) {
    return ((uint64_t)type << 61) | ((uint64_t)from << 58) | ((uint64_t)to << 55) | payload;
  }
  static DSL_HD int m_type(uint64_t m) { return (int)(m >> 61); }
  static DSL_HD int m_from(uint64_t m) { return (int)((m >> 58) & 7); }
  static DSL_HD int m_to(uint64_t m) { return (int)((m >> 55) & 7); }
  // comparable ballot (round<<2|leader) <-> message field round:4 @0 | leader:2 @4
  static DSL_HD uint64_t m_ballot_field(int cb_) { return (uint64_t)(cb_ >> 2) | ((uint64_t)(cb_ & 3) << 4); }
  static DSL_HD int m_ballot(uint64_t m) { return (int)(((m & 0xf) << 2) | ((m >> 4) & 3)); }

  static DSL_HD int net_size(const State& st) { return (int)st.w[kNetCount]; }
  static DSL_HD uint64_t net_at(const State& st, int i) {
    return (uint64_t)st.w[kNetBase + 2 * i] | ((uint64_t)st.w[kNetBase + 2 * i + 1] << 32);
  }
  static DSL_HD bool send(State& st, uint64_t r) {  // network.add (set semantics, sorted)
    int n = net_size(st), pos = 0;
    while (pos < n && net_at(st, pos) < r) pos++;
    if (pos < n && net_at(st, pos) == r) return true;
    if (n >= kNetCap) return false;
    for (int j = n; j > pos; j--) {
      st.w[kNetBase + 2 * j] = st.w[kNetBase + 2 * j - 2];
      st.w[kNetBase + 2 * j + 1] = st.w[kNetBase + 2 * j - 1];
    }
    st.w[kNetBase + 2 * pos] = (uint32_t)r;
    st.w[kNetBase + 2 * pos + 1] = (uint32_t)(r >> 32);
    st.w[kNetCount] = (uint32_t)(n + 1);
    return true;
  }
  static DSL_HD bool bcast_servers(State& st, const Params& p, int from, int type, uint64_t payload) {
    bool ok = true;
    for (int s = 0; s < p.servers; s++)
      if (s != from) ok &= send(st, msg(type, from, s, payload));
    return ok;
  }

  // ---- application: the executed prefix --------------------------------------------------------
  static DSL_HD int cmd_client(int cmd) { return (cmd - 1) >> 1; }
  static DSL_HD int cmd_seq(int cmd) { return ((cmd - 1) & 1) + 1; }
  static DSL_HD uint32_t res_push(uint32_t r, int v) {  // append value id to a result encoding
    int len = r & 7;
    return (uint32_t)(len + 1) | (r & ~7u) | ((uint32_t)v << (3 + 2 * len));
  }
  // Executed sequence (result encoding) and AMO last seq per client for slots < upto.
  static DSL_HD uint32_t executed(const State& st, const Params& p, int s, int upto, int* last_seq) {
    uint32_t seqv = 0;
    for (int c = 0; c < kMaxClients; c++) last_seq[c] = 0;
    for (int slot = 1; slot < upto; slot++) {
      int cmd = e_cmd(entry(st, s, slot));
      if (!cmd) continue;
      int c = cmd_client(cmd), q = cmd_seq(cmd);
      if (last_seq[c] < q) {
        seqv = res_push(seqv, p.vals[c][q - 1]);
        last_seq[c] = q;
      }
    }
    return seqv;
  }

  static DSL_HD bool execute(State& st, const Params& p, int s) {
    int last_seq[kMaxClients];
    int out = slot_out(st, s);
    uint32_t seqv = executed(st, p, s, out, last_seq);
    bool ok = true;
    while (out <= kSlots && e_status(entry(st, s, out)) == CHOSEN) {
      int cmd = e_cmd(entry(st, s, out));
      if (cmd) {
        int c = cmd_client(cmd), q = cmd_seq(cmd);
        if (last_seq[c] < q) {
          seqv = res_push(seqv, p.vals[c][q - 1]);
          last_seq[c] = q;
          if (active(st, s))
            ok &= send(st, msg(M_REPLY, s, p.servers + c, (uint64_t)q | ((uint64_t)seqv << 2)));
        }
      }
      out++;
    }
    st.set(sb(s) + 14, 3, out);
    return ok;
  }

  static DSL_HD void step_down_to(State& st, int s, int b) {  // adopt: b > current ballot
    set_ballot(st, s, b);
    st.set(sb(s) + 6, 2, 0);   // active, electing
    st.set(sb(s) + 11, 3, 0);  // p1bVotes
    st.w[6 * s + 3] = 0;       // p2bVotes
    st.w[6 * s + 4] = 0;       // p1bLog
    st.w[6 * s + 5] = 0;
  }
  static DSL_HD void adopt(State& st, int s, int b) {
    if (b > cmp_ballot(st, s)) step_down_to(st, s, b);
  }
  static DSL_HD bool majority(const Params& p, int votes) { return __builtin_popcount(votes) * 2 > p.servers; }

  static DSL_HD bool choose(State& st, const Params& p, int s, int slot) {
    int cmd = e_cmd(entry(st, s, slot));
    set_entry(st, s, slot, mk_entry(CHOSEN, 0, cmd));
    set_votes2(st, s, slot, 0);
    bool ok = bcast_servers(st, p, s, M_DECISION, (uint64_t)slot | ((uint64_t)cmd << 3));
    return execute(st, p, s) && ok;
  }
  static DSL_HD bool propose(State& st, const Params& p, int s, int slot, int cmd) {
    const int b = cmp_ballot(st, s);
    set_entry(st, s, slot, mk_entry(ACCEPTED, b, cmd));
    set_votes2(st, s, slot, 1 << s);
    bool ok = bcast_servers(st, p, s, M_P2A, m_ballot_field(b) | ((uint64_t)slot << 6) | ((uint64_t)cmd << 9));
    if (majority(p, 1 << s)) ok &= choose(st, p, s, slot);
    return ok;
  }
  static DSL_HD void merge(State& st, int s, int slot, uint32_t e) {
    uint32_t m = p1entry(st, s, slot);
    if (e_status(e) == CHOSEN) {
      set_p1entry(st, s, slot, mk_entry(CHOSEN, 0, e_cmd(e)));
    } else if (e_status(e) == ACCEPTED && e_status(m) != CHOSEN &&
               (e_status(m) == EMPTY || e_ballot(m) < e_ballot(e))) {
      set_p1entry(st, s, slot, e);
    }
  }
  static DSL_HD bool become_leader(State& st, const Params& p, int s) {
    st.set(sb(s) + 6, 1, 1);   // active
    st.set(sb(s) + 7, 1, 0);   // electing
    st.set(sb(s) + 11, 3, 0);  // p1bVotes
    int last = 0;
    uint32_t merged[kSlots + 1];
    for (int i = 1; i <= kSlots; i++) {
      merged[i] = p1entry(st, s, i);
      if (e_status(merged[i]) != EMPTY || e_status(entry(st, s, i)) != EMPTY) last = i;
    }
    st.w[6 * s + 4] = 0;
    st.w[6 * s + 5] = 0;
    bool ok = true;
    for (int i = 1; i <= last; i++) {
      if (e_status(entry(st, s, i)) == CHOSEN) continue;
      if (e_status(merged[i]) == CHOSEN) {
        set_entry(st, s, i, mk_entry(CHOSEN, 0, e_cmd(merged[i])));
        set_votes2(st, s, i, 0);
      } else {
        ok &= propose(st, p, s, i, e_status(merged[i]) == ACCEPTED ? e_cmd(merged[i]) : 0);
      }
    }
    st.set(sb(s) + 17, 3, last + 1);
    return execute(st, p, s) && ok;
  }

  // ---- clients (PaxosClient inside ClientWorker) -------------------------------------------------
  static DSL_HD bool client_send(State& st, const Params& p, int c, int q) {
    const int b = cb(c);
    st.set(b, 2, q);
    st.set(b + 2, 1, 1);
    st.set(b + 3, 12, 0);
    const int cmd = 1 + 2 * c + (q - 1);
    bool ok = true;
    for (int s = 0; s < p.servers; s++) ok &= send(st, msg(M_REQUEST, p.servers + c, s, (uint64_t)cmd));
    int n = st.get(b + 17, 2);
    if (n >= 2) return false;
    st.set(b + 19 + 2 * n, 2, q);
    st.set(b + 17, 2, n + 1);
    return ok;
  }
  static DSL_HD bool client_worker_continue(State& st, const Params& p, int c) {
    const int b = cb(c);
    int nres = st.get(b + 15, 2);
    uint32_t res = st.get(b + 3, 12);
    if (nres < p.ncmds[c] && res != 0) {
      st.set(b + 32 + 12 * nres, 12, res);
      nres++;
      st.set(b + 15, 2, nres);
      if (nres < p.ncmds[c]) return client_send(st, p, c, nres + 1);
    }
    return true;
  }

  static DSL_HD void init(State& st, const Params& p) {
    for (int i = 0; i < kWords; i++) st.w[i] = 0;
    for (int s = 0; s < p.servers; s++) {
      st.set(sb(s) + 14, 3, 1);
      st.set(sb(s) + 17, 3, 1);
    }
    st.set(sb(0) + 6, 1, 1);  // server1 leads ballot (0, server1)
    for (int c = 0; c < p.clients; c++) client_send(st, p, c, 1);
  }

  // ---- events -----------------------------------------------------------------------------------
  static DSL_HD int num_events(const State& st, const Params& p, const DevSettings& set) {
    int n = 0;
    const int cnt = net_size(st);
    for (int i = 0; i < cnt; i++) {
      uint64_t m = net_at(st, i);
      n += should_deliver(set, m_from(m), m_to(m));
    }
    for (int s = 0; s < p.servers; s++) n += deliver_timers(set, s);
    for (int c = 0; c < p.clients; c++) n += deliver_timers(set, p.servers + c) && st.get(cb(c) + 17, 2) > 0;
    return n;
  }
  // k-th enabled event: >= 0 message index into the network; -1-s server tick; -100-c client timer
  static DSL_HD int locate(const State& st, const Params& p, const DevSettings& set, int k) {
    const int cnt = net_size(st);
    for (int i = 0; i < cnt; i++) {
      uint64_t m = net_at(st, i);
      if (should_deliver(set, m_from(m), m_to(m)) && k-- == 0) return i;
    }
    for (int s = 0; s < p.servers; s++)
      if (deliver_timers(set, s) && k-- == 0) return -1 - s;
    for (int c = 0; c < p.clients; c++)
      if (deliver_timers(set, p.servers + c) && st.get(cb(c) + 17, 2) > 0 && k-- == 0) return -100 - c;
    return -1000;
  }

  static DSL_HD int server_msg(State& st, const Params& p, uint64_t m) {
    const int s = m_to(m), from = m_from(m);
    const int type = m_type(m);
    bool ok = true;
    if (type == M_REQUEST) {
      const int cmd = (int)(m & 7), c = cmd_client(cmd), q = cmd_seq(cmd);
      int last_seq[kMaxClients];
      const uint32_t seqv = executed(st, p, s, slot_out(st, s), last_seq);
      (void)seqv;
      if (last_seq[c] >= q) {
        if (active(st, s) && last_seq[c] == q) {
          // cached AMO result: the executed sequence right after this command
          int ls2[kMaxClients];
          uint32_t r = 0;
          for (int upto = 1; upto <= slot_out(st, s); upto++) {
            r = executed(st, p, s, upto, ls2);
            if (ls2[c] == q) break;
          }
          ok = send(st, msg(M_REPLY, s, p.servers + c, (uint64_t)q | ((uint64_t)r << 2)));
        }
        return ok ? STEP_OK : STEP_OVERFLOW;
      }
      // a new proposal goes after every slot this server knows to be in use (a stale leader may
      // have learned later slots through Decision / P2a); no free slot -> ignore (clients retry)
      int slot = slot_in(st, s);
      for (int i = 1; i <= kSlots; i++)
        if (e_status(entry(st, s, i)) != EMPTY && i + 1 > slot) slot = i + 1;
      if (active(st, s) && slot <= kSlots) {
        for (int i = 1; i <= kSlots; i++) {
          uint32_t e = entry(st, s, i);
          if (e_status(e) != EMPTY && e_cmd(e) == cmd) return STEP_OK;  // already in the log
        }
        st.set(sb(s) + 17, 3, slot + 1);
        ok = propose(st, p, s, slot, cmd);
      }
      return ok ? STEP_OK : STEP_OVERFLOW;
    }
    const int b = m_ballot(m);
    switch (type) {
      case M_P2A: {
        if (b < cmp_ballot(st, s)) return STEP_OK;
        adopt(st, s, b);
        st.set(sb(s) + 8, 1, 1);
        const int slot = (int)((m >> 6) & 7), cmd = (int)((m >> 9) & 7);
        if (e_status(entry(st, s, slot)) != CHOSEN) set_entry(st, s, slot, mk_entry(ACCEPTED, b, cmd));
        ok = send(st, msg(M_P2B, s, from, m_ballot_field(b) | ((uint64_t)slot << 6)));
        break;
      }
      case M_P2B: {
        const int slot = (int)((m >> 6) & 7);
        if (!active(st, s) || b != cmp_ballot(st, s) || e_status(entry(st, s, slot)) != ACCEPTED) return STEP_OK;
        const int v = votes2(st, s, slot) | (1 << from);
        set_votes2(st, s, slot, v);
        if (majority(p, v)) ok = choose(st, p, s, slot);
        break;
      }
      case M_DECISION: {
        const int slot = (int)(m & 7), cmd = (int)((m >> 3) & 7);
        if (e_status(entry(st, s, slot)) != CHOSEN) {
          set_entry(st, s, slot, mk_entry(CHOSEN, 0, cmd));
          set_votes2(st, s, slot, 0);
          ok = execute(st, p, s);
        }
        break;
      }
      case M_HEARTBEAT:
        if (b < cmp_ballot(st, s)) return STEP_OK;
        adopt(st, s, b);
        st.set(sb(s) + 8, 1, 1);
        break;
      case M_P1A: {
        if (b < cmp_ballot(st, s)) return STEP_OK;
        adopt(st, s, b);
        st.set(sb(s) + 8, 1, 1);
        uint64_t logbits = 0;
        for (int i = 1; i <= kSlots; i++) logbits |= (uint64_t)(entry(st, s, i) & 0x7ff) << (11 * (i - 1));
        ok = send(st, msg(M_P1B, s, from, m_ballot_field(b) | (logbits << 6)));
        break;
      }
      case M_P1B: {
        if (!electing(st, s) || b != cmp_ballot(st, s)) return STEP_OK;
        const int v = p1votes(st, s) | (1 << from);
        st.set(sb(s) + 11, 3, v);
        for (int i = 1; i <= kSlots; i++) merge(st, s, i, (uint32_t)((m >> (6 + 11 * (i - 1))) & 0x7ff));
        if (majority(p, v)) ok = become_leader(st, p, s);
        break;
      }
      default:
        return STEP_NULL;
    }
    return ok ? STEP_OK : STEP_OVERFLOW;
  }

  static DSL_HD int server_tick(State& st, const Params& p, int s) {
    bool ok = true;
    if (active(st, s)) {
      ok = bcast_servers(st, p, s, M_HEARTBEAT, m_ballot_field(cmp_ballot(st, s)));
    } else if (heard(st, s)) {
      st.set(sb(s) + 8, 1, 0);
      st.set(sb(s) + 9, 2, 0);
    } else {
      int mis = missed(st, s) + 1;
      if (mis > 2) mis = 2;
      st.set(sb(s) + 9, 2, mis);
      const int b = cmp_ballot(st, s);
      if (mis >= 2 && (b >> 2) < kMaxRound) {
        st.set(sb(s) + 9, 2, 0);
        st.set(sb(s) + 8, 1, 0);
        set_ballot(st, s, (((b >> 2) + 1) << 2) | s);
        st.set(sb(s) + 7, 1, 1);  // electing
        st.set(sb(s) + 6, 1, 0);  // active
        st.w[6 * s + 3] = 0;      // p2bVotes
        st.set(sb(s) + 11, 3, 1 << s);
        st.w[6 * s + 4] = 0;
        st.w[6 * s + 5] = 0;
        for (int i = 1; i <= kSlots; i++) merge(st, s, i, entry(st, s, i));
        ok = bcast_servers(st, p, s, M_P1A, m_ballot_field(cmp_ballot(st, s)));
        if (majority(p, 1 << s)) ok &= become_leader(st, p, s);
      }
    }
    return ok ? STEP_OK : STEP_OVERFLOW;  // set(t, 100) then remove(t): the queue stays [Tick]
  }

  static DSL_HD int step(const State& in, int k, State& st, const Params& p, const DevSettings& set) {
    st = in;
    const int e = locate(in, p, set, k);
    if (e == -1000) return STEP_NULL;
    if (e >= 0) {
      const uint64_t m = net_at(in, e);
      const int to = m_to(m);
      if (to < p.servers) return server_msg(st, p, m);
      // client: PaxosClient.handlePaxosReply, then the ClientWorker loop
      const int c = to - p.servers, b = cb(c);
      const int q = (int)(m & 3);
      if (st.get(b + 2, 1) && q == st.get(b, 2)) {
        st.set(b + 3, 12, (uint32_t)((m >> 2) & 0xfff));
        st.set(b + 2, 1, 0);
      }
      return client_worker_continue(st, p, c) ? STEP_OK : STEP_OVERFLOW;
    }
    if (e > -100) return server_tick(st, p, -1 - e);
    // client timer (head of the queue): onClientTimer, ClientWorker loop, remove first equal
    const int c = -100 - e, b = cb(c);
    const int t = st.get(b + 19, 2);
    bool ok = true;
    if (st.get(b + 2, 1) && t == st.get(b, 2)) {
      const int cmd = 1 + 2 * c + (t - 1);
      for (int s = 0; s < p.servers; s++) ok &= send(st, msg(M_REQUEST, p.servers + c, s, (uint64_t)cmd));
      int n = st.get(b + 17, 2);
      if (n >= 2) return STEP_OVERFLOW;
      st.set(b + 19 + 2 * n, 2, t);
      st.set(b + 17, 2, n + 1);
    }
    ok &= client_worker_continue(st, p, c);
    int n = st.get(b + 17, 2);
    // remove the head (the first entry equal to the fired timer)
    int t1 = st.get(b + 21, 2);
    st.set(b + 19, 2, n > 1 ? t1 : 0);
    st.set(b + 21, 2, 0);
    st.set(b + 17, 2, n - 1);
    return ok ? STEP_OK : STEP_OVERFLOW;
  }

  // ---- predicates ---------------------------------------------------------------------------------
  static DSL_HD int value_of(const Params& p, int cmd) { return cmd ? p.vals[cmd_client(cmd)][cmd_seq(cmd) - 1] : 0; }

  static DSL_HD int logs_consistent(const State& st, const Params& p) {
    int max_ne = 0;
    for (int s = 0; s < p.servers; s++)
      for (int i = 1; i <= kSlots; i++)
        if (e_status(entry(st, s, i)) != EMPTY && i > max_ne) max_ne = i;
    for (int slot = 1; slot <= max_ne; slot++) {
      bool is_chosen = false;
      int chosen = 0;
      for (int s = 0; s < p.servers; s++) {
        uint32_t e = entry(st, s, slot);
        if (e_status(e) == CHOSEN) {
          const int v = value_of(p, e_cmd(e));
          if (is_chosen && v != chosen) return PV_FALSE;
          chosen = v;
          is_chosen = true;
        }
      }
      if (!is_chosen) continue;
      int count = 0;
      for (int s = 0; s < p.servers; s++) {
        uint32_t e = entry(st, s, slot);
        if (e_status(e) != EMPTY && (e_status(e) != ACCEPTED || value_of(p, e_cmd(e)) == chosen)) count++;
      }
      if (2 * count <= p.servers) return PV_FALSE;
    }
    return PV_TRUE;
  }

  static DSL_HD int appends_linearizable(const State& st, const Params& p) {
    uint32_t all[kMaxClients * kMaxCmds];
    int n = 0;
    for (int c = 0; c < p.clients; c++) {
      const int nres = st.get(cb(c) + 15, 2);
      for (int k = 0; k < nres; k++) {
        const uint32_t r = st.get(cb(c) + 32 + 12 * k, 12);
        const int len = r & 7;
        if (len == 0 || (int)((r >> (3 + 2 * (len - 1))) & 3) != p.vals[c][k]) return PV_FALSE;  // endsWith
        all[n++] = r;
      }
    }
    // sort by length (stable), then each must be a strict prefix of the next
    for (int i = 1; i < n; i++)
      for (int j = i; j > 0 && (all[j] & 7) < (all[j - 1] & 7); j--) {
        uint32_t t = all[j];
        all[j] = all[j - 1];
        all[j - 1] = t;
      }
    for (int i = 0; i + 1 < n; i++) {
      const int la = all[i] & 7, lb = all[i + 1] & 7;
      if (la == lb) return PV_FALSE;  // equal (same length and prefix) or not a prefix
      const uint32_t mask = (1u << (2 * la)) - 1;
      if (((all[i] >> 3) & mask) != ((all[i + 1] >> 3) & mask)) return PV_FALSE;
    }
    return PV_TRUE;
  }

  static DSL_HD int eval(const DevPred& pr, const State& st, const Params& p) {
    switch (pr.id) {
      case DSL_PRED_RESULTS_OK:
        for (int c = 0; c < p.clients; c++) {
          const int nres = st.get(cb(c) + 15, 2);
          for (int k = 0; k < nres; k++)
            if (p.expected[c][k] >= 0 && st.get(cb(c) + 32 + 12 * k, 12) != (uint32_t)p.expected[c][k])
              return PV_FALSE;
        }
        return PV_TRUE;
      case DSL_PRED_CLIENTS_DONE:
        for (int c = 0; c < p.clients; c++)
          if (st.get(cb(c) + 15, 2) < p.ncmds[c]) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_DONE: {
        const int c = (int)pr.arg0 - p.servers;
        if (c < 0 || c >= p.clients) return PV_THREW;
        return st.get(cb(c) + 15, 2) >= p.ncmds[c] ? PV_TRUE : PV_FALSE;
      }
      case DSL_PRED_NONE_DECIDED:
        for (int c = 0; c < p.clients; c++)
          if (st.get(cb(c) + 15, 2) > 0) return PV_FALSE;
        return PV_TRUE;
      case DSL_PRED_CLIENT_HAS_RESULTS: {
        const int c = (int)pr.arg0 - p.servers;
        if (c < 0 || c >= p.clients) return PV_THREW;
        return st.get(cb(c) + 15, 2) == pr.arg1 ? PV_TRUE : PV_FALSE;
      }
      case DSL_PRED_LOGS_CONSISTENT:
        return logs_consistent(st, p);
      case DSL_PRED_APPENDS_LINEARIZABLE:
        return appends_linearizable(st, p);
      default:
        return PV_THREW;
    }
  }

  static bool known_predicate(int id) {
    return (id >= DSL_PRED_RESULTS_OK && id <= DSL_PRED_CLIENT_HAS_RESULTS) || id == DSL_PRED_LOGS_CONSISTENT ||
           id == DSL_PRED_APPENDS_LINEARIZABLE;
  }
  static int num_nodes(const Params& p) { return p.servers + p.clients; }
  static bool valid(const Params& p) {
    if (p.servers < 1 || p.servers > kMaxServers || p.clients < 1 || p.clients > kMaxClients) return false;
    for (int c = 0; c < p.clients; c++) {
      if (p.ncmds[c] < 1 || p.ncmds[c] > kMaxCmds) return false;
      for (int k = 0; k < p.ncmds[c]; k++)
        if (p.vals[c][k] < 1 || p.vals[c][k] > 3) return false;
    }
    return true;
  }
  // params: servers, clients, then per client: ncmds, val[0], val[1], expected[0], expected[1]
  static Params from_desc(const dsl_protocol_desc& d) {
    Params p{};
    p.servers = (int32_t)d.params[0];
    p.clients = (int32_t)d.params[1];
    for (int c = 0; c < kMaxClients; c++) {
      const int b = 2 + 5 * c;
      p.ncmds[c] = (int32_t)d.params[b];
      for (int k = 0; k < kMaxCmds; k++) {
        p.vals[c][k] = (int32_t)d.params[b + 1 + k];
        p.expected[c][k] = (int32_t)d.params[b + 3 + k];
      }
    }
    return p;
  }

  static void describe(const State& st, const Params& p, const DevSettings& set, int k, dsl_event* ev) {
    *ev = dsl_event{};
    const int e = locate(st, p, set, k);
    if (e < 0) {
      ev->is_timer = 1;
      ev->timer_min = ev->timer_max = 100;
      if (e > -100) {
        ev->from = ev->to = -1 - e;
        ev->type = T_TICK;
      } else {
        const int c = -100 - e;
        ev->from = ev->to = p.servers + c;
        ev->type = T_CLIENT;
        ev->n_fields = 1;
        ev->fields[0] = st.get(cb(c) + 19, 2);
      }
      return;
    }
    const uint64_t m = net_at(st, e);
    ev->from = m_from(m);
    ev->to = m_to(m);
    ev->type = m_type(m);
    ev->n_fields = 1;
    ev->fields[0] = (int64_t)(m & ((1ull << 55) - 1));
  }
};

}  // namespace dsl
