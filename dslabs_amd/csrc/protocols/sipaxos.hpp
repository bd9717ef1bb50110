// sipaxos.hpp -- the reference's single-instance "Paxos Made Simple" as device transitions.
//
// Re-expresses framework/tst/dslabs/framework/testing/visualization/examples/paxosmadesimple/
// SingleInstancePaxos.java:177-293 (Proposer.onPropose / handlePrepareAck / handleAcceptAck,
// Acceptor.handlePrepare / handleAccept), :296-323 (messages, Propose timer = 100 ms) and the
// buggy acceptor of IncorrectSingleInstancePaxos.java:29-64 (accepts regardless of promise).
//
// Nodes: proposers 0..P-1 ("proposer1".."), acceptors P..P+A-1 ("acceptor1..").
// Proposal values are interned: value id v in 1..P = the initial proposal of proposer v.
//
// Packed state (64 words = 256 B):
//   proposer p (3 words at w[3p]):
//     w0: hasProposed:1 | prepareFinished:1 | value:2 | decision:2 (0 = null) | acceptAcks:5 (bit a)
//         | proposalNumber:8 @16
//     w1,w2: prepareAcks[a] for a < 5, 11 bits each at bit 11*a of the 64-bit pair:
//         present:1 | accepted.n:8 (0 = null) | accepted.v:2
//         (entries are only stored for m.proposalNumber == proposalNumber, so the ack's own
//          proposal number is implied by the proposer's)
//   acceptor a (1 word at w[9 + a]): highestPrepared:8 (0 = null) | accepted.n:8 | accepted.v:2
//   network (w[14] = count, w[15..62] = sorted records), record =
//     type:2 @30 | from:3 @27 | to:3 @24 | n:8 @16 | an:8 @8 | av:2 @0
//     types: 0 Prepare(n), 1 PrepareAck(n, (an, av) | null), 2 Accept(n, av), 3 AcceptAck(n)
// The Propose timer queue of each proposer is always exactly [Propose(100ms)]: onPropose
// re-sets it and stepTimer then removes the first equal entry (SearchState.java:357), so the
// queue is constant and not stored. Proposal numbers above 255 are reported as overflow.
#pragma once
#include "../common.hpp"
#include "../netset.hpp"

namespace dsl {

struct SIPaxos {
  static constexpr int kWords = 64;
  static constexpr int kMaxP = 3, kMaxA = 5;
  static constexpr int kNetBase = 14, kNetCap = 48;
  using State = Packed<kWords>;
  using Net = NetSet<kNetBase, kNetCap>;

  struct Params {
    int32_t proposers, acceptors;
    int32_t incorrect;
  };
  enum { T_PREPARE = 0, T_PREPARE_ACK = 1, T_ACCEPT = 2, T_ACCEPT_ACK = 3, T_PROPOSE_TIMER = 4 };

  static DSL_HD uint32_t rec(int type, int from, int to, int n, int an, int av) {
    return ((uint32_t)type << 30) | ((uint32_t)from << 27) | ((uint32_t)to << 24) | ((uint32_t)n << 16) |
           ((uint32_t)an << 8) | (uint32_t)av;
  }
  static DSL_HD int r_type(uint32_t r) { return r >> 30; }
  static DSL_HD int r_from(uint32_t r) { return (r >> 27) & 7; }
  static DSL_HD int r_to(uint32_t r) { return (r >> 24) & 7; }
  static DSL_HD int r_n(uint32_t r) { return (r >> 16) & 0xff; }
  static DSL_HD int r_an(uint32_t r) { return (r >> 8) & 0xff; }
  static DSL_HD int r_av(uint32_t r) { return r & 3; }

  // proposer fields
  static DSL_HD int pb(int p) { return 3 * p * 32; }
  static DSL_HD int has_proposed(const State& s, int p) { return s.get(pb(p), 1); }
  static DSL_HD int prep_fin(const State& s, int p) { return s.get(pb(p) + 1, 1); }
  static DSL_HD int value(const State& s, int p) { return s.get(pb(p) + 2, 2); }
  static DSL_HD int decision(const State& s, int p) { return s.get(pb(p) + 4, 2); }
  static DSL_HD int accept_acks(const State& s, int p) { return s.get(pb(p) + 6, 5); }
  static DSL_HD int pnum(const State& s, int p) { return s.get(pb(p) + 16, 8); }
  static DSL_HD uint64_t acks64(const State& s, int p) {
    return (uint64_t)s.w[3 * p + 1] | ((uint64_t)s.w[3 * p + 2] << 32);
  }
  static DSL_HD void set_acks64(State& s, int p, uint64_t v) {
    s.w[3 * p + 1] = (uint32_t)v;
    s.w[3 * p + 2] = (uint32_t)(v >> 32);
  }
  // acceptor fields
  static DSL_HD int ab(int a) { return (9 + a) * 32; }

  static DSL_HD int broadcast(State& s, const Params& prm, int from, uint32_t proto_rec) {
    for (int a = 0; a < prm.acceptors; a++) {
      int to = prm.proposers + a;
      uint32_t r = (proto_rec & ~(uint32_t)(0x3f << 24)) | ((uint32_t)from << 27) | ((uint32_t)to << 24);
      if (Net::insert(s, r) < 0) return STEP_OVERFLOW;
    }
    return STEP_OK;
  }

  static DSL_HD void init(State& s, const Params& prm) {
    for (int i = 0; i < kWords; i++) s.w[i] = 0;
    for (int p = 0; p < prm.proposers; p++) {
      s.set(pb(p) + 2, 2, p + 1);    // proposalValue = values[p]
      s.set(pb(p) + 16, 8, p + 1);   // proposalNumber = p + 1
      // init(): set(new Propose(), 100) -- constant queue, not stored
    }
  }

  static DSL_HD int num_events(const State& s, const Params& prm, const DevSettings& set) {
    int n = 0;
    const int cnt = Net::size(s);
    for (int i = 0; i < cnt; i++) {
      uint32_t r = Net::at(s, i);
      n += should_deliver(set, r_from(r), r_to(r));
    }
    for (int p = 0; p < prm.proposers; p++) n += deliver_timers(set, p);
    return n;
  }

  // k-th enabled event: returns the record (messages) or -1-p (timer of proposer p).
  static DSL_HD int64_t locate(const State& s, const Params& prm, const DevSettings& set, int k) {
    const int cnt = Net::size(s);
    for (int i = 0; i < cnt; i++) {
      uint32_t r = Net::at(s, i);
      if (should_deliver(set, r_from(r), r_to(r)) && k-- == 0) return (int64_t)r;
    }
    for (int p = 0; p < prm.proposers; p++)
      if (deliver_timers(set, p) && k-- == 0) return -1 - p;
    return INT64_MIN;
  }

  static DSL_HD int on_propose(State& s, const Params& prm, int p) {
    int n = pnum(s, p);
    if (has_proposed(s, p)) n += prm.proposers;
    if (n > 255) return STEP_OVERFLOW;
    s.set(pb(p) + 16, 8, n);
    s.set(pb(p), 1, 1);
    set_acks64(s, p, 0);         // prepareAcks.clear()
    s.set(pb(p) + 6, 5, 0);      // acceptAcks.clear()
    s.set(pb(p) + 1, 1, 0);      // prepareFinished = false
    return broadcast(s, prm, p, rec(T_PREPARE, 0, 0, n, 0, 0));
  }

  static DSL_HD int prepare_ack(State& s, const Params& prm, int p, int a, uint32_t m) {
    const int n = pnum(s, p);
    if (r_n(m) != n || prep_fin(s, p)) return STEP_OK;
    uint64_t acks = acks64(s, p);
    const int sh = 11 * a;
    acks &= ~((uint64_t)0x7ff << sh);
    acks |= ((uint64_t)(1 | (r_an(m) << 1) | (r_av(m) << 9))) << sh;
    int count = 0;
    for (int i = 0; i < prm.acceptors; i++) count += (acks >> (11 * i)) & 1;
    if (count * 2 > prm.acceptors) {
      s.set(pb(p) + 1, 1, 1);
      // value of the highest accepted ballot among the acks (equal ballots carry equal values)
      int best_n = 0, best_v = 0;
      for (int i = 0; i < prm.acceptors; i++) {
        uint32_t e = (uint32_t)(acks >> (11 * i)) & 0x7ff;
        if (!(e & 1)) continue;
        int an = (e >> 1) & 0xff, av = (e >> 9) & 3;
        if (an != 0 && an >= best_n) best_n = an, best_v = av;
      }
      if (best_n != 0) s.set(pb(p) + 2, 2, best_v);
      acks = 0;  // prepareAcks.clear()
      set_acks64(s, p, acks);
      return broadcast(s, prm, p, rec(T_ACCEPT, 0, 0, n, 0, value(s, p)));
    }
    set_acks64(s, p, acks);
    return STEP_OK;
  }

  static DSL_HD int step(const State& in, int k, State& s, const Params& prm, const DevSettings& set) {
    s = in;
    const int64_t e = locate(in, prm, set, k);
    if (e == INT64_MIN) return STEP_NULL;
    if (e < 0) return on_propose(s, prm, (int)(-1 - e));
    const uint32_t m = (uint32_t)e;
    const int from = r_from(m), to = r_to(m);
    switch (r_type(m)) {
      case T_PREPARE: {  // Acceptor.handlePrepare
        const int b = ab(to - prm.proposers);
        const int hp = s.get(b, 8);
        if (hp != 0 && hp >= r_n(m)) return STEP_OK;
        s.set(b, 8, r_n(m));
        const uint32_t ack = rec(T_PREPARE_ACK, to, from, r_n(m), s.get(b + 8, 8), s.get(b + 16, 2));
        return Net::insert(s, ack) < 0 ? STEP_OVERFLOW : STEP_OK;
      }
      case T_PREPARE_ACK:
        return prepare_ack(s, prm, to, from - prm.proposers, m);
      case T_ACCEPT: {  // Acceptor.handleAccept
        const int b = ab(to - prm.proposers);
        const int hp = s.get(b, 8);
        if (!prm.incorrect && hp != 0 && hp > r_n(m)) return STEP_OK;
        if (Net::insert(s, rec(T_ACCEPT_ACK, to, from, r_n(m), 0, 0)) < 0) return STEP_OVERFLOW;
        const int han = s.get(b + 8, 8);
        if (han == 0 || han < r_n(m)) {
          s.set(b + 8, 8, r_n(m));
          s.set(b + 16, 2, r_av(m));
        }
        return STEP_OK;
      }
      default: {  // T_ACCEPT_ACK: Proposer.handleAcceptAck
        const int p = to;
        if (pnum(s, p) != r_n(m)) return STEP_OK;
        int acks = accept_acks(s, p) | (1 << (from - prm.proposers));
        s.set(pb(p) + 6, 5, acks);
        if (__builtin_popcount(acks) * 2 > prm.acceptors) s.set(pb(p) + 4, 2, value(s, p));
        return STEP_OK;
      }
    }
  }

  static DSL_HD int eval(const DevPred& pr, const State& s, const Params& prm) {
    switch (pr.id) {
      case DSL_PRED_SIP_AGREEMENT: {
        int d = 0;
        for (int p = 0; p < prm.proposers; p++) {
          int x = decision(s, p);
          if (x && d && x != d) return PV_FALSE;
          if (x) d = x;
        }
        return PV_TRUE;
      }
      case DSL_PRED_SIP_INTEGRITY:
        for (int p = 0; p < prm.proposers; p++) {
          int x = decision(s, p);
          if (x && (x < 1 || x > prm.proposers)) return PV_FALSE;
        }
        return PV_TRUE;
      case DSL_PRED_SIP_TERMINATION:
        for (int p = 0; p < prm.proposers; p++)
          if (!decision(s, p)) return PV_FALSE;
        return PV_TRUE;
      default:
        return PV_THREW;
    }
  }

  static bool known_predicate(int id) { return id >= DSL_PRED_SIP_AGREEMENT && id <= DSL_PRED_SIP_TERMINATION; }
  static int num_nodes(const Params& p) { return p.proposers + p.acceptors; }
  static bool valid(const Params& p) {
    return p.proposers >= 1 && p.proposers <= kMaxP && p.acceptors >= 1 && p.acceptors <= kMaxA;
  }
  static Params from_desc(const dsl_protocol_desc& d) {
    Params p{};
    p.proposers = (int32_t)d.params[0];
    p.acceptors = (int32_t)d.params[1];
    p.incorrect = d.n_params > 2 ? (int32_t)d.params[2] : 0;
    return p;
  }
  static void describe(const State& s, const Params& prm, const DevSettings& set, int k, dsl_event* e) {
    *e = dsl_event{};
    const int64_t x = locate(s, prm, set, k);
    if (x < 0) {
      e->is_timer = 1;
      e->from = e->to = (int)(-1 - x);
      e->type = T_PROPOSE_TIMER;
      e->timer_min = e->timer_max = 100;
      return;
    }
    const uint32_t m = (uint32_t)x;
    e->from = r_from(m);
    e->to = r_to(m);
    e->type = r_type(m);
    e->n_fields = 3;
    e->fields[0] = r_n(m);
    e->fields[1] = r_an(m);
    e->fields[2] = r_av(m);
  }
};

}  // namespace dsl
