// sipaxos.hpp -- the reference's single-instance "Paxos Made Simple" as node-local device handlers.
//
// Re-expresses framework/tst/dslabs/framework/testing/visualization/examples/paxosmadesimple/
// SingleInstancePaxos.java:177-293 (Proposer.onPropose / handlePrepareAck / handleAcceptAck,
// Acceptor.handlePrepare / handleAccept), :296-323 (messages, Propose timer = 100 ms) and the
// BadProposer of IncorrectSingleInstancePaxos.java:42-64 (decides once acceptAcks * 2 >=
// acceptors - 1, i.e. without a majority).
//
// Nodes: proposers 0..P-1 ("proposer1.."), acceptors P..P+A-1 ("acceptor1..").
// Proposal values are interned: value id v in 1..P = the initial proposal of proposer v.
// Node words (3):
//   proposer: w0 = hasProposed:1 | prepareFinished:1 | value:2 @2 | decision:2 @4 (0 = null) |
//                  acceptAcks:5 @6 (bit a) | proposalNumber:8 @16
//             w1,w2 = prepareAcks[a], 11 bits each at bit 11a of the 64-bit pair:
//                  present:1 | accepted.n:8 (0 = null) | accepted.v:2  (the ack's proposal number
//                  always equals the proposer's, so it is implied)
//   acceptor: w0 = highestPrepared:8 (0 = null) | accepted.n:8 @8 | accepted.v:2 @16
// The Propose queue of a proposer is always exactly [Propose(100 ms)] (onPropose re-sets it and
// stepTimer removes the first equal entry, SearchState.java:357), so it is not stored.
// Records (32 bit): type:2 @30 | from:3 @27 | to:3 @24 | n:8 @16 | an:8 @8 | av:2
//   0 Prepare(n), 1 PrepareAck(n, (an, av) | null), 2 Accept(n, av), 3 AcceptAck(n)
#pragma once
#include "../nodestate.hpp"

namespace dsl {

struct SIPaxos {
  static constexpr int kMaxP = 3, kMaxA = 5;
  static constexpr int kNodes = kMaxP + kMaxA, kNodeWords = 3, kNetCap = 48, kMaxSends = kMaxA;
  static constexpr int kMsgClasses = 4;  // handler classes of messages (message types 0..3); timers: class 4
  using Rec = uint32_t;
  using State = StateOf<SIPaxos>;

  struct Params {
    int32_t proposers, acceptors, incorrect;
  };
  enum { T_PREPARE = 0, T_PREPARE_ACK = 1, T_ACCEPT = 2, T_ACCEPT_ACK = 3, T_PROPOSE_TIMER = 4 };

  static DSL_HD Rec rec(int type, int from, int to, int n, int an, int av) {
    return ((Rec)type << 30) | ((Rec)from << 27) | ((Rec)to << 24) | ((Rec)n << 16) | ((Rec)an << 8) | (Rec)av;
  }
  static DSL_HD int r_type(Rec r) { return r >> 30; }
  static DSL_HD int rec_from(Rec r) { return (r >> 27) & 7; }
  static DSL_HD int rec_to(Rec r) { return (r >> 24) & 7; }
  static DSL_HD int r_n(Rec r) { return (r >> 16) & 0xff; }
  static DSL_HD int r_an(Rec r) { return (r >> 8) & 0xff; }
  static DSL_HD int r_av(Rec r) { return r & 3; }

  // Handler class of a message (< kMsgClasses; timers are class kMsgClasses): k_level groups a chunk's work items
  // by class so that the lanes of a wavefront run the same handler.
  static DSL_HD int msg_class(Rec r) { return r_type(r); }
  static DSL_HD int get(const uint32_t* w, int bit, int width) { return field_get<kNodeWords>(w, bit, width); }
  static DSL_HD void put(uint32_t* w, int bit, int width, int v) { field_put<kNodeWords>(w, bit, width, v); }
  // proposer fields
  static DSL_HD int has_proposed(const uint32_t* w) { return get(w, 0, 1); }
  static DSL_HD int prep_fin(const uint32_t* w) { return get(w, 1, 1); }
  static DSL_HD int value(const uint32_t* w) { return get(w, 2, 2); }
  static DSL_HD int decision(const uint32_t* w) { return get(w, 4, 2); }
  static DSL_HD int accept_acks(const uint32_t* w) { return get(w, 6, 5); }
  static DSL_HD int pnum(const uint32_t* w) { return get(w, 16, 8); }
  static DSL_HD uint64_t acks64(const uint32_t* w) { return (uint64_t)w[1] | ((uint64_t)w[2] << 32); }
  static DSL_HD void set_acks64(uint32_t* w, uint64_t v) {
    w[1] = (uint32_t)v;
    w[2] = (uint32_t)(v >> 32);
  }

  template <class O>
  static DSL_HD void broadcast(int from, const Params& p, Rec proto, O& out) {
    for (int a = 0; a < p.acceptors; a++) out.send((proto & ~(Rec)(0x3f << 24)) | ((Rec)from << 27) | ((Rec)(p.proposers + a) << 24));
  }

  static DSL_HD int num_nodes(const Params& p) { return p.proposers + p.acceptors; }
  template <class O>
  static DSL_HD void init_node(int i, uint32_t* w, O&, const Params& p) {
    if (i < p.proposers) {
      put(w, 2, 2, i + 1);   // proposalValue = values[i]
      put(w, 16, 8, i + 1);  // proposalNumber = i + 1; init(): set(Propose, 100) (constant queue)
    }
  }
  static DSL_HD int num_timer_events(int i, const uint32_t*, const Params& p) { return i < p.proposers; }

  // Proposer.onPropose (the Propose queue stays [Propose]).
  template <class O>
  static DSL_HD int on_timer(int i, uint32_t* w, int, O& out, const Params& p) {
    int n = pnum(w);
    if (has_proposed(w)) n += p.proposers;
    if (n > 255) return STEP_OVERFLOW;
    put(w, 16, 8, n);
    put(w, 0, 1, 1);
    set_acks64(w, 0);  // prepareAcks.clear()
    put(w, 6, 5, 0);   // acceptAcks.clear()
    put(w, 1, 1, 0);   // prepareFinished = false
    broadcast(i, p, rec(T_PREPARE, 0, 0, n, 0, 0), out);
    return STEP_OK;
  }

  template <class O>
  static DSL_HD int on_message(int i, uint32_t* w, Rec m, O& out, const Params& p) {
    const int from = rec_from(m);
    switch (r_type(m)) {
      case T_PREPARE: {  // Acceptor.handlePrepare
        const int hp = get(w, 0, 8);
        if (hp != 0 && hp >= r_n(m)) return STEP_OK;
        put(w, 0, 8, r_n(m));
        out.send(rec(T_PREPARE_ACK, i, from, r_n(m), get(w, 8, 8), get(w, 16, 2)));
        return STEP_OK;
      }
      case T_PREPARE_ACK: {  // Proposer.handlePrepareAck
        const int n = pnum(w), a = from - p.proposers;
        if (r_n(m) != n || prep_fin(w)) return STEP_OK;
        uint64_t acks = acks64(w);
        acks &= ~((uint64_t)0x7ff << (11 * a));
        acks |= ((uint64_t)(1 | (r_an(m) << 1) | (r_av(m) << 9))) << (11 * a);
        int count = 0;
        for (int k = 0; k < p.acceptors; k++) count += (acks >> (11 * k)) & 1;
        if (count * 2 > p.acceptors) {
          put(w, 1, 1, 1);
          int best_n = 0, best_v = 0;  // value of the highest accepted ballot among the acks
          for (int k = 0; k < p.acceptors; k++) {
            uint32_t e = (uint32_t)(acks >> (11 * k)) & 0x7ff;
            if (!(e & 1)) continue;
            int an = (e >> 1) & 0xff, av = (e >> 9) & 3;
            if (an != 0 && an >= best_n) best_n = an, best_v = av;
          }
          if (best_n != 0) put(w, 2, 2, best_v);
          set_acks64(w, 0);  // prepareAcks.clear()
          broadcast(i, p, rec(T_ACCEPT, 0, 0, n, 0, value(w)), out);
          return STEP_OK;
        }
        set_acks64(w, acks);
        return STEP_OK;
      }
      case T_ACCEPT: {  // Acceptor.handleAccept
        const int hp = get(w, 0, 8);
        if (hp != 0 && hp > r_n(m)) return STEP_OK;
        out.send(rec(T_ACCEPT_ACK, i, from, r_n(m), 0, 0));
        const int han = get(w, 8, 8);
        if (han == 0 || han < r_n(m)) {
          put(w, 8, 8, r_n(m));
          put(w, 16, 2, r_av(m));
        }
        return STEP_OK;
      }
      default: {  // Proposer.handleAcceptAck (BadProposer: acks * 2 >= acceptors - 1)
        if (pnum(w) != r_n(m)) return STEP_OK;
        const int acks = accept_acks(w) | (1 << (from - p.proposers));
        put(w, 6, 5, acks);
        const int acks2 = __builtin_popcount(acks) * 2;
        if (p.incorrect ? acks2 >= p.acceptors - 1 : acks2 > p.acceptors) put(w, 4, 2, value(w));
        return STEP_OK;
      }
    }
  }

  static DSL_HD int eval(const DevPred& pr, const NodeView& v, const Params& p) {
    switch (pr.id) {
      case DSL_PRED_SIP_AGREEMENT: {
        int d = 0;
        for (int i = 0; i < p.proposers; i++) {
          int x = decision(v.node(i));
          if (x && d && x != d) return PV_FALSE;
          if (x) d = x;
        }
        return PV_TRUE;
      }
      case DSL_PRED_SIP_INTEGRITY:
        for (int i = 0; i < p.proposers; i++) {
          int x = decision(v.node(i));
          if (x && (x < 1 || x > p.proposers)) return PV_FALSE;
        }
        return PV_TRUE;
      case DSL_PRED_SIP_TERMINATION:
        for (int i = 0; i < p.proposers; i++)
          if (!decision(v.node(i))) return PV_FALSE;
        return PV_TRUE;
      default:
        return PV_THREW;
    }
  }

  // Read sets (judge_view's incremental check): the predicates read proposer nodes only.
  static uint32_t pred_reads(const DevPred& pr, const Params& p) {
    return (pr.id >= DSL_PRED_SIP_AGREEMENT && pr.id <= DSL_PRED_SIP_TERMINATION) ? ((1u << p.proposers) - 1u)
                                                                                   : kReadsAll;
  }
  static bool known_predicate(int id) { return id >= DSL_PRED_SIP_AGREEMENT && id <= DSL_PRED_SIP_TERMINATION; }
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
  static void describe_message(Rec m, dsl_event* e) {
    e->from = rec_from(m);
    e->to = rec_to(m);
    e->type = r_type(m);
    e->n_fields = 3;
    e->fields[0] = r_n(m);
    e->fields[1] = r_an(m);
    e->fields[2] = r_av(m);
  }
  static void describe_timer(int i, const uint32_t*, int, const Params&, dsl_event* e) {
    e->is_timer = 1;
    e->from = e->to = i;
    e->type = T_PROPOSE_TIMER;
    e->timer_min = e->timer_max = 100;
  }
};

}  // namespace dsl
