// minitest.hpp -- the two-node fixture of the reference's trace-minimizer tests
// (framework/tst-self/dslabs/framework/testing/search/SearchAndTraceMinimizerTest.java:430-471:
// nodes A and B, messages Foo and Bar; predicates foo / fooException :104-126 and
// alwaysException :255-260). It pins dsl_replay's minimization to the reference's own
// known answers; object-style in oracle/proto_minitest.hpp.
//
// Nodes: 0 = "a", 1 = "b". Node word of a: bit 0 = foo. b has no fields.
// A.init sends Foo to b (twice: one envelope, the network is a set). B on Foo: send Foo and Bar
// back. A on Foo: throws. A on Bar: foo = true.
// Records (32 bit): type:1 @30 (0 Foo, 1 Bar) | from:1 @29 | to:1 @28 | marker bit 0.
#pragma once
#include "../nodestate.hpp"

namespace dsl {

struct MiniTest {
  static constexpr int kNodes = 2, kNodeWords = 1, kNetCap = 4, kMaxSends = 2;
  static constexpr int kMsgClasses = 2;  // handler classes of messages (Foo, Bar); timers: class 2
  using Rec = uint32_t;
  using State = StateOf<MiniTest>;

  struct Params {
    int32_t pad;
  };
  enum { M_FOO = 0, M_BAR = 1 };

  static DSL_HD Rec rec(int type, int from, int to) {
    return ((Rec)type << 30) | ((Rec)from << 29) | ((Rec)to << 28) | 1u;
  }
  static DSL_HD int rec_type(Rec r) { return (int)((r >> 30) & 1); }
  static DSL_HD int rec_from(Rec r) { return (int)((r >> 29) & 1); }
  static DSL_HD int rec_to(Rec r) { return (int)((r >> 28) & 1); }
  static DSL_HD int msg_class(Rec r) { return rec_type(r); }

  static DSL_HD int num_nodes(const Params&) { return 2; }
  template <class O>
  static DSL_HD void init_node(int i, uint32_t* w, O& out, const Params&) {
    w[0] = 0;
    if (i == 0) {  // A.init: send(new Foo(), b) twice
      out.send(rec(M_FOO, 0, 1));
      out.send(rec(M_FOO, 0, 1));
    }
  }
  static DSL_HD int num_timer_events(int, const uint32_t*, const Params&) { return 0; }
  template <class O>
  static DSL_HD int on_timer(int, uint32_t*, int, O&, const Params&) { return STEP_EXCEPTION; }

  template <class O>
  static DSL_HD int on_message(int i, uint32_t* w, Rec m, O& out, const Params&) {
    if (i == 0) {
      if (rec_type(m) == M_FOO) return STEP_EXCEPTION;  // A.handleFoo: throw new RuntimeException()
      w[0] = 1;                                         // A.handleBar: foo = true
      return STEP_OK;
    }
    if (rec_type(m) != M_FOO) return STEP_EXCEPTION;  // B has no Bar handler
    out.send(rec(M_FOO, 1, rec_from(m)));            // B.handleFoo: send(foo, sender)
    out.send(rec(M_BAR, 1, rec_from(m)));            //              send(new Bar(), sender)
    return STEP_OK;
  }

  static DSL_HD int eval(const DevPred& pr, const NodeView& v, const Params&) {
    const bool foo = v.node(0)[0] & 1u;
    switch (pr.id) {
      case DSL_PRED_MINI_FOO:
        return foo ? PV_FALSE : PV_TRUE;
      case DSL_PRED_MINI_FOO_EXCEPTION:
        return foo ? PV_THREW : PV_TRUE;
      default:  // DSL_PRED_MINI_ALWAYS_EXCEPTION
        return PV_THREW;
    }
  }
  static uint32_t pred_reads(const DevPred& pr, const Params&) {
    return pr.id == DSL_PRED_MINI_ALWAYS_EXCEPTION ? kReadsAll : 1u;
  }
  static bool known_predicate(int id) { return id >= DSL_PRED_MINI_FOO && id <= DSL_PRED_MINI_ALWAYS_EXCEPTION; }
  static bool valid(const Params&) { return true; }
  static Params from_desc(const dsl_protocol_desc&) { return Params{}; }
  static void describe_message(Rec r, dsl_event* e) {
    e->from = rec_from(r);
    e->to = rec_to(r);
    e->type = rec_type(r);
    e->n_fields = 0;
  }
  static void describe_timer(int i, const uint32_t*, int, const Params&, dsl_event* e) {
    e->is_timer = 1;
    e->from = e->to = i;
  }
};

}  // namespace dsl
