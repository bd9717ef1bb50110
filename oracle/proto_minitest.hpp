// oracle/proto_minitest.hpp -- TEST INFRASTRUCTURE ONLY (see oracle_core.hpp).
// Restates the two-node fixture of the reference's minimizer tests
// (framework/tst-self/dslabs/framework/testing/search/SearchAndTraceMinimizerTest.java:55-67,
// :104-126 predicates foo / fooException, :255-260 alwaysException, :430-471 nodes A and B,
// messages Foo and Bar): A sends Foo to B twice at init (one envelope: the network is a set);
// B answers a Foo with Foo and Bar; A throws on Foo and sets foo on Bar.
#pragma once
#include "oracle_core.hpp"

namespace oracle {
namespace minitest {

struct A : Node {
  bool foo = false;
  std::shared_ptr<Node> clone() const override { return std::make_shared<A>(*this); }
  void key(std::string& out) const override { out += foo ? "A{foo=true}" : "A{foo=false}"; }
  std::string str() const override { return foo ? "A(foo=true)" : "A(foo=false)"; }
  void init(Ctx& ctx) override {
    ctx.send(Rec{"Foo", {}}, 1);
    ctx.send(Rec{"Foo", {}}, 1);
  }
  void handleMessage(const Rec& m, int, int, Ctx&) override {
    if (m.type == "Foo") throw HandlerException("RuntimeException");  // A.handleFoo
    if (m.type != "Bar") throw HandlerException("no handler");
    foo = true;  // A.handleBar
  }
  void onTimer(const Rec&, Ctx&) override { throw HandlerException("no timer handler"); }
};

struct B : Node {
  std::shared_ptr<Node> clone() const override { return std::make_shared<B>(*this); }
  void key(std::string& out) const override { out += "B{}"; }
  std::string str() const override { return "B()"; }
  void handleMessage(const Rec& m, int from, int, Ctx& ctx) override {
    if (m.type != "Foo") throw HandlerException("no handler");
    ctx.send(m, from);  // B.handleFoo: send(foo, sender); send(new Bar(), sender)
    ctx.send(Rec{"Bar", {}}, from);
  }
  void onTimer(const Rec&, Ctx&) override { throw HandlerException("no timer handler"); }
};

// Address 0 = "a", 1 = "b" (both servers, added in that order: setupSearchTest :66-71).
inline std::shared_ptr<State> initial(Names& names) {
  names.addr = {"a", "b"};
  return makeInitial({std::make_shared<A>(), std::make_shared<B>()}, {Kind::Server, Kind::Server});
}

inline Predicate foo() {  // value = !a.foo
  return Predicate{"foo", [](const State& s) {
                     PredResult r;
                     r.value = !dynamic_cast<const A&>(*s.nodes[0]).foo;
                     r.detail = r.value ? "1234" : "asdf";
                     return r;
                   }};
}
inline Predicate fooException() {  // throws when a.foo
  return Predicate{"fooException", [](const State& s) {
                     if (dynamic_cast<const A&>(*s.nodes[0]).foo) throw std::runtime_error("RuntimeException");
                     PredResult r;
                     r.detail = "1234";
                     return r;
                   }};
}
inline Predicate alwaysException() {
  return Predicate{"alwaysException", [](const State&) -> PredResult { throw std::runtime_error("RuntimeException"); }};
}

}  // namespace minitest
}  // namespace oracle
