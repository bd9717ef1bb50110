// oracle/proto_synthetic.hpp -- TEST INFRASTRUCTURE ONLY (see oracle_core.hpp).
//
// The synthetic table-driven protocol of BASELINE config C3 (builder-defined: the reference has no
// analogue; DESIGN.md §10 is the specification shared with the packed device form in
// dslabs_amd/csrc/protocols/synthetic.hpp). Written object-style on the oracle's Node / Ctx /
// TimerQueue model, like any DSLabs node: fields v and pokes, timers set with ctx.set, pokes sent
// with ctx.send; queue order, removal of the fired timer and the network set are the framework's
// (SearchState.stepTimer / stepMessage semantics restated in oracle_core.hpp).
#pragma once
#include <cstdint>

#include "oracle_core.hpp"

namespace oracle {
namespace synthetic {

constexpr int kTimerMin = 1, kTimerMax = 100;

struct Table {  // the seeded transition function
  int nodes = 5, K = 64, P = 7;
  uint64_t seed = 0x5EEDD51AB5ull;
  static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  int mix(int i, int t, int v) const {
    return (int)(splitmix64(seed ^ ((uint64_t)i << 48) ^ ((uint64_t)t << 40) ^ (uint64_t)v) % (uint64_t)K);
  }
};

struct SynthNode : Node {
  int self = 0;
  Table tab;
  int v = 0, pokes = 0;
  std::shared_ptr<Node> clone() const override { return std::make_shared<SynthNode>(*this); }
  void key(std::string& out) const override {
    out += "SynthNode{v=" + std::to_string(v) + ",pokes=" + std::to_string(pokes) + "}";
  }
  std::string str() const override { return "SynthNode(v=" + std::to_string(v) + ", pokes=" + std::to_string(pokes) + ")"; }
  void init(Ctx& ctx) override {
    for (int t = 0; t < 4; t++) ctx.set(Rec{"SynthTimer", {std::to_string(t)}}, kTimerMin, kTimerMax);
  }
  void onTimer(const Rec& tm, Ctx& ctx) override {
    if (tm.type != "SynthTimer") throw HandlerException("no timer handler");
    const int t = std::stoi(tm.f[0]);
    v = tab.mix(self, t, v);
    if (v % tab.P == 0) ctx.send(Rec{"Poke", {}}, (self + 1) % tab.nodes);
    ctx.set(tm, kTimerMin, kTimerMax);
  }
  void handleMessage(const Rec& m, int, int, Ctx&) override {
    if (m.type != "Poke") throw HandlerException("no handler");
    pokes = (pokes + 1) % 4;
    v = tab.mix(self, 4 + pokes, v);
  }
};

inline std::shared_ptr<State> initial(const Table& tab, Names& names) {
  std::vector<std::shared_ptr<Node>> nodes;
  std::vector<Kind> kinds;
  for (int i = 0; i < tab.nodes; i++) {
    names.addr.push_back("node" + std::to_string(i + 1));
    auto n = std::make_shared<SynthNode>();
    n->self = i;
    n->tab = tab;
    nodes.push_back(n);
    kinds.push_back(Kind::Server);
  }
  return makeInitial(nodes, kinds);
}

inline Predicate notAllMax(const Table& tab) {
  return {"NOT_ALL_MAX", [tab](const State& s) {
            PredResult r;
            r.value = false;
            for (int i = 0; i < tab.nodes; i++)
              if (dynamic_cast<const SynthNode*>(s.nodes[i].get())->v != tab.K - 1) r.value = true;
            return r;
          }};
}
inline Predicate counterLt(int node, int bound) {
  return {"COUNTER_LT:" + std::to_string(node) + ":" + std::to_string(bound), [node, bound](const State& s) {
            PredResult r;
            r.value = dynamic_cast<const SynthNode*>(s.nodes[node].get())->v < bound;
            return r;
          }};
}

}  // namespace synthetic
}  // namespace oracle
