// oracle/proto_sipaxos.hpp -- TEST INFRASTRUCTURE ONLY (see oracle_core.hpp).
// Restates the reference's only complete Paxos, "Paxos Made Simple" single-instance Paxos:
// framework/tst/dslabs/framework/testing/visualization/examples/paxosmadesimple/
//   SingleInstancePaxos.java:50-127 (initial state: proposers "proposer1..", acceptors
//   "acceptor1.."; invariants Integrity/Agreement, goal Termination), :177-293 (Proposer /
//   Acceptor handlers), :296-323 (messages, Propose timer).
//   IncorrectSingleInstancePaxos.java:29-64 (BadProposer.handleAcceptAck, :54-63: decides once
//   acceptAcks.size() * 2 >= acceptors.length - 1, i.e. without a majority).
// Lombok equality: Proposer includes hasProposed, numProposers, acceptors, proposalValue,
// proposalNumber, prepareFinished, prepareAcks (map), acceptAcks (set), decision.
#pragma once
#include "oracle_core.hpp"

namespace oracle {
namespace sipaxos {

// PrepareAck.accepted is Pair<Integer,String> or null -> encoded as "null" or "n:v".
struct Proposer : Node {
  std::vector<int> acceptors;
  bool hasProposed = false;
  int numProposers = 0;
  std::string proposalValue;
  int proposalNumber = 0;
  bool prepareFinished = false;
  std::map<int, Rec> prepareAcks;  // sender -> PrepareAck
  std::set<int> acceptAcks;
  std::optional<std::string> decision;
  bool incorrect = false;  // IncorrectSingleInstancePaxos BadProposer

  std::shared_ptr<Node> clone() const override { return std::make_shared<Proposer>(*this); }
  void key(std::string& out) const override {
    out += "P{" + std::to_string(hasProposed) + "," + proposalValue + "," + std::to_string(proposalNumber) +
           "," + std::to_string(prepareFinished) + ",PA[";
    for (auto& kv : prepareAcks) out += std::to_string(kv.first) + "=" + kv.second.str() + ",";
    out += "],AA[";
    for (int a : acceptAcks) out += std::to_string(a) + ",";
    out += "]," + (decision ? *decision : std::string("null")) + "}";
  }
  std::string str() const override {
    return "Proposer(proposalValue=" + proposalValue + ", proposalNumber=" + std::to_string(proposalNumber) +
           ", decision=" + (decision ? *decision : "null") + ")";
  }
  void init(Ctx& ctx) override { ctx.set(Rec{"Propose", {}}, 100); }
  void onTimer(const Rec& t, Ctx& ctx) override {
    if (hasProposed) proposalNumber += numProposers;
    hasProposed = true;
    prepareAcks.clear();
    acceptAcks.clear();
    prepareFinished = false;
    ctx.broadcast(Rec{"Prepare", {std::to_string(proposalNumber)}}, acceptors);
    ctx.set(t, 100);
  }
  void handleMessage(const Rec& m, int from, int, Ctx& ctx) override {
    if (m.type == "PrepareAck") {
      int n = std::stoi(m.f[0]);
      if (n != proposalNumber || prepareFinished) return;
      prepareAcks[from] = m;
      if (prepareAcks.size() * 2 > acceptors.size()) {
        prepareFinished = true;
        // reduce((p1,p2) -> p1.accepted.left > p2.accepted.left ? p1 : p2) over non-null
        // accepted values, in HashMap value order; ties on ballot keep the later element.
        // Accepted values with equal ballots carry the same value in this protocol, so the
        // iteration order does not change the chosen value.
        const Rec* best = nullptr;
        int bestN = 0;
        for (auto& kv : prepareAcks) {
          if (kv.second.f[1] == "null") continue;
          int an = std::stoi(kv.second.f[1]);
          if (!best || !(bestN > an)) {
            best = &kv.second;
            bestN = an;
          }
        }
        if (best) proposalValue = best->f[2];
        prepareAcks.clear();
        ctx.broadcast(Rec{"Accept", {std::to_string(proposalNumber), proposalValue}}, acceptors);
      }
    } else if (m.type == "AcceptAck") {
      int n = std::stoi(m.f[0]);
      if (proposalNumber != n) return;
      acceptAcks.insert(from);
      const size_t acks2 = acceptAcks.size() * 2;
      if (incorrect ? acks2 + 1 >= acceptors.size() : acks2 > acceptors.size()) decision = proposalValue;
    } else {
      throw HandlerException("no handler");
    }
  }
};

struct Acceptor : Node {
  std::optional<int> highestPrepared;
  std::optional<std::pair<int, std::string>> highestAccepted;

  std::shared_ptr<Node> clone() const override { return std::make_shared<Acceptor>(*this); }
  void key(std::string& out) const override {
    out += "A{" + (highestPrepared ? std::to_string(*highestPrepared) : "null") + "," +
           (highestAccepted ? std::to_string(highestAccepted->first) + ":" + highestAccepted->second : "null") +
           "}";
  }
  std::string str() const override { return "Acceptor()"; }
  void onTimer(const Rec&, Ctx&) override { throw HandlerException("no timer handler"); }
  void handleMessage(const Rec& m, int from, int, Ctx& ctx) override {
    int n = std::stoi(m.f[0]);
    if (m.type == "Prepare") {
      if (highestPrepared && *highestPrepared >= n) return;
      highestPrepared = n;
      Rec ack{"PrepareAck", {std::to_string(n), "null", ""}};
      if (highestAccepted) ack.f = {std::to_string(n), std::to_string(highestAccepted->first), highestAccepted->second};
      ctx.send(ack, from);
    } else if (m.type == "Accept") {
      if (highestPrepared && *highestPrepared > n) return;
      ctx.send(Rec{"AcceptAck", {std::to_string(n)}}, from);
      if (!highestAccepted || highestAccepted->first < n) highestAccepted = std::make_pair(n, m.f[1]);
    } else {
      throw HandlerException("no handler");
    }
  }
};

// Addresses: proposers 0..P-1 ("proposer1".."), acceptors P..P+A-1 ("acceptor1..").
inline std::shared_ptr<State> initial(int P, int A, const std::vector<std::string>& values, bool incorrect,
                                      Names& names) {
  std::vector<std::shared_ptr<Node>> nodes;
  std::vector<Kind> kinds;
  std::vector<int> acc;
  for (int a = 0; a < A; a++) acc.push_back(P + a);
  for (int p = 0; p < P; p++) {
    names.addr.push_back("proposer" + std::to_string(p + 1));
    auto n = std::make_shared<Proposer>();
    n->acceptors = acc;
    n->numProposers = P;
    n->proposalNumber = p + 1;
    n->proposalValue = values[p];
    n->incorrect = incorrect;
    nodes.push_back(n);
    kinds.push_back(Kind::Server);
  }
  for (int a = 0; a < A; a++) {
    names.addr.push_back("acceptor" + std::to_string(a + 1));
    auto n = std::make_shared<Acceptor>();
    nodes.push_back(n);
    kinds.push_back(Kind::Server);
  }
  return makeInitial(nodes, kinds);
}

inline Predicate agreement(int P) {
  return {"Agreement", [P](const State& s) {
            PredResult r;
            std::optional<std::string> decided;
            for (int p = 0; p < P; p++) {
              auto* n = dynamic_cast<const Proposer*>(s.nodes[p].get());
              if (n->decision && decided && *n->decision != *decided) r.value = false;
              if (n->decision) decided = n->decision;
            }
            return r;
          }};
}
inline Predicate integrity(int P, std::vector<std::string> values) {
  return {"Integrity", [P, values](const State& s) {
            PredResult r;
            for (int p = 0; p < P; p++) {
              auto* n = dynamic_cast<const Proposer*>(s.nodes[p].get());
              if (n->decision && std::find(values.begin(), values.end(), *n->decision) == values.end())
                r.value = false;
            }
            return r;
          }};
}
inline Predicate termination(int P) {
  return {"Termination", [P](const State& s) {
            PredResult r;
            for (int p = 0; p < P; p++)
              if (!dynamic_cast<const Proposer*>(s.nodes[p].get())->decision) r.value = false;
            return r;
          }};
}

}  // namespace sipaxos
}  // namespace oracle
