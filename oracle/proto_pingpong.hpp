// oracle/proto_pingpong.hpp -- TEST INFRASTRUCTURE ONLY (see oracle_core.hpp).
// Restates lab0 PingPong: labs/lab0-pingpong/src/dslabs/pingpong/PingServer.java:29-32,
// PingClient.java:41-87, Timers.java:7-11 (PingTimer, RETRY_MILLIS = 10),
// PingApplication.java (Pong = Ping value), and the test workload
// labs/lab0-pingpong/tst/dslabs/pingpong/PingTest.java:44-51 (repeatedPings: "ping-%i" x n).
// Mutants restate the README's "When Things Go Wrong" edits
// (labs/lab0-pingpong/README.md:299-306 no timer re-set, :342-347 no pong-value check).
#pragma once
#include "oracle_core.hpp"

namespace oracle {
namespace pingpong {

constexpr int RETRY_MILLIS = 10;

struct PingServer : Node {
  std::shared_ptr<Node> clone() const override { return std::make_shared<PingServer>(*this); }
  void key(std::string& out) const override { out += "PingServer{}"; }  // app has no fields
  std::string str() const override { return "PingServer()"; }
  void handleMessage(const Rec& m, int from, int, Ctx& ctx) override {
    if (m.type != "PingRequest") throw HandlerException("no handler");
    ctx.send(Rec{"PongReply", {m.f[0]}}, from);  // Pong(p.value()) back to the sender
  }
  void onTimer(const Rec&, Ctx&) override { throw HandlerException("no timer handler"); }
};

struct PingClient : Client {
  int server = 0;
  bool checkValue = true;  // false = README mutant :342-347
  bool resetTimer = true;  // false = README mutant :299-306
  std::optional<std::string> ping, pong;

  std::shared_ptr<Node> clone() const override { return std::make_shared<PingClient>(*this); }
  void key(std::string& out) const override {
    out += "PingClient{ping=" + (ping ? *ping : "null") + ",pong=" + (pong ? *pong : "null") + "}";
  }
  std::string str() const override {
    return "PingClient(ping=" + (ping ? "Ping(" + *ping + ")" : "null") +
           ", pong=" + (pong ? "Pong(" + *pong + ")" : "null") + ")";
  }
  void sendCommand(const Rec& cmd, Ctx& ctx) override {
    ping = cmd.f[0];
    pong.reset();
    ctx.send(Rec{"PingRequest", {*ping}}, server);
    ctx.set(Rec{"PingTimer", {*ping}}, RETRY_MILLIS);
  }
  bool hasResult() const override { return pong.has_value(); }
  Rec getResult() const override { return Rec{"Pong", {*pong}}; }
  void handleMessage(const Rec& m, int, int, Ctx&) override {
    if (m.type != "PongReply") throw HandlerException("no handler");
    if (!checkValue || (ping && *ping == m.f[0])) pong = m.f[0];
  }
  void onTimer(const Rec& t, Ctx& ctx) override {
    if (t.type != "PingTimer") throw HandlerException("no timer handler");
    if (ping && *ping == t.f[0] && !pong) {
      ctx.send(Rec{"PingRequest", {*ping}}, server);
      if (resetTimer) ctx.set(t, RETRY_MILLIS);
    }
  }
};

// Address 0 = "pingserver", 1..n = "client1".."clientN".
inline std::shared_ptr<State> initial(int clients, int pings, bool checkValue, bool resetTimer, Names& names) {
  std::vector<std::shared_ptr<Node>> nodes;
  std::vector<Kind> kinds;
  names.addr = {"pingserver"};
  nodes.push_back(std::make_shared<PingServer>());
  kinds.push_back(Kind::Server);
  for (int c = 1; c <= clients; c++) {
    names.addr.push_back("client" + std::to_string(c));
    auto pc = std::make_shared<PingClient>();
    pc->checkValue = checkValue;
    pc->resetTimer = resetTimer;
    auto cw = std::make_shared<ClientWorker>();
    cw->client = pc;
    cw->addrName = names.addr.back();
    cw->workload.cmds = {"ping-%i"};
    cw->workload.results = {"ping-%i"};
    cw->workload.numTimes = pings;
    cw->workload.parser = [](const std::string& c, const std::string& r) {
      return std::make_pair(Rec{"Ping", {c}}, Rec{"Pong", {r}});
    };
    nodes.push_back(cw);
    kinds.push_back(Kind::ClientWorker);
  }
  return makeInitial(nodes, kinds);
}

}  // namespace pingpong
}  // namespace oracle
