// oracle/proto_amokv.hpp -- TEST INFRASTRUCTURE ONLY (see oracle_core.hpp).
//
// lab1 at-most-once client/server KV store (BASELINE config C2). The reference ships the classes
// as stubs (labs/lab1-clientserver/src/dslabs/clientserver/SimpleClient.java, SimpleServer.java,
// Messages.java, Timers.java; atmostonce/AMOApplication.java, AMOCommand.java, AMOResult.java;
// kvstore/KVStore.java); this is the builder-authored solution specified in DESIGN.md §11, written
// object-style on the oracle's Node model. The KVStore semantics (Get / Put / Append and their
// results) and the workloads follow labs/lab1-clientserver/tst/dslabs/kvstore/KVStoreWorkload.java
// (:40-66 constructors, :76-133 parse, :202-216 appendDifferentKeyWorkload, :282-340
// APPENDS_LINEARIZABLE) and ClientServerPart2Test.java:221-263 (test09 / test10).
//
//   SimpleClient: seq++, pending = AMOCommand(cmd, seq), send Request(cmd, seq) to the server,
//     set ClientTimer(seq) 100 ms; Reply(result, seq) for the pending seq stores the result;
//     ClientTimer(seq) for the pending seq without a result re-sends and re-sets.
//   SimpleServer(AMOApplication(KVStore)): Request(cmd, seq) from c: seq < last[c] -> ignored;
//     seq == last[c] -> the cached result again; else execute, cache, reply Reply(result, seq).
#pragma once
#include "oracle_core.hpp"

namespace oracle {
namespace amokv {

constexpr int CLIENT_RETRY_MILLIS = 100;

struct Config {
  int clients = 2;
  std::vector<std::string> cmds, results;  // workload templates (%a = address, %i = 1-based index)
  int numTimes = 1;
  static Config fromArgs(int clients, const std::string& workload) {
    Config c;
    c.clients = clients;
    if (workload == "diffkey3") {  // appendDifferentKeyWorkload(3) (test09)
      c.cmds = {"APPEND:KEY-%a:0", "APPEND:KEY-%a:1", "APPEND:KEY-%a:2"};
      c.results = {"0", "01", "012"};
    } else if (workload == "diffkey2") {
      c.cmds = {"APPEND:KEY-%a:0", "APPEND:KEY-%a:1"};
      c.results = {"0", "01"};
    } else if (workload == "samekey3") {  // APPEND:foo:%i x 3 (test10)
      c.cmds = {"APPEND:foo:%i"};
      c.numTimes = 3;
    } else if (workload == "samekey2") {
      c.cmds = {"APPEND:foo:%i"};
      c.numTimes = 2;
    } else if (workload == "appendappendget") {  // KVStoreWorkload.appendAppendGet (test08)
      c.cmds = {"APPEND:foo:bar", "APPEND:foo:bar", "GET:foo"};
      c.results = {"bar", "barbar", "barbar"};
    } else if (workload == "putappendget") {  // KVStoreWorkload.putAppendGetWorkload
      c.cmds = {"PUT:foo:bar", "APPEND:foo:baz", "GET:foo"};
      c.results = {"Ok", "barbaz", "barbaz"};
    } else if (workload == "putget") {  // KVStoreWorkload.putGetWorkload (PrimaryBackupTest test17)
      c.cmds = {"PUT:foo:bar", "GET:foo"};
      c.results = {"Ok", "bar"};
    } else if (workload == "getput") {  // a GET before any PUT: KeyNotFound
      c.cmds = {"GET:foo", "PUT:foo:bar", "GET:foo"};
      c.results = {"KeyNotFound", "Ok", "bar"};
    } else {
      throw std::runtime_error("unknown workload " + workload);
    }
    return c;
  }
};

// Inverse of Rec::str() for the flat records carried inside messages ("Type(a, b)"; the KV
// values and keys of the workloads contain no ", " or parentheses).
inline Rec parseRec(const std::string& s) {
  Rec r;
  const size_t o = s.find('(');
  r.type = s.substr(0, o);
  const std::string body = s.substr(o + 1, s.size() - o - 2);
  size_t p = 0;
  while (!body.empty() && p <= body.size()) {
    const size_t q = body.find(", ", p);
    r.f.push_back(body.substr(p, q == std::string::npos ? std::string::npos : q - p));
    if (q == std::string::npos) break;
    p = q + 2;
  }
  return r;
}

// KVStoreWorkload.parse (KVStoreWorkload.java:76-133)
inline std::pair<Rec, Rec> parse(const std::string& c, const std::string& r) {
  std::vector<std::string> sp;
  size_t p = 0;
  for (int k = 0; k < 2; k++) {
    size_t q = c.find(':', p);
    if (q == std::string::npos) break;
    sp.push_back(c.substr(p, q - p));
    p = q + 1;
  }
  sp.push_back(c.substr(p));
  Rec cmd, res;
  if (sp[0] == "GET") {
    cmd = Rec{"Get", {sp.size() == 2 ? sp[1] : sp[1] + sp[2]}};
    if (!r.empty()) res = r == "KeyNotFound" ? Rec{"KeyNotFound", {}} : Rec{"GetResult", {r}};
  } else if (sp[0] == "PUT") {
    cmd = Rec{"Put", {sp[1], sp[2]}};
    if (r == "Ok") res = Rec{"PutOk", {}};
  } else {
    cmd = Rec{"Append", {sp[1], sp[2]}};
    if (!r.empty()) res = Rec{"AppendResult", {r}};
  }
  return {cmd, res};
}

struct SimpleClient : Client {
  int server = 0;
  int seq = 0;
  std::optional<Rec> pending;  // the AMOCommand's command (its seq is `seq`)
  std::optional<Rec> result;

  std::shared_ptr<Node> clone() const override { return std::make_shared<SimpleClient>(*this); }
  void key(std::string& out) const override {
    out += "SC{" + std::to_string(seq) + "," + (pending ? pending->str() : "null") + "," +
           (result ? result->str() : "null") + "}";
  }
  std::string str() const override { return "SimpleClient(seq=" + std::to_string(seq) + ")"; }
  void sendCommand(const Rec& cmd, Ctx& ctx) override {
    seq++;
    pending = cmd;
    result.reset();
    ctx.send(Rec{"Request", {cmd.str(), std::to_string(seq)}}, server);
    ctx.set(Rec{"ClientTimer", {std::to_string(seq)}}, CLIENT_RETRY_MILLIS);
  }
  bool hasResult() const override { return result.has_value(); }
  Rec getResult() const override { return *result; }
  void handleMessage(const Rec& m, int, int, Ctx&) override {
    if (m.type != "Reply") throw HandlerException("no handler");
    if (pending && !result && std::stoi(m.f[1]) == seq) result = parseRec(m.f[0]);
  }
  void onTimer(const Rec& t, Ctx& ctx) override {
    if (t.type != "ClientTimer") throw HandlerException("no timer handler");
    if (pending && !result && std::stoi(t.f[0]) == seq) {
      ctx.send(Rec{"Request", {pending->str(), std::to_string(seq)}}, server);
      ctx.set(t, CLIENT_RETRY_MILLIS);
    }
  }
};

struct SimpleServer : Node {
  std::map<std::string, std::string> kv;                  // KVStore
  std::map<int, std::pair<int, std::string>> amo;         // client -> (last seq, result)
  std::shared_ptr<Node> clone() const override { return std::make_shared<SimpleServer>(*this); }
  void key(std::string& out) const override {
    out += "SS{";
    for (auto& e : kv) out += e.first + "=" + e.second + ",";
    out += "|";
    for (auto& e : amo) out += std::to_string(e.first) + ":" + std::to_string(e.second.first) + ":" + e.second.second + ",";
    out += "}";
  }
  std::string str() const override { return "SimpleServer()"; }
  Rec executeKV(const Rec& c) {  // KVStore.execute
    if (c.type == "Get") {
      auto it = kv.find(c.f[0]);
      return it == kv.end() ? Rec{"KeyNotFound", {}} : Rec{"GetResult", {it->second}};
    }
    if (c.type == "Put") {
      kv[c.f[0]] = c.f[1];
      return Rec{"PutOk", {}};
    }
    kv[c.f[0]] += c.f[1];
    return Rec{"AppendResult", {kv[c.f[0]]}};
  }
  void handleMessage(const Rec& m, int from, int, Ctx& ctx) override {
    if (m.type != "Request") throw HandlerException("no handler");
    const int seq = std::stoi(m.f[1]);
    auto it = amo.find(from);
    const int last = it == amo.end() ? 0 : it->second.first;
    if (seq < last) return;  // an older command: already superseded, no reply
    std::string res;
    if (seq == last) {
      res = it->second.second;
    } else {
      res = executeKV(parseRec(m.f[0])).str();
      amo[from] = {seq, res};
    }
    ctx.send(Rec{"Reply", {res, std::to_string(seq)}}, from);
  }
  void onTimer(const Rec&, Ctx&) override { throw HandlerException("no timer handler"); }
};

// Address 0 = "server", 1..n = "client1".."clientN" (ClientServerBaseTest.java: SA = "server").
inline std::shared_ptr<State> initial(const Config& cfg, Names& names) {
  std::vector<std::shared_ptr<Node>> nodes;
  std::vector<Kind> kinds;
  names.addr = {"server"};
  nodes.push_back(std::make_shared<SimpleServer>());
  kinds.push_back(Kind::Server);
  for (int c = 1; c <= cfg.clients; c++) {
    names.addr.push_back("client" + std::to_string(c));
    auto sc = std::make_shared<SimpleClient>();
    auto cw = std::make_shared<ClientWorker>();
    cw->client = sc;
    cw->addrName = names.addr.back();
    cw->workload.cmds = cfg.cmds;
    cw->workload.results = cfg.results;
    cw->workload.numTimes = cfg.numTimes;
    cw->workload.parser = parse;
    nodes.push_back(cw);
    kinds.push_back(Kind::ClientWorker);
  }
  return makeInitial(nodes, kinds);
}

// KVStoreWorkload.APPENDS_LINEARIZABLE (KVStoreWorkload.java:282-340): the i-th result of a
// client worker belongs to its i-th sent command (the workload's i-th command).
inline Predicate appendsLinearizable(const Config& cfg, const Names& names) {
  return {"Sequence of appends to the same key is linearizable", [cfg, names](const State& s) {
            PredResult r;
            std::vector<std::string> all;
            for (int a : s.clientWorkers()) {
              const ClientWorker* cw = s.cw(a);
              Workload w = cw->workload;
              w.i = 0;
              for (size_t k = 0; k < cw->results.size(); k++) {
                Rec c = w.next(names.addr[a]).first;
                if (c.type != "Append") throw std::runtime_error("Client workers have non-Append Commands");
                const Rec& res = cw->results[k];
                if (res.type != "AppendResult") {
                  r.value = false;
                  return r;
                }
                const std::string& v = res.f[0];
                const std::string& app = c.f[1];
                if (v.size() < app.size() || v.compare(v.size() - app.size(), app.size(), app) != 0) {
                  r.value = false;
                  return r;
                }
                all.push_back(v);
              }
            }
            std::stable_sort(all.begin(), all.end(),
                             [](const std::string& x, const std::string& y) { return x.size() < y.size(); });
            for (size_t i = 0; i + 1 < all.size(); i++)
              if (all[i + 1].rfind(all[i], 0) != 0 || all[i + 1] == all[i]) {
                r.value = false;
                return r;
              }
            return r;
          }};
}

}  // namespace amokv
}  // namespace oracle
