// oracle/proto_multipaxos.hpp -- TEST INFRASTRUCTURE ONLY (see oracle_core.hpp).
//
// Builder-authored Multi-Paxos for lab3 (the reference ships only stubs:
// labs/lab3-paxos/src/dslabs/paxos/PaxosServer.java:16-127, PaxosClient.java:16-62). It follows
// the lab3 README (labs/lab3-paxos/README.md:25-106): PMMC roles in one PaxosServer, a stable
// leader with a heartbeat-check timer (a follower starts phase 1 after two ticks without
// hearing from the leader), clients broadcasting requests (README hint :176-177), an
// at-most-once KV application, and the PaxosServer interface status/command/firstNonCleared/
// lastNonEmpty that PaxosTest's predicates call (PaxosTest.java:113-346). Garbage collection is
// not modelled (firstNonCleared() == 1), which keeps MARKERS_VALID trivially satisfied.
//
// The SAME protocol is re-expressed independently as packed device transitions in
// dslabs_amd/csrc/protocols/multipaxos.hpp; DESIGN.md §9 is the shared specification.
//
//   ballot = (round, leader index), ordered lexicographically; initial ballot (0, server1) with
//   server1 active (phase 1 of ballot 0 is vacuous: nothing can have been accepted before it).
//   Request(cmd)      client->all servers. A server that already executed cmd (AMO) and is the
//                     active leader replies with the cached result; an active leader proposes a
//                     cmd not yet in its log at slotIn (self-accept, P2a to the others).
//   P2a(b,slot,cmd)   acceptor: if b >= ballot: adopt b (step down if b > ballot), heard, accept
//                     unless the slot is chosen, reply P2b(b,slot).
//   P2b(b,slot)       leader (active, b == ballot, slot not chosen): vote; majority -> chosen,
//                     Decision(slot,cmd) to the others, execute.
//   Decision(slot,c)  follower: mark chosen, execute.
//   Tick (100 ms)     active leader: Heartbeat(ballot) to the others. Follower: if heard, clear
//                     heard and missed; else missed++, and at 2 start phase 1 with ballot
//                     (round+1, me): P1a to the others.
//   Heartbeat(b)      if b >= ballot: adopt b (step down if b > ballot), heard.
//   P1a(b)            if b >= ballot: adopt b (step down if b > ballot), heard, P1b(b, log).
//   P1b(b,log)        candidate (electing, b == ballot): vote, merge (chosen wins, else the
//                     highest accepted ballot); majority -> active: re-propose merged slots (holes
//                     become no-ops), slotIn = last merged slot + 1.
//   Execute           in slot order while chosen; AMO: a client's command executes once. Only an
//                     active leader replies to clients.
//   Client            PaxosClient: seq++, broadcast Request, ClientTimer(seq) 100 ms; on timer for
//                     the pending seq re-broadcast and re-set; accept Reply with the pending seq.
#pragma once
#include "oracle_core.hpp"

namespace oracle {
namespace multipaxos {

constexpr int kMaxSlots = 4;
constexpr int kMaxRound = 15;
constexpr int kTick = 100, kClientRetry = 100;

// Workloads are KVStoreWorkload command / result templates on the key "foo"
// (labs/lab1-clientserver/tst/dslabs/kvstore/KVStoreWorkload.java:40-66, :76-133).
struct Config {
  int servers = 3, clients = 2;
  std::vector<std::vector<std::string>> cmds;      // per client: "APPEND:foo:X" / "PUT:foo:bar" / "GET:foo"
  std::vector<std::vector<std::string>> expected;  // per client: expected results (may be empty)
  static Config fromArgs(int servers, int clients, const std::string& workload, bool) {
    Config c;
    c.servers = servers;
    c.clients = clients;
    if (workload == "append-xy") {  // BASELINE C5: concurrent appends, results checked by linearizability
      c.cmds = {{"APPEND:foo:X"}, {"APPEND:foo:Y"}};
      c.expected = {{}, {}};
    } else if (workload == "append-xy-expect") {  // PaxosTest.test22: client1 -> X, client2 -> XY
      c.cmds = {{"APPEND:foo:X"}, {"APPEND:foo:Y"}};
      c.expected = {{"X"}, {"XY"}};
    } else if (workload == "append-x") {  // single client
      c.cmds = {{"APPEND:foo:X"}};
      c.expected = {{"X"}};
    } else if (workload == "append-xz") {  // two commands from client1, one from client2
      c.cmds = {{"APPEND:foo:X", "APPEND:foo:Z"}, {"APPEND:foo:Y"}};
      c.expected = {{}, {}};
    } else if (workload == "put-append-get") {  // KVStoreWorkload.putAppendGetWorkload (PaxosTest.test27)
      c.cmds = {{"PUT:foo:bar", "APPEND:foo:baz", "GET:foo"}};
      c.expected = {{"Ok", "barbaz", "barbaz"}};
    } else {
      throw std::runtime_error("unknown workload " + workload);
    }
    c.cmds.resize(clients);
    c.expected.resize(clients);
    return c;
  }
};

// KVStoreWorkload.parse for the templates above (the same forms as lab1's, proto_amokv.hpp).
inline std::pair<Rec, Rec> parseKv(const std::string& c, const std::string& r) {
  Rec cmd, res;
  if (c.rfind("GET:", 0) == 0) {
    cmd = Rec{"Get", {c.substr(4)}};
    if (!r.empty()) res = r == "KeyNotFound" ? Rec{"KeyNotFound", {}} : Rec{"GetResult", {r}};
  } else if (c.rfind("PUT:", 0) == 0) {
    const size_t k = c.find(':', 4);
    cmd = Rec{"Put", {c.substr(4, k - 4), c.substr(k + 1)}};
    if (r == "Ok") res = Rec{"PutOk", {}};
  } else {
    const size_t k = c.find(':', 7);
    cmd = Rec{"Append", {c.substr(7, k - 7), c.substr(k + 1)}};
    if (!r.empty()) res = Rec{"AppendResult", {r}};
  }
  return {cmd, res};
}

struct Ballot {
  int round = 0, leader = 0;
  bool operator<(const Ballot& o) const { return round != o.round ? round < o.round : leader < o.leader; }
  bool operator==(const Ballot& o) const { return round == o.round && leader == o.leader; }
  bool operator<=(const Ballot& o) const { return !(o < *this); }
  std::string str() const { return "(" + std::to_string(round) + "," + std::to_string(leader) + ")"; }
  static Ballot parse(const std::string& s) {
    Ballot b;
    sscanf(s.c_str(), "(%d,%d)", &b.round, &b.leader);
    return b;
  }
};

// An AMO command: (client address, seq, KV command on "foo"). client < 0 = no-op. String form:
// "c#s:X" for Append(foo, X), "c#s:=X" for Put(foo, X), "c#s:?" for Get(foo).
struct Cmd {
  int client = -1, seq = 0;
  char op = 'A';  // 'A'ppend, 'P'ut, 'G'et
  std::string value;
  bool noop() const { return client < 0; }
  bool operator==(const Cmd& o) const {
    return client == o.client && seq == o.seq && op == o.op && value == o.value;
  }
  // PaxosServer.command(i): the KV command (Lombok equals: type and fields), null for a no-op
  bool sameKv(const Cmd& o) const { return noop() == o.noop() && (noop() || (op == o.op && value == o.value)); }
  std::string str() const {
    if (noop()) return "noop";
    const std::string pre = std::to_string(client) + "#" + std::to_string(seq) + ":";
    return op == 'P' ? pre + "=" + value : op == 'G' ? pre + "?" : pre + value;
  }
  static Cmd parse(const std::string& s) {
    Cmd c;
    if (s == "noop") return c;
    size_t h = s.find('#'), k = s.find(':');
    c.client = std::stoi(s.substr(0, h));
    c.seq = std::stoi(s.substr(h + 1, k - h - 1));
    std::string v = s.substr(k + 1);
    if (!v.empty() && v[0] == '=') {
      c.op = 'P';
      c.value = v.substr(1);
    } else if (v == "?") {
      c.op = 'G';
    } else {
      c.value = v;
    }
    return c;
  }
};

enum Status { EMPTY = 0, ACCEPTED = 1, CHOSEN = 2 };

struct Entry {
  Status status = EMPTY;
  Ballot ballot;  // acceptance ballot (unused once chosen)
  Cmd cmd;
  std::string str() const {
    if (status == EMPTY) return "E";
    if (status == CHOSEN) return "C:" + cmd.str();
    return "A" + ballot.str() + ":" + cmd.str();
  }
};

// Log snapshot carried by P1b: "E|C:cmd|A(r,l):cmd" per slot, separated by ';'.
inline std::string logStr(const std::vector<Entry>& log) {
  std::string s;
  for (size_t i = 1; i < log.size(); i++) s += (i > 1 ? ";" : "") + log[i].str();
  return s;
}
inline std::vector<Entry> parseLog(const std::string& s) {
  std::vector<Entry> log(kMaxSlots + 1);
  size_t pos = 0;
  for (int i = 1; i <= kMaxSlots; i++) {
    size_t e = s.find(';', pos);
    std::string t = s.substr(pos, e == std::string::npos ? std::string::npos : e - pos);
    pos = e == std::string::npos ? s.size() : e + 1;
    if (t == "E") continue;
    if (t[0] == 'C') {
      log[i].status = CHOSEN;
      log[i].cmd = Cmd::parse(t.substr(2));
    } else {
      size_t c = t.find(')');
      log[i].status = ACCEPTED;
      log[i].ballot = Ballot::parse(t.substr(1, c));
      log[i].cmd = Cmd::parse(t.substr(c + 2));
    }
  }
  return log;
}

struct PaxosServer : Node {
  int me = 0, n = 3;
  Ballot ballot;
  bool active = false, electing = false, heard = false;
  int missed = 0;
  std::set<int> p1bVotes;
  std::vector<Entry> p1bLog = std::vector<Entry>(kMaxSlots + 1);
  std::vector<Entry> log = std::vector<Entry>(kMaxSlots + 1);
  std::vector<std::set<int>> p2bVotes = std::vector<std::set<int>>(kMaxSlots + 1);
  int slotOut = 1, slotIn = 1;
  // application (derived from the executed prefix, kept explicitly like an AMOApplication)
  std::map<int, std::pair<int, std::string>> amo;  // client -> (last seq, result)
  std::string foo;
  bool fooSet = false;  // the key exists (a Put or Append executed)

  std::shared_ptr<Node> clone() const override { return std::make_shared<PaxosServer>(*this); }
  void key(std::string& out) const override {
    out += "PS{" + ballot.str() + (active ? "A" : "") + (electing ? "E" : "") + (heard ? "H" : "") + "m" +
           std::to_string(missed) + "v";
    for (int v : p1bVotes) out += std::to_string(v);
    out += "|" + logStr(p1bLog) + "|" + logStr(log) + "|";
    for (int i = 1; i <= kMaxSlots; i++) {
      for (int v : p2bVotes[i]) out += std::to_string(v);
      out += ",";
    }
    out += "|" + std::to_string(slotOut) + "," + std::to_string(slotIn) + "|" + (fooSet ? foo : "-") + "}";
  }
  std::string str() const override { return "PaxosServer(" + ballot.str() + ")"; }

  std::vector<int> others() const {
    std::vector<int> v;
    for (int s = 0; s < n; s++)
      if (s != me) v.push_back(s);
    return v;
  }
  bool majority(size_t k) const { return (int)k * 2 > n; }

  void adopt(const Ballot& b) {  // b >= ballot; a higher ballot steps this server down
    if (ballot < b) {
      ballot = b;
      active = false;
      electing = false;
      p1bVotes.clear();
      p1bLog = std::vector<Entry>(kMaxSlots + 1);
      for (auto& v : p2bVotes) v.clear();
    }
  }

  // KVStore.execute on "foo" (KVStore.java:59-78 as lab1 specifies it); the result as the reply
  // carries it: "Ok" (PutOk), "KeyNotFound", or the value (AppendResult / GetResult).
  std::string kvExecute(const Cmd& c) {
    if (c.op == 'P') {
      foo = c.value;
      fooSet = true;
      return "Ok";
    }
    if (c.op == 'A') {
      foo += c.value;
      fooSet = true;
      return foo;
    }
    return fooSet ? foo : "KeyNotFound";
  }

  void execute(Ctx& ctx) {
    while (slotOut <= kMaxSlots && log[slotOut].status == CHOSEN) {
      const Cmd& c = log[slotOut].cmd;
      if (!c.noop()) {
        auto it = amo.find(c.client);
        if (it == amo.end() || it->second.first < c.seq) {
          const std::string res = kvExecute(c);
          amo[c.client] = {c.seq, res};
          if (active) ctx.send(Rec{"PaxosReply", {std::to_string(c.seq), res}}, c.client);
        }
      }
      slotOut++;
    }
  }

  bool inLog(const Cmd& c) const {
    for (int i = 1; i <= kMaxSlots; i++)
      if (log[i].status != EMPTY && log[i].cmd == c) return true;
    return false;
  }

  void propose(int slot, const Cmd& c, Ctx& ctx) {
    if (slot > kMaxSlots) throw Overflow{"log capacity exceeded"};
    log[slot] = Entry{ACCEPTED, ballot, c};
    p2bVotes[slot] = {me};
    ctx.broadcast(Rec{"P2a", {ballot.str(), std::to_string(slot), c.str()}}, others());
    if (majority(p2bVotes[slot].size())) choose(slot, ctx);
  }

  void choose(int slot, Ctx& ctx) {
    log[slot].status = CHOSEN;
    log[slot].ballot = Ballot{};
    p2bVotes[slot].clear();
    ctx.broadcast(Rec{"Decision", {std::to_string(slot), log[slot].cmd.str()}}, others());
    execute(ctx);
  }

  void init(Ctx& ctx) override {
    if (me == 0) active = true;
    ctx.set(Rec{"TickTimer", {}}, kTick);
  }

  void onTimer(const Rec& t, Ctx& ctx) override {
    if (active) {
      ctx.broadcast(Rec{"Heartbeat", {ballot.str()}}, others());
    } else if (heard) {
      heard = false;
      missed = 0;
    } else if ((missed = std::min(missed + 1, 2)) >= 2 && ballot.round < kMaxRound) {
      // two ticks without hearing from the leader: phase 1 (bounded ballots: none past kMaxRound)
      missed = 0;
      heard = false;
      ballot = Ballot{ballot.round + 1, me};
      electing = true;
      active = false;
      for (auto& v : p2bVotes) v.clear();
      p1bVotes = {me};
      p1bLog = std::vector<Entry>(kMaxSlots + 1);
      merge(log);
      ctx.broadcast(Rec{"P1a", {ballot.str()}}, others());
      if (majority(p1bVotes.size())) becomeLeader(ctx);
    }
    ctx.set(t, kTick);
  }

  void merge(const std::vector<Entry>& other) {
    for (int i = 1; i <= kMaxSlots; i++) {
      const Entry& e = other[i];
      Entry& m = p1bLog[i];
      if (e.status == CHOSEN) {
        m = Entry{CHOSEN, Ballot{}, e.cmd};
      } else if (e.status == ACCEPTED && m.status != CHOSEN && (m.status == EMPTY || m.ballot < e.ballot)) {
        m = e;
      }
    }
  }

  void becomeLeader(Ctx& ctx) {
    electing = false;
    active = true;
    p1bVotes.clear();
    int last = 0;
    for (int i = 1; i <= kMaxSlots; i++)
      if (p1bLog[i].status != EMPTY || log[i].status != EMPTY) last = i;
    std::vector<Entry> merged = p1bLog;
    p1bLog = std::vector<Entry>(kMaxSlots + 1);
    for (int i = 1; i <= last; i++) {
      if (log[i].status == CHOSEN) continue;
      if (merged[i].status == CHOSEN) {
        log[i] = Entry{CHOSEN, Ballot{}, merged[i].cmd};
        p2bVotes[i].clear();
      } else {
        propose(i, merged[i].status == ACCEPTED ? merged[i].cmd : Cmd{}, ctx);
      }
    }
    slotIn = last + 1;
    execute(ctx);
  }

  void handleMessage(const Rec& m, int from, int, Ctx& ctx) override {
    if (m.type == "PaxosRequest") {
      Cmd c = Cmd::parse(m.f[0]);
      auto it = amo.find(c.client);
      if (it != amo.end() && it->second.first >= c.seq) {
        if (active && it->second.first == c.seq)
          ctx.send(Rec{"PaxosReply", {std::to_string(c.seq), it->second.second}}, c.client);
        return;
      }
      // new proposals go after every slot this server knows to be in use (a stale leader may
      // have learned later slots through Decision / P2a); bounded log: with no free slot the
      // leader ignores the request (clients retry)
      const int slot = std::max(slotIn, lastNonEmpty() + 1);
      if (active && !inLog(c) && slot <= kMaxSlots) {
        slotIn = slot + 1;
        propose(slot, c, ctx);
      }
    } else if (m.type == "P2a") {
      Ballot b = Ballot::parse(m.f[0]);
      if (b < ballot) return;
      adopt(b);
      heard = true;
      int slot = std::stoi(m.f[1]);
      if (log[slot].status != CHOSEN) log[slot] = Entry{ACCEPTED, b, Cmd::parse(m.f[2])};
      ctx.send(Rec{"P2b", {b.str(), m.f[1]}}, from);
    } else if (m.type == "P2b") {
      Ballot b = Ballot::parse(m.f[0]);
      int slot = std::stoi(m.f[1]);
      if (!active || !(b == ballot) || log[slot].status != ACCEPTED) return;
      p2bVotes[slot].insert(from);
      if (majority(p2bVotes[slot].size())) choose(slot, ctx);
    } else if (m.type == "Decision") {
      int slot = std::stoi(m.f[0]);
      if (log[slot].status != CHOSEN) {
        log[slot] = Entry{CHOSEN, Ballot{}, Cmd::parse(m.f[1])};
        p2bVotes[slot].clear();
        execute(ctx);
      }
    } else if (m.type == "Heartbeat") {
      Ballot b = Ballot::parse(m.f[0]);
      if (b < ballot) return;
      adopt(b);
      heard = true;
    } else if (m.type == "P1a") {
      Ballot b = Ballot::parse(m.f[0]);
      if (b < ballot) return;
      adopt(b);
      heard = true;
      ctx.send(Rec{"P1b", {b.str(), logStr(log)}}, from);
    } else if (m.type == "P1b") {
      Ballot b = Ballot::parse(m.f[0]);
      if (!electing || !(b == ballot)) return;
      p1bVotes.insert(from);
      merge(parseLog(m.f[1]));
      if (majority(p1bVotes.size())) becomeLeader(ctx);
    } else {
      throw HandlerException("no handler for " + m.type);
    }
  }

  // PaxosServer interface (PaxosServer.java:54-108)
  Status status(int i) const { return (i >= 1 && i <= kMaxSlots) ? log[i].status : EMPTY; }
  int lastNonEmpty() const {
    int ne = 0;
    for (int i = 1; i <= kMaxSlots; i++)
      if (log[i].status != EMPTY) ne = i;
    return ne;
  }
};

struct PaxosClient : Client {
  std::vector<int> servers;
  int me = 0;
  int seq = 0;
  std::optional<Cmd> pending;
  char pendingOp = 'A';  // the op of the last command sent (transient: implied by seq and the workload)
  std::optional<std::string> result;

  std::shared_ptr<Node> clone() const override { return std::make_shared<PaxosClient>(*this); }
  void key(std::string& out) const override {
    out += "PC{" + std::to_string(seq) + "," + (pending ? pending->str() : "null") + "," + (result ? *result : "null") +
           "}";
  }
  std::string str() const override { return "PaxosClient(seq=" + std::to_string(seq) + ")"; }
  void sendCommand(const Rec& cmd, Ctx& ctx) override {
    seq++;
    Cmd c{me, seq, cmd.type == "Put" ? 'P' : cmd.type == "Get" ? 'G' : 'A', cmd.type == "Get" ? "" : cmd.f[1]};
    pending = c;
    pendingOp = c.op;
    result.reset();
    ctx.broadcast(Rec{"PaxosRequest", {pending->str()}}, servers);
    ctx.set(Rec{"ClientTimer", {std::to_string(seq)}}, kClientRetry);
  }
  bool hasResult() const override { return result.has_value(); }
  Rec getResult() const override {  // typed by the command it answers
    if (pendingOp == 'P') return Rec{"PutOk", {}};
    if (pendingOp == 'G') return *result == "KeyNotFound" ? Rec{"KeyNotFound", {}} : Rec{"GetResult", {*result}};
    return Rec{"AppendResult", {*result}};
  }
  void handleMessage(const Rec& m, int, int, Ctx&) override {
    if (m.type != "PaxosReply") throw HandlerException("no handler");
    if (pending && std::stoi(m.f[0]) == seq) {
      result = m.f[1];
      pending.reset();
    }
  }
  void onTimer(const Rec& t, Ctx& ctx) override {
    if (pending && std::stoi(t.f[0]) == seq) {
      ctx.broadcast(Rec{"PaxosRequest", {pending->str()}}, servers);
      ctx.set(t, kClientRetry);
    }
  }
};

// Addresses: server1..serverN (0..N-1), client1..clientC (N..N+C-1).
inline std::shared_ptr<State> initial(const Config& cfg, Names& names) {
  std::vector<std::shared_ptr<Node>> nodes;
  std::vector<Kind> kinds;
  std::vector<int> servers;
  for (int s = 0; s < cfg.servers; s++) servers.push_back(s);
  for (int s = 0; s < cfg.servers; s++) {
    names.addr.push_back("server" + std::to_string(s + 1));
    auto p = std::make_shared<PaxosServer>();
    p->me = s;
    p->n = cfg.servers;
    nodes.push_back(p);
    kinds.push_back(Kind::Server);
  }
  for (int c = 0; c < cfg.clients; c++) {
    names.addr.push_back("client" + std::to_string(c + 1));
    auto pc = std::make_shared<PaxosClient>();
    pc->servers = servers;
    pc->me = cfg.servers + c;
    auto cw = std::make_shared<ClientWorker>();
    cw->client = pc;
    cw->addrName = names.addr.back();
    cw->workload.cmds = cfg.cmds[c];
    cw->workload.results = cfg.expected[c];
    cw->workload.numTimes = 1;
    cw->workload.parser = parseKv;
    nodes.push_back(cw);
    kinds.push_back(Kind::ClientWorker);
  }
  return makeInitial(nodes, kinds);
}

inline const PaxosServer* server(const State& s, int i) { return dynamic_cast<const PaxosServer*>(s.nodes[i].get()); }

// PaxosTest.slotValid(st, i) (PaxosTest.java:215-279). No garbage collection: firstNonCleared()
// == 1, no slot is CLEARED, and command(i) is the KV command (null for EMPTY slots and no-ops).
inline bool slotValid(const State& s, int N, int i, std::string* why) {
  std::optional<Cmd> chosen;
  bool isChosen = false;
  for (int k = 0; k < N; k++) {
    const PaxosServer* p = server(s, k);
    const int nc = 1, ne = p->lastNonEmpty();
    const Status st = p->status(i);
    if (i < nc) {  // status(i) is not CLEARED (nothing ever is)
      *why = "slot " + std::to_string(i) + " below the first non-cleared slot is not cleared";
      return false;
    }
    if (i > ne && st != EMPTY) {
      *why = "slot past the last non-empty one is not empty";
      return false;
    }
    if (st == CHOSEN) {
      const Cmd& c = p->log[i].cmd;
      if (isChosen && !chosen->sameKv(c)) {
        *why = "Two different commands chosen for slot " + std::to_string(i);
        return false;
      }
      chosen = c;
      isChosen = true;
    }
  }
  if (!isChosen) return true;
  int count = 0;
  for (int k = 0; k < N; k++) {
    const PaxosServer* p = server(s, k);
    const Status st = p->status(i);
    if (st != EMPTY && (st != ACCEPTED || p->log[i].cmd.sameKv(*chosen))) count++;
  }
  if (2 * count <= N) {
    *why = "chosen for slot " + std::to_string(i) + " without a majority accepting";
    return false;
  }
  return true;
}

// PaxosTest.LOGS_CONSISTENT_ALL_SLOTS (:302-322) and LOGS_CONSISTENT (:282-300; from the smallest
// firstNonCleared(), i.e. 1, so the two coincide), each with MARKERS_VALID (:128-193), which holds
// by construction here (firstNonCleared() == 1, lastNonEmpty() the last non-EMPTY slot).
inline Predicate logsConsistent(const Config& cfg, bool active = false) {
  int N = cfg.servers;
  return {active ? "Active log slots consistent" : "Non-empty log slots consistent", [N](const State& s) {
            PredResult r;
            int maxNe = 0;
            for (int i = 0; i < N; i++) maxNe = std::max(maxNe, server(s, i)->lastNonEmpty());
            for (int slot = 1; slot <= maxNe; slot++)
              if (!slotValid(s, N, slot, &r.detail)) {
                r.value = false;
                return r;
              }
            return r;
          }};
}
inline Predicate slotValidPred(const Config& cfg, int i) {
  int N = cfg.servers;
  return {"Logs consistent for slot " + std::to_string(i), [N, i](const State& s) {
            PredResult r;
            r.value = slotValid(s, N, i, &r.detail);
            return r;
          }};
}
// PaxosTest.hasStatus(a, i, s) (:113-117): ((PaxosServer) st.server(a)).status(i) == s.
inline Predicate hasStatus(const Config& cfg, int a, int i, Status want) {
  int N = cfg.servers;
  return {"has status", [N, a, i, want](const State& s) {
            if (a < 0 || a >= N) throw HandlerException("not a PaxosServer");
            PredResult r;
            r.value = server(s, a)->status(i) == want;
            return r;
          }};
}
// PaxosTest.hasCommand(a, i, c) (:119-123): Objects.equals(command(i), c); c as a Cmd ("noop" =
// null; only its KV command is compared).
inline Predicate hasCommand(const Config& cfg, int a, int i, const Cmd& want) {
  int N = cfg.servers;
  return {"has command", [N, a, i, want](const State& s) {
            if (a < 0 || a >= N) throw HandlerException("not a PaxosServer");
            const PaxosServer* p = server(s, a);
            Cmd have;  // null unless the slot holds a (non-no-op) command
            if (p->status(i) != EMPTY) have = p->log[i].cmd;
            PredResult r;
            r.value = have.sameKv(want);
            return r;
          }};
}

// KVStoreWorkload.APPENDS_LINEARIZABLE (labs/lab1-clientserver/tst/dslabs/kvstore/KVStoreWorkload.java:282-340)
inline Predicate appendsLinearizable(const Config& cfg) {
  return {"Sequence of appends to the same key is linearizable", [cfg](const State& s) {
            PredResult r;
            std::vector<std::string> all;
            for (int a : s.clientWorkers()) {
              const ClientWorker* cw = s.cw(a);
              int ci = a - cfg.servers;
              for (size_t k = 0; k < cw->results.size(); k++) {
                const std::string& tmpl = cfg.cmds[ci][k];
                if (tmpl.rfind("APPEND:", 0) != 0) throw std::runtime_error("Client workers have non-Append Commands");
                const std::string val = tmpl.substr(tmpl.find(':', 7) + 1);
                if (cw->results[k].type != "AppendResult") {
                  r.value = false;
                  return r;
                }
                const std::string& res = cw->results[k].f[0];
                if (res.size() < val.size() || res.compare(res.size() - val.size(), val.size(), val) != 0) {
                  r.value = false;
                  return r;
                }
                all.push_back(res);
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

}  // namespace multipaxos
}  // namespace oracle
