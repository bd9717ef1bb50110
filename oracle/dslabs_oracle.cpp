// oracle/dslabs_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see oracle_core.hpp header).
//
// Command-line front end of the CPU oracle. Prints one JSON object on stdout.
//
//   dslabs_oracle bfs --proto pingpong --clients 1 --pings 10 --inv RESULTS_OK --prune CLIENTS_DONE
//   dslabs_oracle bfs --proto sipaxos --proposers 2 --acceptors 3 --values a,b --max-depth 9
//   dslabs_oracle replay --proto pingpong ... --trace-file events.txt
//   dslabs_oracle replaysearch --proto minitest --inv foo --trace-file events.txt [--minimize]
//                [--human-readable]   (the reported state's trace reordered, SearchState.humanReadableTrace)
//   dslabs_oracle timerqueue        (TimerQueueTest.randomTimers truth table)
//
// Options common to bfs/replay:
//   --inv NAME / --goal NAME / --prune NAME   (repeatable, insertion order kept; prefix "!" = negate)
//   --max-depth N, --finish-level (level-synchronous terminal rule), --max-secs S,
//   --no-timers ADDR, --partition a,b|c (link filter), --print-states
#include <cstring>
#include <fstream>
#include <iostream>

#include "oracle_core.hpp"
#include "proto_amokv.hpp"
#include "proto_minitest.hpp"
#include "proto_multipaxos.hpp"
#include "proto_pb.hpp"
#include "proto_pingpong.hpp"
#include "proto_sipaxos.hpp"
#include "proto_synthetic.hpp"
#include "gen/proto_pingpong_ir.hpp"  // generated from the protocol IR (tools/gen_ir.py)
#include "gen/proto_amokv_ir.hpp"
#include "gen/proto_multipaxos_ir.hpp"
#include "gen/proto_pb_ir.hpp"

using namespace oracle;

static std::string jsonEsc(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += c;
    } else if (c == '\n') {
      o += "\\n";
    } else {
      o += c;
    }
  }
  return o;
}

struct Args {
  std::string mode, proto = "pingpong";
  std::map<std::string, std::vector<std::string>> kv;
  bool has(const std::string& k) const { return kv.count(k) > 0; }
  std::string get(const std::string& k, const std::string& d = "") const {
    auto it = kv.find(k);
    return it == kv.end() ? d : it->second.back();
  }
  int geti(const std::string& k, int d) const { return has(k) ? std::stoi(get(k)) : d; }
  std::vector<std::string> all(const std::string& k) const {
    auto it = kv.find(k);
    return it == kv.end() ? std::vector<std::string>{} : it->second;
  }
};

static std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  out.push_back(cur);
  return out;
}

struct Scenario {
  std::shared_ptr<State> init;
  Names names;
  std::function<Predicate(const std::string&)> pred;  // protocol predicate registry
};

static int addrOf(const Names& n, const std::string& s) {
  for (size_t i = 0; i < n.addr.size(); i++)
    if (n.addr[i] == s) return (int)i;
  throw std::runtime_error("unknown address " + s);
}

static Scenario build(const Args& a) {
  Scenario sc;
  auto common = [&sc](const std::string& name) -> std::optional<Predicate> {
    if (name == "RESULTS_OK") return RESULTS_OK(sc.names);
    if (name == "CLIENTS_DONE") return CLIENTS_DONE();
    if (name == "NONE_DECIDED") return NONE_DECIDED();
    if (name.rfind("clientDone:", 0) == 0) return clientDone(sc.names, addrOf(sc.names, name.substr(11)));
    return std::nullopt;
  };
  if (a.proto == "pingpong") {
    sc.init = pingpong::initial(a.geti("clients", 1), a.geti("pings", 10), !a.has("mutant-no-check"),
                                !a.has("mutant-no-reset"), sc.names);
    sc.pred = [common](const std::string& n) {
      auto p = common(n);
      if (!p) throw std::runtime_error("unknown predicate " + n);
      return *p;
    };
  } else if (a.proto == "pingpong_ir") {  // the same protocol, generated from the IR
    pingpong_ir::Params prm;
    prm.clients = a.geti("clients", 1);
    prm.pings = a.geti("pings", 10);
    prm.check_value = a.has("mutant-no-check") ? 0 : 1;
    prm.reset_timer = a.has("mutant-no-reset") ? 0 : 1;
    sc.init = pingpong_ir::initial(prm, sc.names);
    sc.pred = [common](const std::string& n) {
      auto p = common(n);
      if (!p) throw std::runtime_error("unknown predicate " + n);
      return *p;
    };
  } else if (a.proto == "amokv_ir") {  // --ir-params: the engine's parameter vector, comma-separated
    std::vector<long long> v;
    for (auto& x : split(a.get("ir-params"), ',')) v.push_back(std::stoll(x));
    sc.init = amokv_ir::initial(amokv_ir::from_vector(v), sc.names);
    sc.pred = [common](const std::string& n) {
      auto p = common(n);
      if (!p) throw std::runtime_error("unknown predicate " + n);
      return *p;
    };
  } else if (a.proto == "multipaxos_ir") {  // --ir-params: the engine's parameter vector, comma-separated
    std::vector<long long> v;
    for (auto& x : split(a.get("ir-params"), ',')) v.push_back(std::stoll(x));
    const auto prm = multipaxos_ir::from_vector(v);
    sc.init = multipaxos_ir::initial(prm, sc.names);
    sc.pred = [common, prm](const std::string& n) {
      auto p = common(n);
      if (!p) p = multipaxos_ir::predicate(n, prm);
      if (!p) throw std::runtime_error("unknown predicate " + n);
      return *p;
    };
  } else if (a.proto == "pb_ir") {  // --ir-params: the engine's parameter vector, comma-separated
    std::vector<long long> v;
    for (auto& x : split(a.get("ir-params"), ',')) v.push_back(std::stoll(x));
    const auto prm = pb_ir::from_vector(v);
    sc.init = pb_ir::initial(prm, sc.names);
    sc.pred = [common, prm](const std::string& n) {
      auto p = common(n);
      if (!p) p = pb_ir::predicate(n, prm);
      if (!p) throw std::runtime_error("unknown predicate " + n);
      return *p;
    };
  } else if (a.proto == "sipaxos") {
    int P = a.geti("proposers", 2), A = a.geti("acceptors", 3);
    auto values = split(a.get("values", "a,b"), ',');
    sc.init = sipaxos::initial(P, A, values, a.has("incorrect"), sc.names);
    sc.pred = [P, values](const std::string& n) -> Predicate {
      if (n == "Agreement") return sipaxos::agreement(P);
      if (n == "Integrity") return sipaxos::integrity(P, values);
      if (n == "Termination") return sipaxos::termination(P);
      throw std::runtime_error("unknown predicate " + n);
    };
  } else if (a.proto == "multipaxos") {
    multipaxos::Config cfg = multipaxos::Config::fromArgs(a.geti("servers", 3), a.geti("clients", 2),
                                                          a.get("workload", "append-xy"), false);
    sc.init = multipaxos::initial(cfg, sc.names);
    sc.pred = [common, cfg](const std::string& n) -> Predicate {
      auto p = common(n);
      if (p) return *p;
      if (n == "LOGS_CONSISTENT_ALL_SLOTS") return multipaxos::logsConsistent(cfg);
      if (n == "LOGS_CONSISTENT") return multipaxos::logsConsistent(cfg, true);
      if (n == "APPENDS_LINEARIZABLE") return multipaxos::appendsLinearizable(cfg);
      auto parts = split(n, ':');
      if (parts[0] == "slotValid" && parts.size() == 2) return multipaxos::slotValidPred(cfg, std::stoi(parts[1]));
      if (parts[0] == "hasStatus" && parts.size() == 4) {  // hasStatus:serverK:slot:STATUS
        static const std::map<std::string, multipaxos::Status> st = {
            {"EMPTY", multipaxos::EMPTY}, {"ACCEPTED", multipaxos::ACCEPTED}, {"CHOSEN", multipaxos::CHOSEN}};
        if (parts[3] == "CLEARED")  // never cleared (no garbage collection): always false
          return Predicate{n, [](const State&) { PredResult r; r.value = false; return r; }};
        return multipaxos::hasStatus(cfg, std::stoi(parts[1].substr(6)) - 1, std::stoi(parts[2]), st.at(parts[3]));
      }
      if (parts[0] == "hasCommand" && parts.size() >= 4) {  // hasCommand:serverK:slot:CMD (Cmd string form)
        const std::string c = n.substr(n.find(':', n.find(':', 11) + 1) + 1);
        return multipaxos::hasCommand(cfg, std::stoi(parts[1].substr(6)) - 1, std::stoi(parts[2]),
                                      c == "null" ? multipaxos::Cmd{} : multipaxos::Cmd::parse("0#0:" + c));
      }
      throw std::runtime_error("unknown predicate " + n);
    };
  } else if (a.proto == "amokv") {
    amokv::Config cfg = amokv::Config::fromArgs(a.geti("clients", 2), a.get("workload", "diffkey3"));
    sc.init = amokv::initial(cfg, sc.names);
    Names* nm = &sc.names;
    sc.pred = [common, cfg, nm](const std::string& n) -> Predicate {
      auto p = common(n);
      if (p) return *p;
      if (n == "APPENDS_LINEARIZABLE") return amokv::appendsLinearizable(cfg, *nm);
      throw std::runtime_error("unknown predicate " + n);
    };
  } else if (a.proto == "pb") {
    pb::Config cfg;
    cfg.servers = a.geti("servers", 2);
    cfg.clients = a.geti("clients", 1);
    cfg.kv = amokv::Config::fromArgs(cfg.clients, a.get("workload", "putget"));
    sc.init = pb::initial(cfg, sc.names);
    sc.pred = [common, &sc](const std::string& n) -> Predicate {
      auto p = common(n);
      if (p) return *p;
      if (n.rfind("hasViewReply:", 0) == 0) {  // hasViewReply:N or hasViewReply:N:P:B
        auto parts = split(n, ':');
        if (parts.size() == 2) return pb::hasViewReply(std::stoi(parts[1]));
        return pb::hasViewReplyExact(std::stoi(parts[1]), std::stoi(parts[2]), std::stoi(parts[3]));
      }
      if (n.rfind("viewRepliesSent:", 0) == 0) {  // viewRepliesSent:N:P:B:addr1+addr2+...
        auto parts = split(n, ':');
        std::vector<int> to;
        for (auto& nm : split(parts[4], '+')) to.push_back(addrOf(sc.names, nm));
        return pb::viewRepliesSent(std::stoi(parts[1]), std::stoi(parts[2]), std::stoi(parts[3]), to);
      }
      throw std::runtime_error("unknown predicate " + n);
    };
  } else if (a.proto == "synthetic") {
    synthetic::Table tab;
    tab.nodes = a.geti("nodes", 5);
    tab.K = a.geti("values", 64);
    tab.P = a.geti("poke-mod", 7);
    if (a.has("seed")) tab.seed = std::stoull(a.get("seed"), nullptr, 0);
    sc.init = synthetic::initial(tab, sc.names);
    sc.pred = [tab](const std::string& n) -> Predicate {
      if (n == "NOT_ALL_MAX") return synthetic::notAllMax(tab);
      if (n.rfind("COUNTER_LT:", 0) == 0) {
        auto parts = split(n, ':');
        return synthetic::counterLt(std::stoi(parts[1]), std::stoi(parts[2]));
      }
      throw std::runtime_error("unknown predicate " + n);
    };
  } else if (a.proto == "minitest") {
    sc.init = minitest::initial(sc.names);
    sc.pred = [](const std::string& n) -> Predicate {
      if (n == "foo") return minitest::foo();
      if (n == "fooException") return minitest::fooException();
      if (n == "alwaysException") return minitest::alwaysException();
      throw std::runtime_error("unknown predicate " + n);
    };
  } else {
    throw std::runtime_error("unknown protocol " + a.proto);
  }
  return sc;
}

// A predicate argument: NAME, !P (negate), and(P,Q), or(P,Q), implies(P,Q), nested.
static Predicate parsePred(const std::string& raw, Scenario& sc) {
  if (!raw.empty() && raw[0] == '!') return parsePred(raw.substr(1), sc).negate();
  for (const char* op : {"and(", "or(", "implies("}) {
    const std::string o(op);
    if (raw.rfind(o, 0) == 0 && raw.back() == ')') {
      const std::string in = raw.substr(o.size(), raw.size() - o.size() - 1);
      int depth = 0;
      for (size_t k = 0; k < in.size(); k++) {
        if (in[k] == '(') depth++;
        else if (in[k] == ')') depth--;
        else if (in[k] == ',' && depth == 0) {
          Predicate x = parsePred(in.substr(0, k), sc), y = parsePred(in.substr(k + 1), sc);
          return o == "and(" ? x.and_(y) : o == "or(" ? x.or_(y) : x.implies(y);
        }
      }
      throw std::runtime_error("bad predicate " + raw);
    }
  }
  return sc.pred(raw);
}

static Settings settingsFrom(const Args& a, Scenario& sc) {
  Settings st;
  auto mk = [&](const std::string& raw) { return parsePred(raw, sc); };
  for (auto& n : a.all("inv")) st.invariants.push_back(mk(n));
  for (auto& n : a.all("goal")) st.goals.push_back(mk(n));
  for (auto& n : a.all("prune")) st.prunes.push_back(mk(n));
  st.maxDepth = a.geti("max-depth", -1);
  for (auto& n : a.all("no-timers")) st.timersActive[addrOf(sc.names, n)] = false;
  for (auto& n : a.all("inactive")) {  // TestSettings.nodeActive(n, false)
    st.senderActive[addrOf(sc.names, n)] = false;
    st.receiverActive[addrOf(sc.names, n)] = false;
  }
  if (a.has("network-off")) st.networkActive = false;  // TestSettings.networkActive(false)
  for (auto& n : a.all("active")) {  // TestSettings.nodeActive(n, true)
    st.senderActive[addrOf(sc.names, n)] = true;
    st.receiverActive[addrOf(sc.names, n)] = true;
  }
  for (auto& l : a.all("link")) {  // TestSettings.linkActive(from, to, true): "from,to"
    auto ft = split(l, ',');
    st.linkActive[{addrOf(sc.names, ft[0]), addrOf(sc.names, ft[1])}] = true;
  }
  if (a.has("partition")) {  // TestSettings.partition: network off, links inside each group on
    st.networkActive = false;
    for (auto& group : split(a.get("partition"), '|')) {
      auto members = split(group, ',');
      for (auto& x : members)
        for (auto& y : members)
          if (x != y) st.linkActive[{addrOf(sc.names, x), addrOf(sc.names, y)}] = true;
    }
  }
  return st;
}

static void printTerminal(const Terminal& t, const Names& names, bool printStates) {
  std::cout << "{\"kind\":\"" << endName(t.kind) << "\",\"depth\":" << t.state->depth << ",\"predicate\":\""
            << jsonEsc(t.predicate) << "\",\"detail\":\"" << jsonEsc(t.detail) << "\",\"trace\":[";
  auto tr = trace(t.state);
  bool first = true;
  for (auto& s : tr) {
    if (!s->previousEvent) continue;
    std::cout << (first ? "" : ",") << "\"" << jsonEsc(eventStr(*s->previousEvent, names)) << "\"";
    first = false;
  }
  std::cout << "]";
  if (printStates) {
    std::cout << ",\"state\":\"" << jsonEsc(t.state->key()) << "\"";
  }
  std::cout << "}";
}

// --start-trace FILE: replay the events (one per line, unfiltered) from the initial state and
// start the search there (bfs(goalStateOfAnEarlierSearch), e.g. PaxosTest.java:898-910); lines
// starting with '#' apply dropPendingMessages / undropMessages* to the state reached so far
// (PaxosTest.java:1065, :1092, :1132).
static std::shared_ptr<const State> replayStart(const Args& a, Scenario& sc) {
  std::shared_ptr<const State> s = sc.init;
  if (!a.has("start-trace")) return s;
  Settings all;  // events are matched without delivery filters
  std::ifstream in(a.get("start-trace"));
  std::string line;
  auto addrOf = [&](const std::string& n) {
    for (size_t i = 0; i < sc.names.addr.size(); i++)
      if (sc.names.addr[i] == n) return (int)i;
    throw std::runtime_error("unknown address " + n);
  };
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    // state operations between searches (SearchState.java:538-561): "#DROP" = dropPendingMessages,
    // "#UNDROP" / "#UNDROP_FROM a" / "#UNDROP_TO a" = undropMessages / ...From / ...To
    if (line[0] == '#') {
      auto ns = std::make_shared<State>(*s);
      if (line == "#DROP") {
        ns->dropped.insert(ns->network.begin(), ns->network.end());
        ns->network.clear();
      } else {
        const bool from = line.rfind("#UNDROP_FROM ", 0) == 0, to = line.rfind("#UNDROP_TO ", 0) == 0;
        if (!from && !to && line != "#UNDROP") throw std::runtime_error("unknown start-trace directive " + line);
        const int x = (from || to) ? addrOf(line.substr(line.find(' ') + 1)) : -1;
        for (auto& m : ns->dropped)
          if ((!from || m.from == x) && (!to || m.to == x)) ns->network.insert(m);
      }
      s = ns;
      continue;
    }
    bool found = false;
    for (auto& ev : events(*s, all))
      if (eventStr(ev, sc.names) == line) {
        s = stepEvent(s, ev);
        found = true;
        break;
      }
    if (!found) throw std::runtime_error("start trace event not enabled: " + line);
  }
  auto fresh = std::make_shared<State>(*s);  // the start state keeps its depth
  return fresh;
}

static int runBfs(const Args& a) {
  Scenario sc = build(a);
  Settings st = settingsFrom(a, sc);
  std::shared_ptr<const State> start = replayStart(a, sc);
  int reps = a.geti("repeat", 1);
  Results R;
  for (int r = 0; r < reps; r++) R = bfs(start, st, a.has("finish-level"), a.has("max-secs") ? std::stod(a.get("max-secs")) : -1);
  std::cout << "{\"end\":\"" << endName(R.end) << "\",\"states\":" << R.states << ",\"max_depth\":" << R.maxDepth
            << ",\"successors\":" << R.successorsGenerated << ",\"elapsed_s\":" << R.elapsed << ",\"per_depth\":[";
  for (size_t d = 0; d < R.perDepth.size(); d++) std::cout << (d ? "," : "") << R.perDepth[d];
  std::cout << "],\"terminals\":[";
  size_t lim = std::min<size_t>(R.terminals.size(), (size_t)a.geti("max-terminals", 64));
  for (size_t i = 0; i < lim; i++) {
    if (i) std::cout << ",";
    printTerminal(R.terminals[i], sc.names, a.has("print-states"));
  }
  std::cout << "],\"num_terminals\":" << R.terminals.size() << "}" << std::endl;
  return 0;
}

// Replays a list of event strings from the initial state (TraceReplaySearch.java:76-101 /
// stepEvent(skipChecks=false): every event must be enabled in the state it is applied to).
// ViewServerTest (labs/lab2-primarybackup/tst/dslabs/primarybackup/ViewServerTest.java:156-303)
// replayed against the oracle's ViewServer: the reference's own known-answer tests for the view
// service. Addresses: 0 = viewserver, 1..3 = server1..3, 9 = the test client.
static int runVsTest(const Args&) {
  using namespace pb;
  struct Harness {
    std::shared_ptr<ViewServer> vs = std::make_shared<ViewServer>();
    std::vector<TimerEnv> timers;
    bool ok = true;
    std::string why;
    Harness() {
      Ctx c{0, {}, {}};
      vs->init(c);
      timers = c.timers;
    }
    void ping(int n, int from) {
      Ctx c{0, {}, {}};
      vs->handleMessage(Rec{"Ping", {std::to_string(n)}}, from, 0, c);
    }
    void timeout() {
      if (timers.empty()) { ok = false; why = "no timer"; return; }
      TimerEnv t = timers.front();
      timers.erase(timers.begin());
      Ctx c{0, {}, {}};
      vs->onTimer(t.t, c);
      for (auto& x : c.timers) timers.push_back(x);
    }
    View get() {
      Ctx c{0, {}, {}};
      vs->handleMessage(Rec{"GetView", {}}, 9, 0, c);
      return View::parse(c.sent.back().m.f[0]);
    }
    void check(int p, int b, int n) {
      View v = get();
      if (v.primary != p || v.backup != b || (n >= 0 && v.num != n)) {
        if (ok) why = "expected (" + std::to_string(n) + "," + std::to_string(p) + "," + std::to_string(b) + ") got " + v.str();
        ok = false;
      }
    }
    void setup(int p, int b, bool ack) {
      ping(STARTUP_VIEWNUM, p);
      check(p, -1, INITIAL_VIEWNUM);
      if (b >= 0) {
        ping(INITIAL_VIEWNUM, p);
        ping(STARTUP_VIEWNUM, b);
        check(p, b, INITIAL_VIEWNUM + 1);
      }
      if (ack) ping(b < 0 ? INITIAL_VIEWNUM : INITIAL_VIEWNUM + 1, p);
    }
    void timeoutFully(std::vector<int> pingers) {
      View cur = get();
      for (int i = 0; i < 2; i++) {
        for (int x : pingers) ping(cur.num, x);
        timeout();
      }
    }
  };
  std::vector<std::pair<std::string, std::function<void(Harness&)>>> tests = {
      {"test01StartupViewCorrect", [](Harness& h) { h.check(-1, -1, STARTUP_VIEWNUM); }},
      {"test02firstPrimary", [](Harness& h) { h.setup(1, -1, false); }},
      {"test03FirstBackup", [](Harness& h) { h.setup(1, 2, false); }},
      {"test04BackupPingsFirst", [](Harness& h) {
         h.setup(1, -1, false); h.ping(STARTUP_VIEWNUM, 2); h.ping(INITIAL_VIEWNUM, 1);
         h.check(1, 2, INITIAL_VIEWNUM + 1); }},
      {"test05BackupTakesOver", [](Harness& h) {
         h.setup(1, 2, true);
         h.ping(INITIAL_VIEWNUM + 1, 2); h.check(1, 2, INITIAL_VIEWNUM + 1); h.timeout();
         h.ping(INITIAL_VIEWNUM + 1, 2); h.check(1, 2, INITIAL_VIEWNUM + 1); h.timeout();
         h.check(2, -1, INITIAL_VIEWNUM + 2); }},
      {"test06OldServerBecomesBackup", [](Harness& h) {
         h.setup(1, 2, true); h.timeoutFully({2}); h.check(2, -1, INITIAL_VIEWNUM + 2);
         h.ping(INITIAL_VIEWNUM + 2, 2); h.ping(INITIAL_VIEWNUM + 1, 1); h.check(2, 1, INITIAL_VIEWNUM + 3); }},
      {"test07IdleThirdServerBecomesBackup", [](Harness& h) {
         h.setup(1, 2, true); h.timeoutFully({2, 3}); h.check(2, 3, INITIAL_VIEWNUM + 2); }},
      {"test08WaitForPrimaryAck", [](Harness& h) {
         h.ping(STARTUP_VIEWNUM, 1); h.ping(STARTUP_VIEWNUM, 2); h.check(1, -1, INITIAL_VIEWNUM);
         h.ping(INITIAL_VIEWNUM, 1); h.check(1, 2, INITIAL_VIEWNUM + 1); h.ping(INITIAL_VIEWNUM, 2);
         h.timeoutFully({2}); h.check(1, 2, INITIAL_VIEWNUM + 1); }},
      {"test09DeadBackupRemoved", [](Harness& h) {
         h.setup(1, 2, true); h.timeoutFully({1}); h.check(1, -1, INITIAL_VIEWNUM + 2); }},
      {"test10UninitializedNotPromoted", [](Harness& h) {
         h.setup(1, 2, true); h.timeoutFully({2, 3}); h.check(2, 3, INITIAL_VIEWNUM + 2);
         h.timeoutFully({3}); h.check(2, 3, INITIAL_VIEWNUM + 2); }},
      {"test11DeadServerNotMadeBackup", [](Harness& h) {
         h.setup(1, -1, false); h.ping(STARTUP_VIEWNUM, 2); h.timeoutFully({}); h.ping(INITIAL_VIEWNUM, 1);
         h.check(1, -1, INITIAL_VIEWNUM); }},
      {"test12NewViewNotStarted", [](Harness& h) {
         h.setup(1, -1, false); h.timeoutFully({1}); h.check(1, -1, INITIAL_VIEWNUM);
         h.timeoutFully({}); h.check(1, -1, INITIAL_VIEWNUM); h.ping(INITIAL_VIEWNUM, 1);
         h.timeoutFully({1}); h.check(1, -1, INITIAL_VIEWNUM); h.timeoutFully({}); h.check(1, -1, INITIAL_VIEWNUM);
         h.ping(STARTUP_VIEWNUM, 2); h.check(1, 2, INITIAL_VIEWNUM + 1); h.ping(INITIAL_VIEWNUM + 1, 1);
         h.check(1, 2, INITIAL_VIEWNUM + 1); h.timeoutFully({1, 2}); h.check(1, 2, INITIAL_VIEWNUM + 1);
         h.timeoutFully({});
         View v = h.get();
         if (v.primary == 1 && v.backup == 2 && v.num != INITIAL_VIEWNUM + 1) h.ok = false; }},
  };
  std::cout << "{\"results\":[";
  for (size_t i = 0; i < tests.size(); i++) {
    Harness h;
    tests[i].second(h);
    std::cout << (i ? "," : "") << "{\"name\":\"" << tests[i].first << "\",\"ok\":" << (h.ok ? "true" : "false")
              << ",\"why\":\"" << jsonEsc(h.why) << "\"}";
  }
  std::cout << "]}" << std::endl;
  return 0;
}

static int runReplay(const Args& a) {
  Scenario sc = build(a);
  Settings st = settingsFrom(a, sc);
  std::ifstream in(a.get("trace-file"));
  std::string line;
  std::shared_ptr<const State> s = replayStart(a, sc);  // --start-trace: an earlier search's state
  int step = 0;
  bool ok = true;
  std::string err;
  auto addrOf = [&](const std::string& n) {
    for (size_t i = 0; i < sc.names.addr.size(); i++)
      if (sc.names.addr[i] == n) return (int)i;
    throw std::runtime_error("unknown address " + n);
  };
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    // state operations between searches (SearchState.java:538-561): "#DROP" = dropPendingMessages,
    // "#UNDROP" / "#UNDROP_FROM a" / "#UNDROP_TO a" = undropMessages / ...From / ...To
    if (line[0] == '#') {
      auto ns = std::make_shared<State>(*s);
      if (line == "#DROP") {
        ns->dropped.insert(ns->network.begin(), ns->network.end());
        ns->network.clear();
      } else {
        const bool from = line.rfind("#UNDROP_FROM ", 0) == 0, to = line.rfind("#UNDROP_TO ", 0) == 0;
        if (!from && !to && line != "#UNDROP") throw std::runtime_error("unknown start-trace directive " + line);
        const int x = (from || to) ? addrOf(line.substr(line.find(' ') + 1)) : -1;
        for (auto& m : ns->dropped)
          if ((!from || m.from == x) && (!to || m.to == x)) ns->network.insert(m);
      }
      s = ns;
      continue;
    }
    bool found = false;
    for (auto& ev : events(*s, st)) {
      if (eventStr(ev, sc.names) == line) {
        s = stepEvent(s, ev);
        found = true;
        break;
      }
    }
    if (!found) {
      ok = false;
      err = "event " + std::to_string(step) + " not enabled: " + line;
      break;
    }
    step++;
  }
  std::cout << "{\"ok\":" << (ok ? "true" : "false") << ",\"error\":\"" << jsonEsc(err) << "\",\"depth\":" << s->depth
            << ",\"exception\":" << (s->exception ? "true" : "false") << ",\"invariants\":[";
  bool first = true;
  for (auto& p : st.invariants) {
    PredResult r = p.test(*s);
    std::cout << (first ? "" : ",") << "{\"name\":\"" << jsonEsc(p.name) << "\",\"value\":" << (r.value ? "true" : "false")
              << ",\"threw\":" << (r.threw ? "true" : "false") << ",\"detail\":\"" << jsonEsc(r.detail) << "\"}";
    first = false;
  }
  std::cout << "],\"goals\":[";
  first = true;
  for (auto& p : st.goals) {
    PredResult r = p.test(*s);
    std::cout << (first ? "" : ",") << "{\"name\":\"" << jsonEsc(p.name) << "\",\"value\":" << (r.value ? "true" : "false")
              << ",\"threw\":" << (r.threw ? "true" : "false") << "}";
    first = false;
  }
  std::cout << "],\"state\":\"" << jsonEsc(s->key()) << "\"}" << std::endl;
  return 0;
}

// Trace-replay search (TraceReplaySearch.java:76-101 / ReplaySearch): replays the trace's events
// with checkState after every step; --minimize runs TraceMinimizer on a terminal
// (Search.checkState(s, true)). An event string names a message in the network or a queued timer;
// one that names neither, or cannot be delivered, ends the replay (SPACE_EXHAUSTED).
static int runReplaySearch(const Args& a) {
  Scenario sc = build(a);
  Settings st = settingsFrom(a, sc);
  std::shared_ptr<const State> s0 = replayStart(a, sc);
  std::vector<std::string> lines;
  {
    std::ifstream in(a.get("trace-file"));
    std::string line;
    while (std::getline(in, line))
      if (!line.empty()) lines.push_back(line);
  }
  // events are resolved against the state each one is applied to, on an unfiltered replay
  std::vector<Event> evs;
  std::shared_ptr<const State> s = s0;
  for (auto& line : lines) {
    std::optional<Event> found;
    for (auto& m : s->network) {
      Event e;
      e.msg = m;
      if (eventStr(e, sc.names) == line) found = e;
    }
    for (size_t n = 0; n < s->timers.size() && !found; n++)
      for (auto& t : s->timers[n].timers) {
        Event e;
        e.isTimer = true;
        e.timer = t;
        if (eventStr(e, sc.names) == line) found = e;
      }
    if (!found) break;
    evs.push_back(*found);
    auto n = stepChecked(s, *found, nullptr);
    if (!n) break;
    s = n;
  }
  ReplayOutcome R = replaySearch(s0, st, evs, a.has("minimize"));
  if (a.has("human-readable")) R.state = humanReadableTrace(R.state);
  std::cout << "{\"end\":\"" << endName(R.end) << "\",\"depth\":" << R.state->depth << ",\"predicate_index\":"
            << R.predIndex << ",\"predicate\":\"" << jsonEsc(R.predicate) << "\",\"trace\":[";
  bool first = true;
  for (auto& x : trace(R.state)) {
    if (!x->previousEvent || x->depth <= s0->depth) continue;
    std::cout << (first ? "" : ",") << "\"" << jsonEsc(eventStr(*x->previousEvent, sc.names)) << "\"";
    first = false;
  }
  std::cout << "],\"state\":\"" << jsonEsc(R.state->key()) << "\"}" << std::endl;
  return 0;
}

// TimerQueueTest.randomTimers (framework/tst-self/.../search/TimerQueueTest.java:153-175) as a
// truth table: for te1=(i,j), te2=(k,l) added in order, is te2 deliverable?
static int runTimerQueue() {
  std::cout << "{\"cases\":[";
  bool first = true;
  for (int i = 1; i <= 4; i++)
    for (int j = i; j <= 4; j++)
      for (int k = 1; k <= 4; k++)
        for (int l = k; l <= 4; l++) {
          TimerQueue tq;
          TimerEnv t1{1, Rec{"T", {}}, i, j}, t2{2, Rec{"T", {}}, k, l};
          tq.add(t1);
          tq.add(t2);
          auto d = tq.deliverable();
          bool d1 = std::find(d.begin(), d.end(), t1) != d.end() && tq.isDeliverable(t1);
          bool d2l = std::find(d.begin(), d.end(), t2) != d.end();
          bool d2i = tq.isDeliverable(t2);
          std::cout << (first ? "" : ",") << "[" << i << "," << j << "," << k << "," << l << "," << d1 << "," << d2l
                    << "," << d2i << "]";
          first = false;
        }
  std::cout << "]}" << std::endl;
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::cerr << "usage: dslabs_oracle bfs|replay|timerqueue [--opts]\n";
    return 2;
  }
  Args a;
  a.mode = argv[1];
  for (int i = 2; i < argc; i++) {
    std::string k = argv[i];
    if (k.rfind("--", 0) != 0) {
      std::cerr << "bad arg " << k << "\n";
      return 2;
    }
    k = k.substr(2);
    std::string v = "1";
    if (i + 1 < argc && std::strncmp(argv[i + 1], "--", 2) != 0) v = argv[++i];
    a.kv[k].push_back(v);
  }
  a.proto = a.get("proto", "pingpong");
  try {
    if (a.mode == "bfs") return runBfs(a);
    if (a.mode == "replay") return runReplay(a);
    if (a.mode == "replaysearch") return runReplaySearch(a);
    if (a.mode == "vstest") return runVsTest(a);
    if (a.mode == "timerqueue") return runTimerQueue();
  } catch (const std::exception& e) {
    std::cout << "{\"error\":\"" << jsonEsc(e.what()) << "\"}" << std::endl;
    return 1;
  } catch (const Overflow& o) {
    std::cout << "{\"error\":\"overflow: " << jsonEsc(o.msg) << "\"}" << std::endl;
    return 3;
  }
  std::cerr << "unknown mode\n";
  return 2;
}
