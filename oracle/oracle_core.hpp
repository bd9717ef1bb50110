// oracle/oracle_core.hpp -- TEST INFRASTRUCTURE ONLY.
//
// A plain-C++ restatement of the DSLabs search semantics (Jay686/dslabs, read-only at
// /root/reference) used as the parity ORACLE for the MI355X engine. Only tests/, the
// smoke() check in __graft_entry__.py and bench.py's cpu_baseline leg may run it; the
// product path (dslabs_amd/, libdslabs_hip.so) never links, loads or calls it.
//
// The restatement is deliberately written against Java-like object semantics (strings,
// std::set / std::map, copy-on-write node objects, canonical-key equality) and shares no
// code or encoding with the GPU engine's packed states, so agreement between the two is
// evidence, not tautology.
//
// Reference sections followed (paths relative to /root/reference,
// T = framework/tst/dslabs/framework/testing):
//   T/search/Search.java:162-231   checkState order (exception > invariant > goal > prune > depth)
//   T/search/Search.java:233-388   run() / end-condition priority
//   T/search/Search.java:405-505   BFS: counting rules, FIFO levels, TERMINAL -> return
//   T/search/SearchState.java:108-122, 189-224  successor construction, send/broadcast/set capture
//   T/search/SearchState.java:226-252  events(): network (shouldDeliver) then deliverable timers
//   T/search/SearchState.java:282-303, 336-359  stepMessage (message stays), stepTimer (remove after)
//   T/search/SearchState.java:575-619  search-equivalence wrapper (exception / dropped network)
//   T/search/TimerQueue.java:45-134     deliverable(), isDeliverable(), remove(first equal)
//   T/TestSettings.java:76-94, 130-138, 224-245  timer masks, invariants, shouldDeliver precedence
//   T/search/SearchSettings.java:77-135  prunes (throwing prunes), goals (throwing ignored)
//   T/ClientWorker.java:49-297          ClientWorker equality {client, results}, command loop
//   T/Workload.java:112-349             "%i" replacement (1-based), numTimes repetition
//   F = framework/src/dslabs/framework/Node.java:190-352  send/broadcast/set (set rejects min<1, min>max)
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_set>
#include <vector>

namespace oracle {

// ---------------------------------------------------------------------------------------------
// Values: messages, timers, commands and results are "records": a type name plus string fields.
// Equality / ordering is field-wise, like Lombok @Data (the ordering is only for std::set).
// ---------------------------------------------------------------------------------------------
struct Rec {
  std::string type;
  std::vector<std::string> f;
  bool operator<(const Rec& o) const { return type != o.type ? type < o.type : f < o.f; }
  bool operator==(const Rec& o) const { return type == o.type && f == o.f; }
  bool operator!=(const Rec& o) const { return !(*this == o); }
  std::string str() const {
    std::string s = type + "(";
    for (size_t i = 0; i < f.size(); i++) s += (i ? ", " : "") + f[i];
    return s + ")";
  }
};

struct Envelope {  // MessageEnvelope record {from, to, message}
  int from, to;
  Rec m;
  bool operator<(const Envelope& o) const {
    if (from != o.from) return from < o.from;
    if (to != o.to) return to < o.to;
    return m < o.m;
  }
  bool operator==(const Envelope& o) const { return from == o.from && to == o.to && m == o.m; }
};

struct TimerEnv {  // TimerEnvelope, equality {to, timer, min, max} (TimerEnvelope.java:40)
  int to;
  Rec t;
  int min, max;
  bool operator==(const TimerEnv& o) const {
    return to == o.to && t == o.t && min == o.min && max == o.max;
  }
};

// A bounded container of a restated protocol overflowed: a hard error of the oracle run (the
// engine reports DSL_ERR_STATE_OVERFLOW for the same situation). Deliberately NOT a
// std::exception, so stepEvent does not capture it as a handler exception.
struct Overflow {
  std::string msg;
};

// Exceptions thrown by handlers (captured into the state, SearchState.java:218-222).
struct HandlerException : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ---------------------------------------------------------------------------------------------
// TimerQueue (TimerQueue.java:45-134): ordered list, list equality.
// ---------------------------------------------------------------------------------------------
struct TimerQueue {
  std::vector<TimerEnv> timers;
  void add(const TimerEnv& t) { timers.push_back(t); }
  // deliverable(): yield in order; after yielding t, minMax = min(minMax, t.max); skip entries
  // with min >= minMax.
  std::vector<TimerEnv> deliverable() const {
    std::vector<TimerEnv> out;
    std::optional<int> minMax;
    size_t i = 0;
    while (i < timers.size()) {
      const TimerEnv& n = timers[i++];
      if (!minMax || n.max < *minMax) minMax = n.max;
      out.push_back(n);
      while (i < timers.size() && minMax && timers[i].min >= *minMax) i++;
    }
    return out;
  }
  bool isDeliverable(const TimerEnv& te) const {
    for (const auto& t : timers) {
      if (t == te) return true;
      if (te.min >= t.max) return false;
    }
    return false;
  }
  void remove(const TimerEnv& te) {  // removes the FIRST equal entry (List.remove(Object))
    for (size_t i = 0; i < timers.size(); i++)
      if (timers[i] == te) {
        timers.erase(timers.begin() + i);
        return;
      }
  }
};

// ---------------------------------------------------------------------------------------------
// Handler context: captures send / broadcast / set like SearchState.configNode.
// ---------------------------------------------------------------------------------------------
struct Ctx {
  int self;
  std::vector<Envelope> sent;
  std::vector<TimerEnv> timers;
  void send(const Rec& m, int to) { sent.push_back({self, to, m}); }
  void broadcast(const Rec& m, const std::vector<int>& to) {
    for (int a : to) sent.push_back({self, a, m});
  }
  void set(const Rec& t, int ms) { set(t, ms, ms); }
  void set(const Rec& t, int mn, int mx) {
    if (mn > mx) throw HandlerException("Minimum timer length greater than maximum timer length");
    if (mn < 1) throw HandlerException("Minimum timer length < 1ms");
    timers.push_back({self, t, mn, mx});
  }
};

struct Node {
  virtual ~Node() = default;
  virtual std::shared_ptr<Node> clone() const = 0;
  // Canonical key of the fields that take part in Lombok equality (address excluded).
  virtual void key(std::string& out) const = 0;
  virtual std::string str() const = 0;
  virtual void init(Ctx&) {}
  virtual void handleMessage(const Rec& m, int from, int to, Ctx& ctx) = 0;
  virtual void onTimer(const Rec& t, Ctx& ctx) = 0;
};

struct Client : Node {
  virtual void sendCommand(const Rec& cmd, Ctx& ctx) = 0;
  virtual bool hasResult() const = 0;
  virtual Rec getResult() const = 0;
};

// Workload.StandardWorkload with command/result strings and "%i" (1-based) replacement.
struct Workload {
  std::vector<std::string> cmds, results;  // templates
  int numTimes = 1;
  int i = 0;
  std::function<std::pair<Rec, Rec>(const std::string&, const std::string&)> parser;
  bool hasNext() const { return i < (int)cmds.size() * numTimes; }
  bool hasResults() const { return cmds.size() == results.size(); }
  static std::string replace(const std::string& s, int idx, const std::string& addr) {
    std::string out;
    for (size_t k = 0; k < s.size(); k++) {
      if (s[k] == '%' && k + 1 < s.size() && s[k + 1] == 'i') {
        out += std::to_string(idx);
        k++;
      } else if (s[k] == '%' && k + 1 < s.size() && s[k + 1] == 'a') {
        out += addr;
        k++;
      } else {
        out += s[k];
      }
    }
    return out;
  }
  std::pair<Rec, Rec> next(const std::string& addr) {
    if (!hasNext()) throw HandlerException("Workload finished.");
    int index = i % (int)cmds.size();
    std::string c = replace(cmds[index], i + 1, addr);
    std::string r = hasResults() ? replace(results[index], i + 1, addr) : std::string();
    i++;
    return parser(c, r);
  }
};

// ClientWorker (ClientWorker.java): equality is ONLY {client, results}.
struct ClientWorker : Node {
  std::shared_ptr<Client> client;
  Workload workload;
  std::string addrName;
  bool initialized = false, waitingOnResult = false;
  std::optional<Rec> lastCommand, expectedResult;
  std::vector<Rec> results;
  bool resultsOk = true;
  std::optional<std::pair<Rec, Rec>> expectedAndReceived;

  std::shared_ptr<Node> clone() const override {
    auto c = std::make_shared<ClientWorker>(*this);
    c->client = std::static_pointer_cast<Client>(client->clone());
    return c;
  }
  void key(std::string& out) const override {
    out += "CW{";
    client->key(out);
    out += "|R[";
    for (auto& r : results) out += r.str() + ",";
    out += "]}";
  }
  std::string str() const override {
    std::string s = "ClientWorker(client=" + client->str() + ", results=[";
    for (size_t k = 0; k < results.size(); k++) s += (k ? ", " : "") + results[k].str();
    return s + "])";
  }
  bool done() const { return !waitingOnResult && !workload.hasNext(); }
  void sendNextCommandWhilePossible(Ctx& ctx) {
    if (!initialized) return;
    while (true) {
      if (waitingOnResult && client->hasResult()) {
        Rec result = client->getResult();
        results.push_back(result);
        if (workload.hasResults() && !(expectedResult && *expectedResult == result)) {
          resultsOk = false;
          if (!expectedAndReceived) expectedAndReceived = std::make_pair(*expectedResult, result);
        }
        waitingOnResult = false;
        lastCommand.reset();
        expectedResult.reset();
      }
      if (waitingOnResult || !workload.hasNext()) break;
      auto cr = workload.next(addrName);
      lastCommand = cr.first;
      expectedResult = cr.second;
      client->sendCommand(cr.first, ctx);
      waitingOnResult = true;
    }
  }
  void init(Ctx& ctx) override {
    initialized = true;
    client->init(ctx);
    sendNextCommandWhilePossible(ctx);
  }
  void handleMessage(const Rec& m, int from, int to, Ctx& ctx) override {
    client->handleMessage(m, from, to, ctx);
    sendNextCommandWhilePossible(ctx);
  }
  void onTimer(const Rec& t, Ctx& ctx) override {
    client->onTimer(t, ctx);
    sendNextCommandWhilePossible(ctx);
  }
};

// ---------------------------------------------------------------------------------------------
// Search state (SearchState.java / AbstractState.java).
// ---------------------------------------------------------------------------------------------
enum class Kind { Server, ClientWorker };

struct Event {
  bool isTimer = false;
  Envelope msg{};
  TimerEnv timer{};
};

struct Names {
  std::vector<std::string> addr;  // address index -> name
};

struct State {
  std::vector<std::shared_ptr<Node>> nodes;  // index = address
  std::vector<Kind> kinds;
  std::set<Envelope> network, dropped;
  std::vector<TimerQueue> timers;
  int depth = 0;
  bool exception = false;
  std::string exceptionMsg;
  uint64_t exceptionId = 0;  // Throwable identity: exceptional states never merge
  std::shared_ptr<const State> previous;
  std::optional<Event> previousEvent;
  std::vector<Envelope> newMessages;  // every send of the step that made this state (SearchState.newMessages)

  const ClientWorker* cw(int a) const { return dynamic_cast<const ClientWorker*>(nodes[a].get()); }
  std::vector<int> clientWorkers() const {
    std::vector<int> v;
    for (size_t a = 0; a < nodes.size(); a++)
      if (kinds[a] == Kind::ClientWorker) v.push_back((int)a);
    return v;
  }
  // Search-equivalence key (SearchState.java:575-619 + AbstractState/SearchState equality):
  // SearchState equality plus Throwable identity.
  std::string key() const {
    std::string k = contentKey();
    if (exception) k += "EXC#" + std::to_string(exceptionId);
    return k;
  }
  // SearchState.equals (nodes, network, timers; thrownException is transient, SearchState.java:67-89)
  std::string contentKey() const {
    std::string k;
    for (size_t a = 0; a < nodes.size(); a++) {
      k += "N" + std::to_string(a) + ":";
      nodes[a]->key(k);
      k += ";";
    }
    k += "NET{";
    std::set<Envelope> u = network;
    u.insert(dropped.begin(), dropped.end());
    for (auto& e : u) k += std::to_string(e.from) + ">" + std::to_string(e.to) + ":" + e.m.str() + ",";
    k += "}T{";
    for (size_t a = 0; a < timers.size(); a++) {
      k += std::to_string(a) + "[";
      for (auto& t : timers[a].timers)
        k += t.t.str() + "/" + std::to_string(t.min) + "/" + std::to_string(t.max) + ",";
      k += "]";
    }
    k += "}";
    if (!dropped.empty()) {
      k += "UNDROPPED{";
      for (auto& e : network) k += std::to_string(e.from) + ">" + std::to_string(e.to) + ":" + e.m.str() + ",";
      k += "}";
    }
    return k;
  }
};

inline std::string eventStr(const Event& e, const Names& n) {
  if (e.isTimer) return "Timer(-> " + n.addr[e.timer.to] + ", " + e.timer.t.str() + ")";
  return "Message(" + n.addr[e.msg.from] + " -> " + n.addr[e.msg.to] + ", " + e.msg.m.str() + ")";
}

// ---------------------------------------------------------------------------------------------
// Settings (TestSettings / SearchSettings).
// ---------------------------------------------------------------------------------------------
struct PredResult {
  bool threw = false;
  bool value = true;
  std::string detail;
};
struct Predicate {
  std::string name;
  std::function<PredResult(const State&)> fn;
  PredResult test(const State& s) const {
    try {
      return fn(s);
    } catch (const std::exception& e) {
      PredResult r;
      r.threw = true;
      r.detail = e.what();
      return r;
    }
  }
  Predicate negate() const {
    Predicate p;
    p.name = "¬(" + name + ")";
    auto f = fn;
    p.fn = [f](const State& s) {
      PredResult r = f(s);
      r.value = !r.value;
      return r;
    };
    return p;
  }
  // StatePredicate.and / or / implies (StatePredicate.java:397-431): the operands' functions are
  // applied directly, so an exception in an evaluated operand propagates (the right operand is
  // evaluated only when the left one does not decide).
  Predicate and_(const Predicate& o) const {
    Predicate p;
    p.name = "(" + name + ") ∧ (" + o.name + ")";
    auto f = fn, g = o.fn;
    p.fn = [f, g](const State& s) {
      PredResult r1 = f(s);
      if (!r1.value) return r1;
      PredResult r2 = g(s);
      if (!r2.value) return r2;
      PredResult r;
      r.detail = "(" + r1.detail + ") and (" + r2.detail + ")";
      return r;
    };
    return p;
  }
  Predicate or_(const Predicate& o) const {
    Predicate p;
    p.name = "(" + name + ") ∨ (" + o.name + ")";
    auto f = fn, g = o.fn;
    p.fn = [f, g](const State& s) {
      PredResult r1 = f(s);
      if (r1.value) return r1;
      PredResult r2 = g(s);
      if (r2.value) return r2;
      PredResult r;
      r.value = false;
      r.detail = "(" + r1.detail + ") or (" + r2.detail + ")";
      return r;
    };
    return p;
  }
  Predicate implies(const Predicate& o) const {
    Predicate p = negate().or_(o);
    p.name = "(" + name + ") → (" + o.name + ")";
    return p;
  }
};

struct Settings {
  std::vector<Predicate> invariants, goals, prunes;
  int maxDepth = -1;
  bool networkActive = true;
  std::map<std::pair<int, int>, bool> linkActive;
  std::map<int, bool> senderActive, receiverActive;
  bool deliverTimersDefault = true;
  std::map<int, bool> timersActive;

  bool deliverTimers(int a) const {
    auto it = timersActive.find(a);
    return it == timersActive.end() ? deliverTimersDefault : it->second;
  }
  // TestSettings.shouldDeliver precedence: self-send, link, sender, receiver, network.
  bool shouldDeliver(const Envelope& e) const {
    if (e.from == e.to) return true;
    auto l = linkActive.find({e.from, e.to});
    if (l != linkActive.end()) return l->second;
    auto s = senderActive.find(e.from);
    if (s != senderActive.end()) return s->second;
    auto r = receiverActive.find(e.to);
    if (r != receiverActive.end()) return r->second;
    return networkActive;
  }
};

// ---------------------------------------------------------------------------------------------
// Stepping (SearchState.events / stepMessage / stepTimer).
// ---------------------------------------------------------------------------------------------
inline uint64_t& exceptionCounter() {
  static uint64_t c = 0;
  return c;
}

inline std::vector<Event> events(const State& s, const Settings& st) {
  std::vector<Event> ev;
  for (auto& m : s.network)
    if (m.to < (int)s.nodes.size() && st.shouldDeliver(m)) {
      Event e;
      e.msg = m;
      ev.push_back(e);
    }
  for (size_t a = 0; a < s.nodes.size(); a++)
    if (st.deliverTimers((int)a))
      for (auto& t : s.timers[a].deliverable()) {
        Event e;
        e.isTimer = true;
        e.timer = t;
        ev.push_back(e);
      }
  return ev;
}

inline void applyCtx(State& ns, const Ctx& ctx) {
  ns.newMessages = ctx.sent;
  for (auto& e : ctx.sent) ns.network.insert(e);
  for (auto& t : ctx.timers) ns.timers[t.to].add(t);
}

inline std::shared_ptr<State> successor(const std::shared_ptr<const State>& s, int addr, const Event& ev) {
  auto ns = std::make_shared<State>(*s);  // copies maps / sets; node pointers are shared (COW)
  ns->previous = s;
  ns->previousEvent = ev;
  ns->depth = s->depth + 1;
  ns->nodes[addr] = s->nodes[addr]->clone();
  return ns;
}

inline std::shared_ptr<State> stepEvent(const std::shared_ptr<const State>& s, const Event& ev) {
  int to = ev.isTimer ? ev.timer.to : ev.msg.to;
  if (to < 0 || to >= (int)s->nodes.size()) return nullptr;
  auto ns = successor(s, to, ev);
  Ctx ctx{to, {}, {}};
  try {
    if (ev.isTimer)
      ns->nodes[to]->onTimer(ev.timer.t, ctx);
    else
      ns->nodes[to]->handleMessage(ev.msg.m, ev.msg.from, ev.msg.to, ctx);
    applyCtx(*ns, ctx);
  } catch (const std::exception& e) {
    applyCtx(*ns, ctx);
    ns->exception = true;
    ns->exceptionMsg = e.what();
    ns->exceptionId = ++exceptionCounter();
  }
  if (ev.isTimer) ns->timers[to].remove(ev.timer);  // AFTER the handler (SearchState.java:357)
  return ns;
}

// Builds an initial state: every node is added and init()-ed in address order
// (AbstractState.addServer / addClientWorker -> SearchState.setupNode).
inline std::shared_ptr<State> makeInitial(const std::vector<std::shared_ptr<Node>>& nodes,
                                          const std::vector<Kind>& kinds) {
  auto s = std::make_shared<State>();
  s->nodes = nodes;
  s->kinds = kinds;
  s->timers.resize(nodes.size());
  for (size_t a = 0; a < nodes.size(); a++) {
    Ctx ctx{(int)a, {}, {}};
    s->nodes[a]->init(ctx);
    applyCtx(*s, ctx);
  }
  return s;
}

// ---------------------------------------------------------------------------------------------
// BFS (Search.java:405-505 / checkState :162-231 / run :370-385).
// ---------------------------------------------------------------------------------------------
enum class Status { VALID, TERMINAL, PRUNED };
enum class End { EXCEPTION_THROWN, INVARIANT_VIOLATED, GOAL_FOUND, SPACE_EXHAUSTED, TIME_EXHAUSTED };
inline const char* endName(End e) {
  switch (e) {
    case End::EXCEPTION_THROWN: return "EXCEPTION_THROWN";
    case End::INVARIANT_VIOLATED: return "INVARIANT_VIOLATED";
    case End::GOAL_FOUND: return "GOAL_FOUND";
    case End::SPACE_EXHAUSTED: return "SPACE_EXHAUSTED";
    default: return "TIME_EXHAUSTED";
  }
}

struct Terminal {
  End kind;
  std::shared_ptr<const State> state;
  std::string predicate, detail;
};

struct Results {
  End end = End::SPACE_EXHAUSTED;
  uint64_t states = 0;
  int maxDepth = 0;
  std::vector<uint64_t> perDepth;  // unique states discovered per depth (initial state included)
  std::vector<Terminal> terminals;  // first = the one the reference would report first
  double elapsed = 0;
  uint64_t successorsGenerated = 0;
};

// finishLevel=false: exactly Search.java single-threaded (stop at the first TERMINAL state).
// finishLevel=true : after the first TERMINAL state at depth d, still generate every depth-d
//                    successor of the remaining depth-(d-1) states (nothing deeper), so the
//                    depth-d count is complete; this is the level-synchronous engine's rule.
inline Results bfs(std::shared_ptr<const State> init, const Settings& st, bool finishLevel,
                   double maxSecs = -1) {
  auto t0 = std::chrono::steady_clock::now();
  Results R;
  std::deque<std::shared_ptr<const State>> queue;
  std::unordered_set<std::string> discovered;
  queue.push_back(init);
  discovered.insert(init->key());
  int initialDepth = init->depth;
  R.maxDepth = init->depth;
  auto count = [&](int d) {
    if ((int)R.perDepth.size() <= d) R.perDepth.resize(d + 1, 0);
    R.perDepth[d]++;
    R.states++;
    R.maxDepth = std::max(R.maxDepth, d);
  };
  auto check = [&](const std::shared_ptr<const State>& s) -> Status {
    if (s->exception) {
      R.terminals.push_back({End::EXCEPTION_THROWN, s, "", s->exceptionMsg});
      return Status::TERMINAL;
    }
    for (auto& p : st.invariants) {
      PredResult r = p.test(*s);
      if (r.threw || !r.value) {
        R.terminals.push_back({End::INVARIANT_VIOLATED, s, p.name, r.detail});
        return Status::TERMINAL;
      }
    }
    for (auto& p : st.goals) {
      PredResult r = p.test(*s);
      if (r.threw) continue;
      if (r.value) {
        R.terminals.push_back({End::GOAL_FOUND, s, p.name, r.detail});
        return Status::TERMINAL;
      }
    }
    for (auto& p : st.prunes) {
      PredResult r = p.test(*s);
      if (r.threw || r.value) return Status::PRUNED;
    }
    if (st.maxDepth >= 0 && s->depth >= st.maxDepth) return Status::PRUNED;
    return Status::VALID;
  };

  int terminalDepth = -1;
  bool timeUp = false;
  while (!queue.empty()) {
    if (maxSecs > 0 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > maxSecs) {
      timeUp = true;
      break;
    }
    auto node = queue.front();
    if (terminalDepth >= 0 && (!finishLevel || node->depth + 1 > terminalDepth)) break;
    queue.pop_front();
    if (node->depth == initialDepth) {
      count(node->depth);
      if (check(node) == Status::TERMINAL) {
        terminalDepth = node->depth;
        break;
      }
    }
    for (auto& ev : events(*node, st)) {
      auto succ = stepEvent(node, ev);
      if (!succ) continue;
      R.successorsGenerated++;
      if (!discovered.insert(succ->key()).second) continue;
      count(succ->depth);
      Status stt = check(succ);
      if (stt == Status::TERMINAL) {
        if (terminalDepth < 0) terminalDepth = succ->depth;
        if (!finishLevel) break;
        continue;
      }
      if (stt == Status::PRUNED) continue;
      queue.push_back(succ);
    }
    if (terminalDepth >= 0 && !finishLevel) break;
  }
  R.elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (!R.terminals.empty()) {
    // End-condition priority (Search.java:370-385): EXCEPTION > INVARIANT > GOAL.
    End best = R.terminals[0].kind;
    for (auto& t : R.terminals) best = std::min(best, t.kind);
    R.end = best;
  } else {
    R.end = timeUp ? End::TIME_EXHAUSTED : End::SPACE_EXHAUSTED;
  }
  return R;
}

inline std::vector<std::shared_ptr<const State>> trace(std::shared_ptr<const State> s) {
  std::vector<std::shared_ptr<const State>> t;
  for (; s; s = s->previous) t.push_back(s);
  std::reverse(t.begin(), t.end());
  return t;
}

// ---------------------------------------------------------------------------------------------
// Trace minimization (TraceMinimizer.java:32-108) and trace-replay search
// (TraceReplaySearch.java:76-101, ReplaySearch in SearchAndTraceMinimizerTest.java:520-548, with
// Search.checkState(s, shouldMinimize), Search.java:162-231).
// ---------------------------------------------------------------------------------------------
// stepEvent(e, settings, skipChecks=false) (SearchState.java:282-303, :316-359): the message must
// be in the network and pass shouldDeliver / the timer must pass canStepTimer, else null.
// settings == nullptr: default SearchSettings (everything delivered), as TraceMinimizer uses.
inline std::shared_ptr<State> stepChecked(const std::shared_ptr<const State>& s, const Event& ev, const Settings* st) {
  if (ev.isTimer) {
    const int to = ev.timer.to;
    if (to < 0 || to >= (int)s->nodes.size()) return nullptr;
    if ((st && !st->deliverTimers(to)) || !s->timers[to].isDeliverable(ev.timer)) return nullptr;
  } else {
    if (ev.msg.to < 0 || ev.msg.to >= (int)s->nodes.size()) return nullptr;
    if (!s->network.count(ev.msg) || (st && !st->shouldDeliver(ev.msg))) return nullptr;
  }
  return stepEvent(s, ev);
}

// The result a minimized state must keep (TraceMinimizer.stateMatches :51-61): the same
// exception class (minimizeExceptionCausingTrace :70-91; every handler exception here is one
// class), or the predicate with the same value / again throwing.
struct Expected {
  bool exception = false;
  const Predicate* pred = nullptr;
  bool threw = false, value = false;
};

inline bool stateMatches(const State* s, const Expected& x) {
  if (!s) return false;
  if (x.exception) return s->exception;
  PredResult r = x.pred->test(*s);
  if (x.threw) return r.threw;
  return !r.threw && r.value == x.value;
}

// applyEvents (:93-108): steps until an event cannot be applied; returns the last state reached.
inline std::shared_ptr<const State> applyEvents(std::shared_ptr<const State> s, const std::deque<Event>& events) {
  for (auto& e : events) {
    auto n = stepChecked(s, e, nullptr);
    if (!n) break;
    s = n;
  }
  return s;
}

// minimizeTrace (:32-49): walking back from the end, drop an event when replaying the kept
// suffix from its predecessor still matches; repeat until a pass drops nothing.
inline std::shared_ptr<const State> minimizeTrace(std::shared_ptr<const State> state, const Expected& x) {
  bool shortened;
  do {
    shortened = false;
    std::deque<Event> events;
    for (auto s = state; s->previous; s = s->previous) {
      auto test = applyEvents(s->previous, events);
      if (stateMatches(test.get(), x)) {
        shortened = true;
        state = test;
      } else {
        events.push_front(*s->previousEvent);
      }
    }
  } while (shortened);
  return state;
}

// humanReadableTrace (SearchState.java:373-470): the trace's events as a causal graph -- an edge
// from the step that first sent a message to its delivery, and from each step of a node to its
// next step -- emitted in depth-first topological order, then replayed (skipChecks = true) from
// the initial state, dropping steps that leave the state unchanged. Where the reference iterates
// a HashSet of successors (order unspecified), successors are pushed in trace order here; the
// engine (csrc/replay.hpp) uses the same rule. Returns the new end state (its trace is the
// human-readable one), or `end` itself if a reordered event cannot be taken.
inline std::shared_ptr<const State> humanReadableTrace(const std::shared_ptr<const State>& end) {
  std::vector<std::shared_ptr<const State>> orig;
  for (auto s = end; s; s = s->previous) orig.push_back(s);
  std::reverse(orig.begin(), orig.end());
  const int L = (int)orig.size() - 1;  // events 1..L
  std::vector<std::set<int>> next(L + 1), prev(L + 1);
  std::map<Envelope, int> whenSent;
  std::map<int, int> lastStep;
  std::vector<int> initSteps;
  for (int i = 1; i <= L; i++) {
    const Event& ev = *orig[i]->previousEvent;
    if (!ev.isTimer) {
      auto it = whenSent.find(ev.msg);
      if (it != whenSent.end()) {
        next[it->second].insert(i);
        prev[i].insert(it->second);
      }
    }
    const int a = ev.isTimer ? ev.timer.to : ev.msg.to;  // locationRootAddress
    auto ls = lastStep.find(a);
    if (ls != lastStep.end()) {
      next[ls->second].insert(i);
      prev[i].insert(ls->second);
    }
    lastStep[a] = i;
    for (auto& me : orig[i]->newMessages) whenSent.emplace(me, i);
    if (prev[i].empty()) initSteps.push_back(i);
  }
  std::vector<int> order, stack(initSteps.rbegin(), initSteps.rend());
  while (!stack.empty()) {
    const int n = stack.back();
    stack.pop_back();
    order.push_back(n);
    for (int x : next[n]) {  // ascending trace order
      prev[x].erase(n);
      if (prev[x].empty()) stack.push_back(x);
    }
  }
  std::shared_ptr<const State> s = orig[0];
  for (int n : order) {
    const Event& ev = *orig[n]->previousEvent;
    auto nx = stepEvent(s, ev);
    if (!nx) return end;
    if (nx->contentKey() == s->contentKey()) continue;  // next.equals(previous): a step that changes nothing
    s = nx;
  }
  return s;
}

struct ReplayOutcome {
  End end = End::SPACE_EXHAUSTED;
  std::shared_ptr<const State> state;  // terminal (possibly minimized) or the last state reached
  int predIndex = -1;
  std::string predicate;
};

// Replays events from init with checkState after every step; a terminal is minimized when
// `minimize` (TraceReplaySearch passes true; ReplaySearch passes its flag). An event that cannot
// be delivered ends the replay with SPACE_EXHAUSTED (eventsExhausted). PRUNED states do not stop
// it (TraceReplaySearch only asserts they do not occur).
inline ReplayOutcome replaySearch(std::shared_ptr<const State> init, const Settings& st, const std::vector<Event>& evs,
                                  bool minimize) {
  ReplayOutcome out;
  auto check = [&](std::shared_ptr<const State> s, bool mini) -> bool {
    if (s->exception) {
      Expected x;
      x.exception = true;
      out.end = End::EXCEPTION_THROWN;
      out.state = mini ? minimizeTrace(s, x) : s;
      return true;
    }
    for (size_t i = 0; i < st.invariants.size(); i++) {
      PredResult r = st.invariants[i].test(*s);
      if (r.threw || !r.value) {
        Expected x{false, &st.invariants[i], r.threw, r.value};
        out.end = End::INVARIANT_VIOLATED;
        out.predIndex = (int)i;
        out.predicate = st.invariants[i].name;
        out.state = mini ? minimizeTrace(s, x) : s;
        return true;
      }
    }
    for (size_t i = 0; i < st.goals.size(); i++) {
      PredResult r = st.goals[i].test(*s);
      if (r.threw || !r.value) continue;
      Expected x{false, &st.goals[i], false, true};
      out.end = End::GOAL_FOUND;
      out.predIndex = (int)i;
      out.predicate = st.goals[i].name;
      out.state = mini ? minimizeTrace(s, x) : s;
      return true;
    }
    return false;
  };
  std::shared_ptr<const State> s = init;
  if (check(s, false)) return out;  // the initial state has no trace to minimize
  for (auto& e : evs) {
    auto n = stepChecked(s, e, &st);
    if (!n) break;
    s = n;
    if (check(s, minimize)) return out;
  }
  out.end = End::SPACE_EXHAUSTED;
  out.state = s;
  return out;
}

// Standard predicates (StatePredicate.java:52-83).
inline Predicate RESULTS_OK(const Names& n) {
  return {"Clients got expected results", [n](const State& s) {
            for (int a : s.clientWorkers()) {
              const ClientWorker* c = s.cw(a);
              if (!c->resultsOk) {
                PredResult r;
                r.value = false;
                if (c->expectedAndReceived)
                  r.detail = n.addr[a] + " got " + c->expectedAndReceived->second.str() + ", expected " +
                             c->expectedAndReceived->first.str();
                else
                  r.detail = n.addr[a] + " got an unexpected result";
                return r;
              }
            }
            return PredResult{};
          }};
}
inline Predicate CLIENTS_DONE() {
  return {"All clients' workloads finished", [](const State& s) {
            PredResult r;
            for (int a : s.clientWorkers())
              if (!s.cw(a)->done()) r.value = false;
            return r;
          }};
}
inline Predicate clientDone(const Names& n, int a) {
  return {n.addr[a] + "'s workload finished", [a](const State& s) {
            PredResult r;
            r.value = s.cw(a)->done();
            return r;
          }};
}
inline Predicate NONE_DECIDED() {
  return {"No results returned", [](const State& s) {
            PredResult r;
            for (int a : s.clientWorkers())
              if (!s.cw(a)->results.empty()) r.value = false;
            return r;
          }};
}

}  // namespace oracle
