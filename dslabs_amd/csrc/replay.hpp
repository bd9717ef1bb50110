// replay.hpp -- trace replay and trace minimization on the host, over the same packed
// transition functions (nodestate.hpp + protocols/) that the device kernels run.
//
//   TraceReplaySearch.replayTrace   T/junit/TraceReplaySearch.java:76-101
//   TraceMinimizer.minimizeTrace    T/search/TraceMinimizer.java:32-49, stateMatches :51-61,
//                                   minimizeExceptionCausingTrace :70-91, applyEvents :93-108
//   SearchState.stepEvent(e, settings, skipChecks = false)  T/search/SearchState.java:275-359
//   SearchState.humanReadableTrace  T/search/SearchState.java:373-470
//
// Events are identified by content (dsl_event), so a trace taken from one state can be applied
// to another: an event is applied iff it is among the enabled events of the state it meets.
// Exceptional successors: every handler here throws at dispatch, before changing anything, so a
// state produced by a throwing step has its parent's content (plus the exception mark).
#pragma once
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <vector>

#include "nodestate.hpp"

namespace dsl {

inline bool same_event(const dsl_event& a, const dsl_event& b) {
  if (a.is_timer != b.is_timer || a.from != b.from || a.to != b.to || a.type != b.type || a.n_fields != b.n_fields ||
      a.timer_min != b.timer_min || a.timer_max != b.timer_max)
    return false;
  for (int i = 0; i < a.n_fields && i < DSL_MAX_EVENT_FIELDS; i++)
    if (a.fields[i] != b.fields[i]) return false;
  return true;
}

template <class P>
struct TraceTool {
  using State = typename P::State;
  struct Step {
    State s;
    bool exc;  // the step that produced s threw (SearchState.thrownException)
  };
  // What a minimized state must keep (stateMatches): the exception, or the predicate's outcome
  // (PV_FALSE / PV_TRUE, or PV_THREW).
  struct Expected {
    bool exception;
    DevProg pred;
    int outcome;
  };

  const typename P::Params& prm;
  const DevSettings& search;  // the search's settings: delivery filters and predicates
  DevSettings open;           // default SearchSettings (every message and timer delivered)

  TraceTool(const typename P::Params& p, const DevSettings& s) : prm(p), search(s), open(s) {
    open.all_deliver = 1;
    for (int i = 0; i < DSL_MAX_NODES; i++) open.deliver[i] = 0xffffffffu;
    open.timer_mask = 0xffffffffu;
  }

  // stepEvent(e, settings, skipChecks = false): 1 = stepped, 0 = null (not deliverable here),
  // -1 = a bounded container overflowed.
  int step(const DevSettings& st, const State& s, const dsl_event& e, Step* out) const {
    const int n = count_events<P>(s.w, prm, st);
    for (int k = 0; k < n; k++) {
      dsl_event d;
      describe_event<P>(s.w, k, prm, st, &d);
      if (!same_event(d, e)) continue;
      const int rc = full_step<P>(s.w, k, out->s.w, prm, st);
      if (rc == STEP_OVERFLOW) return -1;
      if (rc == STEP_NULL) return 0;
      out->exc = rc == STEP_EXCEPTION;
      if (out->exc) out->s = s;
      return 1;
    }
    return 0;
  }

  int eval(DevProg g, const State& s) const {
    const NodeView v{s.w, P::kNodeWords, -1, nullptr};
    return eval_prog<P>(search, g, v, prm);
  }

  // checkState (Search.java:162-231) of one state: Verdict and the predicate index.
  int judge(const Step& x, int depth, int* pi) const {
    *pi = -1;
    if (x.exc) return V_TERM_EXCEPTION;
    const NodeView v{x.s.w, P::kNodeWords, -1, nullptr};
    return judge_view<P>(v, prm, search, depth, pi);
  }

  // The result the minimized trace must keep, for a terminal verdict v / predicate pi of `last`.
  Expected expected(int v, int pi, const State& last) const {
    if (v == V_TERM_EXCEPTION) return Expected{true, DevProg{0, 0}, 0};
    const DevProg g = v == V_TERM_INVARIANT ? search.inv[pi] : search.goal[pi];
    return Expected{false, g, eval(g, last)};
  }

  bool matches(const Step& x, const Expected& e) const {
    if (e.exception) return x.exc;
    return eval(e.pred, x.s) == e.outcome;
  }

  // The event matching e among the enabled events of s under st (-1: none).
  int find_event(const DevSettings& st, const State& s, const dsl_event& e) const {
    const int n = count_events<P>(s.w, prm, st);
    for (int k = 0; k < n; k++) {
      dsl_event d;
      describe_event<P>(s.w, k, prm, st, &d);
      if (same_event(d, e)) return k;
    }
    return -1;
  }

  // Every send of event k of s, in send order and with repeats (SearchState.newMessages): the
  // handler as delta_step runs it, without the canonicalization of the send list.
  void raw_sends(const State& s, int k, std::vector<typename P::Rec>* out) const {
    out->clear();
    const int e = locate_event<P>(s.w, prm, open, k);
    if (e == INT32_MIN) return;
    Delta<P> d;
    d.out.n = 0;
    d.out.overflow = false;
    if (e >= 0) {
      const auto r = Net<P>::at(s.w, e);
      d.node = P::rec_to(r);
      if (d.node >= P::num_nodes(prm)) return;
      for (int i = 0; i < P::kNodeWords; i++) d.nw[i] = s.w[d.node * P::kNodeWords + i];
      P::on_message(d.node, d.nw, r, d.out, prm);
    } else {
      const int x = -1 - e;
      d.node = x >> 8;
      for (int i = 0; i < P::kNodeWords; i++) d.nw[i] = s.w[d.node * P::kNodeWords + i];
      P::on_timer(d.node, d.nw, x & 255, d.out, prm);
    }
    for (int j = 0; j < d.out.n; j++) out->push_back(d.out.r[j]);
  }

  // humanReadableTrace (SearchState.java:373-470): a causal graph of the trace's events -- from
  // the step that first sent a message to its delivery, and from each step of a node to its
  // next step -- emitted in depth-first topological order (successors pushed in trace order where
  // the reference iterates a HashSet), then replayed from `start` without delivery checks,
  // dropping steps that leave the state unchanged. On return evs is the reordered trace and *last
  // its end state; both stay as they were if a reordered event cannot be taken.
  void human_readable(const State& start, std::vector<dsl_event>& evs, State* last) const {
    using Rec = typename P::Rec;
    const int L = (int)evs.size();
    std::vector<std::set<int>> next(L + 1), prev(L + 1);
    std::map<Rec, int> when_sent;
    std::map<int, int> last_step;
    std::vector<int> init_steps;
    State s = start;
    std::vector<Rec> sent;
    for (int i = 1; i <= L; i++) {
      const int k = find_event(open, s, evs[i - 1]);
      if (k < 0) return;  // not a trace of `start`
      const int loc = locate_event<P>(s.w, prm, open, k);
      if (loc >= 0) {  // a message: the edge from its first sender
        auto it = when_sent.find(Net<P>::at(s.w, loc));
        if (it != when_sent.end()) {
          next[it->second].insert(i);
          prev[i].insert(it->second);
        }
      }
      const int a = evs[i - 1].to;  // locationRootAddress
      auto ls = last_step.find(a);
      if (ls != last_step.end()) {
        next[ls->second].insert(i);
        prev[i].insert(ls->second);
      }
      last_step[a] = i;
      raw_sends(s, k, &sent);
      for (Rec r : sent) when_sent.emplace(r, i);
      if (prev[i].empty()) init_steps.push_back(i);
      Step n;
      if (step(open, s, evs[i - 1], &n) != 1) return;
      s = n.s;
    }
    std::vector<int> order, stack(init_steps.rbegin(), init_steps.rend());
    while (!stack.empty()) {
      const int n = stack.back();
      stack.pop_back();
      order.push_back(n);
      for (int x : next[n]) {  // ascending trace order
        prev[x].erase(n);
        if (prev[x].empty()) stack.push_back(x);
      }
    }
    std::vector<dsl_event> out;
    State cur = start;
    for (int n : order) {
      Step nx;
      if (step(open, cur, evs[n - 1], &nx) != 1) return;  // the reference returns the original trace
      if (std::memcmp(nx.s.w, cur.w, sizeof(cur.w)) == 0) continue;  // next.equals(previous)
      cur = nx.s;
      out.push_back(evs[n - 1]);
    }
    evs = out;
    *last = cur;
  }

  // minimizeTrace from `start` over `evs` (each applicable in turn). On return evs is the
  // minimized trace and *last the state it reaches.
  void minimize(const Step& start, std::vector<dsl_event>& evs, Step* last, const Expected& x) const {
    bool shortened;
    do {
      shortened = false;
      std::vector<Step> chain(1, start);  // chain[i] = state after evs[0..i)
      for (const auto& e : evs) {
        Step n;
        if (step(open, chain.back().s, e, &n) != 1) break;  // cannot happen for a replayed chain
        chain.push_back(n);
      }
      evs.resize(chain.size() - 1);
      std::deque<dsl_event> kept;  // the suffix of events kept so far
      std::vector<dsl_event> best;
      Step best_last{};
      for (size_t i = evs.size(); i >= 1; i--) {
        // applyEvents(s.previous, kept): s = chain[i], s.previous = chain[i - 1]
        Step t = chain[i - 1];
        std::vector<dsl_event> applied;
        for (const auto& e : kept) {
          Step n;
          if (step(open, t.s, e, &n) != 1) break;
          t = n;
          applied.push_back(e);
        }
        if (matches(t, x)) {
          shortened = true;
          best.assign(evs.begin(), evs.begin() + (i - 1));
          best.insert(best.end(), applied.begin(), applied.end());
          best_last = t;
        } else {
          kept.push_front(evs[i - 1]);
        }
      }
      if (shortened) {
        evs = best;
        *last = best_last;
      }
    } while (shortened);
  }
};

}  // namespace dsl
