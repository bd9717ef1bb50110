// settings.hpp -- dsl_settings (TestSettings + SearchSettings) -> DevSettings, host side.
// Shared by the engine (engine.hip) and the host-only CPU baseline (tools/cpu_bfs.cpp).
#pragma once
#include <functional>
#include <string>

#include "common.hpp"

namespace dsl {

// TestSettings.shouldDeliver precedence (TestSettings.java:224-245): self-send always; then
// link override, sender override, receiver override, global networkActive.
// TestSettings.deliverTimers(a): per-address override else the global flag (:87-89).
inline int resolve_settings(const dsl_settings& in, int num_nodes, bool (*known)(int), DevSettings* out,
                            std::string* why_out) {
  DevSettings d{};
  if (num_nodes > DSL_MAX_NODES) return *why_out = "too many nodes", DSL_ERR_ARG;
  if (in.do_checks < DSL_CHECKS_NONE || in.do_checks > DSL_CHECKS_ALL || in.check_sample < 0)
    return *why_out = "do_checks must be DSL_CHECKS_NONE / _ERRORS / _ALL and check_sample >= 0", DSL_ERR_ARG;
  for (int f = 0; f < num_nodes; f++) {
    uint32_t row = 0;
    for (int t = 0; t < num_nodes; t++) {
      bool ok;
      if (f == t) ok = true;
      else if (in.link_active[f][t] >= 0) ok = in.link_active[f][t] != 0;
      else if (in.sender_active[f] >= 0) ok = in.sender_active[f] != 0;
      else if (in.receiver_active[t] >= 0) ok = in.receiver_active[t] != 0;
      else ok = in.network_active != 0;
      if (ok) row |= 1u << t;
    }
    d.deliver[f] = row;
  }
  d.all_deliver = 1;
  for (int f = 0; f < num_nodes; f++)
    if ((d.deliver[f] & ((num_nodes >= 32 ? 0u : (1u << num_nodes)) - 1u)) != ((num_nodes >= 32 ? 0u : (1u << num_nodes)) - 1u))
      d.all_deliver = 0;
  for (int a = 0; a < num_nodes; a++) {
    bool ok = in.timers_active[a] >= 0 ? in.timers_active[a] != 0 : in.deliver_timers != 0;
    if (ok) d.timer_mask |= 1u << a;
  }
  d.max_depth = in.max_depth;
  if (in.n_invariants < 0 || in.n_invariants > DSL_MAX_PREDICATES || in.n_goals < 0 ||
      in.n_goals > DSL_MAX_PREDICATES || in.n_prunes < 0 || in.n_prunes > DSL_MAX_PREDICATES || in.n_pool < 0 ||
      in.n_pool > DSL_MAX_POOL)
    return *why_out = "predicate counts out of range", DSL_ERR_ARG;
  d.n_inv = in.n_invariants;
  d.n_goal = in.n_goals;
  d.n_prune = in.n_prunes;
  // predicate trees (leaves + DSL_PRED_AND / _OR / _IMPLIES over pool entries) -> postfix programs
  std::string why;
  std::function<bool(const dsl_predicate&, int, int*)> emit = [&](const dsl_predicate& p, int level, int* sp) -> bool {
    if (level > 16) return why = "predicate nesting too deep", false;
    const bool comb = p.pred_id == DSL_PRED_AND || p.pred_id == DSL_PRED_OR || p.pred_id == DSL_PRED_IMPLIES;
    if (comb) {
      if (p.arg0 < 0 || p.arg0 >= in.n_pool || p.arg1 < 0 || p.arg1 >= in.n_pool)
        return why = "combinator operand outside dsl_settings.pool", false;
      if (!emit(in.pool[p.arg0], level + 1, sp)) return false;
      auto push_op = [&](int32_t op) {
        if (d.n_ops >= kMaxProgOps) return why = "predicate programs too long", false;
        d.ops[d.n_ops++] = DevPred{op, 0, 0, 0, 0u, 0u};
        return true;
      };
      if (p.pred_id == DSL_PRED_IMPLIES && !push_op(kOpNot)) return false;  // or(negate(a), b)
      if (!emit(in.pool[p.arg1], level + 1, sp)) return false;
      if (!push_op(p.pred_id == DSL_PRED_AND ? kOpAnd : kOpOr)) return false;
      (*sp)--;
      if (p.negate && !push_op(kOpNot)) return false;
      return true;
    }
    if (!known(p.pred_id)) return why = "predicate not supported by this protocol's device predicates", false;
    if (d.n_ops >= kMaxProgOps) return why = "predicate programs too long", false;
    d.ops[d.n_ops++] = DevPred{p.pred_id, p.negate, (int32_t)p.arg0, (int32_t)p.arg1, 0u, 0u};
    if (++*sp > kMaxProgStack) return why = "predicate too wide", false;
    return true;
  };
  auto compile = [&](const dsl_predicate* src, int n, DevProg* dst) {
    for (int i = 0; i < n; i++) {
      const int start = d.n_ops;
      int sp = 0;
      if (!emit(src[i], 0, &sp)) return false;
      dst[i] = DevProg{(int16_t)start, (int16_t)(d.n_ops - start)};
    }
    return true;
  };
  if (!compile(in.invariants, d.n_inv, d.inv) || !compile(in.goals, d.n_goal, d.goal) ||
      !compile(in.prunes, d.n_prune, d.prune)) {
    *why_out = why;
    return why.rfind("predicate not supported", 0) == 0 ? DSL_ERR_UNKNOWN_PREDICATE : DSL_ERR_ARG;
  }
  d.flat = d.n_ops == d.n_inv + d.n_goal + d.n_prune ? 1 : 0;  // one leaf per program
  *out = d;
  return DSL_OK;
}

}  // namespace dsl
