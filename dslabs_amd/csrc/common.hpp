// common.hpp -- shared device/host types of the MI355X BFS engine.
//
// Every protocol is a struct with static __host__ __device__ transition functions over a
// fixed-width packed State (uint32 words). The engine (engine.hip) is templated on it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dslabs_hip.h"

#define DSL_HD __host__ __device__ __forceinline__

namespace dsl {

// Outcome of applying the k-th enabled event to a state.
enum StepRc : int {
  STEP_OK = 0,
  STEP_NULL = 1,       // destination node missing (SearchState.stepMessage returns null)
  STEP_EXCEPTION = 2,  // handler "threw": exceptional, terminal, never equal to another state
  STEP_OVERFLOW = 3    // bounded container exceeded: hard engine error, never truncated
};

// Predicate value (StatePredicate.test): false / true / threw.
enum PredVal : int { PV_FALSE = 0, PV_TRUE = 1, PV_THREW = 2 };

struct DevPred {
  int32_t id;
  int32_t negate;
  int64_t arg0, arg1;
  uint32_t reads;  // nodes whose words the predicate reads (bit i = node i; bit 31 = the network)
  uint32_t pad;
};
constexpr uint32_t kReadsAll = 0xffffffffu;

// Device form of SearchSettings/TestSettings. The tri-state precedence of
// TestSettings.shouldDeliver (TestSettings.java:224-245) is resolved on the host into a
// boolean matrix deliver[from] bit `to`; timers into timer_mask bit a = deliverTimers(a).
struct DevSettings {
  uint32_t deliver[DSL_MAX_NODES];
  uint32_t timer_mask;
  int32_t all_deliver;  // every (from, to) pair of the protocol's nodes delivers
  int32_t max_depth;
  int32_t n_inv, n_goal, n_prune;
  DevPred inv[DSL_MAX_PREDICATES];
  DevPred goal[DSL_MAX_PREDICATES];
  DevPred prune[DSL_MAX_PREDICATES];
};

DSL_HD bool should_deliver(const DevSettings& s, int from, int to) {
  return (s.deliver[from] >> to) & 1u;
}
DSL_HD bool deliver_timers(const DevSettings& s, int a) { return (s.timer_mask >> a) & 1u; }

// Bit-field access into a packed state. Fields never straddle a 32-bit word.
template <int W>
struct Packed {
  uint32_t w[W];
  DSL_HD uint32_t get(int bitoff, int width) const {
    return (w[bitoff >> 5] >> (bitoff & 31)) & ((width == 32) ? 0xffffffffu : ((1u << width) - 1u));
  }
  DSL_HD void set(int bitoff, int width, uint32_t v) {
    uint32_t m = ((width == 32) ? 0xffffffffu : ((1u << width) - 1u)) << (bitoff & 31);
    uint32_t& x = w[bitoff >> 5];
    x = (x & ~m) | ((v << (bitoff & 31)) & m);
  }
  DSL_HD bool bit(int b) const { return (w[b >> 5] >> (b & 31)) & 1u; }
  DSL_HD void setbit(int b) { w[b >> 5] |= 1u << (b & 31); }
};

// Word i of a node's N words for a run-time i: a select chain, so a node held in a per-lane
// array stays in VGPRs (a dynamically indexed private array is placed in scratch, and every
// handler access would then be a memory round trip). A constant i folds to one access.
template <int N>
DSL_HD uint32_t sel_word(const uint32_t* w, int i) {
  uint32_t v = w[0];
#pragma unroll
  for (int k = 1; k < N; k++) {
    uint32_t x = w[k];
#ifdef __HIP_DEVICE_COMPILE__
    // keeps the selection on VALUES: otherwise the optimizer folds the chain into one load
    // from a selected address, i.e. back into a dynamically indexed (scratch) array
    asm("" : "+v"(x));
#endif
    v = (i == k) ? x : v;
  }
  return v;
}
template <int N>
DSL_HD void sel_put(uint32_t* w, int i, uint32_t v) {
#pragma unroll
  for (int k = 0; k < N; k++) w[k] = (i == k) ? v : w[k];
}
// Bit-field get/put over a node's N words (fields never straddle a word).
template <int N>
DSL_HD int field_get(const uint32_t* w, int bit, int width) {
  return (int)((sel_word<N>(w, bit >> 5) >> (bit & 31)) & ((1u << width) - 1u));
}
template <int N>
DSL_HD void field_put(uint32_t* w, int bit, int width, int v) {
  const uint32_t m = ((1u << width) - 1u) << (bit & 31);
  const int i = bit >> 5;
  sel_put<N>(w, i, (sel_word<N>(w, i) & ~m) | (((uint32_t)v << (bit & 31)) & m));
}

// How a successor is judged (Search.checkState, Search.java:162-231).
enum Verdict : int { V_VALID = 0, V_PRUNED = 1, V_TERM_EXCEPTION = 2, V_TERM_INVARIANT = 3, V_TERM_GOAL = 4 };

}  // namespace dsl
