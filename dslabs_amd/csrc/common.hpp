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

// One step of a predicate program: a leaf (a standard or protocol predicate, optionally
// negated) or a combinator over the values on the program's stack (StatePredicate.and / or /
// implies / negate, T/StatePredicate.java:382-432). Programs are postfix; resolve_settings
// compiles the C ABI's predicate trees into them.
struct DevPred {
  int32_t id;      // leaf: dsl_predicate_id (> 0); combinator: kOpAnd / kOpOr / kOpNot
  int32_t negate;  // leaf: StatePredicate.negate()
  int32_t arg0, arg1;
  uint32_t reads;  // leaf: nodes whose words it reads (bit i = node i; bit 31 = the network)
  uint32_t pad;
};
constexpr int32_t kOpAnd = -1, kOpOr = -2, kOpNot = -3;
constexpr uint32_t kReadsAll = 0xffffffffu;
constexpr int kMaxProgOps = 64;   // ops of all the programs of one search
constexpr int kMaxProgStack = 16;  // values on a program's stack (2 bits each in one word)
constexpr int kFlatUnroll = 4;     // leaves judge_view unrolls on a flat program list

// A top-level predicate (an invariant, goal or prune): ops [start, start + len) of the pool.
struct DevProg {
  int16_t start, len;
};

// Device form of SearchSettings/TestSettings. The tri-state precedence of
// TestSettings.shouldDeliver (TestSettings.java:224-245) is resolved on the host into a
// boolean matrix deliver[from] bit `to`; timers into timer_mask bit a = deliverTimers(a).
struct DevSettings {
  uint32_t deliver[DSL_MAX_NODES];
  uint32_t timer_mask;
  int32_t all_deliver;  // every (from, to) pair of the protocol's nodes delivers
  int32_t max_depth;
  int32_t n_inv, n_goal, n_prune, n_ops;
  // 1: every program is a single leaf (no combinator), so ops[t] is program t in checkState order
  // -- invariants, goals, prunes (resolve_settings emits them in that order); judge_view then walks
  // the leaves directly (no program descriptors, no stack)
  int32_t flat;
  int32_t pad_flat;
  DevProg inv[DSL_MAX_PREDICATES];
  DevProg goal[DSL_MAX_PREDICATES];
  DevProg prune[DSL_MAX_PREDICATES];
  DevPred ops[kMaxProgOps];
  // SearchState.droppedNetwork (dsl_set_dropped): the records network predicates see beside the
  // state's own (network() = network + droppedNetwork, SearchState.java:153-157); the same
  // records in device memory (kernels) and host memory (host-side judging), P::Rec-typed.
  const void* dropped_dev;
  const void* dropped_host;
  int32_t n_dropped;
  int32_t pad_dropped;
  DSL_HD const void* dropped() const {
#ifdef __HIP_DEVICE_COMPILE__
    return dropped_dev;
#else
    return dropped_host;
#endif
  }
};

// True when no active lane of the wavefront has `p` (device; one thread on the host): the exit of
// a fixed-trip loop over a per-lane list once every lane is past its end (the unrolled iterations
// after it would each still pay their exec-mask test and branch).
DSL_HD bool wave_none(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ballot(p) == 0ull;
#else
  return !p;
#endif
}

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
// An opaque copy of v: per-element selects over a private array stay selects of VALUES (the
// optimizer would otherwise merge them into one access at a computed address, and a dynamically
// addressed private array -- or a kernel-argument struct -- is copied to scratch memory).
template <class T>
DSL_HD T keep_value(T v) {
#ifdef __HIP_DEVICE_COMPILE__
  asm("" : "+v"(v));
#endif
  return v;
}
// a[r][c] of a small parameter table for run-time r, c (a select chain, see keep_value).
template <int R, int C>
DSL_HD int sel_param(const int32_t (&a)[R][C], int r, int c) {
  int v = 0;
#pragma unroll
  for (int i = 0; i < R; i++)
#pragma unroll
    for (int j = 0; j < C; j++) v = (i == r && j == c) ? keep_value((int)a[i][j]) : v;
  return v;
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
