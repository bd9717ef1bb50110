// nodestate.hpp -- generic packed search state + incremental set fingerprint.
//
// A packed state is [kNodes x kNodeWords node words][net count][records, sorted, distinct].
// Node words hold a node's fields and its timer queue; the network is the SET of sent messages
// (delivery never removes, duplicates collapse: SearchState.java:71, :300-301).
//
// Protocols are node-local, as DSLabs handlers are (F/Node.java:387-562): a handler sees only
// its node's words and the delivered message / fired timer, updates the words and emits sends.
// A successor is therefore a DELTA of its parent: one node's new words + a short send list.
//
// Fingerprint (128 bit): the XOR over nodes i of H_node(i, words_i) and over the network's
// records r of H_msg(r), with H = MurmurHash3_x64_128 block/finalizer structure under domain
// seeds. It is order-independent over the record set, so
//     fp(successor) = fp(parent) ^ H_node(i, old) ^ H_node(i, new) ^ XOR_{r new to the set} H_msg(r)
// is computed without materializing the successor. For n distinct states the chance that two
// share a fingerprint is ~ n^2 / 2^129 (each pair of distinct states differs in a non-empty
// set of hashed components).
#pragma once
#include <type_traits>

#include "common.hpp"
#include "fingerprint.hpp"

namespace dsl {

template <class P>
struct Layout {
  using Rec = typename P::Rec;
  static constexpr int kRecWords = (int)(sizeof(Rec) / 4);
  static constexpr int kNetCount = P::kNodes * P::kNodeWords;
  static constexpr int kRecBase = ((kNetCount + 1 + kRecWords - 1) / kRecWords) * kRecWords;
  static constexpr int kWords = ((kRecBase + P::kNetCap * kRecWords) + 3) / 4 * 4;
};

template <class P>
using StateOf = Packed<Layout<P>::kWords>;

template <class P>
struct Net {
  using L = Layout<P>;
  using Rec = typename P::Rec;
  static DSL_HD int size(const uint32_t* w) { return (int)w[L::kNetCount]; }
  static DSL_HD Rec at(const uint32_t* w, int i) {
    if constexpr (sizeof(Rec) == 8) {
      return (Rec)w[L::kRecBase + 2 * i] | ((Rec)w[L::kRecBase + 2 * i + 1] << 32);
    } else {
      return (Rec)w[L::kRecBase + i];
    }
  }
  static DSL_HD void put(uint32_t* w, int i, Rec r) {
    if constexpr (sizeof(Rec) == 8) {
      w[L::kRecBase + 2 * i] = (uint32_t)r;
      w[L::kRecBase + 2 * i + 1] = (uint32_t)((uint64_t)r >> 32);
    } else {
      w[L::kRecBase + i] = (uint32_t)r;
    }
  }
  static DSL_HD bool contains(const uint32_t* w, Rec r) {
    int lo = 0, hi = size(w);
    while (lo < hi) {
      int mid = (lo + hi) >> 1;
      Rec x = at(w, mid);
      if (x == r) return true;
      if (x < r) lo = mid + 1; else hi = mid;
    }
    return false;
  }
  // 0 inserted, 1 present, -1 overflow
  static DSL_HD int insert(uint32_t* w, Rec r) {
    int n = size(w), lo = 0, hi = n;
    while (lo < hi) {
      int mid = (lo + hi) >> 1;
      if (at(w, mid) < r) lo = mid + 1; else hi = mid;
    }
    if (lo < n && at(w, lo) == r) return 1;
    if (n >= P::kNetCap) return -1;
    for (int j = n; j > lo; j--) put(w, j, at(w, j - 1));
    put(w, lo, r);
    w[L::kNetCount] = (uint32_t)(n + 1);
    return 0;
  }
};

// P::kNetPreds: some predicate of P reads the network (StatePredicate.containsMessageMatching),
// so the judge's view must carry the successor's new records.
template <class P, class = void>
struct NetPreds : std::false_type {};
template <class P>
struct NetPreds<P, std::void_t<decltype(P::kNetPreds)>> : std::integral_constant<bool, P::kNetPreds> {};
// P::kSendsDistinct: no handler of P sends one record twice in one step (tests/hostcheck checks
// it on every explored step), so Sender needs no duplicate check.
template <class P, class = void>
struct SendsDistinct : std::false_type {};
template <class P>
struct SendsDistinct<P, std::void_t<decltype(P::kSendsDistinct)>> : std::integral_constant<bool, P::kSendsDistinct> {};

// Sends emitted by one handler invocation (duplicates collapse, as in the network set).
// Every access to r[] uses a compile-time index (fully unrolled loops predicated on i < n), so
// the list lives in VGPRs; a dynamically indexed per-lane array would be placed in scratch and
// every send would pay a memory round trip.
template <class P>
struct Sender {
  using Rec = typename P::Rec;
  static constexpr int K = P::kMaxSends;
  int n = 0;
  bool overflow = false;
  Rec r[K];
  DSL_HD void send(Rec x) {
    if constexpr (!SendsDistinct<P>::value) {
      bool dup = false;
#pragma unroll
      for (int i = 0; i < K; i++)
        if (i < n && r[i] == x) dup = true;
      if (dup) return;
    }
    if (n >= K) {
      overflow = true;
      return;
    }
#ifdef DSL_SENDER_SHIFT
    // shift register: the newest record at r[0] (the lanes at this send site move, the others keep
    // their registers under the exec mask; no compare with n per slot)
#pragma unroll
    for (int i = K - 1; i > 0; i--) r[i] = r[i - 1];
    r[0] = x;
#else
#pragma unroll
    for (int i = 0; i < K; i++) {
      if (wave_none(i <= n)) break;  // every sending lane's slot is behind
      r[i] = keep_value(i == n ? x : r[i]);
    }
#endif
    n++;
  }
};

// Read access to a state's node words (what predicates and handlers see).
struct NodeView {
  const uint32_t* base;     // node words of the parent state
  int nw;                   // words per node
  int changed;              // node replaced by `over` (-1: none)
  const uint32_t* over;
  // network predicates (P::kNetPreds): the state's records are the parent row's (base is a whole
  // row) plus `nsends` new records of type P::Rec at `sends`
  const void* sends = nullptr;
  int nsends = 0;
  // the dropped network (DevSettings::dropped, set by judge_view): part of network() for
  // predicates, never an event
  const void* dropped = nullptr;
  int ndropped = 0;
  DSL_HD const uint32_t* node(int i) const { return i == changed ? over : base + i * nw; }
};

// Any record of the viewed state's network() -- parent records, the view's new records and the
// dropped records (SearchState.network() = network + droppedNetwork, SearchState.java:153-157;
// StatePredicate.containsMessageMatching reads it, T/StatePredicate.java:146-149) -- satisfying f.
template <class P, class F>
DSL_HD bool view_any_record(const NodeView& v, F f) {
  const int n = Net<P>::size(v.base);
  for (int j = 0; j < n; j++)
    if (f(Net<P>::at(v.base, j))) return true;
  const auto* r = static_cast<const typename P::Rec*>(v.sends);
  for (int j = 0; j < v.nsends; j++)
    if (f(r[j])) return true;
  const auto* x = static_cast<const typename P::Rec*>(v.dropped);
  for (int j = 0; j < v.ndropped; j++)
    if (f(x[j])) return true;
  return false;
}

// ---- fingerprint ------------------------------------------------------------------------------
DSL_HD Fp fp_xor(Fp a, Fp b) { return Fp{a.hi ^ b.hi, a.lo ^ b.lo}; }

template <int NW>
DSL_HD Fp hash_words(const uint32_t* w, uint64_t seed) {
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  uint64_t h1 = seed ^ 0x9368e53c2f6af274ULL, h2 = seed ^ 0x586dcd208f7cd3fdULL;
#pragma unroll
  for (int i = 0; i < NW; i += 4) {
    const uint64_t k1 = (uint64_t)w[i] | ((uint64_t)(i + 1 < NW ? w[i + 1] : 0u) << 32);
    const uint64_t k2 = (uint64_t)(i + 2 < NW ? w[i + 2] : 0u) | ((uint64_t)(i + 3 < NW ? w[i + 3] : 0u) << 32);
    uint64_t a = k1 * c1;
    a = rotl64(a, 31) * c2;
    h1 ^= a;
    h1 = rotl64(h1, 27) + h2;
    h1 = h1 * 5 + 0x52dce729;
    uint64_t b = k2 * c2;
    b = rotl64(b, 33) * c1;
    h2 ^= b;
    h2 = rotl64(h2, 31) + h1;
    h2 = h2 * 5 + 0x38495ab5;
  }
  h1 ^= (uint64_t)(NW * 4);
  h2 ^= (uint64_t)(NW * 4);
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  h2 += h1;
  return Fp{h1, h2};
}

template <class P>
DSL_HD Fp node_hash(int i, const uint32_t* w) {
  return hash_words<P::kNodeWords>(w, 0x5EED00000000ull + (uint64_t)i);
}

template <class P>
DSL_HD Fp msg_hash(typename P::Rec r) {
  uint32_t w[2] = {(uint32_t)(uint64_t)r, (uint32_t)((uint64_t)r >> 32)};
  return hash_words<2>(w, 0x0E7A5E7ull);
}

template <class P>
DSL_HD Fp full_fingerprint(const uint32_t* w) {
  Fp f{0, 0};
  for (int i = 0; i < P::kNodes; i++) f = fp_xor(f, node_hash<P>(i, w + i * P::kNodeWords));
  const int n = Net<P>::size(w);
  for (int j = 0; j < n; j++) f = fp_xor(f, msg_hash<P>(Net<P>::at(w, j)));
  return f;
}

// ---- events -------------------------------------------------------------------------------------
// Enabled events of a state (SearchState.events, SearchState.java:226-252): every network record
// whose (from, to) passes shouldDeliver and whose destination exists, in record order; then for
// every node with deliverTimers(node), its deliverable timers (TimerQueue.deliverable()).
template <class P>
DSL_HD int count_events(const uint32_t* w, const typename P::Params& prm, const DevSettings& set) {
  int n = 0;
  const int cnt = Net<P>::size(w);
  const int nodes = P::num_nodes(prm);
  if (set.all_deliver) {
    n = cnt;
  } else {
    for (int j = 0; j < cnt; j++) {
      const auto r = Net<P>::at(w, j);
      n += should_deliver(set, P::rec_from(r), P::rec_to(r));
    }
  }
  for (int i = 0; i < nodes; i++)
    if (deliver_timers(set, i)) n += P::num_timer_events(i, w + i * P::kNodeWords, prm);
  return n;
}

// Locates event k: returns >= 0 = record index, or -1 - (node * 256 + j) for timer j of node.
template <class P>
DSL_HD int locate_event(const uint32_t* w, const typename P::Params& prm, const DevSettings& set, int k) {
  const int cnt = Net<P>::size(w);
  if (set.all_deliver) {
    if (k < cnt) return k;
    k -= cnt;
  } else {
    for (int j = 0; j < cnt; j++) {
      const auto r = Net<P>::at(w, j);
      if (should_deliver(set, P::rec_from(r), P::rec_to(r)) && k-- == 0) return j;
    }
  }
  const int nodes = P::num_nodes(prm);
  for (int i = 0; i < nodes; i++) {
    if (!deliver_timers(set, i)) continue;
    const int t = P::num_timer_events(i, w + i * P::kNodeWords, prm);
    if (k < t) return -1 - (i * 256 + k);
    k -= t;
  }
  return INT32_MIN;
}

// Handler classes (k_level sorts a chunk's work items by class, so a wavefront mostly runs one
// handler): messages [0, kMsgClasses) by P::msg_class; timers from kMsgClasses on, one class, or
// TimerClasses<P> of them when the protocol splits its timer handlers by node kind
// (P::kTimerClasses + P::timer_class(node): Multi-Paxos's server Tick and client ClientTimer,
// which a wave of mixed timer items would otherwise both run); last the skip class (NoopFilter).
template <class P, class = void>
struct TimerClasses : std::integral_constant<int, 1> {
  static DSL_HD int of(int, const typename P::Params&) { return 0; }
};
template <class P>
struct TimerClasses<P, std::void_t<decltype(P::kTimerClasses)>> : std::integral_constant<int, P::kTimerClasses> {
  static DSL_HD int of(int node, const typename P::Params& prm) { return P::timer_class(node, prm); }
};
template <class P>
struct Classes {
  static constexpr int kTimer0 = P::kMsgClasses;
  static constexpr int kSkip = P::kMsgClasses + TimerClasses<P>::value;
  static constexpr int kCount = kSkip + 1;
  static_assert(P::kMsgClasses >= 1 && kCount <= 16, "at most 16 handler classes, the skip class included");
};

// Events whose handler surely changes nothing: a protocol may provide
//   static bool surely_noop(int node, const uint32_t* w, Rec r, const Params&)
//   static bool surely_noop_timer(int node, const uint32_t* w, int timer, const Params&)
// (w = the whole state row) returning true only when the event surely returns STEP_OK with the
// node's words unchanged and every send already in the network (the successor is the parent;
// `false` whenever unsure). k_level counts such an event as a successor (Search.java:481-485: it
// is generated, then found in the visited set) without running its handler; tests/hostcheck
// checks the implication on every explored event. event_class_skip returns Classes<P>::kSkip for them.
template <class P, class = void>
struct NoopFilter {
  static DSL_HD bool msg(int, const uint32_t*, typename P::Rec, const typename P::Params&) { return false; }
};
template <class P>
struct NoopFilter<P, std::void_t<decltype(&P::surely_noop)>> {
  static DSL_HD bool msg(int i, const uint32_t* w, typename P::Rec r, const typename P::Params& prm) {
    return P::surely_noop(i, w, r, prm);
  }
};
template <class P, class = void>
struct NoopTimerFilter {
  static DSL_HD bool timer(int, const uint32_t*, int, const typename P::Params&) { return false; }
};
template <class P>
struct NoopTimerFilter<P, std::void_t<decltype(&P::surely_noop_timer)>> {
  static DSL_HD bool timer(int i, const uint32_t* w, int t, const typename P::Params& prm) {
    return P::surely_noop_timer(i, w, t, prm);
  }
};

template <class P>
DSL_HD int event_class_skip(const uint32_t* w, const typename P::Params& prm, const DevSettings& set, int k,
                            int* located = nullptr) {
  const int e = locate_event<P>(w, prm, set, k);
  if (located) *located = e;  // k_level keeps it for delta_step_located (no second walk)
  if (e < 0) {
    if (e == INT32_MIN) return Classes<P>::kTimer0;
    const int x = -1 - e;
    return NoopTimerFilter<P>::timer(x >> 8, w, x & 255, prm) ? Classes<P>::kSkip
                                                                : Classes<P>::kTimer0 + TimerClasses<P>::of(x >> 8, prm);
  }
  const auto r = Net<P>::at(w, e);
  const int i = P::rec_to(r);
  if (i < P::num_nodes(prm) && NoopFilter<P>::msg(i, w, r, prm)) return Classes<P>::kSkip;
  return P::msg_class(r);
}

// A successor as a delta of its parent: one node's new words and the handler's sends (distinct);
// bit i of `keep` marks send i as new to the parent's network set. The records the successor adds
// are exactly the kept sends; they stay in send order (nothing is moved or sorted), and every
// consumer that needs the merged order ranks them itself (delta_rank).
template <class P>
struct Delta {
  int node;
  uint32_t nw[P::kNodeWords];
  Sender<P> out;
  uint32_t keep;
};

template <class P>
DSL_HD int delta_new_count(const Delta<P>& d) { return __builtin_popcount(d.keep); }

// Marks the sends that are not already in the parent's network set (canonical successor: the
// set union). No reordering: the send list stays where the handler wrote it, in VGPRs.
// Membership by a fixed-trip lower bound over the sorted records (log2(kNetCap) + 1 dependent LDS
// reads, selects instead of a data-dependent loop: C5 d12 -1.5 % against Net::contains).
template <class P>
DSL_HD bool net_contains_fixed(const uint32_t* w, int n, typename P::Rec r) {
  int pos = 0;
#pragma unroll
  for (int step = 1 << (31 - __builtin_clz((unsigned)P::kNetCap)); step > 0; step >>= 1) {
    const int q = pos + step;
    pos = (q <= n && Net<P>::at(w, q - 1) < r) ? q : pos;
  }
  return pos < n && Net<P>::at(w, pos) == r;
}

template <class P>
DSL_HD void canon_sends(const uint32_t* w, Delta<P>& d) {
  constexpr int K = P::kMaxSends;
  const int n = d.out.n;
  uint32_t keep = 0;
  const int nr = Net<P>::size(w);
#pragma unroll
  for (int i = 0; i < K; i++) {
    if (wave_none(i < n)) break;
    if (i < n && !net_contains_fixed<P>(w, nr, d.out.r[i])) keep |= 1u << i;
  }
  d.keep = keep;
}

// The kept sends, compacted in send order into out[]; returns their number (host code and LDS views).
template <class P>
DSL_HD int delta_sends(const Delta<P>& d, typename P::Rec* out) {
  int m = 0;
  for (int i = 0; i < P::kMaxSends; i++)
    if ((d.keep >> i) & 1u) out[m++] = d.out.r[i];
  return m;
}

// Applies event k of parent w: fills the delta (its send list canonical); returns a StepRc.
template <class P>
DSL_HD int delta_step_located(const uint32_t* w, int e, Delta<P>& d, const typename P::Params& prm,
                              const DevSettings& set);
template <class P>
DSL_HD int delta_step(const uint32_t* w, int k, Delta<P>& d, const typename P::Params& prm, const DevSettings& set) {
  return delta_step_located<P>(w, locate_event<P>(w, prm, set, k), d, prm, set);
}
// The same for an event already located (locate_event's code e).
template <class P>
DSL_HD int delta_step_located(const uint32_t* w, int e, Delta<P>& d, const typename P::Params& prm,
                              const DevSettings& set) {
  if (e == INT32_MIN) return STEP_NULL;
  d.out.n = 0;
  d.out.overflow = false;
  d.keep = 0;
  int rc;
  if (e >= 0) {
    const auto r = Net<P>::at(w, e);
    d.node = P::rec_to(r);
    if (d.node >= P::num_nodes(prm)) return STEP_NULL;
    for (int i = 0; i < P::kNodeWords; i++) d.nw[i] = w[d.node * P::kNodeWords + i];
    rc = P::on_message(d.node, d.nw, r, d.out, prm);
  } else {
    const int x = -1 - e;
    d.node = x >> 8;
    for (int i = 0; i < P::kNodeWords; i++) d.nw[i] = w[d.node * P::kNodeWords + i];
    rc = P::on_timer(d.node, d.nw, x & 255, d.out, prm);
  }
  if (d.out.overflow && rc == STEP_OK) rc = STEP_OVERFLOW;
  if (rc == STEP_OK) canon_sends<P>(w, d);
  else d.keep = (1u << d.out.n) - 1u;  // an exceptional state keeps what was sent before the throw
  return rc;
}

// Successor fingerprint from the parent's: node delta + the sends not already in the set.
template <class P>
DSL_HD Fp delta_fingerprint(const uint32_t* w, Fp parent, const Delta<P>& d) {
  Fp f = fp_xor(parent, node_hash<P>(d.node, w + d.node * P::kNodeWords));
  f = fp_xor(f, node_hash<P>(d.node, d.nw));
#pragma unroll
  for (int j = 0; j < P::kMaxSends; j++) {
    if (wave_none((d.keep >> j) != 0u)) break;
    if ((d.keep >> j) & 1u) f = fp_xor(f, msg_hash<P>(d.out.r[j]));  // the records new to the set
  }
  return f;
}

// The same from the parent's fingerprint with the changed node's old hash already removed
// (k_level caches the parents' node hashes in LDS).
template <class P>
DSL_HD Fp delta_fingerprint_cached(Fp parent_without_node, const Delta<P>& d) {
  Fp f = fp_xor(parent_without_node, node_hash<P>(d.node, d.nw));
#pragma unroll
  for (int j = 0; j < P::kMaxSends; j++) {
    if (wave_none((d.keep >> j) != 0u)) break;
    if ((d.keep >> j) & 1u) f = fp_xor(f, msg_hash<P>(d.out.r[j]));
  }
  return f;
}

// Enabled events of the successor, from the parent's count and the delta: the changed node's
// timer events are replaced, records new to the set add their deliverable ones.
template <class P>
DSL_HD int delta_event_count(const uint32_t* w, int parent_events, const Delta<P>& d, const typename P::Params& prm,
                             const DevSettings& set) {
  int n = parent_events;
  if (deliver_timers(set, d.node))
    n += P::num_timer_events(d.node, d.nw, prm) - P::num_timer_events(d.node, w + d.node * P::kNodeWords, prm);
#pragma unroll
  for (int j = 0; j < P::kMaxSends; j++) {  // the records new to the set
    if (wave_none((d.keep >> j) != 0u)) break;
    if ((d.keep >> j) & 1u) {
      const auto r = d.out.r[j];
      if (set.all_deliver || should_deliver(set, P::rec_from(r), P::rec_to(r))) n++;
    }
  }
  return n;
}

// ---- merged-row emission ----------------------------------------------------------------------
// The successor row = parent row with one node's words replaced and the canonical sends merged
// into the sorted record array. The kernels write it lane-parallel (kernels.hpp: wave_emit):
// header word o is the parent's word o, the replaced node's word, or the new record count; the
// merged record array is written by element: the parent's record q goes to slot q + (new records
// below it), a new record r to slot (parent records below r) + (new records below r) -- its rank
// among all the elements, as the records are distinct -- and the slots past n + m are zero.
// emit_row restates exactly that element-wise rule on the host (tests/hostcheck checks it
// against materialize(), which inserts the records one by one).
template <class P>
DSL_HD bool emit_row(const uint32_t* pw, const Delta<P>& d, uint32_t* out) {
  using L = Layout<P>;
  using Rec = typename P::Rec;
  Rec s[P::kMaxSends];
  const int n = Net<P>::size(pw), m = delta_sends<P>(d, s);
  if (n + m > P::kNetCap) return false;
  for (int o = 0; o < L::kRecBase; o++) {
    uint32_t v = o < L::kNetCount ? pw[o] : o == L::kNetCount ? (uint32_t)(n + m) : 0u;
    const int rel = o - d.node * P::kNodeWords;
    if (rel >= 0 && rel < P::kNodeWords) v = d.nw[rel];
    out[o] = v;
  }
  for (int o = L::kRecBase; o < L::kWords; o++) out[o] = 0u;
  auto put = [&](int slot, Rec r) {
    if constexpr (sizeof(Rec) == 8) {
      out[L::kRecBase + 2 * slot] = (uint32_t)r;
      out[L::kRecBase + 2 * slot + 1] = (uint32_t)((uint64_t)r >> 32);
    } else {
      out[L::kRecBase + slot] = (uint32_t)r;
    }
  };
  for (int q = 0; q < n; q++) {
    const Rec e = Net<P>::at(pw, q);
    int rk = q;
    for (int i = 0; i < m; i++) rk += s[i] < e;
    put(rk, e);
  }
  for (int i = 0; i < m; i++) {
    int pos = 0;
    for (int q = 0; q < n; q++) pos += Net<P>::at(pw, q) < s[i];
    for (int j = 0; j < m; j++) pos += s[j] < s[i];
    put(pos, s[i]);
  }
  return true;
}

// Materializes the successor (parent w + delta) into out; false on network overflow.
template <class P>
DSL_HD bool materialize(const uint32_t* w, const Delta<P>& d, uint32_t* out) {
  for (int i = 0; i < Layout<P>::kWords; i++) out[i] = w[i];
  for (int i = 0; i < P::kNodeWords; i++) out[d.node * P::kNodeWords + i] = d.nw[i];
  for (int j = 0; j < d.out.n; j++)
    if (((d.keep >> j) & 1u) && Net<P>::insert(out, d.out.r[j]) < 0) return false;
  return true;
}

// Whole-state step (host-side trace replay, initial states).
template <class P>
DSL_HD int full_step(const uint32_t* w, int k, uint32_t* out, const typename P::Params& prm, const DevSettings& set) {
  Delta<P> d;
  int rc = delta_step<P>(w, k, d, prm, set);
  if (rc == STEP_NULL) return rc;
  if (!materialize<P>(w, d, out)) return STEP_OVERFLOW;
  return rc;
}

// Initial state: every node added and init()-ed in address order (SearchState.setupNode).
template <class P>
DSL_HD bool init_state(uint32_t* w, const typename P::Params& prm) {
  for (int i = 0; i < Layout<P>::kWords; i++) w[i] = 0;
  for (int i = 0; i < P::num_nodes(prm); i++) {
    Sender<P> out;
    P::init_node(i, w + i * P::kNodeWords, out, prm);
    if (out.overflow) return false;
    for (int j = 0; j < out.n; j++)
      if (Net<P>::insert(w, out.r[j]) < 0) return false;
  }
  return true;
}

// Decodes event k of state w for traces (MessageEnvelope / TimerEnvelope fields).
template <class P>
void describe_event(const uint32_t* w, int k, const typename P::Params& prm, const DevSettings& set, dsl_event* e) {
  *e = dsl_event{};
  const int x = locate_event<P>(w, prm, set, k);
  if (x == INT32_MIN) return;
  if (x >= 0) {
    P::describe_message(Net<P>::at(w, x), e);
  } else {
    const int y = -1 - x, node = y >> 8;
    P::describe_timer(node, w + node * P::kNodeWords, y & 255, prm, e);
  }
}

// Incremental predicate evaluation (judge_view below): a leaf that reads neither the changed node
// nor the network keeps the parent's value. A leaf reading the changed node is also unchanged
// when the words it reads are: the
// protocol's pred_same(pr, old, new) says so (e.g. Multi-Paxos LOGS_CONSISTENT reads only the
// servers' log words); without one, the node's words must all be equal.
template <int N>
DSL_HD bool same_words(const uint32_t* a, const uint32_t* b) {
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < N; i++) d |= a[i] ^ b[i];
  return d == 0;
}
template <class P, class = void>
struct PredSame {
  static DSL_HD bool same(const DevPred&, const uint32_t* a, const uint32_t* b) { return same_words<P::kNodeWords>(a, b); }
};
template <class P>
struct PredSame<P, std::void_t<decltype(&P::pred_same)>> {
  static DSL_HD bool same(const DevPred& pr, const uint32_t* a, const uint32_t* b) { return P::pred_same(pr, a, b); }
};

template <class P>
DSL_HD bool leaf_unchanged(const DevPred& pr, const NodeView& v) {
  if (pr.reads >> 31) return false;
  if (!((pr.reads >> v.changed) & 1u)) return true;
  return PredSame<P>::same(pr, v.base + v.changed * v.nw, v.over);
}
// A program is unchanged when every leaf is.
template <class P>
DSL_HD bool prog_unchanged(const DevSettings& set, DevProg g, const NodeView& v, bool incremental) {
  if (!incremental || v.changed < 0) return false;
  for (int i = 0; i < g.len; i++) {
    const DevPred& op = set.ops[g.start + i];
    if (op.id > 0 && !leaf_unchanged<P>(op, v)) return false;
  }
  return true;
}

// StatePredicate.test of a program (false / true / threw): postfix over a stack of 2-bit values
// kept in one word (no indexed private array). Combinators follow StatePredicate.java:397-431: a
// throwing left operand throws; and(a, b) is a when a is false, else b; or(a, b) is a when a is
// true, else b; negate keeps a throw.
template <class P>
DSL_HD int eval_prog(const DevSettings& set, DevProg g, const NodeView& v, const typename P::Params& prm) {
  uint32_t st = 0;
  for (int i = 0; i < g.len; i++) {
    const DevPred& op = set.ops[g.start + i];
    int x;
    if (op.id == kOpAnd || op.id == kOpOr) {
      const int b = (int)(st & 3u);
      st >>= 2;
      const int a = (int)(st & 3u);
      st >>= 2;
      x = a == PV_THREW ? PV_THREW : op.id == kOpAnd ? (a == PV_FALSE ? PV_FALSE : b) : (a == PV_TRUE ? PV_TRUE : b);
    } else if (op.id == kOpNot) {
      const int a = (int)(st & 3u);
      st >>= 2;
      x = a == PV_THREW ? PV_THREW : !a;
    } else {
      x = P::eval(op, v, prm);
      if (x != PV_THREW && op.negate) x = !x;
    }
    st = (st << 2) | (uint32_t)x;
  }
  return (int)(st & 3u);
}

// A leaf known to hold on the parent (an invariant, not negated, of an expanded parent: the view is
// incremental) may be evaluated on the successor from what the changed node's words changed: a
// protocol may provide
//   static int eval_held(const DevPred&, const NodeView&, const Params&, bool held)
// (Multi-Paxos LOGS_CONSISTENT: only the slots whose entries the changed server changed, the other
// slots are as valid as on the parent); it must equal eval whenever held is true of the parent
// (tests/hostcheck compares the incremental verdict with the full one on every explored successor).
template <class P, class = void>
struct EvalHeld {
  static DSL_HD int eval(const DevPred& pr, const NodeView& v, const typename P::Params& prm, bool) {
    return P::eval(pr, v, prm);
  }
};
#ifndef DSL_NO_EVAL_HELD  // (measurement builds: -DDSL_NO_EVAL_HELD evaluates every leaf in full)
template <class P>
struct EvalHeld<P, std::void_t<decltype(&P::eval_held)>> {
  static DSL_HD int eval(const DevPred& pr, const NodeView& v, const typename P::Params& prm, bool held) {
    return P::eval_held(pr, v, prm, held);
  }
};
#endif

// checkState order over a node view (Search.java:162-231).
// incremental: the view is a successor of an EXPANDED, non-initial parent, which therefore had
// every invariant true, every goal false or throwing (ignored) and every prune false (a state
// that violated, matched or was pruned is never expanded; only the initial state is expanded
// when pruned, Search.java:475). A predicate whose leaves read neither the changed node's
// relevant words nor the network has the parent's value, so it is skipped with that outcome.
// tests/hostcheck checks the incremental verdict against the full one on every successor.
// The invariants, goals and prunes are walked as ONE sequence (programs [0, n_inv) are the
// invariants, then the goals, then the prunes), so the protocol's predicate code is inlined once
// rather than once per kind.
template <class P>
DSL_HD Verdict judge_view(const NodeView& v0, const typename P::Params& prm, const DevSettings& set, int depth,
                          int* pred_index, bool incremental = false) {
  NodeView v = v0;
  if constexpr (NetPreds<P>::value) {
    v.dropped = set.dropped();
    v.ndropped = set.n_dropped;
  }
  const int ng = set.n_inv + set.n_goal, nt = ng + set.n_prune;
#ifdef DSL_NO_FLAT  // measurement variant: the program interpreter for every predicate list
  if (false) {
#else
  if (set.flat) {
#endif
    // every program is one leaf (resolve_settings): program t IS ops[t], in checkState order
    // (invariants, goals, prunes) -- no program descriptors, no stack machine
#ifdef DSL_FLAT_UNROLL
#pragma unroll
    for (int t = 0; t < kFlatUnroll; t++) {
      if (t >= nt) break;
#else
    for (int t = 0; t < nt; t++) {
#endif
      const DevPred& op = set.ops[t];
      if (incremental && v.changed >= 0 && leaf_unchanged<P>(op, v)) continue;
      int x = EvalHeld<P>::eval(op, v, prm, incremental && v.changed >= 0 && t < set.n_inv && !op.negate);
      if (x != PV_THREW && op.negate) x = !x;
      if (t < set.n_inv) {
        if (x != PV_TRUE) {  // a false or throwing invariant is violated
          *pred_index = t;
          return V_TERM_INVARIANT;
        }
      } else if (t < ng) {
        if (x == PV_TRUE) {  // throwing goals are ignored
          *pred_index = t - set.n_inv;
          return V_TERM_GOAL;
        }
      } else if (x != PV_FALSE) {
        return V_PRUNED;  // true or throwing
      }
    }
#ifdef DSL_FLAT_UNROLL
    for (int t = kFlatUnroll; t < nt; t++) {
      const DevPred& op = set.ops[t];
      if (incremental && v.changed >= 0 && leaf_unchanged<P>(op, v)) continue;
      int x = EvalHeld<P>::eval(op, v, prm, incremental && v.changed >= 0 && t < set.n_inv && !op.negate);
      if (x != PV_THREW && op.negate) x = !x;
      if (t < set.n_inv) {
        if (x != PV_TRUE) {
          *pred_index = t;
          return V_TERM_INVARIANT;
        }
      } else if (t < ng) {
        if (x == PV_TRUE) {
          *pred_index = t - set.n_inv;
          return V_TERM_GOAL;
        }
      } else if (x != PV_FALSE) {
        return V_PRUNED;
      }
    }
#endif
    if (set.max_depth >= 0 && depth >= set.max_depth) return V_PRUNED;
    return V_VALID;
  }
  for (int t = 0; t < nt; t++) {
    const int kind = t < set.n_inv ? 0 : t < ng ? 1 : 2;
    const int i = kind == 0 ? t : kind == 1 ? t - set.n_inv : t - ng;
    const DevProg g = kind == 0 ? set.inv[i] : kind == 1 ? set.goal[i] : set.prune[i];
    if (prog_unchanged<P>(set, g, v, incremental)) continue;
    const int x = eval_prog<P>(set, g, v, prm);
    if (kind == 0 && x != PV_TRUE) {  // a false or throwing invariant is violated
      *pred_index = i;
      return V_TERM_INVARIANT;
    }
    if (kind == 1 && x == PV_TRUE) {  // throwing goals are ignored
      *pred_index = i;
      return V_TERM_GOAL;
    }
    if (kind == 2 && x != PV_FALSE) return V_PRUNED;  // true or throwing
  }
  if (set.max_depth >= 0 && depth >= set.max_depth) return V_PRUNED;
  return V_VALID;
}

// Fills DevPred::reads of every leaf from the protocol's read sets (host, after resolve_settings).
template <class P>
void set_pred_reads(DevSettings& d, const typename P::Params& prm) {
  for (int i = 0; i < d.n_ops; i++)
    if (d.ops[i].id > 0) d.ops[i].reads = P::pred_reads(d.ops[i], prm);
}

}  // namespace dsl
