// synthetic.hpp -- the table-driven synthetic protocol of BASELINE config C3 (a dedup /
// all-to-all stress test with no reference analogue; specification in DESIGN.md §10 and,
// object-style, oracle/proto_synthetic.hpp).
//
// N <= 5 nodes "node1".."nodeN". Node i holds v in [0, K) and pokes in [0, 4), and a timer queue
// of the four timers SynthTimer(0..3), each set with bounds (1, 100) ms, so all four are always
// deliverable (TimerQueue.deliverable: an entry is skipped only if its min >= the smallest max
// yielded before it). SynthTimer(t) fires: v = mix(i, t, v) mod K; if v mod P == 0, send Poke to
// node i+1 (mod N); re-set SynthTimer(t) (the fired entry is removed after the handler, so t
// moves to the back of the queue). Poke delivered to node i: pokes = pokes+1 mod 4, v =
// mix(i, 4 + pokes, v) mod K. mix = splitmix64 of (seed ^ i << 48 ^ t << 40 ^ v): the seeded
// transition table. Branching: 4N timer events + up to N pokes (~20-25 at N = 5).
//
// Packed node (2 words): w0 = v:16 | pokes:2 @16; w1 = timer queue, 4 types x 2 bits in order.
// Records (32 bit): Poke = from:3 @27 | to:3 @24. State: 10 node words + count + 5 records = 64 B.
#pragma once
#include "../nodestate.hpp"

namespace dsl {

// k_level at 6 waves per SIMD (80 VGPRs): as fast as 8 (64 VGPRs) on C3 d10 with half the scratch
// (60 vs 124 B per lane; profiles/r06_c3_dedup_waves_ab.txt)
#ifndef DSL_SYNTH_WAVES
#define DSL_SYNTH_WAVES 6
#endif

struct Synthetic {
  static constexpr int kMaxNodes = 5;
  static constexpr int kNodes = kMaxNodes, kNodeWords = 2, kNetCap = kMaxNodes, kMaxSends = 1;
  static constexpr int kLevelWaves = DSL_SYNTH_WAVES;  // k_level waves per SIMD (kernels.hpp LevelWaves)
// k_level's in-chunk duplicate filter (kernels.hpp ChunkDedup): off. 18 % of C3's probes are
// in-chunk duplicates (profiles/r06_chunk_census.txt), but the filter measured 7 % slower on C3 d10
// (profiles/r06_c3_dedup_waves_ab.txt): every probing lane pays its LDS CAS chain, and a
// duplicate's global probe is cheap (its line was just touched by the first occurrence).
#ifndef DSL_SYNTH_DEDUP
#define DSL_SYNTH_DEDUP 0
#endif
  static constexpr bool kChunkDedup = DSL_SYNTH_DEDUP;
  // on sharded levels the filter would keep duplicates off the links (16 B each) and the owners'
  // probes -- but the device's frontier order leaves few of them in a chunk (siblings are emitted
  // by different waves and passes, interleaved with other workgroups' rows): with the filter on, C3
  // d9 at W = 8 routed 549.7 M instead of 551.5 M records, while its k_level took 13 % longer
  // (profiles/r06_shard_scale.txt). Off.
#ifndef DSL_SYNTH_ROUTE_DEDUP
#define DSL_SYNTH_ROUTE_DEDUP 0
#endif
  static constexpr bool kRouteDedup = DSL_SYNTH_ROUTE_DEDUP;
  static constexpr int kMsgClasses = 1;  // handler classes of messages (Poke); timers: class 1
  static constexpr int kTimerMin = 1, kTimerMax = 100;
  using Rec = uint32_t;
  using State = StateOf<Synthetic>;

  struct Params {
    int32_t nodes, K, P, pad;
    uint64_t seed;
  };
  enum { M_POKE = 0, T_SYNTH = 1 };

  static DSL_HD uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  static DSL_HD int mix(const Params& p, int i, int t, int v) {
    return (int)(splitmix64(p.seed ^ ((uint64_t)i << 48) ^ ((uint64_t)t << 40) ^ (uint64_t)v) % (uint64_t)p.K);
  }
  static DSL_HD Rec poke(int from, int to) { return ((Rec)from << 27) | ((Rec)to << 24); }
  static DSL_HD int rec_from(Rec r) { return (int)((r >> 27) & 7); }
  static DSL_HD int rec_to(Rec r) { return (int)((r >> 24) & 7); }
  static DSL_HD int msg_class(Rec) { return 0; }

  static DSL_HD int v_of(const uint32_t* w) { return (int)(w[0] & 0xffff); }
  static DSL_HD int pokes_of(const uint32_t* w) { return (int)((w[0] >> 16) & 3); }
  static DSL_HD int timer_at(const uint32_t* w, int j) { return (int)((w[1] >> (2 * j)) & 3); }

  static DSL_HD int num_nodes(const Params& p) { return p.nodes; }
  template <class O>
  static DSL_HD void init_node(int, uint32_t* w, O&, const Params&) {
    w[0] = 0;
    w[1] = 0 | (1 << 2) | (2 << 4) | (3 << 6);  // init(): set SynthTimer(0), (1), (2), (3)
  }
  static DSL_HD int num_timer_events(int, const uint32_t*, const Params&) { return 4; }

  template <class O>
  static DSL_HD int on_timer(int i, uint32_t* w, int j, O& out, const Params& p) {
    const int t = timer_at(w, j);
    const int v = mix(p, i, t, v_of(w));
    w[0] = (w[0] & ~0xffffu) | (uint32_t)v;
    if (v % p.P == 0) out.send(poke(i, (i + 1) % p.nodes));
    // re-set SynthTimer(t) (appended), then the fired entry j is removed: t moves to the back
    const uint32_t q = w[1];
    const uint32_t lo = q & ((1u << (2 * j)) - 1u), hi = (q >> (2 * j + 2)) << (2 * j);
    w[1] = (lo | hi | ((uint32_t)t << 6)) & 0xffu;
    return STEP_OK;
  }
  template <class O>
  static DSL_HD int on_message(int i, uint32_t* w, Rec, O&, const Params& p) {
    const int k = (pokes_of(w) + 1) & 3;
    const int v = mix(p, i, 4 + k, v_of(w));
    w[0] = (uint32_t)v | ((uint32_t)k << 16);
    return STEP_OK;
  }

  static DSL_HD int eval(const DevPred& pr, const NodeView& vw, const Params& p) {
    switch (pr.id) {
      case DSL_PRED_SYNTH_NOT_ALL_MAX:
        for (int i = 0; i < p.nodes; i++)
          if (v_of(vw.node(i)) != p.K - 1) return PV_TRUE;
        return PV_FALSE;
      case DSL_PRED_SYNTH_COUNTER_LT:
        if (pr.arg0 < 0 || pr.arg0 >= p.nodes) return PV_THREW;
        return v_of(vw.node((int)pr.arg0)) < pr.arg1 ? PV_TRUE : PV_FALSE;
      default:
        return PV_THREW;
    }
  }
  static uint32_t pred_reads(const DevPred& pr, const Params& p) {
    if (pr.id == DSL_PRED_SYNTH_COUNTER_LT && pr.arg0 >= 0 && pr.arg0 < p.nodes) return 1u << pr.arg0;
    if (pr.id == DSL_PRED_SYNTH_NOT_ALL_MAX) return (1u << p.nodes) - 1u;
    return kReadsAll;
  }
  static bool known_predicate(int id) { return id == DSL_PRED_SYNTH_NOT_ALL_MAX || id == DSL_PRED_SYNTH_COUNTER_LT; }
  static bool valid(const Params& p) {
    return p.nodes >= 1 && p.nodes <= kMaxNodes && p.K >= 1 && p.K <= 65536 && p.P >= 1;
  }
  // params: nodes, K, P, seed (64 bit)
  static Params from_desc(const dsl_protocol_desc& d) {
    Params p{};
    p.nodes = (int32_t)d.params[0];
    p.K = (int32_t)d.params[1];
    p.P = (int32_t)d.params[2];
    p.seed = (uint64_t)d.params[3];
    return p;
  }
  static void describe_message(Rec r, dsl_event* e) {
    e->from = rec_from(r);
    e->to = rec_to(r);
    e->type = M_POKE;
    e->n_fields = 0;
  }
  static void describe_timer(int i, const uint32_t* w, int j, const Params&, dsl_event* e) {
    e->is_timer = 1;
    e->from = e->to = i;
    e->timer_min = kTimerMin;
    e->timer_max = kTimerMax;
    e->type = T_SYNTH;
    e->n_fields = 1;
    e->fields[0] = timer_at(w, j);
  }
};

}  // namespace dsl
