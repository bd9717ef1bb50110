// tests/hostcheck/protocheck.cpp -- TEST TOOL, not part of the product.
//
// Runs a protocol's packed-state transition functions (the same __host__ __device__ code the
// HIP kernels execute) in a plain host BFS with EXACT state equality (no fingerprints), so a
// protocol encoding can be checked against the oracle's per-depth vectors on a machine with no
// GPU. It also cross-checks the incremental (delta) fingerprint against a full recomputation on
// every generated successor. It never stands in for the engine: the Search API only runs the
// libdslabs_hip.so kernels.
//
// usage: protocheck <proto> <params...> -- <inv ids> / <goal ids> / <prune ids> maxdepth
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../dslabs_amd/csrc/protocols/all.hpp"

using namespace dsl;

// Every send of one step, duplicates kept (the check behind P::kSendsDistinct).
template <class P>
struct RawSender {
  typename P::Rec r[64];
  int n = 0;
  bool overflow = false;
  void send(typename P::Rec x) {
    if (n < 64) r[n] = x;
    n++;
  }
};
template <class P>
static bool sends_distinct(const uint32_t* w, int k, const typename P::Params& prm, const DevSettings& set) {
  const int e = locate_event<P>(w, prm, set, k);
  if (e == INT32_MIN) return true;
  uint32_t nw[P::kNodeWords];
  RawSender<P> out;
  if (e >= 0) {
    const auto r = Net<P>::at(w, e);
    const int node = P::rec_to(r);
    if (node >= P::num_nodes(prm)) return true;
    for (int i = 0; i < P::kNodeWords; i++) nw[i] = w[node * P::kNodeWords + i];
    P::on_message(node, nw, r, out, prm);
  } else {
    const int x = -1 - e, node = x >> 8;
    for (int i = 0; i < P::kNodeWords; i++) nw[i] = w[node * P::kNodeWords + i];
    P::on_timer(node, nw, x & 255, out, prm);
  }
  for (int a = 0; a < out.n && a < 64; a++)
    for (int b = a + 1; b < out.n && b < 64; b++)
      if (out.r[a] == out.r[b]) return false;
  return true;
}

template <class P>
static int run(const dsl_protocol_desc& d, DevSettings set) {
  typename P::Params prm = P::from_desc(d);
  set_pred_reads<P>(set, prm);
  if (!P::valid(prm)) {
    printf("{\"error\":\"invalid params\"}\n");
    return 1;
  }
  using S = typename P::State;
  constexpr int NWORDS = Layout<P>::kWords;
  struct Node {
    S s;
    int depth;
    long long id;
    Fp fp;
  };
  std::vector<std::pair<long long, int>> parent{{-1, -1}};
  long long first_term_parent = -2;
  int first_term_event = -1;
  auto key = [](const S& s) { return std::string((const char*)s.w, sizeof(S)); };
  S init;
  if (!init_state<P>(init.w, prm)) {
    printf("{\"error\":\"init overflow\"}\n");
    return 1;
  }
  std::unordered_set<std::string> seen;
  std::deque<Node> q;
  std::vector<unsigned long long> per;
  seen.insert(key(init));
  per.push_back(1);
  int pi = -1;
  NodeView v0{init.w, P::kNodeWords, -1, nullptr};
  int v = judge_view<P>(v0, prm, set, 0, &pi);
  const char* end = "SPACE_EXHAUSTED";
  int tdepth = -1;
  long long nterm[3] = {0, 0, 0};
  long long fp_mismatch = 0, emit_mismatch = 0, judge_mismatch = 0, noop = 0, succ = 0, dup_sends = 0, skipped = 0, skip_mismatch = 0;
  if (v >= V_TERM_EXCEPTION) {
    end = v == V_TERM_INVARIANT ? "INVARIANT_VIOLATED" : "GOAL_FOUND";
    tdepth = 0;
  } else {
    q.push_back({init, 0, 0, full_fingerprint<P>(init.w)});
  }
  int best = 99;
  while (!q.empty()) {
    Node n = q.front();
    if (tdepth >= 0 && n.depth + 1 > tdepth) break;
    q.pop_front();
    const int ne = count_events<P>(n.s.w, prm, set);
    for (int k = 0; k < ne; k++) {
      Delta<P> dl;
      const int rc = delta_step<P>(n.s.w, k, dl, prm, set);
      if (event_class_skip<P>(n.s.w, prm, set, k) == Classes<P>::kSkip) {  // the kernels skip its handler
        skipped++;
        if (rc != STEP_OK || dl.keep != 0 || !same_words<P::kNodeWords>(dl.nw, n.s.w + dl.node * P::kNodeWords))
          skip_mismatch++;
      }
      if (rc == STEP_NULL) continue;
      if (rc == STEP_OVERFLOW) {
        printf("{\"error\":\"overflow\"}\n");
        return 1;
      }
      const int d = n.depth + 1;
      succ++;
      if (rc == STEP_EXCEPTION) {
        if ((int)per.size() <= d) per.resize(d + 1, 0);
        per[d]++;
        if (tdepth < 0) tdepth = d;
        if (d == tdepth) nterm[0]++;
        best = std::min(best, (int)V_TERM_EXCEPTION);
        continue;
      }
      const bool is_noop = dl.keep == 0 && same_words<P::kNodeWords>(dl.nw, n.s.w + dl.node * P::kNodeWords);
      if (is_noop) noop++;

      if constexpr (SendsDistinct<P>::value) {  // P::kSendsDistinct: no record sent twice in one step
        if (!sends_distinct<P>(n.s.w, k, prm, set)) dup_sends++;
      }
      S t;
      if (!materialize<P>(n.s.w, dl, t.w)) {
        printf("{\"error\":\"overflow\"}\n");
        return 1;
      }
      {  // the kernels' lane-parallel merge (emit_row: wave_emit's rank rule) must produce the same row
        S e;
        if (!emit_row<P>(n.s.w, dl, e.w) || std::memcmp(e.w, t.w, sizeof(S)) != 0) emit_mismatch++;
      }
      const Fp f = delta_fingerprint<P>(n.s.w, n.fp, dl);
      const Fp g = full_fingerprint<P>(t.w);
      if (f.hi != g.hi || f.lo != g.lo) fp_mismatch++;
      {  // k_level's form: the parent's node hash cached per parent (LDS), removed once
        const Fp c = delta_fingerprint_cached<P>(
            fp_xor(n.fp, node_hash<P>(dl.node, n.s.w + dl.node * P::kNodeWords)), dl);
        if (c.hi != g.hi || c.lo != g.lo) fp_mismatch++;
      }
      if (!seen.insert(key(t)).second) continue;
      if ((int)per.size() <= d) per.resize(d + 1, 0);
      per[d]++;
      NodeView view{n.s.w, P::kNodeWords, dl.node, dl.nw};
      typename P::Rec news[P::kMaxSends];
      view.sends = news;
      view.nsends = delta_sends<P>(dl, news);
      v = judge_view<P>(view, prm, set, d, &pi);
      if (n.depth > 0) {  // the kernels' incremental check must give the same verdict
        int pi2 = -1;
        const int v2 = judge_view<P>(view, prm, set, d, &pi2, true);
        if (v2 != v || (v >= V_TERM_EXCEPTION && pi2 != pi)) judge_mismatch++;
      }
      if (v >= V_TERM_EXCEPTION) {
        if (tdepth < 0) tdepth = d;
        if (d == tdepth) nterm[v - V_TERM_EXCEPTION]++;
        if (first_term_parent == -2) first_term_parent = n.id, first_term_event = k;
        best = std::min(best, v);
        continue;
      }
      if (v == V_PRUNED) continue;
      parent.push_back({n.id, k});
      q.push_back({t, d, (long long)parent.size() - 1, g});
    }
  }
  if (best != 99)
    end = best == V_TERM_EXCEPTION ? "EXCEPTION_THROWN" : best == V_TERM_INVARIANT ? "INVARIANT_VIOLATED" : "GOAL_FOUND";
  unsigned long long total = 0;
  printf("{\"end\":\"%s\",\"terminal_depth\":%d,\"state_bytes\":%d,\"fp_mismatch\":%lld,\"emit_mismatch\":%lld,"
         "\"judge_mismatch\":%lld,\"dup_sends\":%lld,\"skip_mismatch\":%lld,\"skipped\":%lld,\"per_depth\":[", end, tdepth,
         (int)sizeof(S), fp_mismatch, emit_mismatch, judge_mismatch, dup_sends, skip_mismatch, skipped);
  for (size_t i = 0; i < per.size(); i++) {
    printf("%s%llu", i ? "," : "", per[i]);
    total += per[i];
  }
  printf("],\"terminals_at_depth\":[%lld,%lld,%lld],\"states\":%llu,\"successors\":%lld,\"noop_successors\":%lld", nterm[0], nterm[1], nterm[2], total, succ, noop);
  if (first_term_parent >= 0) {
    std::vector<int> evs{first_term_event};
    for (long long id = first_term_parent; id > 0; id = parent[id].first) evs.push_back(parent[id].second);
    std::reverse(evs.begin(), evs.end());
    printf(",\"trace\":[");
    S s = init, t;
    for (size_t i = 0; i < evs.size(); i++) {
      dsl_event e;
      describe_event<P>(s.w, evs[i], prm, set, &e);
      printf("%s[%d,%d,%d,%d,%lld]", i ? "," : "", e.is_timer, e.from, e.to, e.type, (long long)e.fields[0]);
      full_step<P>(s.w, evs[i], t.w, prm, set);
      s = t;
    }
    printf("]");
  }
  (void)NWORDS;
  printf("}\n");
  return 0;
}

// ViewServerTest (labs/lab2-primarybackup/tst/dslabs/primarybackup/ViewServerTest.java:156-303)
// against a DEVICE ViewServer handler (PB node 0), the same scenarios the oracle replays: the
// hand-written one (csrc/protocols/pb.hpp) or the IR-generated one (csrc/protocols/gen/pb_ir.hpp).
// Both reply with the view as num | p << 4 | b << 6 in the record's low byte.
struct VsHand {
  using P = PB;
  static PB::Rec ping(int n, int from) { return PB::msg(PB::M_PING, from, 0, (uint64_t)n); }
  static PB::Rec getview() { return PB::msg(PB::M_GETVIEW, 4, 0, 0); }
  static void init(uint32_t*, const PB::Params&) {}
};
struct VsIR {  // records: type << 60 | from << 57 | to << 54 | fields; Ping = 0 (num: bits 0-3), GetView = 1
  using P = PBIR;
  static PBIR::Rec ping(int n, int from) { return ((PBIR::Rec)from << 57) | (PBIR::Rec)(n & 15); }
  static PBIR::Rec getview() { return ((PBIR::Rec)1 << 60) | ((PBIR::Rec)4 << 57); }
  static void init(uint32_t* w, const PBIR::Params& p) {  // the ViewServer's init: its PingCheckTimer
    Sender<PBIR> out;
    PBIR::init_viewserver(0, w, out, p);
  }
};

template <class V>
static int vstest() {
  using P = typename V::P;
  struct H {
    typename P::Params p{};
    uint32_t w[P::kNodeWords] = {};
    bool ok = true;
    H() {
      p.servers = 3; p.clients = 1; p.ncmds = 1;
      V::init(w, p);
    }
    void ping(int n, int from) {
      Sender<P> out;
      if (P::on_message(0, w, V::ping(n, from), out, p) != STEP_OK) ok = false;
    }
    void timeout() {
      Sender<P> out;
      if (P::on_timer(0, w, 0, out, p) != STEP_OK) ok = false;
    }
    int get() {  // GetView: the ViewReply's view (num | p << 4 | b << 6)
      Sender<P> out;
      if (P::on_message(0, w, V::getview(), out, p) != STEP_OK || out.n != 1) ok = false;
      return (int)(out.r[0] & 0xff);
    }
    void check(int pr, int b, int n) {
      const int v = get();
      if (PB::v_p(v) != pr || PB::v_b(v) != b || (n >= 0 && PB::v_num(v) != n)) ok = false;
    }
    void setup(int pr, int b, bool ack) {
      ping(0, pr);
      check(pr, 0, 1);
      if (b) {
        ping(1, pr);
        ping(0, b);
        check(pr, b, 2);
      }
      if (ack) ping(b ? 2 : 1, pr);
    }
    void full(std::vector<int> ps) {
      const int n = PB::v_num(get());
      for (int i = 0; i < 2; i++) {
        for (int x : ps) ping(n, x);
        timeout();
      }
    }
  };
  std::vector<std::pair<const char*, void (*)(H&)>> t = {
      {"test01StartupViewCorrect", [](H& h) { h.check(0, 0, 0); }},
      {"test02firstPrimary", [](H& h) { h.setup(1, 0, false); }},
      {"test03FirstBackup", [](H& h) { h.setup(1, 2, false); }},
      {"test04BackupPingsFirst", [](H& h) { h.setup(1, 0, false); h.ping(0, 2); h.ping(1, 1); h.check(1, 2, 2); }},
      {"test05BackupTakesOver", [](H& h) {
         h.setup(1, 2, true); h.ping(2, 2); h.check(1, 2, 2); h.timeout(); h.ping(2, 2); h.check(1, 2, 2);
         h.timeout(); h.check(2, 0, 3); }},
      {"test06OldServerBecomesBackup", [](H& h) {
         h.setup(1, 2, true); h.full({2}); h.check(2, 0, 3); h.ping(3, 2); h.ping(2, 1); h.check(2, 1, 4); }},
      {"test07IdleThirdServerBecomesBackup", [](H& h) { h.setup(1, 2, true); h.full({2, 3}); h.check(2, 3, 3); }},
      {"test08WaitForPrimaryAck", [](H& h) {
         h.ping(0, 1); h.ping(0, 2); h.check(1, 0, 1); h.ping(1, 1); h.check(1, 2, 2); h.ping(1, 2); h.full({2});
         h.check(1, 2, 2); }},
      {"test09DeadBackupRemoved", [](H& h) { h.setup(1, 2, true); h.full({1}); h.check(1, 0, 3); }},
      {"test10UninitializedNotPromoted", [](H& h) {
         h.setup(1, 2, true); h.full({2, 3}); h.check(2, 3, 3); h.full({3}); h.check(2, 3, 3); }},
      {"test11DeadServerNotMadeBackup", [](H& h) {
         h.setup(1, 0, false); h.ping(0, 2); h.full({}); h.ping(1, 1); h.check(1, 0, 1); }},
      {"test12NewViewNotStarted", [](H& h) {
         h.setup(1, 0, false); h.full({1}); h.check(1, 0, 1); h.full({}); h.check(1, 0, 1); h.ping(1, 1);
         h.full({1}); h.check(1, 0, 1); h.full({}); h.check(1, 0, 1); h.ping(0, 2); h.check(1, 2, 2); h.ping(2, 1);
         h.check(1, 2, 2); h.full({1, 2}); h.check(1, 2, 2); h.full({});
         const int v = h.get();
         if (PB::v_p(v) == 1 && PB::v_b(v) == 2 && PB::v_num(v) != 2) h.ok = false; }},
  };
  printf("{\"results\":[");
  for (size_t i = 0; i < t.size(); i++) {
    H h;
    t[i].second(h);
    printf("%s{\"name\":\"%s\",\"ok\":%s}", i ? "," : "", t[i].first, h.ok ? "true" : "false");
  }
  printf("]}\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && strcmp(argv[1], "vstest") == 0) return vstest<VsHand>();
  if (argc > 1 && strcmp(argv[1], "vstest_ir") == 0) return vstest<VsIR>();
  dsl_protocol_desc d{};
  int i = 1;
  d.protocol = atoi(argv[i++]);
  while (i < argc && strcmp(argv[i], "--") != 0) d.params[d.n_params++] = atoll(argv[i++]);
  i++;
  DevSettings set{};
  for (int a = 0; a < DSL_MAX_NODES; a++) set.deliver[a] = 0xffffffffu;
  set.timer_mask = 0xffffffffu;
  set.all_deliver = 1;
  DevProg* lists[3] = {set.inv, set.goal, set.prune};
  int* counts[3] = {&set.n_inv, &set.n_goal, &set.n_prune};
  int which = 0;
  for (; i < argc - 1; i++) {
    if (strcmp(argv[i], "/") == 0) {
      which++;
      continue;
    }
    // predicate token: a leaf [-]id[:arg0[:arg1]] (leading '-' = negated), or a postfix program of
    // leaves and the combinators "and" / "or" / "not" joined by commas
    const int start = set.n_ops;
    for (const char* tok = argv[i]; *tok;) {
      const char* end = strchr(tok, ',');
      std::string t(tok, end ? (size_t)(end - tok) : strlen(tok));
      DevPred p{};
      if (t == "and") p.id = kOpAnd;
      else if (t == "or") p.id = kOpOr;
      else if (t == "not") p.id = kOpNot;
      else {
        int id = 0, a0 = 0, a1 = 0;
        sscanf(t.c_str(), "%d:%d:%d", &id, &a0, &a1);
        p.negate = id < 0;
        p.id = id < 0 ? -id : id;
        p.arg0 = a0;
        p.arg1 = a1;
      }
      set.ops[set.n_ops++] = p;
      tok = end ? end + 1 : tok + t.size();
    }
    lists[which][(*counts[which])++] = DevProg{(int16_t)start, (int16_t)(set.n_ops - start)};
  }
  set.max_depth = atoi(argv[argc - 1]);
  switch (d.protocol) {
    case DSL_PROTO_PINGPONG: return run<PingPong>(d, set);
    case DSL_PROTO_SIPAXOS: return run<SIPaxos>(d, set);
    case DSL_PROTO_MULTIPAXOS: return run<MultiPaxos>(d, set);
    case DSL_PROTO_SYNTHETIC: return run<Synthetic>(d, set);
    case DSL_PROTO_AMOKV: return run<AmoKV>(d, set);
    case DSL_PROTO_PB: return run<PB>(d, set);
    case DSL_PROTO_MINITEST: return run<MiniTest>(d, set);
    case DSL_PROTO_PINGPONG_IR: return run<PingPongIR>(d, set);
    case DSL_PROTO_AMOKV_IR: return run<AmoKVIR>(d, set);
    case DSL_PROTO_MULTIPAXOS_IR: return run<MultiPaxosIR>(d, set);
    case DSL_PROTO_PB_IR: return run<PBIR>(d, set);
  }
  return 2;
}
