// tools/cpu_bfs.cpp -- the multithreaded CPU baseline of bench.py: the
// reference's level-synchronous BFS (Search.java:241-348: worker threads take states of the
// current level from a shared queue, expand them, add unseen successors to a concurrent visited
// set and the next level) on the host's cores, over the SAME packed transition functions the HIP
// kernels run (dslabs_amd/csrc/protocols/*.hpp compiled for the host). It is a measurement tool,
// never a fallback: the Search API only runs libdslabs_hip.so.
//
// Per level: T threads claim chunks of the frontier with one atomic counter; each successor is
// built as a delta of its parent (delta_step), no-op successors (node unchanged, nothing sent)
// are dropped as the kernels drop them, the rest are fingerprinted incrementally and inserted into
// a lock-free open-addressing set of 64-bit keys (one CAS per new state, the kernels' key), then
// judged (checkState order); VALID states go to the thread's part of the next frontier. The
// counts follow exploreNode (every new successor counts, terminal and pruned ones included), so
// per-depth vectors equal the GPU's and the oracle's (tests/test_cpu_bfs.py).
//
// usage: cpu_bfs <blob> <threads> <table_log2> [repeat [min_seconds]]
//   blob = dsl_protocol_desc bytes followed by dsl_settings bytes (bench.py writes it); with
//   repeat > 1 the search runs that many times on the same buffers and the runs after the first
//   are timed (the first one grows the frontier buffers, as bench.py's GPU warmup step does);
//   min_seconds > 0 repeats the timed runs until they add up to that much time
// prints one JSON line: end, per_depth, states (per run), elapsed_s (last run), threads,
// states_per_s (timed runs' states / their time), runs, timed_s
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unordered_set>
#include <vector>

#include "../dslabs_amd/csrc/protocols/all.hpp"
#include "../dslabs_amd/csrc/settings.hpp"

using namespace dsl;

namespace {

struct VisitedSet {
  std::vector<std::atomic<uint64_t>> slots;
  uint64_t mask;
  explicit VisitedSet(int log2) : slots(1ull << log2), mask((1ull << log2) - 1) {}
  // 1 = inserted, 0 = present, -1 = full
  int insert(const Fp& f) {
    const uint64_t key = f.hi | 1ull;
    uint64_t i = f.lo & mask;
    for (uint64_t n = 0; n <= mask; n++, i = (i + 1) & mask) {
      uint64_t cur = slots[i].load(std::memory_order_relaxed);
      if (cur == key) return 0;
      if (cur == 0) {
        if (slots[i].compare_exchange_strong(cur, key, std::memory_order_relaxed)) return 1;
        if (cur == key) return 0;
      }
    }
    return -1;
  }
};

template <class P>
int run(const dsl_protocol_desc& d, const dsl_settings& hs, int threads, int table_log2, int repeat,
        double min_s, const std::vector<uint8_t>& start, int depth0) {
  const typename P::Params prm = P::from_desc(d);
  if (!P::valid(prm)) return fprintf(stderr, "invalid params\n"), 2;
  DevSettings set;
  std::string why;
  if (resolve_settings(hs, P::num_nodes(prm), &P::known_predicate, &set, &why))
    return fprintf(stderr, "settings: %s\n", why.c_str()), 2;
  set_pred_reads<P>(set, prm);
  constexpr int NW = Layout<P>::kWords;
  struct Row {
    uint32_t w[NW];
    Fp fp;
  };
  Row init;
  if (!init_state<P>(init.w, prm)) return fprintf(stderr, "init overflow\n"), 2;
  if (!start.empty()) {  // a start state of an earlier search (the engine's dsl_set_initial)
    if (start.size() != sizeof(init.w)) return fprintf(stderr, "start state size\n"), 2;
    std::memcpy(init.w, start.data(), sizeof(init.w));
  }
  init.fp = full_fingerprint<P>(init.w);

  VisitedSet seen(table_log2);
  // frontier buffers, one per thread and level parity: kept (with their capacity) across levels
  // and runs, as the engine keeps its device buffers across searches
  std::vector<std::vector<Row>> buf_a(threads), buf_b(threads);
  std::vector<unsigned long long> per;
  int best = 99;
  const char* err = nullptr;
  double el = 0, timed = 0;
  int timed_runs = 0;
  // the first run only grows the buffers (the GPU's warmup step); with min_s > 0 the timed runs
  // repeat until they add up to at least min_s seconds (a bounded sample of ~10 s of CPU work)
  for (int run = 0; !err && (run < repeat || (min_s > 0 && timed < min_s)); run++) {
  const auto t0 = std::chrono::steady_clock::now();
  {  // the visited set starts empty (cleared by all threads)
    std::vector<std::thread> pool;
    const uint64_t n = seen.slots.size(), per_t = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++)
      pool.emplace_back([&, t] {
        for (uint64_t i = t * per_t; i < std::min(n, (t + 1) * per_t); i++) seen.slots[i].store(0, std::memory_order_relaxed);
      });
    for (auto& th : pool) th.join();
  }
  seen.insert(init.fp);
  per.assign(1, 1);
  int pi = -1;
  const NodeView v0{init.w, P::kNodeWords, -1, nullptr};
  best = judge_view<P>(v0, prm, set, depth0, &pi);
  auto* cur = &buf_a;
  auto* nxt = &buf_b;
  for (auto& v : *cur) v.clear();
  if (best < V_TERM_EXCEPTION) (*cur)[0].push_back(init);
  best = best >= V_TERM_EXCEPTION ? best : 99;
  // the frontier as (part, index) ranges: parts are the previous level's per-thread vectors
  for (int depth = depth0; best == 99 && !err; depth++) {
    std::vector<uint64_t> start{0};
    for (auto& p : *cur) start.push_back(start.back() + p.size());
    const uint64_t F = start.back();
    if (F == 0) break;
    std::atomic<uint64_t> next_i{0};
    std::atomic<unsigned long long> level_new{0};
    std::atomic<int> level_best{99};
    std::atomic<int> level_err{0};
    // DSL_CPU_CHUNK_CENSUS=PB: chunks of PB consecutive frontier rows (k_level's chunk), and per
    // level the probed successors whose fingerprint an earlier successor of the SAME chunk already
    // had (diamonds among sibling parents: what an in-chunk LDS dedup would take off the global
    // probes), to stderr
    static const uint64_t chunk_census = getenv("DSL_CPU_CHUNK_CENSUS") ? strtoull(getenv("DSL_CPU_CHUNK_CENSUS"), nullptr, 10) : 0;
    const uint64_t kChunk = chunk_census ? chunk_census : 64;
    std::atomic<unsigned long long> cc_probed{0}, cc_dup{0};
    // DSL_CPU_CENSUS: per handler class (event_class_skip), events / filtered as surely no-op /
    // run but no-op / probed / new (a measurement of the no-op filter's reach, to stderr)
    constexpr int NC = Classes<P>::kCount;
    static const bool census = getenv("DSL_CPU_CENSUS") != nullptr;
    std::vector<std::array<unsigned long long, 5 * NC>> cen(threads);
    for (auto& c : cen) c.fill(0);
    auto work = [&](int t) {
      std::vector<Row>& out = (*nxt)[t];
      out.clear();
      unsigned long long c_new = 0;
      int my_best = 99, my_err = 0;
      Row s;
      for (;;) {
        const uint64_t b = next_i.fetch_add(kChunk, std::memory_order_relaxed);
        if (b >= F) break;
        const uint64_t e = std::min(F, b + kChunk);
        std::unordered_set<uint64_t> local;
        size_t part = std::upper_bound(start.begin(), start.end(), b) - start.begin() - 1;
        for (uint64_t g = b; g < e; g++) {
          while (g >= start[part + 1]) part++;
          const Row& r = (*cur)[part][g - start[part]];
          const int ne = count_events<P>(r.w, prm, set);
          for (int k = 0; k < ne; k++) {
            Delta<P> dl;
            int cls = 0, real = 0;
            if (census) {
              cls = event_class_skip<P>(r.w, prm, set, k);
              // the filtered events' real class (the handler a skipped event would have run)
              real = cls;
              if (cls == Classes<P>::kSkip) {
                const int e = locate_event<P>(r.w, prm, set, k);
                real = e < 0 ? Classes<P>::kTimer0 + TimerClasses<P>::of((-1 - e) >> 8, prm) : P::msg_class(Net<P>::at(r.w, e));
              }
              cen[t][5 * real + (cls == Classes<P>::kSkip ? 1 : 0)]++;
            }
            const int rc = delta_step<P>(r.w, k, dl, prm, set);
            if (census && cls != Classes<P>::kSkip) {
              const bool nop = rc == STEP_OK && dl.keep == 0 && same_words<P::kNodeWords>(dl.nw, r.w + dl.node * P::kNodeWords);
              cen[t][5 * real + (nop ? 2 : 3)]++;
            }
            if (rc == STEP_NULL) continue;
            if (rc == STEP_EXCEPTION) {  // never equal to another state: new and terminal
              c_new++;
              my_best = std::min(my_best, (int)V_TERM_EXCEPTION);
              continue;
            }
            if (rc == STEP_OVERFLOW) {
              my_err = 1;
              continue;
            }
            if (dl.keep == 0 && same_words<P::kNodeWords>(dl.nw, r.w + dl.node * P::kNodeWords)) continue;
            const Fp f = delta_fingerprint<P>(r.w, r.fp, dl);
            if (chunk_census) {
              cc_probed++;
              if (!local.insert(f.lo ^ (f.hi * 0x9E3779B97F4A7C15ull)).second) cc_dup++;
            }
            const int ins = seen.insert(f);
            if (ins < 0) {
              my_err = 2;
              continue;
            }
            if (ins == 0) continue;
            c_new++;
            if (census) cen[t][5 * (cls == Classes<P>::kSkip ? 0 : cls) + 4]++;
            int pidx = -1;
            NodeView view{r.w, P::kNodeWords, dl.node, dl.nw};
            typename P::Rec news[P::kMaxSends];
            view.sends = news;
            view.nsends = delta_sends<P>(dl, news);
            const int v = judge_view<P>(view, prm, set, depth + 1, &pidx, depth > depth0);
            if (v >= V_TERM_EXCEPTION) {
              my_best = std::min(my_best, v);
              continue;
            }
            if (v == V_PRUNED) continue;
            if (!emit_row<P>(r.w, dl, s.w)) {
              my_err = 1;
              continue;
            }
            s.fp = f;
            out.push_back(s);
          }
        }
      }
      level_new += c_new;
      int cb = level_best.load();
      while (my_best < cb && !level_best.compare_exchange_weak(cb, my_best)) {
      }
      if (my_err) level_err = my_err;
    };
    const auto lt0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
    if (getenv("DSL_CPU_TRACE"))
      fprintf(stderr, "level %d: %llu parents, %.3f ms\n", depth + 1, (unsigned long long)F,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - lt0).count());
    if (chunk_census)
      fprintf(stderr, "chunk census level %d (PB %llu): probed %llu, in-chunk duplicates %llu (%.1f %%), new %llu\n", depth + 1,
              (unsigned long long)chunk_census, cc_probed.load(), cc_dup.load(),
              cc_probed.load() ? 100.0 * cc_dup.load() / cc_probed.load() : 0.0, level_new.load());
    if (census) {
      fprintf(stderr, "census level %d (class: events filtered run_noop probed new):", depth + 1);
      for (int c = 0; c < NC; c++) {
        unsigned long long v[5] = {0, 0, 0, 0, 0};
        for (auto& x : cen)
          for (int i = 0; i < 5; i++) v[i] += x[5 * c + i];
        if (v[0] || v[1] || v[2] || v[3])
          fprintf(stderr, " | %d: %llu %llu %llu %llu %llu", c, v[0] + v[1], v[1], v[2], v[3], v[4]);
      }
      fprintf(stderr, "\n");
    }
    per.push_back(level_new.load());
    if (level_err) err = level_err == 2 ? "visited table full" : "network overflow";
    best = level_best.load();
    std::swap(cur, nxt);
  }
  el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (run > 0 || repeat == 1) {
    timed += el;
    timed_runs++;
  }
  }
  if (err) return fprintf(stderr, "error: %s\n", err), 3;
  while (per.size() > 1 && per.back() == 0) per.pop_back();
  unsigned long long total = 0;
  for (auto c : per) total += c;
  const char* end = best == 99 ? "SPACE_EXHAUSTED"
                    : best == V_TERM_EXCEPTION ? "EXCEPTION_THROWN"
                    : best == V_TERM_INVARIANT ? "INVARIANT_VIOLATED"
                                               : "GOAL_FOUND";
  printf("{\"end\":\"%s\",\"states\":%llu,\"elapsed_s\":%.6f,\"threads\":%d,\"states_per_s\":%.1f,"
         "\"runs\":%d,\"timed_s\":%.6f,\"per_depth\":[",
         end, total, el, threads, (double)total * timed_runs / timed, timed_runs, timed);
  for (size_t i = 0; i < per.size(); i++) printf("%s%llu", i ? "," : "", per[i]);
  printf("]}\n");
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) return fprintf(stderr, "usage: cpu_bfs <blob> <threads> <table_log2> [repeat [min_seconds]]\n"), 2;
  dsl_protocol_desc d;
  dsl_settings s;
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(&d, sizeof d, 1, f) != 1 || fread(&s, sizeof s, 1, f) != 1)
    return fprintf(stderr, "cannot read %s\n", argv[1]), 2;
  // optional: int32 start depth + the packed start state (tools/cpu_baseline.py)
  int depth0 = 0;
  std::vector<uint8_t> start;
  if (fread(&depth0, sizeof depth0, 1, f) == 1) {
    uint8_t buf[4096];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) start.insert(start.end(), buf, buf + n);
  }
  fclose(f);
  const int threads = std::max(1, atoi(argv[2])), log2 = std::max(10, std::min(36, atoi(argv[3])));
  const int repeat = argc > 4 ? std::max(1, atoi(argv[4])) : 1;
  const double min_s = argc > 5 ? atof(argv[5]) : 0.0;
  switch (d.protocol) {
    case DSL_PROTO_PINGPONG: return run<PingPong>(d, s, threads, log2, repeat, min_s, start, depth0);
    case DSL_PROTO_SIPAXOS: return run<SIPaxos>(d, s, threads, log2, repeat, min_s, start, depth0);
    case DSL_PROTO_MULTIPAXOS: return run<MultiPaxos>(d, s, threads, log2, repeat, min_s, start, depth0);
    case DSL_PROTO_SYNTHETIC: return run<Synthetic>(d, s, threads, log2, repeat, min_s, start, depth0);
    case DSL_PROTO_AMOKV: return run<AmoKV>(d, s, threads, log2, repeat, min_s, start, depth0);
    case DSL_PROTO_PB: return run<PB>(d, s, threads, log2, repeat, min_s, start, depth0);
    case DSL_PROTO_MINITEST: return run<MiniTest>(d, s, threads, log2, repeat, min_s, start, depth0);
    case DSL_PROTO_PINGPONG_IR: return run<PingPongIR>(d, s, threads, log2, repeat, min_s, start, depth0);
    case DSL_PROTO_AMOKV_IR: return run<AmoKVIR>(d, s, threads, log2, repeat, min_s, start, depth0);
    case DSL_PROTO_MULTIPAXOS_IR: return run<MultiPaxosIR>(d, s, threads, log2, repeat, min_s, start, depth0);
    case DSL_PROTO_PB_IR: return run<PBIR>(d, s, threads, log2, repeat, min_s, start, depth0);
  }
  return fprintf(stderr, "unknown protocol\n"), 2;
}
