package dslabs.framework.testing.search;

import dslabs.framework.testing.Event;
import dslabs.framework.testing.StatePredicate;
import dslabs.framework.testing.StatePredicate.PredicateResult;
import dslabs.framework.testing.search.SearchResults.EndCondition;
import dslabs.framework.testing.search.gpu.Dsl;
import dslabs.framework.testing.search.gpu.GpuPredicates;
import dslabs.framework.testing.search.gpu.GpuProtocols;
import java.lang.foreign.MemorySegment;
import java.util.ArrayList;
import java.util.List;

/**
 * Breadth-first search on the MI355X engine (libdslabs_hip.so, include/dslabs_hip.h) as a drop-in
 * for {@link Search#bfs} (Search.java:390-395): a lab test selects it where it calls bfs()
 * (BaseJUnitTest.java:256-262). The engine runs Search.run's BFS with the reference's counting
 * rules and end-condition priority; the terminal state is then rebuilt on the Java Node handlers by
 * replaying the device trace with stepEvent(e, settings, false) (TraceReplaySearch.java:76-101
 * semantics), so trace printing and SerializableTrace work unchanged. A protocol or predicate with
 * no device form (GpuProtocols / GpuPredicates return null), or no visible GPU, runs the JVM search.
 * This file is part of the integration layer (INTEGRATION.md); it is not compiled in this build,
 * whose image has no JDK.
 */
public final class GpuBFS {
  private GpuBFS() {}

  public static SearchResults bfs(SearchState init, SearchSettings settings) {
    if (settings == null) settings = new SearchSettings();
    if (!Dsl.deviceAvailable()) return Search.bfs(init, settings);
    GpuProtocols.Desc desc = GpuProtocols.describe(init);
    if (desc == null || init.depth() > 0) return Search.bfs(init, settings);  // packing a mid-search state: see INTEGRATION.md
    try (Dsl.Engine eng = new Dsl.Engine(desc.protocol())) {
      MemorySegment enc = GpuPredicates.encode(settings, desc.addresses(), desc.leaf(), eng.arena());
      if (enc == null) return Search.bfs(init, settings);
      eng.setSettings(enc);
      Dsl.Result r = eng.run();
      return results(init, settings, desc, r);
    }
  }

  private static SearchResults results(SearchState init, SearchSettings settings, GpuProtocols.Desc desc,
                                       Dsl.Result r) {
    SearchResults res = new SearchResults();
    res.invariantsTested(new ArrayList<>(settings.invariants()));
    res.goalsSought(new ArrayList<>(settings.goals()));
    EndCondition end = switch (r.endCondition()) {
      case Dsl.END_EXCEPTION_THROWN -> EndCondition.EXCEPTION_THROWN;
      case Dsl.END_INVARIANT_VIOLATED -> EndCondition.INVARIANT_VIOLATED;
      case Dsl.END_GOAL_FOUND -> EndCondition.GOAL_FOUND;
      case Dsl.END_TIME_EXHAUSTED -> EndCondition.TIME_EXHAUSTED;
      default -> EndCondition.SPACE_EXHAUSTED;
    };
    res.endCondition(end);
    if (r.terminalDepth() < 0) return res;
    // the terminal on the Java handlers: each device event is the unique matching event of the
    // state it meets (events(settings), SearchState.java:226-252)
    SearchState s = init;
    for (Dsl.Event de : r.trace()) {
      Event match = null;
      for (Event je : s.events(settings))
        if (desc.matcher().matches(je, de, desc.addresses())) {
          match = je;
          break;
        }
      if (match == null) throw new IllegalStateException("device trace event has no Java counterpart: " + de);
      s = s.stepEvent(match, settings, false);
    }
    switch (end) {
      case EXCEPTION_THROWN -> res.exceptionThrown(s);
      case INVARIANT_VIOLATED -> res.invariantViolated(s, fired(settings.invariants(), r.predicateIndex(), s, true));
      case GOAL_FOUND -> res.goalFound(s, fired(settings.goals(), r.predicateIndex(), s, false));
      default -> {}
    }
    return res;
  }

  // The predicate the device reported, re-tested on the Java state for its result and detail.
  private static PredicateResult fired(Iterable<StatePredicate> ps, int index, SearchState s, boolean invariant) {
    List<StatePredicate> list = new ArrayList<>();
    ps.forEach(list::add);
    StatePredicate p = list.get(index);
    return p.test(s, invariant);  // the normal value of an invariant is true, of a goal false
  }
}
