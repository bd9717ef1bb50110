package dslabs.framework.testing.search;

import dslabs.framework.testing.Event;
import dslabs.framework.testing.MessageEnvelope;
import dslabs.framework.testing.StatePredicate;
import dslabs.framework.testing.StatePredicate.PredicateResult;
import dslabs.framework.testing.utils.GlobalSettings;
import dslabs.framework.testing.search.SearchResults.EndCondition;
import dslabs.framework.testing.search.gpu.Dsl;
import dslabs.framework.testing.search.gpu.GpuPredicates;
import dslabs.framework.testing.search.gpu.GpuProtocols;
import java.lang.foreign.MemorySegment;
import java.util.ArrayList;
import java.util.HashSet;
import java.util.List;
import java.util.Set;

/**
 * Breadth-first search on the MI355X engine (libdslabs_hip.so, include/dslabs_hip.h) as a drop-in
 * for {@link Search#bfs} (Search.java:390-395): a lab test selects it where it calls bfs()
 * (BaseJUnitTest.java:256-262). The engine runs Search.run's BFS with the reference's counting
 * rules and end-condition priority; the terminal state is then rebuilt on the Java Node handlers by
 * replaying the device trace with stepEvent(e, settings, false) (TraceReplaySearch.java:76-101
 * semantics), so trace printing and SerializableTrace work unchanged. A mid-search start state is
 * packed by replaying its own trace on the engine (dsl_replay, then dsl_set_initial). A protocol,
 * predicate or event with no device form (GpuProtocols / GpuPredicates return null), or no visible
 * GPU runs the JVM search. A start state with a dropped network (PaxosTest's narrowed searches:
 * dropPendingMessages, then undropMessagesFrom / To, PaxosTest.java:1065-1132) is packed the same
 * way on the engine (dsl_drop_pending_messages, dsl_undrop_messages) and its dropped set handed to
 * the search (dsl_set_dropped); a dropped network no sequence of those calls produces keeps the JVM
 * search.
 * This file is part of the integration layer (INTEGRATION.md); it is not compiled in this build,
 * whose image has no JDK.
 */
public final class GpuBFS {
  private GpuBFS() {}

  public static SearchResults bfs(SearchState init, SearchSettings settings) {
    if (settings == null) settings = new SearchSettings();
    if (!Dsl.deviceAvailable()) return Search.bfs(init, settings);
    // GlobalSettings.doErrorChecks / doAllChecks (Search.java:201-220) re-step every explored state
    // and report each offending event with its starting SearchState through CheckLogger; that
    // state is a Java object the device never holds, so a checked run keeps the JVM search (the
    // engine's own sampled checks, dsl_settings.do_checks, are for its tests and the C ABI)
    if (GlobalSettings.doErrorChecks()) return Search.bfs(init, settings);
    List<SearchState> chain = new ArrayList<>();
    init.trace().forEach(chain::add);
    GpuProtocols.Desc desc = GpuProtocols.describe(chain.get(0));
    if (desc == null) return Search.bfs(init, settings);
    Undrop undrop = undrop(init, desc);
    if (undrop == null) return Search.bfs(init, settings);
    try (Dsl.Engine eng = new Dsl.Engine(desc.protocol())) {
      MemorySegment enc = GpuPredicates.encode(settings, desc.addresses(), desc.leaf(), eng.arena());
      byte[] packed = enc == null ? null : start(eng, desc, chain);
      if (packed == null) return Search.bfs(init, settings);
      eng.setSettings(enc);
      if (undrop.dropped()) {
        if (packed.length == 0) return Search.bfs(init, settings);  // an initial state has nothing to drop
        eng.setDropped(eng.dropPending(packed, undrop.from(), undrop.to()));
      }
      if (packed.length > 0) eng.setInitial(packed, init.depth());
      Dsl.Result r = eng.run();
      return results(init, settings, desc, r);
    }
  }

  /**
   * How a start state's live network follows from its dropped one: every message was dropped
   * (dropPendingMessages), then those from the nodes `from` and to the nodes `to` were undropped.
   * dropped() is false for a state that never dropped anything; null when the live network is not
   * such a union (the JVM search then runs).
   */
  record Undrop(boolean dropped, int[] from, int[] to) {}

  @SuppressWarnings("unchecked")
  private static Undrop undrop(SearchState s, GpuProtocols.Desc desc) {
    // the two sets of SearchState (SearchState.java:71-77): network() is their union
    Set<MessageEnvelope> dropped, live;
    try {
      java.lang.reflect.Field d = SearchState.class.getDeclaredField("droppedNetwork");
      java.lang.reflect.Field n = SearchState.class.getDeclaredField("network");
      d.setAccessible(true);
      n.setAccessible(true);
      dropped = (Set<MessageEnvelope>) d.get(s);
      live = (Set<MessageEnvelope>) n.get(s);
    } catch (ReflectiveOperationException e) {
      return null;
    }
    if (dropped.isEmpty()) return new Undrop(false, new int[0], new int[0]);
    if (!dropped.containsAll(live)) return null;  // sent after the drop: not an undrop
    List<Integer> from = new ArrayList<>(), to = new ArrayList<>();
    Set<MessageEnvelope> union = new HashSet<>();
    for (int i = 0; i < desc.addresses().size(); i++) {
      var a = desc.addresses().get(i);
      Set<MessageEnvelope> sent = new HashSet<>(), got = new HashSet<>();
      for (MessageEnvelope m : dropped) {
        if (m.from().rootAddress().equals(a)) sent.add(m);
        if (m.to().rootAddress().equals(a)) got.add(m);
      }
      if (!sent.isEmpty() && live.containsAll(sent)) {
        from.add(i);
        union.addAll(sent);
      }
      if (!got.isEmpty() && live.containsAll(got)) {
        to.add(i);
        union.addAll(got);
      }
    }
    if (!union.equals(live)) return null;
    return new Undrop(true, from.stream().mapToInt(Integer::intValue).toArray(),
        to.stream().mapToInt(Integer::intValue).toArray());
  }


  /**
   * BaseJUnitTest.traceReplay (BaseJUnitTest.java:279-284, TraceReplaySearch.java:76-101) on the
   * engine: the events are encoded as dsl_events (GpuProtocols.EventEncoder) and replayed by
   * dsl_replay with checkState after every step; a terminal's trace comes back minimized
   * (TraceMinimizer), and the terminal is rebuilt on the Java handlers. Returns null when the
   * protocol, a predicate or an event has no device form: the caller then runs TraceReplaySearch.
   */
  public static SearchResults traceReplay(SearchState init, SearchSettings settings, List<Event> trace) {
    if (settings == null) settings = new SearchSettings();
    if (!Dsl.deviceAvailable()) return null;
    List<SearchState> chain = new ArrayList<>();
    init.trace().forEach(chain::add);
    GpuProtocols.Desc desc = GpuProtocols.describe(chain.get(0));
    if (desc == null || undrop(init, desc) == null || undrop(init, desc).dropped()) return null;
    Dsl.Event[] evs = new Dsl.Event[trace.size()];
    for (int i = 0; i < evs.length; i++)
      if ((evs[i] = desc.encoder().encode(trace.get(i))) == null) return null;
    try (Dsl.Engine eng = new Dsl.Engine(desc.protocol())) {
      MemorySegment enc = GpuPredicates.encode(settings, desc.addresses(), desc.leaf(), eng.arena());
      byte[] packed = enc == null ? null : start(eng, desc, chain);
      if (packed == null) return null;
      eng.setSettings(enc);
      if (packed.length > 0) eng.setInitial(packed, init.depth());
      return results(init, settings, desc, eng.replay(evs, true));
    }
  }

  // The packed form of a mid-search start state (the last of `chain`): its own trace from the
  // initial state, encoded and replayed on the engine with every link and timer enabled
  // (dsl_replay), whose last state dsl_set_initial then takes. The Python mirror builds
  // PrimaryBackupTest.initView's state the same way (dslabs_amd/protocols.py PB.initView).
  // Empty for the initial state itself; null when the trace has no device form.
  private static byte[] start(Dsl.Engine eng, GpuProtocols.Desc desc, List<SearchState> chain) {
    if (chain.size() == 1) return new byte[0];
    Dsl.Event[] evs = new Dsl.Event[chain.size() - 1];
    for (int i = 1; i < chain.size(); i++)
      if ((evs[i - 1] = desc.encoder().encode(chain.get(i).previousEvent())) == null) return null;
    MemorySegment all = GpuPredicates.encode(new SearchSettings(), desc.addresses(), desc.leaf(), eng.arena());
    eng.setSettings(all);
    Dsl.Result r = eng.replay(evs, false);
    if (r.endCondition() != Dsl.END_SPACE_EXHAUSTED || r.trace().length != evs.length || r.terminalState() == null)
      return null;  // a step threw, or the engine could not deliver an event the JVM did
    return r.terminalState();
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
        if (desc.matches(je, de)) {
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
