package dslabs.framework.testing.search.gpu;

import dslabs.framework.Address;
import dslabs.framework.Message;
import dslabs.framework.testing.MessageEnvelope;
import dslabs.framework.testing.StatePredicate;
import dslabs.framework.testing.search.SearchSettings;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.ValueLayout;
import java.util.ArrayList;
import java.util.List;
import java.util.function.Function;

/**
 * SearchSettings -> dsl_settings (include/dslabs_hip.h). Delivery is resolved by asking the
 * settings themselves (TestSettings.shouldDeliver / deliverTimers, TestSettings.java:87-89,
 * :224-245) for every (from, to) pair, so the precedence rules are the reference's by
 * construction. Predicates are matched by name: a leaf through the protocol's registry
 * (GpuProtocols.Desc#leaf), the combinators through the names StatePredicate gives them
 * (StatePredicate.java:382-432: "¬(A)", "(A) ∧ (B)", "(A) ∨ (B)", "(A) → (B)"). Returns null when
 * something has no device form (GpuBFS then runs the JVM search).
 */
public final class GpuPredicates {
  static final int AND = 900, OR = 901, IMPLIES = 902;

  /** A predicate leaf on the device: id and two integer arguments. */
  public record Leaf(int id, long arg0, long arg1) {}

  private record Tree(int id, boolean negate, long arg0, long arg1, Tree left, Tree right) {}

  private GpuPredicates() {}

  /** The fired predicate is reported by index into these lists (same order as the settings). */
  public static MemorySegment encode(SearchSettings s, List<Address> addresses, Function<String, Leaf> leaf,
                                     Arena arena) {
    MemorySegment m = arena.allocate(Dsl.SIZE_SETTINGS, 8);
    m.set(ValueLayout.JAVA_INT, Dsl.OFF_MAX_DEPTH, s.maxDepth());
    m.set(ValueLayout.JAVA_INT, Dsl.OFF_MAX_TIME_MS, s.maxTimeSecs() > 0 ? s.maxTimeSecs() * 1000 : -1);
    m.set(ValueLayout.JAVA_INT, Dsl.OFF_NETWORK_ACTIVE, 1);
    m.set(ValueLayout.JAVA_INT, Dsl.OFF_DELIVER_TIMERS, 1);
    int n = addresses.size();
    if (n > Dsl.MAX_NODES) return null;
    Message probe = new Message() {};
    for (int f = 0; f < Dsl.MAX_NODES; f++)
      for (int t = 0; t < Dsl.MAX_NODES; t++) {
        byte v = -1;
        if (f < n && t < n)
          v = (byte) (s.shouldDeliver(new MessageEnvelope(addresses.get(f), addresses.get(t), probe)) ? 1 : 0);
        m.set(ValueLayout.JAVA_BYTE, Dsl.OFF_LINK_ACTIVE + (long) f * Dsl.MAX_NODES + t, v);
      }
    for (int a = 0; a < Dsl.MAX_NODES; a++) {
      m.set(ValueLayout.JAVA_BYTE, Dsl.OFF_SENDER_ACTIVE + a, (byte) -1);
      m.set(ValueLayout.JAVA_BYTE, Dsl.OFF_RECEIVER_ACTIVE + a, (byte) -1);
      m.set(ValueLayout.JAVA_BYTE, Dsl.OFF_TIMERS_ACTIVE + a,
          a < n ? (byte) (s.deliverTimers(addresses.get(a)) ? 1 : 0) : (byte) -1);
    }
    List<Tree> pool = new ArrayList<>();
    long[][] lists = {{Dsl.OFF_N_INVARIANTS, Dsl.OFF_INVARIANTS}, {Dsl.OFF_N_GOALS, Dsl.OFF_GOALS},
                      {Dsl.OFF_N_PRUNES, Dsl.OFF_PRUNES}};
    List<List<StatePredicate>> preds = List.of(List.copyOf(s.invariants()), List.copyOf(s.goals()),
        List.copyOf(s.prunes()));
    for (int l = 0; l < 3; l++) {
      List<StatePredicate> ps = preds.get(l);
      if (ps.size() > Dsl.MAX_PREDICATES) return null;
      m.set(ValueLayout.JAVA_INT, lists[l][0], ps.size());
      for (int i = 0; i < ps.size(); i++) {
        Tree t = parse(ps.get(i).name(), leaf);
        if (t == null) return null;
        if (!write(m, lists[l][1] + Dsl.SIZE_PREDICATE * i, t, pool)) return null;
      }
    }
    if (pool.size() > Dsl.MAX_POOL) return null;
    m.set(ValueLayout.JAVA_INT, Dsl.OFF_N_POOL, pool.size());
    m.set(ValueLayout.JAVA_INT, Dsl.OFF_TABLE_LOG2, 0);  // automatic
    // GlobalSettings checks (Search.java:201-220) keep the JVM search (GpuBFS.bfs): the device's
    // sampled checks could count offending events but not hand CheckLogger their Java states
    m.set(ValueLayout.JAVA_INT, Dsl.OFF_DO_CHECKS, Dsl.CHECKS_NONE);
    m.set(ValueLayout.JAVA_INT, Dsl.OFF_CHECK_SAMPLE, 0);
    return m;
  }

  // Writes t at `off`; its operands go to the pool first (an operand may reference lower entries).
  private static boolean write(MemorySegment m, long off, Tree t, List<Tree> pool) {
    long a0 = t.arg0(), a1 = t.arg1();
    if (t.left() != null) {
      a0 = pool.size();
      pool.add(t.left());
      if (!write(m, Dsl.OFF_POOL + Dsl.SIZE_PREDICATE * a0, t.left(), pool)) return false;
      a1 = pool.size();
      pool.add(t.right());
      if (!write(m, Dsl.OFF_POOL + Dsl.SIZE_PREDICATE * a1, t.right(), pool)) return false;
    }
    if (pool.size() > Dsl.MAX_POOL) return false;
    m.set(ValueLayout.JAVA_INT, off + Dsl.OFF_PRED_ID, t.id());
    m.set(ValueLayout.JAVA_INT, off + Dsl.OFF_PRED_NEGATE, t.negate() ? 1 : 0);
    m.set(ValueLayout.JAVA_LONG, off + Dsl.OFF_PRED_ARG0, a0);
    m.set(ValueLayout.JAVA_LONG, off + Dsl.OFF_PRED_ARG1, a1);
    return true;
  }

  // The combinator structure back from StatePredicate's names.
  static Tree parse(String name, Function<String, Leaf> leaf) {
    Leaf l = leaf.apply(name);
    if (l != null) return new Tree(l.id(), false, l.arg0(), l.arg1(), null, null);
    if (name.startsWith("¬(") && name.endsWith(")")) {
      Tree t = parse(name.substring(2, name.length() - 1), leaf);
      return t == null ? null : new Tree(t.id(), !t.negate(), t.arg0(), t.arg1(), t.left(), t.right());
    }
    if (!name.startsWith("(")) return null;
    int depth = 0;
    for (int i = 0; i < name.length(); i++) {
      char c = name.charAt(i);
      if (c == '(') depth++;
      else if (c == ')') depth--;
      if (depth == 0) {  // the end of the left operand "(A)"
        String rest = name.substring(i + 1);
        int op = rest.startsWith(" ∧ (") ? AND : rest.startsWith(" ∨ (") ? OR : rest.startsWith(" → (") ? IMPLIES : 0;
        if (op == 0 || !rest.endsWith(")")) return null;
        Tree a = parse(name.substring(1, i), leaf), b = parse(rest.substring(4, rest.length() - 1), leaf);
        return a == null || b == null ? null : new Tree(op, false, 0, 0, a, b);
      }
    }
    return null;
  }
}
