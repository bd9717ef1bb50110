package dslabs.framework.testing.search.gpu;

import dslabs.framework.Address;
import dslabs.framework.Command;
import dslabs.framework.Node;
import dslabs.framework.Result;
import dslabs.framework.testing.ClientWorker;
import dslabs.framework.testing.Event;
import dslabs.framework.testing.MessageEnvelope;
import dslabs.framework.testing.TimerEnvelope;
import dslabs.framework.testing.Workload;
import dslabs.framework.testing.search.SearchState;
import dslabs.framework.testing.utils.Cloning;
import java.lang.reflect.Field;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.Comparator;
import java.util.List;
import java.util.Map;
import java.util.TreeSet;
import java.util.function.Function;
import java.util.regex.Matcher;
import java.util.regex.Pattern;
import org.apache.commons.lang3.tuple.Pair;

/**
 * Which initial states have a device form, and how Java events map to device events. A protocol
 * entry gives the engine's protocol id and parameter vector (the vectors dslabs_amd/protocols.py
 * builds), the addresses in the engine's node order, the predicate leaf registry, and an event
 * encoder: a MessageEnvelope / TimerEnvelope -> the dsl_event the engine describes for it
 * (describe_message / describe_timer of dslabs_amd/csrc/protocols/*.hpp). The encoder serves
 * three ways: matching device trace events to Java events (GpuBFS rebuilding the terminal state),
 * replaying a Java trace on the engine to pack a mid-search start state (dsl_replay, then
 * dsl_set_initial), and replaying a saved trace (GpuBFS.traceReplay).
 *
 * <p>Covered: lab0 PingPong (labs/lab0-pingpong), the reference's single-instance Paxos
 * (T/visualization/examples/paxosmadesimple), lab1 AMO KV (java/src/dslabs/clientserver, the
 * solution of DESIGN.md §11: BASELINE C2), lab2 primary-backup + ViewServer
 * (java/src/dslabs/primarybackup, DESIGN.md §12: C4) and lab3 Multi-Paxos (java/src/dslabs/paxos,
 * DESIGN.md §9: C5). Lab classes are read by reflection (class simple names and field
 * names), since this file is compiled with every lab and each lab has only its own classes.
 * Anything else returns null (GpuBFS then runs the JVM search).
 */
public final class GpuProtocols {
  /** A device protocol for one initial state. */
  public record Desc(Dsl.Protocol protocol, List<Address> addresses, Function<String, GpuPredicates.Leaf> leaf,
                     EventEncoder encoder) {
    /** Whether a Java event is the device event. */
    public boolean matches(Event javaEvent, Dsl.Event deviceEvent) {
      Dsl.Event e = encoder.encode(javaEvent);
      return e != null && e.sameAs(deviceEvent);
    }
  }

  /** A Java event as the engine's dsl_event; null if it has no device form. */
  public interface EventEncoder {
    Dsl.Event encode(Event javaEvent);
  }

  // dsl_pred_id (include/dslabs_hip.h) of the StatePredicate constants (StatePredicate.java:90-148)
  private static final Map<String, Integer> STANDARD = Map.of(
      "Clients got expected results", 1, "All clients' workloads finished", 2, "No results returned", 4);

  private GpuProtocols() {}

  public static Desc describe(SearchState init) {
    // the engine's node order: the server kinds first, then the clients, each by address name
    List<Address> addrs = new ArrayList<>();
    for (Address a : init.addresses()) addrs.add(a);
    addrs.sort(Comparator.comparing((Address a) -> rank(init.node(a))).thenComparing(Address::toString));
    List<Node> nodes = new ArrayList<>();
    for (Address a : addrs) nodes.add(init.node(a));
    if (nodes.isEmpty()) return null;
    String first = simpleName(nodes.get(0));
    try {
      if (first.equals("PingServer")) return pingPong(addrs, nodes);
      if (first.endsWith("Proposer")) return sipaxos(addrs, nodes);
      if (first.equals("PaxosServer")) return multiPaxos(addrs, nodes);
      if (first.equals("SimpleServer")) return amoKV(addrs, nodes);
      if (first.equals("ViewServer")) return primaryBackup(addrs, nodes);
    } catch (ReflectiveOperationException | ClassCastException e) {
      return null;  // a class of that name with another shape: not the protocol the engine has
    }
    return null;
  }

  private static int rank(Node n) {
    String c = simpleName(n);
    return c.equals("PingServer") || c.endsWith("Proposer") || c.equals("PaxosServer") || c.equals("SimpleServer")
        || c.equals("ViewServer") ? 0 : c.equals("Acceptor") || c.equals("PBServer") ? 1 : 2;
  }

  // ---- lab0 PingPong: "pingserver", then ClientWorkers around PingClients (PingTest.java:44-51) ----
  // Device values: "ping-i" -> i (dslabs_amd/csrc/protocols/pingpong.hpp)
  private static Desc pingPong(List<Address> addrs, List<Node> nodes) throws ReflectiveOperationException {
    int pings = -1;
    for (int i = 1; i < nodes.size(); i++) {
      if (!(nodes.get(i) instanceof ClientWorker cw)) return null;
      List<Pair<Command, Result>> w = commands(cw, addrs.get(i));
      if (w == null || (pings >= 0 && w.size() != pings)) return null;
      for (int k = 0; k < w.size(); k++) {  // the repeatedPings workload: ping-1 .. ping-N
        if (!("ping-" + (k + 1)).equals(field(w.get(k).getLeft(), "value"))) return null;
        Result r = w.get(k).getRight();
        if (r != null && !("ping-" + (k + 1)).equals(field(r, "value"))) return null;
      }
      pings = w.size();
    }
    if (pings < 1 || pings > 15 || nodes.size() - 1 > 4) return null;
    long[] params = {nodes.size() - 1, pings, 1, 1};  // clients, pings, value check, timer re-set
    Function<String, GpuPredicates.Leaf> leaf = name -> {
      Integer id = STANDARD.get(name);
      return id == null ? null : new GpuPredicates.Leaf(id, 0, 0);
    };
    EventEncoder enc = je -> {
      try {
        if (je instanceof TimerEnvelope t) {
          if (!simpleName(t.timer()).equals("PingTimer")) return null;
          long v = pingValue(field(t.timer(), "ping"));
          return v < 0 ? null : Dsl.Event.timer(addrs.indexOf(t.to().rootAddress()), 2, t.minTimerLengthMillis(),
              t.maxTimerLengthMillis(), v);
        }
        MessageEnvelope m = (MessageEnvelope) je;
        String c = simpleName(m.message());
        long v = c.equals("PingRequest") ? pingValue(field(m.message(), "ping"))
            : c.equals("PongReply") ? pingValue(field(m.message(), "pong")) : -1;
        return v < 0 ? null : Dsl.Event.message(addrs.indexOf(m.from().rootAddress()),
            addrs.indexOf(m.to().rootAddress()), c.equals("PingRequest") ? 0 : 1, v);
      } catch (ReflectiveOperationException e) {
        return null;
      }
    };
    return new Desc(new Dsl.Protocol(Dsl.PROTO_PINGPONG, params), addrs, leaf, enc);
  }

  private static long pingValue(Object pingOrPong) throws ReflectiveOperationException {
    Object v = field(pingOrPong, "value");
    if (!(v instanceof String s) || !s.startsWith("ping-")) return -1;
    try {
      return Long.parseLong(s.substring(5));
    } catch (NumberFormatException e) {
      return -1;
    }
  }

  // ---- SingleInstancePaxos: proposers then acceptors (SingleInstancePaxos.java:50-127) ----
  // Device values: value id v = the initial proposal of proposer v (dslabs_amd/csrc/protocols/sipaxos.hpp)
  private static Desc sipaxos(List<Address> addrs, List<Node> nodes) throws ReflectiveOperationException {
    int p = 0;
    while (p < nodes.size() && simpleName(nodes.get(p)).endsWith("Proposer")) p++;
    int a = nodes.size() - p;
    if (p < 1 || p > 3 || a < 1 || a > 5) return null;
    boolean incorrect = simpleName(nodes.get(0)).equals("BadProposer");
    List<String> values = new ArrayList<>();
    for (int i = 0; i < p; i++) {
      String v = (String) field(nodes.get(i), "proposalValue");
      if (values.contains(v)) return null;  // interned per proposer on the device
      values.add(v);
    }
    long[] params = {p, a, incorrect ? 1 : 0};
    Function<String, GpuPredicates.Leaf> leaf = name -> switch (name) {
      case "Agreement" -> new GpuPredicates.Leaf(100, 0, 0);
      case "Integrity" -> new GpuPredicates.Leaf(101, 0, 0);
      case "Termination" -> new GpuPredicates.Leaf(102, 0, 0);
      default -> null;
    };
    List<String> types = List.of("Prepare", "PrepareAck", "Accept", "AcceptAck");
    EventEncoder enc = je -> {
      try {
        if (je instanceof TimerEnvelope t)
          return simpleName(t.timer()).equals("Propose") ? Dsl.Event.timer(addrs.indexOf(t.to().rootAddress()), 4,
              t.minTimerLengthMillis(), t.maxTimerLengthMillis()) : null;
        MessageEnvelope m = (MessageEnvelope) je;
        int type = types.indexOf(simpleName(m.message()));
        if (type < 0) return null;
        long n = ((Number) field(m.message(), "proposalNumber")).longValue(), an = 0, av = 0;
        if (type == 1 && field(m.message(), "accepted") instanceof Pair<?, ?> acc) {
          an = ((Number) acc.getLeft()).longValue();
          av = values.indexOf((String) acc.getRight()) + 1;
        } else if (type == 2) {
          av = values.indexOf((String) field(m.message(), "proposalValue")) + 1;
        }
        return Dsl.Event.message(addrs.indexOf(m.from().rootAddress()), addrs.indexOf(m.to().rootAddress()), type, n,
            an, av);
      } catch (ReflectiveOperationException e) {
        return null;
      }
    };
    return new Desc(new Dsl.Protocol(Dsl.PROTO_SIPAXOS, params), addrs, leaf, enc);
  }

  // ---- lab3 Multi-Paxos: servers then ClientWorkers around PaxosClients (DESIGN.md §9) ----
  private static Desc multiPaxos(List<Address> addrs, List<Node> nodes) throws ReflectiveOperationException {
    int n = 0;
    while (n < nodes.size() && simpleName(nodes.get(n)).equals("PaxosServer")) n++;
    int c = nodes.size() - n;
    if (n < 1 || n > MultiPaxosCodec.MAX_SERVERS || c < 1 || c > MultiPaxosCodec.MAX_CLIENTS) return null;
    // a ballot's leader is the index into the server's `servers` array, on the device the node index
    for (int i = 0; i < n; i++)
      if (!Arrays.asList((Object[]) field(nodes.get(i), "servers")).equals(addrs.subList(0, n))) return null;
    List<List<Pair<Command, Result>>> work = new ArrayList<>();
    for (int i = n; i < nodes.size(); i++) {
      if (!(nodes.get(i) instanceof ClientWorker cw) || !simpleName(field(cw, "client")).equals("PaxosClient"))
        return null;
      List<Pair<Command, Result>> w = commands(cw, addrs.get(i));
      if (w == null || w.size() > MultiPaxosCodec.MAX_CMDS) return null;
      work.add(w);
    }
    MultiPaxosCodec codec = MultiPaxosCodec.of(addrs, n, work);
    if (codec == null) return null;
    return new Desc(new Dsl.Protocol(Dsl.PROTO_MULTIPAXOS, codec.params()), addrs, multiPaxosLeaf(addrs, n, codec), codec::encode);
  }

  // ---- lab1 AMO KV: "server", then ClientWorkers around SimpleClients (DESIGN.md §11) ----
  private static Desc amoKV(List<Address> addrs, List<Node> nodes) throws ReflectiveOperationException {
    if (!addrs.get(0).toString().equals("server")) return null;
    List<List<Pair<Command, Result>>> work = new ArrayList<>();
    for (int i = 1; i < nodes.size(); i++) {
      if (!(nodes.get(i) instanceof ClientWorker cw) || !simpleName(field(cw, "client")).equals("SimpleClient"))
        return null;
      List<Pair<Command, Result>> w = commands(cw, addrs.get(i));
      if (w == null) return null;
      work.add(w);
    }
    AmoKVCodec codec = AmoKVCodec.of(addrs, work);
    if (codec == null) return null;
    Function<String, GpuPredicates.Leaf> leaf = name -> {
      Integer id = STANDARD.get(name);
      if (id != null) return new GpuPredicates.Leaf(id, 0, 0);
      return name.equals("Sequence of appends to the same key is linearizable") ? new GpuPredicates.Leaf(300, 0, 0)
          : null;
    };
    return new Desc(new Dsl.Protocol(Dsl.PROTO_AMOKV, codec.params()), addrs, leaf, codec::encode);
  }

  // ---- lab2 primary-backup: "viewserver", PBServers, ClientWorkers around PBClients (DESIGN.md §12) ----
  private static Desc primaryBackup(List<Address> addrs, List<Node> nodes) throws ReflectiveOperationException {
    int n = 0;
    while (1 + n < nodes.size() && simpleName(nodes.get(1 + n)).equals("PBServer")) n++;
    List<List<Pair<Command, Result>>> work = new ArrayList<>();
    for (int i = 1 + n; i < nodes.size(); i++) {
      if (!(nodes.get(i) instanceof ClientWorker cw) || !simpleName(field(cw, "client")).equals("PBClient"))
        return null;
      List<Pair<Command, Result>> w = commands(cw, addrs.get(i));
      if (w == null) return null;
      work.add(w);
    }
    PBCodec codec = PBCodec.of(addrs, n, work);
    if (codec == null) return null;
    return new Desc(new Dsl.Protocol(Dsl.PROTO_PB, codec.params()), addrs, pbLeaf(addrs, n), codec::encode);
  }

  // PrimaryBackupTest's predicates (PrimaryBackupTest.java:104-117, initView's goal :136-156)
  private static final String VIEW = "View\\(viewNum=(\\d+), primary=([^,]+), backup=([^)]+)\\)";
  private static final Pattern HAS_VIEW_REPLY = Pattern.compile("ViewReply with viewNum: (\\d+)");
  private static final Pattern HAS_VIEW_REPLY_EXACT = Pattern.compile("ViewReply with " + VIEW);
  private static final Pattern VIEW_REPLIES_SENT =
      Pattern.compile("ViewReply for " + VIEW + " sent to nodes \\[(.*)\\], primary ack sent");

  private static Function<String, GpuPredicates.Leaf> pbLeaf(List<Address> addrs, int servers) {
    return name -> {
      Integer id = STANDARD.get(name);
      if (id != null) return new GpuPredicates.Leaf(id, 0, 0);
      Matcher m = HAS_VIEW_REPLY.matcher(name);
      if (m.matches()) return new GpuPredicates.Leaf(500, Long.parseLong(m.group(1)), 0);
      m = HAS_VIEW_REPLY_EXACT.matcher(name);
      if (m.matches()) {
        long v = viewBits(addrs, servers, m);
        return v < 0 ? null : new GpuPredicates.Leaf(501, v, 0);
      }
      m = VIEW_REPLIES_SENT.matcher(name);
      if (m.matches()) {
        long v = viewBits(addrs, servers, m), mask = 0;
        for (String a : m.group(4).split(", ")) {
          int i = nodeIndex(addrs, a);
          if (i < 0) return null;
          mask |= 1L << i;
        }
        return v < 0 ? null : new GpuPredicates.Leaf(502, v, mask);
      }
      return null;
    };
  }

  // A View's toString groups (viewNum, primary, backup) as num | primary id << 4 | backup id << 6
  private static long viewBits(List<Address> addrs, int servers, Matcher m) {
    long n = Long.parseLong(m.group(1));
    int p = m.group(2).equals("null") ? 0 : nodeIndex(addrs, m.group(2));
    int b = m.group(3).equals("null") ? 0 : nodeIndex(addrs, m.group(3));
    if (n > 15 || p < 0 || p > servers || b < 0 || b > servers) return -1;
    return n | (long) p << 4 | (long) b << 6;
  }

  // PaxosTest's predicates (PaxosTest.java:113-346) and KVStoreWorkload.APPENDS_LINEARIZABLE
  private static final Pattern HAS_STATUS = Pattern.compile("(\\S+) has status (EMPTY|ACCEPTED|CHOSEN|CLEARED) in slot (\\d+)");
  private static final Pattern HAS_COMMAND = Pattern.compile("(\\S+) has command (.+) in slot (\\d+)");
  private static final Pattern SLOT_VALID = Pattern.compile("Logs consistent for slot (\\d+)");
  private static final List<String> STATUS = List.of("EMPTY", "ACCEPTED", "CHOSEN", "CLEARED");  // PaxosLogSlotStatus

  private static Function<String, GpuPredicates.Leaf> multiPaxosLeaf(List<Address> addrs, int n, MultiPaxosCodec codec) {
    return name -> {
      Integer id = STANDARD.get(name);
      if (id != null) return new GpuPredicates.Leaf(id, 0, 0);
      switch (name) {  // LOGS_CONSISTENT(_ALL_SLOTS) with MARKERS_VALID, which holds with no garbage collection
        case "(Active log slots consistent) ∧ (First non-cleared and last non-empty valid)",
             "Active log slots consistent" -> {
          return new GpuPredicates.Leaf(401, 0, 0);
        }
        case "(Non-empty log slots consistent) ∧ (First non-cleared and last non-empty valid)",
             "Non-empty log slots consistent" -> {
          return new GpuPredicates.Leaf(400, 0, 0);
        }
        case "Sequence of appends to the same key is linearizable" -> {
          return new GpuPredicates.Leaf(300, 0, 0);
        }
        default -> {}
      }
      Matcher m = SLOT_VALID.matcher(name);
      if (m.matches()) return new GpuPredicates.Leaf(402, Long.parseLong(m.group(1)), 0);
      m = HAS_STATUS.matcher(name);
      if (m.matches()) {
        int a = nodeIndex(addrs, m.group(1));
        return a < 0 ? null : new GpuPredicates.Leaf(403, a, (Long.parseLong(m.group(3)) << 4) | STATUS.indexOf(m.group(2)));
      }
      m = HAS_COMMAND.matcher(name);
      if (m.matches()) {
        int a = nodeIndex(addrs, m.group(1));
        long code = codec.kvCodeOf(m.group(2));
        return a < 0 || code < 0 ? null : new GpuPredicates.Leaf(404, a, (Long.parseLong(m.group(3)) << 8) | code);
      }
      return null;
    };
  }

  private static int nodeIndex(List<Address> addrs, String name) {
    for (int i = 0; i < addrs.size(); i++)
      if (addrs.get(i).toString().equals(name)) return i;
    return -1;
  }

  // ---- helpers ----
  static String simpleName(Object o) {
    return o == null ? "" : o.getClass().getSimpleName();
  }

  /** A declared field of o or of a superclass, by name (lab classes are package-private). */
  static Object field(Object o, String name) throws ReflectiveOperationException {
    for (Class<?> k = o.getClass(); k != null; k = k.getSuperclass()) {
      try {
        Field f = k.getDeclaredField(name);
        f.setAccessible(true);
        return f.get(o);
      } catch (NoSuchFieldException e) {
        // try the superclass
      }
    }
    throw new NoSuchFieldException(o.getClass().getName() + "." + name);
  }

  // The commands and expected results of a ClientWorker's workload in order (Workload.java:52-92),
  // read from a copy; null for an infinite workload.
  private static List<Pair<Command, Result>> commands(ClientWorker cw, Address client) {
    if (cw.workload().infinite()) return null;
    Workload w = Cloning.clone(cw.workload());
    w.reset();
    List<Pair<Command, Result>> out = new ArrayList<>();
    while (w.hasNext()) out.add(w.nextCommandAndResult(client));
    return out;
  }

  /** The distinct value strings of a workload's Put / Append commands, sorted. */
  static List<String> tokens(List<List<Pair<Command, Result>>> work) throws ReflectiveOperationException {
    TreeSet<String> t = new TreeSet<>();
    for (List<Pair<Command, Result>> w : work)
      for (Pair<Command, Result> p : w) {
        String op = simpleName(p.getLeft());
        if (op.equals("Put") || op.equals("Append")) t.add((String) field(p.getLeft(), "value"));
      }
    return new ArrayList<>(t);
  }
}
