package dslabs.framework.testing.search.gpu;

import dslabs.framework.Address;
import dslabs.framework.Node;
import dslabs.framework.testing.ClientWorker;
import dslabs.framework.testing.Event;
import dslabs.framework.testing.MessageEnvelope;
import dslabs.framework.testing.TimerEnvelope;
import dslabs.framework.testing.search.SearchState;
import java.util.ArrayList;
import java.util.Comparator;
import java.util.List;
import java.util.Map;
import java.util.function.Function;

/**
 * Which initial states have a device form, and how events of the device trace map back to Java
 * events. A protocol entry gives the engine's protocol id and parameter vector (the same vectors
 * dslabs_amd/protocols.py builds), its addresses in the engine's node order, the predicate leaf
 * registry, and an event matcher. Covered: lab0 PingPong (labs/lab0-pingpong) and the reference's
 * single-instance Paxos (T/visualization/examples/paxosmadesimple); the builder-authored lab1-3
 * solutions exist only on the device and in the oracle, since the reference's lab classes are stubs.
 * Anything else returns null (GpuBFS then runs the JVM search).
 */
public final class GpuProtocols {
  /** A device protocol for one initial state. */
  public record Desc(Dsl.Protocol protocol, List<Address> addresses, Function<String, GpuPredicates.Leaf> leaf,
                     EventMatcher matcher) {}

  /** Whether a Java event is the device event. */
  public interface EventMatcher {
    boolean matches(Event javaEvent, Dsl.Event deviceEvent, List<Address> addresses);
  }

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
    String first = nodes.get(0).getClass().getSimpleName();
    if (first.equals("PingServer")) return pingPong(addrs, nodes);
    if (first.endsWith("Proposer")) return sipaxos(addrs, nodes);
    return null;
  }

  private static int rank(Node n) {
    String c = n.getClass().getSimpleName();
    return c.equals("PingServer") || c.endsWith("Proposer") ? 0 : c.equals("Acceptor") ? 1 : 2;
  }

  // ---- lab0 PingPong: "pingserver", then ClientWorkers around PingClients (PingTest.java:44-51) ----
  private static Desc pingPong(List<Address> addrs, List<Node> nodes) {
    int pings = -1;
    for (int i = 1; i < nodes.size(); i++) {
      if (!(nodes.get(i) instanceof ClientWorker cw)) return null;
      int n = workloadSize(cw);
      if (n < 0 || (pings >= 0 && n != pings)) return null;
      pings = n;
    }
    if (pings < 1 || pings > 15 || nodes.size() - 1 > 4) return null;
    long[] params = {nodes.size() - 1, pings, 1, 1};  // clients, pings, value check, timer re-set
    Function<String, GpuPredicates.Leaf> leaf = name -> {
      Integer id = STANDARD.get(name);
      return id == null ? null : new GpuPredicates.Leaf(id, 0, 0);
    };
    return new Desc(new Dsl.Protocol(1, params), addrs, leaf, (je, de, a) ->
        sameEnds(je, de, a) && classIs(je, de.isTimer() ? "PingTimer" : de.type() == 0 ? "PingRequest" : "PongReply")
            && je.toString().contains("value=ping-" + de.fields()[0] + ")"));
  }

  // ---- SingleInstancePaxos: proposers then acceptors (SingleInstancePaxos.java:50-127) ----
  private static Desc sipaxos(List<Address> addrs, List<Node> nodes) {
    int p = 0;
    while (p < nodes.size() && nodes.get(p).getClass().getSimpleName().endsWith("Proposer")) p++;
    int a = nodes.size() - p;
    if (p < 1 || p > 3 || a < 1 || a > 5) return null;
    boolean incorrect = nodes.get(0).getClass().getSimpleName().equals("BadProposer");
    long[] params = {p, a, incorrect ? 1 : 0};
    Function<String, GpuPredicates.Leaf> leaf = name -> switch (name) {
      case "Agreement" -> new GpuPredicates.Leaf(100, 0, 0);
      case "Integrity" -> new GpuPredicates.Leaf(101, 0, 0);
      case "Termination" -> new GpuPredicates.Leaf(102, 0, 0);
      default -> null;
    };
    String[] types = {"Prepare", "PrepareAck", "Accept", "AcceptAck"};
    return new Desc(new Dsl.Protocol(2, params), addrs, leaf, (je, de, ad) -> {
      if (!sameEnds(je, de, ad)) return false;
      if (de.isTimer()) return classIs(je, "Propose");
      return classIs(je, types[de.type()]) && je.toString().contains("proposalNumber=" + de.fields()[0]);
    });
  }

  // ---- helpers ----
  private static boolean sameEnds(Event je, Dsl.Event de, List<Address> addrs) {
    if (de.isTimer()) return je instanceof TimerEnvelope t && t.to().rootAddress().equals(addrs.get(de.to()));
    return je instanceof MessageEnvelope m && m.from().rootAddress().equals(addrs.get(de.from()))
        && m.to().rootAddress().equals(addrs.get(de.to()));
  }

  private static boolean classIs(Event je, String simpleName) {
    Object body = je instanceof MessageEnvelope m ? m.message() : ((TimerEnvelope) je).timer();
    return body.getClass().getSimpleName().equals(simpleName);
  }

  // ClientWorker's workload size (Workload.size, Workload.java:90), -1 for an infinite workload
  private static int workloadSize(ClientWorker cw) {
    return cw.workload().infinite() ? -1 : cw.workload().size();
  }
}
