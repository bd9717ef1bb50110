package dslabs.framework.testing.search.gpu;

import static dslabs.framework.testing.search.gpu.GpuProtocols.field;
import static dslabs.framework.testing.search.gpu.GpuProtocols.simpleName;

import dslabs.framework.Address;
import dslabs.framework.Command;
import dslabs.framework.Result;
import dslabs.framework.testing.Event;
import dslabs.framework.testing.MessageEnvelope;
import dslabs.framework.testing.TimerEnvelope;
import java.util.ArrayList;
import java.util.List;
import java.util.Map;
import org.apache.commons.lang3.tuple.Pair;

/**
 * The lab2 primary-backup objects (java/src/dslabs/primarybackup) in the engine's packed form
 * (dslabs_amd/csrc/protocols/pb.hpp header): the parameter vector and each message / timer as the
 * dsl_event the engine describes for it (describe_message: fields[0] = the record's 54-bit
 * payload; describe_timer: PingCheckTimer 9 (100 ms), PingTimer 10 (25 ms), ClientTimer(seq) 11
 * (100 ms)). tests/test_java_binding.py checks the constants below against the C header and
 * protocols.py (PB.params, _result_bits, _view_bits).
 *
 * <pre>
 *   nodes      0 = the viewserver, 1..S = the servers, S+1.. = the clients
 *   view       num:4 | primary:2 @4 | backup:2 @6      (server ids = node indices 1..3, 0 = null)
 *   value      len:2 | symbol i (2 bits) @2 + 2i       (<= 3 equal-length value tokens)
 *   result     type:2 | value @2;  AppendResult 0, GetResult 1, KeyNotFound 2, PutOk 3
 *   amo        seq:2 | result:10 @2
 *   0 Ping viewNum    1 GetView    2 ViewReply view    3 Request seq    4 Reply seq | result @2
 *   5 StateTransfer view | app:40 @8 (key 0, key 1 values:8 each, amo[0] @16, amo[1] @28)
 *   6 StateTransferAck viewNum    7 Forward / 8 ForwardAck viewNum | client node @4 | seq @7
 * </pre>
 */
final class PBCodec {
  static final int MAX_SERVERS = 3, MAX_CLIENTS = 2, MAX_CMDS = 3, MAX_KEYS = 2, MAX_SYMS = 4, MAX_LEN = 3;
  static final int OP_GET = 0, OP_PUT = 1, OP_APPEND = 2;
  static final int R_APPEND = 0, R_GET = 1, R_NOTFOUND = 2, R_PUTOK = 3;
  static final int M_PING = 0, M_GETVIEW = 1, M_VIEWREPLY = 2, M_REQUEST = 3, M_REPLY = 4, M_ST = 5, M_STACK = 6,
      M_FORWARD = 7, M_FORWARDACK = 8, T_PINGCHECK = 9, T_PING = 10, T_CLIENT = 11;

  private final List<Address> addrs;
  private final int servers;
  private final List<List<Pair<Command, Result>>> work;
  private final List<String> keys = new ArrayList<>();
  private final List<String> syms = new ArrayList<>();

  private PBCodec(List<Address> addrs, int servers, List<List<Pair<Command, Result>>> work) {
    this.addrs = addrs;
    this.servers = servers;
    this.work = work;
  }

  /** Null when the workload has no device form (AmoKVCodec.of's rules, with 2 keys and values of <= 3 tokens). */
  static PBCodec of(List<Address> addrs, int servers, List<List<Pair<Command, Result>>> work)
      throws ReflectiveOperationException {
    if (servers < 1 || servers > MAX_SERVERS || work.isEmpty() || work.size() > MAX_CLIENTS) return null;
    PBCodec c = new PBCodec(addrs, servers, work);
    int n = work.get(0).size();
    for (List<Pair<Command, Result>> w : work) {
      if (w.size() != n || n < 1 || n > MAX_CMDS) return null;
      for (Pair<Command, Result> p : w) {
        int op = AmoKVCodec.op(p.getLeft());
        if (op < 0) return null;
        String k = (String) field(p.getLeft(), "key");
        if (!c.keys.contains(k)) c.keys.add(k);
        if (op != OP_GET) {
          String v = (String) field(p.getLeft(), "value");
          if (!c.syms.contains(v)) c.syms.add(v);
        }
      }
    }
    if (c.keys.size() > MAX_KEYS || c.syms.size() > MAX_SYMS) return null;
    for (String s : c.syms)
      if (s.isEmpty() || s.length() != c.syms.get(0).length()) return null;
    for (List<Pair<Command, Result>> w : work)
      for (Pair<Command, Result> p : w)
        if (p.getRight() != null && c.resultCode(p.getRight()) < 0) return null;
    return c;
  }

  /** dsl_protocol_desc.params: {servers, clients, ncmds} + per (client < 2, command < 3) {op, key, sym, expected}. */
  long[] params() {
    long[] ps = new long[3 + 4 * MAX_CLIENTS * MAX_CMDS];
    ps[0] = servers;
    ps[1] = work.size();
    ps[2] = work.get(0).size();
    try {
      for (int c = 0; c < MAX_CLIENTS; c++)
        for (int k = 0; k < MAX_CMDS; k++) {
          int b = 3 + 4 * (c * MAX_CMDS + k);
          boolean has = c < work.size() && k < work.get(c).size();
          Command cmd = has ? work.get(c).get(k).getLeft() : null;
          Result res = has ? work.get(c).get(k).getRight() : null;
          ps[b] = cmd == null ? 0 : AmoKVCodec.op(cmd);
          ps[b + 1] = cmd == null ? 0 : keys.indexOf((String) field(cmd, "key"));
          ps[b + 2] = cmd == null || AmoKVCodec.op(cmd) == OP_GET ? 0 : syms.indexOf((String) field(cmd, "value"));
          ps[b + 3] = res == null ? -1 : resultCode(res);
        }
    } catch (ReflectiveOperationException e) {
      throw new IllegalStateException(e);
    }
    return ps;
  }

  long valueCode(String v) {
    if (syms.isEmpty()) return v.isEmpty() ? 0 : -1;
    int w = syms.get(0).length();
    if (v.length() % w != 0 || v.length() / w > MAX_LEN) return -1;
    long r = v.length() / w;
    for (int i = 0; i < v.length() / w; i++) {
      int t = syms.indexOf(v.substring(i * w, (i + 1) * w));
      if (t < 0) return -1;
      r |= (long) t << (2 + 2 * i);
    }
    return r;
  }

  long resultCode(Result r) throws ReflectiveOperationException {
    switch (simpleName(r)) {
      case "PutOk" -> {
        return R_PUTOK;
      }
      case "KeyNotFound" -> {
        return R_NOTFOUND;
      }
      case "AppendResult", "GetResult" -> {
        long v = valueCode((String) field(r, "value"));
        return v < 0 ? -1 : (simpleName(r).equals("AppendResult") ? R_APPEND : R_GET) | v << 2;
      }
      default -> {
        return -1;
      }
    }
  }

  private long serverId(Object address) {
    if (address == null) return 0;
    int i = addrs.indexOf(((Address) address).rootAddress());
    return i >= 1 && i <= servers ? i : -1;
  }

  long viewCode(Object view) throws ReflectiveOperationException {
    long n = ((Number) field(view, "viewNum")).longValue(), p = serverId(field(view, "primary")),
        b = serverId(field(view, "backup"));
    return n > 15 || p < 0 || b < 0 ? -1 : n | p << 4 | b << 6;
  }

  /** An AMOApplication(KVStore) as the 40 bits of a server's words w1 | w2 << 28 (pb.hpp execute). */
  long appCode(Object amoApp) throws ReflectiveOperationException {
    Map<?, ?> data = (Map<?, ?>) field(field(amoApp, "application"), "data");
    Map<?, ?> last = (Map<?, ?>) field(amoApp, "lastResults");
    long bits = 0;
    for (Map.Entry<?, ?> e : data.entrySet()) {
      int k = keys.indexOf((String) e.getKey());
      long v = valueCode((String) e.getValue());
      if (k < 0 || v < 0) return -1;
      bits |= v << (8 * k);
    }
    for (Map.Entry<?, ?> e : last.entrySet()) {
      int c = addrs.indexOf(((Address) e.getKey()).rootAddress()) - 1 - servers;
      long seq = ((Number) field(e.getValue(), "sequenceNum")).longValue();
      long r = resultCode((Result) field(e.getValue(), "result"));
      if (c < 0 || c >= MAX_CLIENTS || r < 0 || seq < 0 || seq > 3) return -1;
      bits |= (seq | r << 2) << (16 + 12 * c);
    }
    return bits;
  }

  private long forwardCode(Object m) throws ReflectiveOperationException {
    Object amo = field(m, "command");
    int ca = addrs.indexOf(((Address) field(amo, "clientAddress")).rootAddress());
    long v = ((Number) field(m, "viewNum")).longValue(), seq = ((Number) field(amo, "sequenceNum")).longValue();
    // the device fields are 4 (view) and 2 (seq) bits (pb.hpp: m & 15, (m >> 7) & 3)
    if (ca <= servers || v < 0 || v > 15 || seq < 0 || seq > 3) return -1;
    return v | (long) ca << 4 | seq << 7;
  }

  /** v when it fits the device field (0..max), else -1: the event then has no encoding (JVM fallback). */
  private static long bounded(long v, long max) {
    return v < 0 || v > max ? -1 : v;
  }

  /** The dsl_event of a Java event; null when it has none. */
  Dsl.Event encode(Event je) {
    try {
      if (je instanceof TimerEnvelope t) {
        int node = addrs.indexOf(t.to().rootAddress());
        int min = t.minTimerLengthMillis(), max = t.maxTimerLengthMillis();
        return switch (simpleName(t.timer())) {
          case "PingCheckTimer" -> node == 0 ? Dsl.Event.timer(node, T_PINGCHECK, min, max, 0) : null;
          case "PingTimer" -> node >= 1 && node <= servers ? Dsl.Event.timer(node, T_PING, min, max, 0) : null;
          case "ClientTimer" -> node > servers
              ? Dsl.Event.timer(node, T_CLIENT, min, max, ((Number) field(t.timer(), "seq")).longValue()) : null;
          default -> null;
        };
      }
      MessageEnvelope me = (MessageEnvelope) je;
      Object m = me.message();
      int type;
      long payload;
      switch (simpleName(m)) {
        case "Ping" -> {
          type = M_PING;
          payload = bounded(((Number) field(m, "viewNum")).longValue(), 15);
        }
        case "GetView" -> {
          type = M_GETVIEW;
          payload = 0;
        }
        case "ViewReply" -> {
          type = M_VIEWREPLY;
          payload = viewCode(field(m, "view"));
        }
        case "Request" -> {
          type = M_REQUEST;
          payload = bounded(((Number) field(field(m, "command"), "sequenceNum")).longValue(), 3);
        }
        case "Reply" -> {
          type = M_REPLY;
          Object amo = field(m, "result");
          long r = resultCode((Result) field(amo, "result"));
          long seq = bounded(((Number) field(amo, "sequenceNum")).longValue(), 3);
          payload = r < 0 || seq < 0 ? -1 : seq | r << 2;
        }
        case "StateTransfer" -> {
          type = M_ST;
          long v = viewCode(field(m, "view")), app = appCode(field(m, "app"));
          payload = v < 0 || app < 0 ? -1 : v | app << 8;
        }
        case "StateTransferAck" -> {
          type = M_STACK;
          payload = bounded(((Number) field(m, "viewNum")).longValue(), 15);
        }
        case "Forward", "ForwardAck" -> {
          type = simpleName(m).equals("Forward") ? M_FORWARD : M_FORWARDACK;
          payload = forwardCode(m);
        }
        default -> {
          return null;
        }
      }
      if (payload < 0) return null;
      return Dsl.Event.message(addrs.indexOf(me.from().rootAddress()), addrs.indexOf(me.to().rootAddress()), type,
          payload);
    } catch (ReflectiveOperationException | ClassCastException e) {
      return null;
    }
  }
}
