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
import org.apache.commons.lang3.tuple.Pair;

/**
 * The lab1 AMO key-value objects (java/src/dslabs/clientserver, atmostonce, kvstore) in the
 * engine's packed form (dslabs_amd/csrc/protocols/amokv.hpp header): the parameter vector and each
 * message / timer as the dsl_event the engine describes for it (describe_message: fields = {seq,
 * result}; describe_timer: ClientTimer = type 2, fields = {seq}). tests/test_java_binding.py checks
 * the constants below against the C header and protocols.py (AmoKV.params, _result_bits).
 *
 * <pre>
 *   nodes        0 = the server, 1..c = the clients (ClientWorkers around SimpleClients)
 *   op           GET 0, PUT 1, APPEND 2;  key: id by first use (<= 3 keys);  sym: value id by first use
 *   value        len:4 | symbol i (2 bits) @4 + 2i   (a sequence of <= 9 equal-length value tokens)
 *   result       type:2 | value @2;  types AppendResult 0, GetResult 1, KeyNotFound 2, PutOk 3
 *   0 Request    {seq, 0}                1 Reply   {seq, result}
 * </pre>
 */
final class AmoKVCodec {
  static final int MAX_CLIENTS = 3, MAX_CMDS = 3, MAX_KEYS = 3, MAX_SYMS = 4, MAX_LEN = 9;
  static final int OP_GET = 0, OP_PUT = 1, OP_APPEND = 2;
  static final int R_APPEND = 0, R_GET = 1, R_NOTFOUND = 2, R_PUTOK = 3;
  static final int M_REQUEST = 0, M_REPLY = 1, T_CLIENT = 2, RETRY_MILLIS = 100;

  private final List<Address> addrs;
  private final List<List<Pair<Command, Result>>> work;
  private final List<String> keys = new ArrayList<>();
  private final List<String> syms = new ArrayList<>();

  private AmoKVCodec(List<Address> addrs, List<List<Pair<Command, Result>>> work) {
    this.addrs = addrs;
    this.work = work;
  }

  /**
   * Null when the workload has no device form: clients with different command counts, more than
   * 3 commands, keys or 4 value tokens, tokens of unequal length, or an expected result the value
   * encoding cannot hold.
   */
  static AmoKVCodec of(List<Address> addrs, List<List<Pair<Command, Result>>> work)
      throws ReflectiveOperationException {
    if (work.isEmpty() || work.size() > MAX_CLIENTS) return null;
    AmoKVCodec c = new AmoKVCodec(addrs, work);
    int n = work.get(0).size();
    for (List<Pair<Command, Result>> w : work) {
      if (w.size() != n || n < 1 || n > MAX_CMDS) return null;  // the device has one command count
      for (Pair<Command, Result> p : w) {
        int op = op(p.getLeft());
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

  static int op(Object kvCommand) {
    return switch (simpleName(kvCommand)) {
      case "Get" -> OP_GET;
      case "Put" -> OP_PUT;
      case "Append" -> OP_APPEND;
      default -> -1;
    };
  }

  /** dsl_protocol_desc.params: {clients, ncmds} + per (client < 3, command < 3) {op, key, sym, expected}. */
  long[] params() {
    long[] ps = new long[2 + 4 * MAX_CLIENTS * MAX_CMDS];
    ps[0] = work.size();
    ps[1] = work.get(0).size();
    try {
      for (int c = 0; c < MAX_CLIENTS; c++)
        for (int k = 0; k < MAX_CMDS; k++) {
          int b = 2 + 4 * (c * MAX_CMDS + k);
          boolean has = c < work.size() && k < work.get(c).size();
          Command cmd = has ? work.get(c).get(k).getLeft() : null;
          Result res = has ? work.get(c).get(k).getRight() : null;
          ps[b] = cmd == null ? 0 : op(cmd);
          ps[b + 1] = cmd == null ? 0 : keys.indexOf((String) field(cmd, "key"));
          ps[b + 2] = cmd == null || op(cmd) == OP_GET ? 0 : syms.indexOf((String) field(cmd, "value"));
          ps[b + 3] = res == null ? -1 : resultCode(res);
        }
    } catch (ReflectiveOperationException e) {
      throw new IllegalStateException(e);
    }
    return ps;
  }

  /** A value string as len:4 | symbols @4; -1 when it is not a sequence of <= 9 workload tokens. */
  long valueCode(String v) {
    if (syms.isEmpty()) return v.isEmpty() ? 0 : -1;
    int w = syms.get(0).length();
    if (v.length() % w != 0 || v.length() / w > MAX_LEN) return -1;
    long r = v.length() / w;
    for (int i = 0; i < v.length() / w; i++) {
      int t = syms.indexOf(v.substring(i * w, (i + 1) * w));
      if (t < 0) return -1;
      r |= (long) t << (4 + 2 * i);
    }
    return r;
  }

  long resultCode(Result r) throws ReflectiveOperationException {
    long v;
    switch (simpleName(r)) {
      case "PutOk" -> {
        return R_PUTOK;
      }
      case "KeyNotFound" -> {
        return R_NOTFOUND;
      }
      case "AppendResult" -> {
        v = valueCode((String) field(r, "value"));
        return v < 0 ? -1 : R_APPEND | v << 2;
      }
      case "GetResult" -> {
        v = valueCode((String) field(r, "value"));
        return v < 0 ? -1 : R_GET | v << 2;
      }
      default -> {
        return -1;
      }
    }
  }

  /** The dsl_event of a Java event; null when it has none. */
  Dsl.Event encode(Event je) {
    try {
      if (je instanceof TimerEnvelope t) {
        if (!simpleName(t.timer()).equals("ClientTimer")) return null;
        return Dsl.Event.timer(addrs.indexOf(t.to().rootAddress()), T_CLIENT, t.minTimerLengthMillis(),
            t.maxTimerLengthMillis(), ((Number) field(t.timer(), "sequenceNum")).longValue());
      }
      MessageEnvelope me = (MessageEnvelope) je;
      Object m = me.message();
      int from = addrs.indexOf(me.from().rootAddress()), to = addrs.indexOf(me.to().rootAddress());
      switch (simpleName(m)) {
        case "Request" -> {
          long seq = ((Number) field(field(m, "command"), "sequenceNum")).longValue();
          return Dsl.Event.message(from, to, M_REQUEST, seq, 0);
        }
        case "Reply" -> {
          Object amo = field(m, "result");
          long r = resultCode((Result) field(amo, "result"));
          return r < 0 ? null
              : Dsl.Event.message(from, to, M_REPLY, ((Number) field(amo, "sequenceNum")).longValue(), r);
        }
        default -> {
          return null;
        }
      }
    } catch (ReflectiveOperationException | ClassCastException e) {
      return null;
    }
  }
}
