package dslabs.framework.testing.search.gpu;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.foreign.ValueLayout;
import java.lang.invoke.MethodHandle;
import java.nio.file.Path;

/**
 * Panama FFM binding of the C ABI in include/dslabs_hip.h (libdslabs_hip.so). Structs are plain
 * byte layouts at the offsets of the C header (x86-64 / gfx950 host ABI); tests/test_java_binding.py
 * checks every OFF_* / SIZE_* constant here against the C structs. Not compiled in this build (no
 * JDK); JDK 22+ (or 21 with --enable-preview). deviceAvailable() refuses a library whose
 * dsl_abi_version() is not ABI_VERSION.
 */
public final class Dsl {
  // dsl_protocol_desc
  public static final long SIZE_PROTOCOL_DESC = 520, OFF_DESC_PROTOCOL = 0, OFF_DESC_N_PARAMS = 4, OFF_DESC_PARAMS = 8;
  public static final int MAX_PARAMS = 64;
  // dsl_predicate
  public static final long SIZE_PREDICATE = 24, OFF_PRED_ID = 0, OFF_PRED_NEGATE = 4, OFF_PRED_ARG0 = 8,
      OFF_PRED_ARG1 = 16;
  // dsl_settings
  public static final long SIZE_SETTINGS = 3488, OFF_MAX_DEPTH = 0, OFF_MAX_TIME_MS = 4, OFF_NETWORK_ACTIVE = 8,
      OFF_DELIVER_TIMERS = 12, OFF_LINK_ACTIVE = 16, OFF_SENDER_ACTIVE = 1040, OFF_RECEIVER_ACTIVE = 1072,
      OFF_TIMERS_ACTIVE = 1104, OFF_N_INVARIANTS = 1136, OFF_N_GOALS = 1140, OFF_N_PRUNES = 1144,
      OFF_INVARIANTS = 1152, OFF_GOALS = 1536, OFF_PRUNES = 1920, OFF_TABLE_LOG2 = 2304, OFF_N_POOL = 2308,
      OFF_MAX_FRONTIER = 2312, OFF_MEMORY_BUDGET = 2320, OFF_POOL = 2328, OFF_DO_CHECKS = 3480,
      OFF_CHECK_SAMPLE = 3484;
  public static final int CHECKS_NONE = 0, CHECKS_ERRORS = 1, CHECKS_ALL = 2;
  public static final int MAX_NODES = 32, MAX_PREDICATES = 16, MAX_POOL = 48;
  // dsl_engine_config
  public static final long SIZE_ENGINE_CONFIG = 160, OFF_CFG_DEVICE = 0, OFF_CFG_RANK = 4, OFF_CFG_WORLD = 8,
      OFF_CFG_VSHARDS = 12, OFF_CFG_COMM_ID = 16, OFF_CFG_REPLICATE_BELOW = 144, OFF_CFG_FLAGS = 152;
  // dsl_event
  public static final long SIZE_EVENT = 96, OFF_EV_IS_TIMER = 0, OFF_EV_FROM = 4, OFF_EV_TO = 8, OFF_EV_TYPE = 12,
      OFF_EV_N_FIELDS = 16, OFF_EV_TIMER_MIN = 20, OFF_EV_TIMER_MAX = 24, OFF_EV_FIELDS = 32;
  // dsl_result
  public static final long SIZE_RESULT = 320, OFF_RES_END = 0, OFF_RES_TERMINAL_DEPTH = 4, OFF_RES_PRED_INDEX = 8,
      OFF_RES_MAX_DEPTH = 12, OFF_RES_STATES = 16, OFF_RES_N_LEVELS = 24, OFF_RES_TRACE_LEN = 28,
      OFF_RES_PER_DEPTH = 32, OFF_RES_TRACE = 40, OFF_RES_TERMINAL_STATE = 48, OFF_RES_STATE_BYTES = 56,
      OFF_RES_INITIAL_DEPTH = 60, OFF_RES_ELAPSED = 64, OFF_RES_CHECKS_RUN = 104, OFF_RES_NOT_DETERMINISTIC = 112,
      OFF_RES_NOT_IDEMPOTENT = 120, OFF_RES_FIRST_NOT_DETERMINISTIC = 128, OFF_RES_FIRST_NOT_IDEMPOTENT = 224;

  // DSL_ABI_VERSION: the struct layout above; a library of another version is refused
  public static final int ABI_VERSION = 5;
  public static final int MAX_EVENT_FIELDS = 8;

  // dsl_protocol_id (include/dslabs_hip.h)
  public static final int PROTO_PINGPONG = 1, PROTO_SIPAXOS = 2, PROTO_AMOKV = 4, PROTO_MULTIPAXOS = 5, PROTO_PB = 6;

  // dsl_end_condition (include/dslabs_hip.h)
  public static final int END_EXCEPTION_THROWN = 0, END_INVARIANT_VIOLATED = 1, END_GOAL_FOUND = 2,
      END_SPACE_EXHAUSTED = 3, END_TIME_EXHAUSTED = 4;

  private static final Linker LINKER = Linker.nativeLinker();
  private static final SymbolLookup LIB = SymbolLookup.libraryLookup(
      Path.of(System.getProperty("dslabs.hip.lib", "libdslabs_hip.so")), Arena.global());

  private static MethodHandle fn(String name, FunctionDescriptor d) {
    return LINKER.downcallHandle(LIB.find(name).orElseThrow(() -> new UnsatisfiedLinkError(name)), d);
  }

  private static final ValueLayout.OfInt I = ValueLayout.JAVA_INT;
  private static final ValueLayout A = ValueLayout.ADDRESS;
  static final MethodHandle CREATE = fn("dsl_create", FunctionDescriptor.of(I, A, A, A));
  static final MethodHandle SET_SETTINGS = fn("dsl_set_settings", FunctionDescriptor.of(I, A, A));
  static final MethodHandle SET_INITIAL =
      fn("dsl_set_initial", FunctionDescriptor.of(I, A, A, ValueLayout.JAVA_LONG, I));
  static final MethodHandle RUN = fn("dsl_run", FunctionDescriptor.of(I, A, A));
  static final MethodHandle RESULT_FREE = fn("dsl_result_free", FunctionDescriptor.ofVoid(A));
  static final MethodHandle DESTROY = fn("dsl_destroy", FunctionDescriptor.ofVoid(A));
  static final MethodHandle LAST_ERROR = fn("dsl_last_error", FunctionDescriptor.of(A));
  static final MethodHandle DEVICE_COUNT = fn("dsl_device_count", FunctionDescriptor.of(I));
  static final MethodHandle ABI = fn("dsl_abi_version", FunctionDescriptor.of(I));
  static final MethodHandle REPLAY = fn("dsl_replay", FunctionDescriptor.of(I, A, A, I, I, A));
  static final MethodHandle SET_DROPPED = fn("dsl_set_dropped", FunctionDescriptor.of(I, A, A, I));
  static final MethodHandle DROP_PENDING =
      fn("dsl_drop_pending_messages", FunctionDescriptor.of(I, A, A, ValueLayout.JAVA_LONG, A, I, A));
  static final MethodHandle UNDROP =
      fn("dsl_undrop_messages", FunctionDescriptor.of(I, A, A, ValueLayout.JAVA_LONG, A, I, I, I));

  private Dsl() {}

  static void check(int rc, String what) {
    if (rc == 0) return;
    String msg;
    try {
      MemorySegment p = (MemorySegment) LAST_ERROR.invokeExact();
      msg = p.reinterpret(4096).getString(0);
    } catch (Throwable t) {
      msg = "?";
    }
    throw new IllegalStateException(what + " failed (" + rc + "): " + msg);
  }

  public static boolean deviceAvailable() {
    try {
      int abi = (int) ABI.invokeExact();
      if (abi != ABI_VERSION)
        throw new IllegalStateException("libdslabs_hip.so has ABI version " + abi + ", this binding needs " + ABI_VERSION);
      return (int) DEVICE_COUNT.invokeExact() > 0;
    } catch (IllegalStateException e) {
      throw e;
    } catch (Throwable t) {
      return false;
    }
  }

  /** A protocol descriptor: the protocol id and its parameter vector (GpuProtocols). */
  public record Protocol(int id, long[] params) {}

  /** One engine (one GPU). */
  public static final class Engine implements AutoCloseable {
    private final Arena arena = Arena.ofConfined();
    private final MemorySegment handle;
    private final MemorySegment desc;

    public Engine(Protocol p) {
      desc = arena.allocate(SIZE_PROTOCOL_DESC, 8);
      desc.set(ValueLayout.JAVA_INT, OFF_DESC_PROTOCOL, p.id());
      desc.set(ValueLayout.JAVA_INT, OFF_DESC_N_PARAMS, p.params().length);
      for (int i = 0; i < p.params().length; i++)
        desc.set(ValueLayout.JAVA_LONG, OFF_DESC_PARAMS + 8L * i, p.params()[i]);
      MemorySegment cfg = arena.allocate(SIZE_ENGINE_CONFIG, 8);
      cfg.set(ValueLayout.JAVA_INT, OFF_CFG_DEVICE, -1);
      cfg.set(ValueLayout.JAVA_INT, OFF_CFG_WORLD, 1);
      cfg.set(ValueLayout.JAVA_LONG, OFF_CFG_REPLICATE_BELOW, -1);
      MemorySegment out = arena.allocate(A);
      try {
        check((int) CREATE.invokeExact(desc, cfg, out), "dsl_create");
      } catch (RuntimeException e) {
        throw e;
      } catch (Throwable t) {
        throw new IllegalStateException(t);
      }
      handle = out.get(A, 0);
    }

    public void setSettings(MemorySegment settings) {
      try {
        check((int) SET_SETTINGS.invokeExact(handle, settings), "dsl_set_settings");
      } catch (RuntimeException e) {
        throw e;
      } catch (Throwable t) {
        throw new IllegalStateException(t);
      }
    }

    public void setInitial(byte[] packed, int depth) {
      MemorySegment buf = arena.allocate(packed.length, 8);
      MemorySegment.copy(MemorySegment.ofArray(packed), 0, buf, 0, packed.length);
      try {
        check((int) SET_INITIAL.invokeExact(handle, buf, (long) packed.length, depth), "dsl_set_initial");
      } catch (RuntimeException e) {
        throw e;
      } catch (Throwable t) {
        throw new IllegalStateException(t);
      }
    }

    /**
     * The start state's dropped network (dsl_set_dropped): packed records, as
     * dsl_drop_pending_messages leaves them; network predicates see them.
     */
    public void setDropped(long[] records) {
      MemorySegment buf = arena.allocate(8L * Math.max(1, records.length), 8);
      for (int i = 0; i < records.length; i++) buf.set(ValueLayout.JAVA_LONG, 8L * i, records[i]);
      try {
        check((int) SET_DROPPED.invokeExact(handle, buf, records.length), "dsl_set_dropped");
      } catch (RuntimeException e) {
        throw e;
      } catch (Throwable t) {
        throw new IllegalStateException(t);
      }
    }

    /**
     * SearchState.dropPendingMessages then undropMessagesFrom / undropMessagesTo
     * (SearchState.java:538-561) on a packed state (dsl_drop_pending_messages, dsl_undrop_messages):
     * every record of its network moves into the returned dropped set (sorted, distinct), then the
     * dropped records sent by each node of `undropFrom` and addressed to each node of `undropTo`
     * (node indices) are live again. `packed` is updated in place.
     */
    public long[] dropPending(byte[] packed, int[] undropFrom, int[] undropTo) {
      final int cap = 4096;
      MemorySegment st = arena.allocate(packed.length, 8);
      MemorySegment.copy(MemorySegment.ofArray(packed), 0, st, 0, packed.length);
      MemorySegment dr = arena.allocate(8L * cap, 8);
      MemorySegment n = arena.allocate(I);
      n.set(I, 0, 0);
      try {
        check((int) DROP_PENDING.invokeExact(desc, st, (long) packed.length, dr, cap, n), "dsl_drop_pending_messages");
        int nd = n.get(I, 0);
        for (int a : undropFrom)
          check((int) UNDROP.invokeExact(desc, st, (long) packed.length, dr, nd, a, -1), "dsl_undrop_messages");
        for (int b : undropTo)
          check((int) UNDROP.invokeExact(desc, st, (long) packed.length, dr, nd, -1, b), "dsl_undrop_messages");
        MemorySegment.copy(st, 0, MemorySegment.ofArray(packed), 0, packed.length);
        long[] out = new long[nd];
        for (int i = 0; i < nd; i++) out[i] = dr.get(ValueLayout.JAVA_LONG, 8L * i);
        return out;
      } catch (RuntimeException e) {
        throw e;
      } catch (Throwable t) {
        throw new IllegalStateException(t);
      }
    }

    /** Runs the BFS; the result is copied out of native memory and freed. */
    public Result run() {
      MemorySegment out = arena.allocate(A);
      try {
        check((int) RUN.invokeExact(handle, out), "dsl_run");
        return take(out);
      } catch (RuntimeException e) {
        throw e;
      } catch (Throwable t) {
        throw new IllegalStateException(t);
      }
    }

    /**
     * TraceReplaySearch on the engine's transitions (dsl_replay): steps `trace` from the start
     * state with checkState after each step; with `minimize` a terminal's trace is minimized.
     * The result's terminalState is the last state reached (also when the trace ran out).
     */
    public Result replay(Event[] trace, boolean minimize) {
      MemorySegment evs = arena.allocate(SIZE_EVENT * Math.max(1, trace.length), 8);
      for (int i = 0; i < trace.length; i++) trace[i].write(evs.asSlice(SIZE_EVENT * i, SIZE_EVENT));
      MemorySegment out = arena.allocate(A);
      try {
        check((int) REPLAY.invokeExact(handle, evs, trace.length, minimize ? 1 : 0, out), "dsl_replay");
        return take(out);
      } catch (RuntimeException e) {
        throw e;
      } catch (Throwable t) {
        throw new IllegalStateException(t);
      }
    }

    private static Result take(MemorySegment out) throws Throwable {
      MemorySegment r = out.get(A, 0).reinterpret(SIZE_RESULT);
      Result res = Result.copyOf(r);
      RESULT_FREE.invokeExact(r);
      return res;
    }

    public Arena arena() {
      return arena;
    }

    @Override
    public void close() {
      try {
        DESTROY.invokeExact(handle);
      } catch (Throwable ignored) {
      }
      arena.close();
    }
  }

  /** A decoded event of a trace (dsl_event). */
  public record Event(boolean isTimer, int from, int to, int type, long[] fields, int timerMin, int timerMax) {
    public static Event message(int from, int to, int type, long... fields) {
      return new Event(false, from, to, type, fields, 0, 0);
    }

    public static Event timer(int node, int type, int min, int max, long... fields) {
      return new Event(true, node, node, type, fields, min, max);
    }

    /** Content equality, as the engine matches events (replay.hpp same_event). */
    public boolean sameAs(Event o) {
      return isTimer == o.isTimer && from == o.from && to == o.to && type == o.type && timerMin == o.timerMin
          && timerMax == o.timerMax && java.util.Arrays.equals(fields, o.fields);
    }

    void write(MemorySegment ev) {
      ev.fill((byte) 0);
      ev.set(ValueLayout.JAVA_INT, OFF_EV_IS_TIMER, isTimer ? 1 : 0);
      ev.set(ValueLayout.JAVA_INT, OFF_EV_FROM, from);
      ev.set(ValueLayout.JAVA_INT, OFF_EV_TO, to);
      ev.set(ValueLayout.JAVA_INT, OFF_EV_TYPE, type);
      ev.set(ValueLayout.JAVA_INT, OFF_EV_N_FIELDS, fields.length);
      ev.set(ValueLayout.JAVA_INT, OFF_EV_TIMER_MIN, timerMin);
      ev.set(ValueLayout.JAVA_INT, OFF_EV_TIMER_MAX, timerMax);
      for (int i = 0; i < fields.length && i < MAX_EVENT_FIELDS; i++)
        ev.set(ValueLayout.JAVA_LONG, OFF_EV_FIELDS + 8L * i, fields[i]);
    }

    static Event at(MemorySegment ev) {
      int n = ev.get(ValueLayout.JAVA_INT, OFF_EV_N_FIELDS);
      long[] f = new long[n];
      for (int i = 0; i < n; i++) f[i] = ev.get(ValueLayout.JAVA_LONG, OFF_EV_FIELDS + 8L * i);
      return new Event(ev.get(ValueLayout.JAVA_INT, OFF_EV_IS_TIMER) != 0, ev.get(ValueLayout.JAVA_INT, OFF_EV_FROM),
          ev.get(ValueLayout.JAVA_INT, OFF_EV_TO), ev.get(ValueLayout.JAVA_INT, OFF_EV_TYPE), f,
          ev.get(ValueLayout.JAVA_INT, OFF_EV_TIMER_MIN), ev.get(ValueLayout.JAVA_INT, OFF_EV_TIMER_MAX));
    }
  }

  /** dsl_result, copied. */
  public record Result(int endCondition, int terminalDepth, int predicateIndex, int maxDepth, long states,
                       long[] perDepth, Event[] trace, byte[] terminalState, int initialDepth, double elapsedSecs,
                       long checksRun, long notDeterministic, long notIdempotent) {
    static Result copyOf(MemorySegment r) {
      int nl = r.get(ValueLayout.JAVA_INT, OFF_RES_N_LEVELS), tl = r.get(ValueLayout.JAVA_INT, OFF_RES_TRACE_LEN);
      long[] pd = new long[nl];
      MemorySegment pdp = r.get(A, OFF_RES_PER_DEPTH).reinterpret(8L * nl);
      for (int i = 0; i < nl; i++) pd[i] = pdp.get(ValueLayout.JAVA_LONG, 8L * i);
      Event[] tr = new Event[tl];
      MemorySegment tp = r.get(A, OFF_RES_TRACE).reinterpret(SIZE_EVENT * Math.max(1, tl));
      for (int i = 0; i < tl; i++) tr[i] = Event.at(tp.asSlice(SIZE_EVENT * i, SIZE_EVENT));
      MemorySegment sp = r.get(A, OFF_RES_TERMINAL_STATE);
      byte[] st = null;
      if (!sp.equals(MemorySegment.NULL))
        st = sp.reinterpret(r.get(ValueLayout.JAVA_INT, OFF_RES_STATE_BYTES)).toArray(ValueLayout.JAVA_BYTE);
      return new Result(r.get(ValueLayout.JAVA_INT, OFF_RES_END), r.get(ValueLayout.JAVA_INT, OFF_RES_TERMINAL_DEPTH),
          r.get(ValueLayout.JAVA_INT, OFF_RES_PRED_INDEX), r.get(ValueLayout.JAVA_INT, OFF_RES_MAX_DEPTH),
          r.get(ValueLayout.JAVA_LONG, OFF_RES_STATES), pd, tr, st, r.get(ValueLayout.JAVA_INT, OFF_RES_INITIAL_DEPTH),
          r.get(ValueLayout.JAVA_DOUBLE, OFF_RES_ELAPSED), r.get(ValueLayout.JAVA_LONG, OFF_RES_CHECKS_RUN),
          r.get(ValueLayout.JAVA_LONG, OFF_RES_NOT_DETERMINISTIC), r.get(ValueLayout.JAVA_LONG, OFF_RES_NOT_IDEMPOTENT));
    }
  }
}
