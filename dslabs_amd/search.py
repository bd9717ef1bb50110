"""Host-side mirror of the reference's search API, running the MI355X engine.

Mirrors (names, argument meaning, error behaviour) of, relative to
/root/reference/framework/tst/dslabs/framework/testing:
  * search/Search.java:390-395            ``Search.bfs(initialState, settings)``
  * search/SearchSettings.java:43-199     ``SearchSettings`` (maxDepth, addGoal/addPrune, ...)
  * TestSettings.java:46-245              invariants, maxTimeSecs, link/sender/receiver filters,
                                          partition, deliverTimers
  * search/SearchResults.java:34-88       ``SearchResults`` / ``EndCondition``
  * StatePredicate.java:52-83, :382-396   standard predicates and ``negate()``

Every search runs on the GPU through libdslabs_hip.so; there is no CPU fallback.
Method names keep the reference's camelCase so that tests read like the reference's tests.
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

from . import _lib
from ._lib import check


class EndCondition(enum.IntEnum):
    EXCEPTION_THROWN = 0
    INVARIANT_VIOLATED = 1
    GOAL_FOUND = 2
    SPACE_EXHAUSTED = 3
    TIME_EXHAUSTED = 4


# dsl_predicate_id
PRED_RESULTS_OK = 1
PRED_CLIENTS_DONE = 2
PRED_CLIENT_DONE = 3
PRED_NONE_DECIDED = 4
PRED_CLIENT_HAS_RESULTS = 5


# combinators (dsl_predicate_id DSL_PRED_AND / _OR / _IMPLIES)
PRED_AND = 900
PRED_OR = 901
PRED_IMPLIES = 902


class StatePredicate:
    """A named state predicate evaluated on the device (StatePredicate.java).

    ``address_args`` names the positional args that are node addresses; they are resolved
    to node indices against the search state's address table when the search starts.
    Combinators follow StatePredicate.and / or / implies (StatePredicate.java:397-431); ``and``
    and ``or`` are Python keywords, so they are spelled ``and_`` / ``or_`` here.
    """

    def __init__(self, name: str, pred_id: int, arg0=0, arg1=0, negated: bool = False,
                 address_args: Sequence[int] = (), operands: Sequence["StatePredicate"] = ()):
        self.name = name
        self.pred_id = pred_id
        self.arg0 = arg0
        self.arg1 = arg1
        self.negated = negated
        self.address_args = tuple(address_args)
        self.operands = tuple(operands)

    def negate(self) -> "StatePredicate":
        # StatePredicate.negate(): "¬(name)" or strip an existing "¬(...)".
        if self.name.startswith("¬(") and self.name.endswith(")"):
            name = self.name[2:-1]
        else:
            name = f"¬({self.name})"
        return StatePredicate(name, self.pred_id, self.arg0, self.arg1, not self.negated, self.address_args,
                              self.operands)

    def and_(self, other: "StatePredicate") -> "StatePredicate":
        return StatePredicate(f"({self.name}) ∧ ({other.name})", PRED_AND, operands=(self, other))

    def or_(self, other: "StatePredicate") -> "StatePredicate":
        return StatePredicate(f"({self.name}) ∨ ({other.name})", PRED_OR, operands=(self, other))

    def implies(self, other: "StatePredicate") -> "StatePredicate":
        return StatePredicate(f"({self.name}) → ({other.name})", PRED_IMPLIES, operands=(self, other))

    def _encode(self, state: "SearchState", pool: list) -> _lib.dsl_predicate:
        """The C ABI form; a combinator's operands are appended to ``pool`` (dsl_settings.pool)."""
        if self.operands:
            idx = []
            for op in self.operands:
                pool.append(op._encode(state, pool))
                idx.append(len(pool) - 1)
            return _lib.dsl_predicate(self.pred_id, 1 if self.negated else 0, idx[0], idx[1])
        args = [self.arg0, self.arg1]
        for i in self.address_args:
            args[i] = state.protocol.address_index(args[i])
        return _lib.dsl_predicate(self.pred_id, 1 if self.negated else 0, int(args[0]), int(args[1]))

    def __repr__(self) -> str:
        return self.name


RESULTS_OK = StatePredicate("Clients got expected results", PRED_RESULTS_OK)
CLIENTS_DONE = StatePredicate("All clients' workloads finished", PRED_CLIENTS_DONE)
NONE_DECIDED = StatePredicate("No results returned", PRED_NONE_DECIDED)


def clientDone(address: str) -> StatePredicate:
    return StatePredicate(f"{address}'s workload finished", PRED_CLIENT_DONE, address, address_args=(0,))


def clientHasResults(address: str, numResults: int) -> StatePredicate:
    return StatePredicate(f"{address} received {numResults} results", PRED_CLIENT_HAS_RESULTS, address,
                          numResults, address_args=(0,))


@dataclass
class PredicateResult:
    """StatePredicate.PredicateResult: which predicate fired and its value."""
    predicate: StatePredicate
    value: Optional[bool]

    def errorMessage(self) -> str:
        verb = "matches" if self.value else "violates"
        return f'State {verb} "{self.predicate.name}"'


class SearchSettings:
    """SearchSettings + TestSettings (fluent setters return self)."""

    def __init__(self):
        self._invariants: List[StatePredicate] = []
        self._goals: List[StatePredicate] = []
        self._prunes: List[StatePredicate] = []
        self._max_depth = -1
        self._max_time_secs = -1
        self._network_active = True
        self._link = {}
        self._sender = {}
        self._receiver = {}
        self._deliver_timers = True
        self._timers_active = {}
        # engine capacity knobs (dsl_settings): the visited table's first size (2^k slots; 0 = 2^20,
        # it grows), a cap on a level's frontier (0 = none), and the device memory the visited
        # table may grow to (bytes; 0 = no limit)
        self.table_log2_slots = 0
        self.max_frontier_states = 0
        self.memory_budget_bytes = 0
        # GlobalSettings.doErrorChecks / doAllChecks (Search.java:201-220): a sample of every level's
        # new states re-derived on the host (determinism) and, for doAllChecks, message deliveries
        # stepped twice (idempotence); counts in SearchResults.checks
        self.do_checks = _lib.DSL_CHECKS_NONE
        self.check_sample = 0

    def doErrorChecks(self, on: bool = True) -> "SearchSettings":
        self.do_checks = _lib.DSL_CHECKS_ERRORS if on else _lib.DSL_CHECKS_NONE
        return self

    def doAllChecks(self, on: bool = True) -> "SearchSettings":
        self.do_checks = _lib.DSL_CHECKS_ALL if on else _lib.DSL_CHECKS_NONE
        return self

    # TestSettings -------------------------------------------------------------------------
    def addInvariant(self, p: StatePredicate) -> "SearchSettings":
        self._invariants.append(p)
        return self

    def clearInvariants(self) -> "SearchSettings":
        self._invariants.clear()
        return self

    def invariants(self) -> List[StatePredicate]:
        return list(self._invariants)

    def maxTimeSecs(self, secs: int) -> "SearchSettings":
        self._max_time_secs = secs
        return self

    def timeLimited(self) -> bool:
        return self._max_time_secs > 0

    def linkActive(self, frm: str, to: str, active: bool) -> "SearchSettings":
        self._link[(frm, to)] = active
        return self

    def senderActive(self, frm: str, active: bool) -> "SearchSettings":
        self._sender[frm] = active
        return self

    def receiverActive(self, to: str, active: bool) -> "SearchSettings":
        self._receiver[to] = active
        return self

    def nodeActive(self, node: str, active: bool) -> "SearchSettings":
        self.receiverActive(node, active)
        return self.senderActive(node, active)

    def networkActive(self, active: bool) -> "SearchSettings":
        self._network_active = active
        return self

    def partition(self, *groups) -> "SearchSettings":
        """TestSettings.partition: network off, links inside each group on.
        Accepts addresses (one group) or sequences of addresses (several groups)."""
        if groups and isinstance(groups[0], str):
            groups = (groups,)
        self._network_active = False
        for g in groups:
            for a in g:
                for b in g:
                    if a != b:
                        self._link[(a, b)] = True
        return self

    def reconnect(self) -> "SearchSettings":
        self._network_active = True
        self._link.clear()
        self._sender.clear()
        self._receiver.clear()
        return self

    def deliverTimers(self, *args) -> "SearchSettings":
        if len(args) == 1:
            self._deliver_timers = bool(args[0])
        else:
            self._timers_active[args[0]] = bool(args[1])
        return self

    def clearDeliverTimers(self) -> "SearchSettings":
        self._deliver_timers = True
        self._timers_active.clear()
        return self

    # SearchSettings ------------------------------------------------------------------------
    def maxDepth(self, depth: int) -> "SearchSettings":
        self._max_depth = depth
        return self

    def depthLimited(self) -> bool:
        return self._max_depth >= 0

    def addGoal(self, p: StatePredicate) -> "SearchSettings":
        self._goals.append(p)
        return self

    def clearGoals(self) -> "SearchSettings":
        self._goals.clear()
        return self

    def goals(self) -> List[StatePredicate]:
        return list(self._goals)

    def addPrune(self, p: StatePredicate) -> "SearchSettings":
        self._prunes.append(p)
        return self

    def clearPrunes(self) -> "SearchSettings":
        self._prunes.clear()
        return self

    def prunes(self) -> List[StatePredicate]:
        return list(self._prunes)

    def clone(self) -> "SearchSettings":
        s = SearchSettings()
        s.__dict__.update({k: (v.copy() if isinstance(v, (list, dict)) else v) for k, v in self.__dict__.items()
                           if k != "_enc_cache"})
        return s

    # encoding -------------------------------------------------------------------------------
    def _signature(self, state: "SearchState") -> tuple:
        """Everything _encode reads (predicates and protocols by identity: they are immutable)."""
        return (state.protocol, self._max_depth, self._max_time_secs, self._network_active, self._deliver_timers,
                tuple(self._link.items()), tuple(self._sender.items()), tuple(self._receiver.items()),
                tuple(self._timers_active.items()), tuple(self._invariants), tuple(self._goals), tuple(self._prunes),
                self.table_log2_slots, self.max_frontier_states, self.memory_budget_bytes, self.do_checks,
                self.check_sample)

    def _encode(self, state: "SearchState") -> _lib.dsl_settings:
        """The C ABI form (dsl_settings); the same object again while nothing it reads changed,
        so a repeated search skips the encoding and the engine skips dsl_set_settings."""
        sig = self._signature(state)
        cached = self.__dict__.get("_enc_cache")
        if cached is not None and cached[0] == sig:
            return cached[1]
        s = self._encode_new(state)
        self.__dict__["_enc_cache"] = (sig, s)
        return s

    def _encode_new(self, state: "SearchState") -> _lib.dsl_settings:
        proto = state.protocol
        s = _lib.dsl_settings()
        s.max_depth = self._max_depth
        s.max_time_ms = max(1, int(round(self._max_time_secs * 1000))) if self._max_time_secs > 0 else -1
        s.network_active = 1 if self._network_active else 0
        s.deliver_timers = 1 if self._deliver_timers else 0
        ctypes.memset(ctypes.addressof(s.link_active), 0xFF, ctypes.sizeof(s.link_active))
        ctypes.memset(ctypes.addressof(s.sender_active), 0xFF, ctypes.sizeof(s.sender_active))
        ctypes.memset(ctypes.addressof(s.receiver_active), 0xFF, ctypes.sizeof(s.receiver_active))
        ctypes.memset(ctypes.addressof(s.timers_active), 0xFF, ctypes.sizeof(s.timers_active))
        for (a, b), v in self._link.items():
            s.link_active[proto.address_index(a)][proto.address_index(b)] = 1 if v else 0
        for a, v in self._sender.items():
            s.sender_active[proto.address_index(a)] = 1 if v else 0
        for a, v in self._receiver.items():
            s.receiver_active[proto.address_index(a)] = 1 if v else 0
        for a, v in self._timers_active.items():
            s.timers_active[proto.address_index(a)] = 1 if v else 0
        pool = []
        for name, lst, arr in (("n_invariants", self._invariants, s.invariants),
                               ("n_goals", self._goals, s.goals), ("n_prunes", self._prunes, s.prunes)):
            if len(lst) > _lib.DSL_MAX_PREDICATES:
                raise ValueError("too many predicates")
            setattr(s, name, len(lst))
            for i, p in enumerate(lst):
                arr[i] = p._encode(state, pool)
        if len(pool) > _lib.DSL_MAX_POOL:
            raise ValueError("too many combinator operands")
        s.n_pool = len(pool)
        for i, p in enumerate(pool):
            s.pool[i] = p
        s.table_log2_slots = self.table_log2_slots
        s.max_frontier_states = self.max_frontier_states
        s.memory_budget_bytes = self.memory_budget_bytes
        s.do_checks = self.do_checks
        s.check_sample = self.check_sample
        return s


class SearchState:
    """A search state handle: the protocol configuration plus (optionally) a packed state.

    ``SearchState`` objects for the initial state are made by the protocol builders in
    ``dslabs_amd.protocols``; terminal states come back from a search with their event trace
    (``trace()``), the analogue of the reference's ``previous`` chain.
    """

    DROPPED_CAP = 4096

    def __init__(self, protocol, packed: Optional[bytes] = None, depth: int = 0,
                 events: Optional[List[str]] = None, raw_events=None, dropped=None):
        self.protocol = protocol
        self.packed = packed
        self._depth = depth
        self._events = events or []
        self._raw_events = raw_events or []
        # SearchState.droppedNetwork (SearchState.java:77): records set aside by
        # dropPendingMessages; successors found by a search from this state inherit the set
        self._dropped = list(dropped or [])

    # ---- dropped network (SearchState.java:538-561) ----------------------------------------------
    def _packed_now(self) -> bytes:
        if self.packed is not None:
            return self.packed
        lib = _lib.load()
        desc = self.protocol.desc()
        n = lib.dsl_state_bytes(ctypes.byref(desc))
        check(n if n < 0 else 0, "dsl_state_bytes")
        buf = (ctypes.c_uint8 * n)()
        check(lib.dsl_init_state(ctypes.byref(desc), buf, n), "dsl_init_state")
        return bytes(buf)

    def dropPendingMessages(self) -> None:
        """Every pending message moves to the dropped set: no longer an event, still part of the
        state's message union (SearchState.dropPendingMessages, :538-541). Mutates this state."""
        lib = _lib.load()
        packed = self._packed_now()
        buf = (ctypes.c_uint8 * len(packed)).from_buffer_copy(packed)
        arr = (ctypes.c_uint64 * self.DROPPED_CAP)(*self._dropped)
        n = ctypes.c_int32(len(self._dropped))
        check(lib.dsl_drop_pending_messages(ctypes.byref(self.protocol.desc()), buf, len(packed), arr,
                                            self.DROPPED_CAP, ctypes.byref(n)), "dsl_drop_pending_messages")
        self.packed = bytes(buf)
        self._dropped = list(arr[:n.value])

    def _undrop(self, frm: int, to: int) -> None:
        lib = _lib.load()
        packed = self._packed_now()
        buf = (ctypes.c_uint8 * len(packed)).from_buffer_copy(packed)
        arr = (ctypes.c_uint64 * max(1, len(self._dropped)))(*self._dropped)
        check(lib.dsl_undrop_messages(ctypes.byref(self.protocol.desc()), buf, len(packed), arr,
                                      len(self._dropped), frm, to), "dsl_undrop_messages")
        self.packed = bytes(buf)

    def undropMessages(self) -> None:
        """SearchState.undropMessages (:543-545): every dropped message is pending again."""
        self._undrop(-1, -1)

    def undropMessagesFrom(self, address: str) -> None:
        """SearchState.undropMessagesFrom (:547-553)."""
        self._undrop(self.protocol.address_index(address), -1)

    def undropMessagesTo(self, address: str) -> None:
        """SearchState.undropMessagesTo (:555-561)."""
        self._undrop(-1, self.protocol.address_index(address))

    def droppedMessages(self) -> List[int]:
        """The dropped set as packed records (sorted)."""
        return list(self._dropped)

    def depth(self) -> int:
        return self._depth

    def trace(self) -> List[str]:
        """Events from the search's initial state to this state (SearchState.trace())."""
        return list(self._events)

    def events(self) -> list:
        """The trace as decoded events (dsl_event copies) from the state the search started at:
        the input of ``Engine.replay`` / ``Search.replay``."""
        return list(self._raw_events)

    def addresses(self) -> List[str]:
        return list(self.protocol.addresses)


class SearchResults:
    def __init__(self, end, states, per_depth, initial_depth, max_depth, terminal: Optional[SearchState],
                 predicate: Optional[PredicateResult], elapsed_s: float, successors: int):
        self._end = end
        self.states = states
        self.per_depth = per_depth
        self.initial_depth = initial_depth
        self.max_depth = max_depth
        self._terminal = terminal
        self._predicate = predicate
        self.elapsed_s = elapsed_s
        self.successors = successors
        self.checks = {"run": 0, "not_deterministic": 0, "not_idempotent": 0, "first_not_deterministic": None,
                       "first_not_idempotent": None}

    def endCondition(self) -> EndCondition:
        return self._end

    def lastState(self) -> Optional[SearchState]:
        """The state a replay ended in (TraceReplaySearch: also when the trace ran out or an event
        could not be delivered); for a search, its terminal state."""
        return getattr(self, "_last", None) or self._terminal

    def invariantViolatingState(self) -> Optional[SearchState]:
        return self._terminal if self._end == EndCondition.INVARIANT_VIOLATED else None

    def invariantViolated(self) -> Optional[PredicateResult]:
        return self._predicate if self._end == EndCondition.INVARIANT_VIOLATED else None

    def goalMatchingState(self) -> Optional[SearchState]:
        return self._terminal if self._end == EndCondition.GOAL_FOUND else None

    def goalMatched(self) -> Optional[PredicateResult]:
        return self._predicate if self._end == EndCondition.GOAL_FOUND else None

    def exceptionalState(self) -> Optional[SearchState]:
        return self._terminal if self._end == EndCondition.EXCEPTION_THROWN else None

    def exceptionThrown(self) -> bool:
        return self._end == EndCondition.EXCEPTION_THROWN

    def statesPerSecond(self) -> float:
        return self.states / self.elapsed_s if self.elapsed_s > 0 else float("inf")

    def status(self) -> str:
        # BFS.status() line (Search.java:426-431)
        return "Explored: %d, Depth: %d (%.2fs, %.2fK states/s)" % (
            self.states, self.max_depth, self.elapsed_s, self.statesPerSecond() / 1000.0)


class Engine:
    """One engine (one GPU, or one shard of a multi-GPU search)."""

    def __init__(self, protocol, device: int = -1, rank: int = 0, world_size: int = 1,
                 virtual_shards: int = 0, comm_id: Optional[bytes] = None, host_comm=None,
                 replicate_below: int = -1, rccl_at_world_1: bool = False):
        """rccl_at_world_1: build the RCCL communicator (comm_id) even at world_size 1
        (DSL_CFG_RCCL_AT_WORLD_1), so the collectives run on a one-GPU box."""
        lib = _lib.load()
        self.lib = lib
        self.protocol = protocol
        self.host_comm = host_comm  # keeps the ctypes callbacks alive
        cfg = _lib.dsl_engine_config()
        cfg.device = device
        cfg.rank = rank
        cfg.world_size = world_size
        cfg.virtual_shards = virtual_shards
        cfg.replicate_below = replicate_below
        cfg.flags = _lib.DSL_CFG_RCCL_AT_WORLD_1 if rccl_at_world_1 else 0
        if comm_id is not None:
            ctypes.memmove(cfg.comm_id, comm_id, 128)
        handle = ctypes.c_void_p()
        if host_comm is not None:
            rc = lib.dsl_create_with_host_comm(ctypes.byref(protocol.desc()), ctypes.byref(cfg),
                                               ctypes.byref(host_comm.struct), ctypes.byref(handle))
            check(rc, "dsl_create_with_host_comm")
        else:
            check(lib.dsl_create(ctypes.byref(protocol.desc()), ctypes.byref(cfg), ctypes.byref(handle)),
                  "dsl_create")
        self.handle = handle

    def close(self):
        if self.handle:
            self.lib.dsl_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def state_bytes(self) -> int:
        return self.lib.dsl_state_bytes(ctypes.byref(self.protocol.desc()))

    def initial_packed(self) -> bytes:
        n = self.state_bytes()
        buf = (ctypes.c_uint8 * n)()
        check(self.lib.dsl_get_initial(self.handle, buf, n), "dsl_get_initial")
        return bytes(buf)

    def kernel_stats(self) -> dict:
        st = _lib.dsl_stats()
        check(self.lib.dsl_kernel_stats(self.handle, ctypes.byref(st)), "dsl_kernel_stats")
        return {name: getattr(st, name) for name, _ in st._fields_}

    def _prepare(self, state: SearchState, settings: SearchSettings):
        lib = self.lib
        enc = settings._encode(state)
        if enc is not getattr(self, "_set_enc", None):  # the engine keeps the settings it was given
            check(lib.dsl_set_settings(self.handle, ctypes.byref(enc)), "dsl_set_settings")
            self._set_enc = enc
            self._set_dropped = None  # dsl_set_settings re-applies the dropped set the engine holds
        if state.packed is not None:
            buf = (ctypes.c_uint8 * len(state.packed)).from_buffer_copy(state.packed)
            check(lib.dsl_set_initial(self.handle, buf, len(state.packed), state.depth()), "dsl_set_initial")
        # the dropped network: part of network() for network predicates (SearchState.java:153-157)
        dr = tuple(state._dropped)
        if dr != getattr(self, "_set_dropped", None):
            arr = (ctypes.c_uint64 * max(1, len(dr)))(*dr)
            check(lib.dsl_set_dropped(self.handle, arr, len(dr)), "dsl_set_dropped")
            self._set_dropped = dr

    def bfs(self, state: SearchState, settings: Optional[SearchSettings] = None) -> SearchResults:
        if settings is None:
            settings = SearchSettings()
        self._prepare(state, settings)
        res_p = ctypes.POINTER(_lib.dsl_result)()
        check(self.lib.dsl_run(self.handle, ctypes.byref(res_p)), "dsl_run")
        return self._results(state, settings, res_p)

    def dfs(self, state: SearchState, settings: Optional[SearchSettings] = None, probes: int = 65536,
            seed: int = 0, max_probes: int = 0, minimize: bool = True, max_trace: int = 0) -> SearchResults:
        """Search.dfs / RandomDFS (Search.java:397-402, :507-583) on the device: `probes` random
        walks at once until a terminal state, settings.maxTimeSecs, or `max_probes` probes. The
        terminal's trace is minimized as RandomDFS does (TraceMinimizer) unless minimize=False."""
        if settings is None:
            settings = SearchSettings()
        self._prepare(state, settings)
        c = _lib.dsl_dfs_config(probes, seed & ((1 << 64) - 1), max_probes, 0, max_trace, 0 if minimize else 1, 0)
        res_p = ctypes.POINTER(_lib.dsl_result)()
        check(self.lib.dsl_run_dfs(self.handle, ctypes.byref(c), ctypes.byref(res_p)), "dsl_run_dfs")
        return self._results(state, settings, res_p)

    def replay(self, state: SearchState, settings: Optional[SearchSettings], events,
               minimize: bool = True) -> SearchResults:
        """TraceReplaySearch (T/junit/TraceReplaySearch.java:76-101): replays `events` (dsl_event
        list, e.g. ``SearchState.events()`` of an earlier result from the same start state) with
        checkState after every step; a terminal is minimized (TraceMinimizer) when `minimize`. An
        event that cannot be delivered, or the end of the trace, ends with SPACE_EXHAUSTED."""
        if settings is None:
            settings = SearchSettings()
        self._prepare(state, settings)
        arr = (_lib.dsl_event * max(1, len(events)))()
        for i, e in enumerate(events):
            ctypes.memmove(ctypes.byref(arr[i]), ctypes.byref(e), ctypes.sizeof(_lib.dsl_event))
        res_p = ctypes.POINTER(_lib.dsl_result)()
        check(self.lib.dsl_replay(self.handle, arr, len(events), 1 if minimize else 0, ctypes.byref(res_p)),
              "dsl_replay")
        return self._results(state, settings, res_p)

    def human_readable_trace(self, state: SearchState, settings: Optional[SearchSettings], events) -> SearchState:
        """SearchState.humanReadableTraceEndState (SearchState.java:373-470): the state reached by
        `events` from `state`, whose trace() is the causally reordered, no-op-free trace."""
        if settings is None:
            settings = SearchSettings()
        self._prepare(state, settings)
        arr = (_lib.dsl_event * max(1, len(events)))()
        for i, e in enumerate(events):
            ctypes.memmove(ctypes.byref(arr[i]), ctypes.byref(e), ctypes.sizeof(_lib.dsl_event))
        res_p = ctypes.POINTER(_lib.dsl_result)()
        check(self.lib.dsl_human_readable_trace(self.handle, arr, len(events), ctypes.byref(res_p)),
              "dsl_human_readable_trace")
        try:
            r = res_p.contents
            raw = [r.trace[i] for i in range(r.trace_len)]
            packed = bytes(ctypes.cast(r.terminal_state, ctypes.POINTER(ctypes.c_uint8 * r.state_bytes)).contents)
            return SearchState(self.protocol, packed, r.terminal_depth, [self.protocol.render_event(e) for e in raw],
                               [_lib.dsl_event.from_buffer_copy(e) for e in raw], state._dropped)
        finally:
            self.lib.dsl_result_free(res_p)

    def _results(self, state: SearchState, settings: SearchSettings, res_p) -> SearchResults:
        lib = self.lib
        try:
            r = res_p.contents
            per_depth = [r.per_depth[i] for i in range(r.n_levels)]
            end = EndCondition(r.end_condition)
            terminal = None
            last = None
            pred = None
            if r.terminal_state:
                raw = [r.trace[i] for i in range(r.trace_len)]
                events = [self.protocol.render_event(e) for e in raw]
                packed = bytes(ctypes.cast(r.terminal_state, ctypes.POINTER(ctypes.c_uint8 * r.state_bytes)).contents)
                base_events = state.trace() if state.packed is not None else []
                last = SearchState(self.protocol, packed, r.terminal_depth if r.terminal_depth >= 0 else r.max_depth,
                                   base_events + events, [_lib.dsl_event.from_buffer_copy(e) for e in raw],
                                   state._dropped)
                if r.terminal_depth >= 0:
                    terminal = last
                if end == EndCondition.INVARIANT_VIOLATED:
                    pred = PredicateResult(settings.invariants()[r.predicate_index], False)
                elif end == EndCondition.GOAL_FOUND:
                    pred = PredicateResult(settings.goals()[r.predicate_index], True)
            res = SearchResults(end, r.states, per_depth, r.initial_depth, r.max_depth, terminal, pred,
                                r.elapsed_s, r.successors)
            res._last = last
            # CheckLogger.notDeterministic / notIdempotent (T/utils/CheckLogger.java:104-121)
            res.checks = {"run": r.checks_run, "not_deterministic": r.not_deterministic,
                          "not_idempotent": r.not_idempotent,
                          "first_not_deterministic": self.protocol.render_event(r.first_not_deterministic)
                          if r.not_deterministic else None,
                          "first_not_idempotent": self.protocol.render_event(r.first_not_idempotent)
                          if r.not_idempotent else None}
            return res
        finally:
            lib.dsl_result_free(res_p)


class Search:
    @staticmethod
    def bfs(initialState: SearchState, settings: Optional[SearchSettings] = None, device: int = -1) -> SearchResults:
        """Search.bfs (Search.java:390-395) on the MI355X engine."""
        eng = Engine(initialState.protocol, device=device)
        try:
            return eng.bfs(initialState, settings)
        finally:
            eng.close()

    @staticmethod
    def replay(initialState: SearchState, settings: Optional[SearchSettings], events, minimize: bool = True,
               device: int = -1) -> SearchResults:
        """TraceReplaySearch on the MI355X engine's transitions (host side, see Engine.replay)."""
        eng = Engine(initialState.protocol, device=device)
        try:
            return eng.replay(initialState, settings, events, minimize)
        finally:
            eng.close()

    @staticmethod
    def dfs(initialState: SearchState, settings: Optional[SearchSettings] = None, device: int = -1,
            **kw) -> SearchResults:
        """Search.dfs (Search.java:397-402): random depth-first probes on the MI355X engine."""
        eng = Engine(initialState.protocol, device=device)
        try:
            return eng.dfs(initialState, settings, **kw)
        finally:
            eng.close()
