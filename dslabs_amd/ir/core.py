"""Protocol IR: a small declarative description of a DSLabs protocol -- node kinds and their fields,
message and timer records, handlers as statement lists -- from which both forms the engine needs
are generated (dslabs_amd/ir/gen_device.py: the packed device protocol for csrc/protocols/;
gen_oracle.py: the object form on the oracle's Node / Ctx / TimerQueue model). The reference
dispatches to handlers by name over Java objects (framework/src/dslabs/framework/Node.java:479-562);
here a handler is a Python function run once at generation time against a recorder, so its
statements become C++ for both targets, and one description is the single source of both.

Scope: integer fields of fixed bit width, bounded lists, messages / timers with integer fields,
sends, timer sets (TimerQueue semantics with static (min, max) per timer type), conditionals and
exceptions; client nodes run inside the reference's ClientWorker command loop (ClientWorker.java:
174-251) with the workload "command k = k" (1-based) and expected results given by an expression
of k. Values are plain integers (interned by the spec author); 0 means null.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple


# ---- expressions -------------------------------------------------------------------------------
class Expr:
    """An integer / boolean expression with its C++ text for the device and the oracle."""

    def __init__(self, dev: str, orc: str):
        self.dev, self.orc = dev, orc

    def _bin(self, o, op):
        o = lit(o)
        return Expr(f"({self.dev} {op} {o.dev})", f"({self.orc} {op} {o.orc})")

    def _rbin(self, o, op):
        return lit(o)._bin(self, op)

    __add__ = lambda s, o: s._bin(o, "+")
    __radd__ = lambda s, o: s._rbin(o, "+")
    __sub__ = lambda s, o: s._bin(o, "-")
    __rsub__ = lambda s, o: s._rbin(o, "-")
    __mul__ = lambda s, o: s._bin(o, "*")
    __eq__ = lambda s, o: s._bin(o, "==")
    __ne__ = lambda s, o: s._bin(o, "!=")
    __lt__ = lambda s, o: s._bin(o, "<")
    __le__ = lambda s, o: s._bin(o, "<=")
    __gt__ = lambda s, o: s._bin(o, ">")
    __ge__ = lambda s, o: s._bin(o, ">=")
    __and__ = lambda s, o: s._bin(o, "&&")
    __or__ = lambda s, o: s._bin(o, "||")

    def __invert__(self):
        return Expr(f"(!{self.dev})", f"(!{self.orc})")

    # bit operations (integers): explicit names, since & and | are the logical connectives
    def shl(self, n):
        return self._bin(n, "<<")

    def shr(self, n):
        return self._bin(n, ">>")

    def band(self, m):
        return self._bin(m, "&")

    def bor(self, m):
        return self._bin(m, "|")

    def __hash__(self):
        return id(self)

    def __bool__(self):
        raise TypeError("IR expressions are symbolic: use h.if_(...) instead of a Python if")


def lit(v) -> Expr:
    if isinstance(v, Expr):
        return v
    if isinstance(v, bool):
        v = int(v)
    return Expr(str(int(v)), str(int(v)))


def select(c, a, b) -> Expr:
    c, a, b = lit(c), lit(a), lit(b)
    return Expr(f"({c.dev} ? {a.dev} : {b.dev})", f"({c.orc} ? {a.orc} : {b.orc})")


# ---- declarations ------------------------------------------------------------------------------
@dataclass
class Param:
    name: str
    default: int
    lo: int
    hi: int


@dataclass
class ParamTable:
    """A per-(row, column) parameter table, e.g. a workload's command table by (client, command).
    A table of small non-negative entries is also packed into one 64-bit word at from_desc time
    (the device reads an entry with a shift, not a select chain over the table)."""
    name: str
    rows: int
    cols: int
    lo: int
    hi: int
    default: int = 0

    def packed_bits(self) -> int:
        """Bits per entry of the packed form, 0 if the table does not pack."""
        if self.lo < 0 or self.default < 0:
            return 0
        b = max(1, int(self.hi).bit_length())
        return b if b * self.rows * self.cols <= 64 else 0


@dataclass
class RecordType:
    """A message or timer type: integer fields of fixed widths, in declaration order."""
    name: str
    fields: List[Tuple[str, int]]
    index: int = 0
    millis: Tuple[int, int] = (0, 0)  # timers: (min, max)


@dataclass
class FieldDecl:
    name: str
    bits: int
    cap: int = 0  # > 0: a bounded list of `cap` elements of `bits` each, with a length
    array: bool = False  # with cap: a fixed-size array (no length), indexed by h.at / h.set_at
    off: int = 0
    len_off: int = 0
    len_bits: int = 0
    per: int = 1  # list / array elements per 32-bit word

    def window_words(self) -> int:
        """Words an array occupies (a 32- or 64-bit window is read with shifts, no select chain)."""
        return (self.cap + self.per - 1) // self.per

    def elem_rel(self, j: str) -> str:
        """Bit offset of element j inside the array's window."""
        if self.per == 1:
            return f"32 * ({j})"
        if 32 % self.bits == 0:
            return f"{self.bits} * ({j})"
        return f"({j}) / {self.per} * 32 + ({j}) % {self.per} * {self.bits}"

    def elem(self, j: str) -> str:
        """C++ bit offset of element j (an index expression)."""
        if self.per == 1:
            return f"{self.off} + 32 * ({j})"
        if 32 % self.bits == 0:
            return f"{self.off} + {self.bits} * ({j})"
        return f"{self.off} + ({j}) / {self.per} * 32 + ({j}) % {self.per} * {self.bits}"


@dataclass
class PredDecl:
    """A protocol state predicate (StatePredicate): `ids` are the engine's DSL_PRED_* ids it
    answers (include/dslabs_hip.h), `names` the oracle CLI names, `full` the reference's
    description; `reads` maps each node kind it reads to the fields it reads (the kernels'
    incremental judge keeps the parent's value when none of those words changed). `nargs`
    integer arguments (dsl_predicate arg0 / arg1; the oracle CLI name NAME:a0[:a1]) are read with
    q.arg(i). A predicate that reads the network (q.any_msg) declares network=True: it is
    re-evaluated for every new state (its read set is everything)."""
    ids: List[int]
    names: List[str]
    full: str
    reads: Dict[str, List[str]]
    fn: Callable
    nargs: int = 0
    network: bool = False


@dataclass
class NodeKind:
    name: str                      # address prefix ("client" -> client1, client2, ...)
    count: object                  # int, or the name of a Param
    max_count: int
    fields: List[FieldDecl] = field(default_factory=list)
    client: bool = False           # runs inside ClientWorker
    single_name: Optional[str] = None  # address of a one-instance kind ("pingserver")
    result_field: str = ""         # client: the field holding the current result (0 = none)
    timer_cap: int = 0
    results_cap: int = 0
    handlers: Dict[str, Callable] = field(default_factory=dict)   # message name -> fn(h)
    timer_handlers: Dict[str, Callable] = field(default_factory=dict)
    init_fn: Optional[Callable] = None
    send_command_fn: Optional[Callable] = None
    noop_fns: Dict[str, Callable] = field(default_factory=dict)  # message name -> fn(h) -> Expr
    tail_fn: Optional[Callable] = None  # common tail of the message handlers (see tail())
    flags: List[str] = field(default_factory=list)
    first: int = 0                 # node index of the first instance (at the maximum counts)
    # a timer queue that is [T] in every reachable state (Protocol.fixed_timer): the device form
    # keeps no queue for it (one deliverable timer, re-armed by its own handler)
    fixed_timer: Optional["RecordType"] = None

    def on(self, msg: RecordType):
        def deco(fn):
            self.handlers[msg.name] = fn
            return fn
        return deco

    def on_timer(self, t: RecordType):
        def deco(fn):
            self.timer_handlers[t.name] = fn
            return fn
        return deco

    def init(self, fn):
        self.init_fn = fn
        return fn

    def send_command(self, fn):
        self.send_command_fn = fn
        return fn

    def tail(self, fn):
        """A common tail run after any message handler of this kind that raised a flag
        (h.flag(name); the tail reads them with h.flagged(name)): one copy of shared work -- e.g.
        Multi-Paxos's execute -- instead of one per handler."""
        self.tail_fn = fn
        return fn

    def flag_bit(self, name: str) -> int:
        if name not in self.flags:
            self.flags.append(name)
        return self.flags.index(name)

    def noop(self, msg: RecordType):
        """The no-op filter of a delivery (nodestate.hpp NoopFilter): fn(h) returns a boolean
        Expr over the node's fields and the message that is true only when the handler (and, for a
        client, the ClientWorker loop after it) surely returns with the node unchanged and sends
        nothing. The kernels count such an event as a successor without running it;
        tests/hostcheck checks the implication on every explored event."""
        def deco(fn):
            self.noop_fns[msg.name] = fn
            return fn
        return deco


class Protocol:
    def __init__(self, name: str, proto_id: int, cxx_name: str, doc: str = ""):
        self.name, self.proto_id, self.cxx_name, self.doc = name, proto_id, cxx_name, doc
        self.params: List[Param] = []
        self.tables: List[ParamTable] = []
        self.messages: List[RecordType] = []
        self.timers: List[RecordType] = []
        self.kinds: List[NodeKind] = []
        self.net_cap = 32
        self.max_sends = 4
        # no handler sends one record twice in one step: the device Sender skips its duplicate
        # check (P::kSendsDistinct; tests/hostcheck/protocheck.cpp counts violations)
        self.sends_distinct = False
        self.workload_size = ""       # Param name: commands per client, or fn(h, c) -> Expr (c from 0)
        self.predicates: List[PredDecl] = []
        # (client index c from 0, command k from 1) -> expected result Expr; < 0: not checked
        self.expected_result: Optional[Callable] = None

    # declarations
    def param(self, name: str, default: int, lo: int = 0, hi: int = 1 << 30) -> Param:
        p = Param(name, default, lo, hi)
        self.params.append(p)
        return p

    def message(self, name: str, **fields: int) -> RecordType:
        r = RecordType(name, list(fields.items()), len(self.messages))
        self.messages.append(r)
        return r

    def timer(self, name: str, millis: Tuple[int, int], **fields: int) -> RecordType:
        r = RecordType(name, list(fields.items()), len(self.timers), millis)
        self.timers.append(r)
        return r

    def param_table(self, name: str, rows: int, cols: int, lo: int = -(1 << 30), hi: int = 1 << 30,
                    default: int = 0) -> ParamTable:
        t = ParamTable(name, rows, cols, lo, hi, default)
        self.tables.append(t)
        return t

    def node(self, name: str, count=1, max_count: int = 1, single_name: Optional[str] = None,
             arrays: Optional[Dict[str, Tuple[int, int]]] = None, **fields: int) -> NodeKind:
        """fields: name -> bits; arrays: name -> (bits, size) fixed-size arrays."""
        fl = [FieldDecl(n, b) for n, b in fields.items()]
        fl += [FieldDecl(n, b, cap, array=True) for n, (b, cap) in (arrays or {}).items()]
        k = NodeKind(name, count, max_count, fl, single_name=single_name)
        self.kinds.append(k)
        return k

    def client_worker(self, name: str, count, max_count: int, result_field: str, results_cap: int, timer_cap: int,
                      arrays=None, **fields: int) -> NodeKind:
        k = self.node(name, count, max_count, arrays=arrays, **fields)
        k.client, k.result_field, k.results_cap, k.timer_cap = True, result_field, results_cap, timer_cap
        return k

    def predicate(self, full: str, ids, names, reads: Dict[str, List[str]], nargs: int = 0, network: bool = False):
        """reads: node kind name -> the fields the predicate reads; nargs: integer arguments
        (q.arg(i)); network: it reads the network (q.any_msg), so it has no node read set."""
        def deco(fn):
            self.predicates.append(PredDecl(list(ids), list(names), full, dict(reads), fn, nargs, network))
            return fn
        return deco

    def net_preds(self) -> bool:
        return any(pd.network for pd in self.predicates)

    def kind(self, name: str) -> NodeKind:
        return next(k for k in self.kinds if k.name == name)

    # derived layout ------------------------------------------------------------------------------
    def layout(self):
        """Node indices (kinds in declaration order, instances consecutive), node word layout
        (fields never straddle a 32-bit word), record layout (type, from, to, fields)."""
        idx = 0
        for k in self.kinds:
            k.first = idx
            idx += k.max_count
        self.max_nodes = idx
        if not getattr(self, "_fixed_done", False):  # once per protocol (handlers are recorded on a first layout)
            self._fixed_done = True
            self._place()
            for k in self.kinds:
                k.fixed_timer = self.fixed_timer(k)
        self._place()

    def fixed_timer(self, k: "NodeKind") -> Optional["RecordType"]:
        """T when k's timer queue is [T] in every reachable state: k handles exactly one timer
        type T, which has no fields; its init sets T once, unconditionally; T's handler re-sets T
        as its last top-level statement, sets no other timer and never returns early; no message
        handler (nor the common tail) sets a timer. Then SearchState.stepTimer's remove of the
        delivered entry and the handler's re-set leave [T] as it was, so the device form keeps
        no queue (the oracle form keeps the TimerQueue and checks the claim by parity)."""
        if not k.timer_cap or k.client or len(k.timer_handlers) != 1 or not k.init_fn:
            return None
        tname, fn = next(iter(k.timer_handlers.items()))
        t = next(x for x in self.timers if x.name == tname)
        if t.fields:
            return None

        def walk(ss):
            for st in ss:
                yield st
                if isinstance(st, IfS):
                    yield from walk(st.then)
                    yield from walk(st.other)
                elif isinstance(st, ForS):
                    yield from walk(st.body)

        def sets(ss):
            return [st for st in walk(ss) if isinstance(st, SetTimerS)]

        init = record(self, k, k.init_fn)
        top = [st for st in init if isinstance(st, SetTimerS)]
        if len(sets(init)) != 1 or len(top) != 1 or top[0].timer is not t:
            return None
        hs = record(self, k, fn, event=t, is_timer=True)
        if not hs or not isinstance(hs[-1], SetTimerS) or hs[-1].timer is not t or len(sets(hs)) != 1:
            return None
        if any(isinstance(st, RetS) for st in walk(hs)):
            return None
        for m in self.messages:
            if m.name in k.handlers and sets(record(self, k, k.handlers[m.name], event=m)):
                return None
        if k.tail_fn and sets(record(self, k, k.tail_fn)):
            return None
        return t

    def _place(self):
        words = 1
        for k in self.kinds:
            if k.fixed_timer is not None:
                k.fields = [f for f in k.fields if f.name != "_timers"]
            elif k.timer_cap and not any(f.name == "_timers" for f in k.fields):
                k.fields.append(FieldDecl("_timers", self.timer_entry_bits(), k.timer_cap))
            if k.client and not any(f.name == "_results" for f in k.fields):
                rb = max(f.bits for f in k.fields if f.name == k.result_field)
                k.fields.append(FieldDecl("_results", rb, k.results_cap))
            bit = 0

            def place(width):
                nonlocal bit
                if (bit % 32) + width > 32:
                    bit = (bit // 32 + 1) * 32
                o = bit
                bit += width
                return o

            for f in k.fields:
                if f.cap:
                    if not f.array:
                        f.len_bits = max(1, f.cap.bit_length())
                        f.len_off = place(f.len_bits)
                    assert f.bits <= 32
                    if f.cap * f.bits <= 32 - bit % 32:
                        # the whole list fits in the rest of the current word: placed inline
                        f.per = f.cap
                        f.off = bit
                        bit += f.cap * f.bits
                    else:
                        # word-aligned; `per` elements per word, none straddling a word
                        f.per = 32 // f.bits
                        bit = (bit + 31) // 32 * 32
                        f.off = bit
                        bit += (f.cap + f.per - 1) // f.per * 32
                else:
                    f.off = place(f.bits)
            words = max(words, (bit + 31) // 32)
        self.node_words = words
        # records
        self.type_bits = max(1, (len(self.messages) - 1).bit_length())
        self.addr_bits = max(1, (self.max_nodes - 1).bit_length())
        width = self.type_bits + 2 * self.addr_bits + max(sum(b for _, b in m.fields) for m in self.messages)
        self.rec_bits = 32 if width <= 32 else 64
        assert width <= 64, "records wider than 64 bits"
        for m in self.messages:
            off, offs = 0, []
            for n, b in m.fields:
                offs.append((n, b, off))
                off += b
            m.offs = offs
        self.type_off = self.rec_bits - self.type_bits
        self.from_off = self.type_off - self.addr_bits
        self.to_off = self.from_off - self.addr_bits

    def timer_entry_bits(self) -> int:
        tb = max(1, (len(self.timers) - 1).bit_length()) if len(self.timers) > 1 else 0
        fb = max([sum(b for _, b in t.fields) for t in self.timers] + [0])
        return tb + fb

    def address_names(self, args: Dict[str, int]) -> List[str]:
        out = []
        for k in self.kinds:
            n = self.count_of(k, args)
            if k.single_name and k.max_count == 1:
                out.append(k.single_name)
            else:
                out += [f"{k.name}{i}" for i in range(1, n + 1)]
        return out

    def count_of(self, k: NodeKind, args: Dict[str, int]) -> int:
        return k.count if isinstance(k.count, int) else int(args[k.count])


# ---- handler recorder ---------------------------------------------------------------------------
class Stmt:
    pass


@dataclass
class Assign(Stmt):
    fld: FieldDecl
    value: Expr


@dataclass
class SendS(Stmt):
    msg: RecordType
    to: Expr
    vals: List[Expr]


@dataclass
class SetTimerS(Stmt):
    timer: RecordType
    vals: List[Expr]


@dataclass
class IfS(Stmt):
    cond: Expr
    then: List[Stmt]
    other: List[Stmt]


@dataclass
class ThrowS(Stmt):
    what: str


@dataclass
class LetS(Stmt):
    name: str
    value: Expr


@dataclass
class VarS(Stmt):
    name: str
    value: Expr
    mutable: bool = True


@dataclass
class SetVarS(Stmt):
    name: str
    value: Expr


@dataclass
class SetAtS(Stmt):
    fld: FieldDecl
    index: Expr
    value: Expr


@dataclass
class RetS(Stmt):
    pass


@dataclass
class OverflowS(Stmt):
    what: str


@dataclass
class ForS(Stmt):
    """A rolled loop: `var` from lo while < hi (one copy of the body in the generated code)."""
    var: str
    lo: Expr
    hi: Expr
    body: List[Stmt]


@dataclass
class SetFlagS(Stmt):
    bit: int


@dataclass
class RetPV(Stmt):
    """A predicate's value: "TRUE", "FALSE" or "THREW"."""
    value: str


class _Fields:
    def __init__(self, h):
        object.__setattr__(self, "_h", h)

    def __getattr__(self, name):
        return self._h._field_expr(name)


class _Rec:
    def __init__(self, h, kind):
        self._h, self._kind = h, kind

    def __getattr__(self, name):
        return self._h._rec_field(self._kind, name)


class Handler:
    """What a handler function sees: h.f.<field> (the node's fields), h.msg.<field> /
    h.timer.<field> (the event's fields), h.sender, h.self, h.param(name), and the statements
    h.set(field, value), h.send(Msg, to, **fields), h.set_timer(Timer, **fields),
    `with h.if_(cond):` / `with h.else_():`, h.throw(why)."""

    def __init__(self, proto: Protocol, kind: NodeKind, event: Optional[RecordType] = None, is_timer=False,
                 cmd: Optional[Expr] = None):
        self.p, self.kind, self.event, self.is_timer = proto, kind, event, is_timer
        self.stmts: List[Stmt] = []
        self._stack = [self.stmts]
        self._last_if: Optional[IfS] = None
        self.f = _Fields(self)
        self.msg = _Rec(self, "msg")
        self.timer = _Rec(self, "timer")
        self.cmd = cmd

    # expressions
    def _fd(self, name) -> FieldDecl:
        for f in self.kind.fields:
            if f.name == name:
                return f
        raise KeyError(f"{self.kind.name} has no field {name}")

    def _field_expr(self, name) -> Expr:
        f = self._fd(name)
        assert not f.cap, "lists are read with h.at(field, i)"
        return Expr(f"get(w, {f.off}, {f.bits})", f"{name}")

    def at(self, name, index) -> Expr:
        """Element `index` of an array field."""
        f, i = self._fd(name), lit(index)
        assert f.array
        if f.window_words() <= 2:
            return Expr(f"arr_{self.kind.name}_{name}(w, {i.dev})", f"{name}[{i.orc}]")
        return Expr(f"get(w, {f.elem(i.dev)}, {f.bits})", f"{name}[{i.orc}]")

    def length(self, name) -> Expr:
        """The length of a bounded list field (e.g. a client's harvested results, "_results")."""
        f = self._fd(name)
        assert f.cap and not f.array
        return Expr(f"get(w, {f.len_off}, {f.len_bits})", f"(int){name}.size()")

    def wsize(self) -> Expr:
        """This client's workload size (commands), for no-op filters."""
        return Expr(f"wsize(i - first_{self.kind.name}(p), p)", f"wsize(self - first_{self.kind.name}(prm), prm)")

    def ptab(self, name, r, c) -> Expr:
        """Parameter table entry [r][c]."""
        r, c = lit(r), lit(c)
        t = next(x for x in self.p.tables if x.name == name)
        b = t.packed_bits()
        if b:
            return Expr(f"(int)((p.{name}_pk >> (({b} * (({r.dev}) * {t.cols} + ({c.dev}))) & 63)) & {(1 << b) - 1}u)",
                        f"prm.{name}[{r.orc}][{c.orc}]")
        return Expr(f"sel_param(p.{name}, {r.dev}, {c.dev})", f"prm.{name}[{r.orc}][{c.orc}]")

    def let(self, name: str, value) -> Expr:
        """A named intermediate value (a local constant in both forms)."""
        self._emit(LetS("l_" + name, lit(value)))
        return Expr("l_" + name, "l_" + name)

    def var(self, name: str, init=0) -> Expr:
        """A mutable local (h.assign(name, value) changes it)."""
        self._emit(VarS("l_" + name, lit(init)))
        return Expr("l_" + name, "l_" + name)

    def assign(self, name: str, value):
        self._emit(SetVarS("l_" + name, lit(value)))

    def set_at(self, name: str, index, value):
        f = self._fd(name)
        assert f.array
        self._emit(SetAtS(f, lit(index), lit(value)))

    def ret(self):
        """Return from the handler (the ClientWorker loop still runs for a client)."""
        self._emit(RetS())

    def flag(self, name: str):
        """Raise a flag of the kind's common tail (NodeKind.tail)."""
        self._emit(SetFlagS(self.kind.flag_bit(name)))

    def flagged(self, name: str) -> Expr:
        b = self.kind.flag_bit(name)
        return Expr(f"((fl >> {b}) & 1)", f"((fl_ >> {b}) & 1)")

    def overflow(self, what: str):
        """A bounded container of the packed form is full: a hard error on the device
        (DSL_ERR_STATE_OVERFLOW); the oracle's objects are unbounded."""
        self._emit(OverflowS(what))

    def _rec_field(self, which, name) -> Expr:
        ev = self.event
        if ev is None:
            raise KeyError("no event")
        for i, (n, b, *rest) in enumerate(getattr(ev, "offs", [(n, b, 0) for n, b in ev.fields])):
            if n == name:
                if which == "msg":
                    off = rest[0]
                    return Expr(f"(int)((r >> {off}) & {(1 << b) - 1}u)", f"std::stoi(m.f[{i}])")
                return Expr(f"tf_{name}", f"std::stoi(t.f[{i}])")
        raise KeyError(f"{ev.name} has no field {name}")

    @property
    def sender(self) -> Expr:
        return Expr("rec_from(r)", "from")

    @property
    def self(self) -> Expr:
        return Expr("i", "self")

    def param(self, name) -> Expr:
        return Expr(f"p.{name}", f"prm.{name}")

    def node(self, kind: NodeKind, k=1) -> Expr:
        """Address of instance k (1-based) of a node kind: kinds in declaration order, instances
        consecutive, by the run's counts (first_<kind>)."""
        k = lit(k)
        return Expr(f"(first_{kind.name}(p) + {k.dev} - 1)", f"(first_{kind.name}(prm) + {k.orc} - 1)")

    def count(self, kind: NodeKind) -> Expr:
        """Instances of a node kind in this run."""
        if isinstance(kind.count, int):
            return lit(kind.count)
        return Expr(f"p.{kind.count}", f"prm.{kind.count}")

    def index(self, kind: NodeKind) -> Expr:
        """This node's instance index (from 0) within its kind."""
        return Expr(f"(i - first_{kind.name}(p))", f"(self - first_{kind.name}(prm))")

    # statements
    def _emit(self, s: Stmt):
        self._stack[-1].append(s)
        if not isinstance(s, IfS):
            self._last_if = None

    def set(self, name: str, value):
        self._emit(Assign(self._fd(name), lit(value)))

    def send(self, msg: RecordType, to, **vals):
        self._emit(SendS(msg, lit(to), [lit(vals[n]) for n, _ in msg.fields]))

    def set_timer(self, t: RecordType, **vals):
        self._emit(SetTimerS(t, [lit(vals[n]) for n, _ in t.fields]))

    def throw(self, why: str):
        self._emit(ThrowS(why))

    def if_(self, cond):
        h = self
        s = IfS(lit(cond), [], [])

        class _Ctx:
            def __enter__(self_):
                h._emit(s)
                h._stack.append(s.then)

            def __exit__(self_, *a):
                h._stack.pop()
                h._last_if = s
        return _Ctx()

    def loop(self, name: str, lo, hi):
        """`with h.loop("j", lo, hi) as j:` -- a rolled loop (j from lo while < hi); its body is
        recorded once, so the generated code holds one copy (Python loops unroll instead)."""
        h = self
        s = ForS("l_" + name, lit(lo), lit(hi), [])

        class _Ctx:
            def __enter__(self_):
                h._emit(s)
                h._stack.append(s.body)
                return Expr("l_" + name, "l_" + name)

            def __exit__(self_, *a):
                h._stack.pop()
                h._last_if = None
        return _Ctx()

    def else_(self):
        h = self
        s = self._last_if
        assert s is not None, "else_ must follow an if_ block"

        class _Ctx:
            def __enter__(self_):
                h._stack.append(s.other)

            def __exit__(self_, *a):
                h._stack.pop()
                h._last_if = None
        return _Ctx()


class PredHandler(Handler):
    """What a predicate function sees: q.field(kind, k, name) / q.at_node(kind, k, name, j) (instance
    k from 0 -- read it only under a `k < q.count(kind)` guard), q.results_len(kind, k) /
    q.result(kind, k, j) (a client's harvested ClientWorker results), params, locals and
    conditionals, and q.ret(True / False / "threw")."""

    def __init__(self, proto: Protocol):
        super().__init__(proto, proto.kinds[0])
        self.cached: List[Tuple[str, int]] = []  # (kind, instance) read at a constant instance

    def _node_dev(self, kind: NodeKind, k) -> str:
        """A constant instance reads a register copy of its words (pn_<kind>_<k>, loaded once at the
        predicate's top: independent LDS reads, none of them under the `k < count` guards, which
        would otherwise keep each read where it is); a run-time instance reads through the view."""
        if isinstance(k, int):
            if (kind.name, k) not in self.cached:
                self.cached.append((kind.name, k))
            return f"pn_{kind.name}_{k}"
        return f"v.node(first_{kind.name}(p) + {lit(k).dev})"

    @staticmethod
    def _node_orc(kind: NodeKind, k) -> str:
        return f"n_{kind.name}(s, first_{kind.name}(prm) + {lit(k).orc})"

    def _kfd(self, kind: NodeKind, name) -> FieldDecl:
        for f in kind.fields:
            if f.name == name:
                return f
        raise KeyError(f"{kind.name} has no field {name}")

    def field(self, kind: NodeKind, k, name) -> Expr:
        fd = self._kfd(kind, name)
        assert not fd.cap
        return Expr(f"get({self._node_dev(kind, k)}, {fd.off}, {fd.bits})", f"{self._node_orc(kind, k)}->{name}")

    def at_node(self, kind: NodeKind, k, name, j) -> Expr:
        fd, j = self._kfd(kind, name), lit(j)
        assert fd.array
        dev = f"arr_{kind.name}_{name}({self._node_dev(kind, k)}, {j.dev})" if fd.window_words() <= 2 else \
            f"get({self._node_dev(kind, k)}, {fd.elem(j.dev)}, {fd.bits})"
        return Expr(dev,
                    f"{self._node_orc(kind, k)}->{name}[{j.orc}]")

    def results_len(self, kind: NodeKind, k) -> Expr:
        rl = self._kfd(kind, "_results")
        return Expr(f"get({self._node_dev(kind, k)}, {rl.len_off}, {rl.len_bits})",
                    f"(int)s.cw(first_{kind.name}(prm) + {lit(k).orc})->results.size()")

    def result(self, kind: NodeKind, k, j) -> Expr:
        rl, j = self._kfd(kind, "_results"), lit(j)
        dev = f"arr_{kind.name}__results({self._node_dev(kind, k)}, {j.dev})" if rl.window_words() <= 2 else \
            f"get({self._node_dev(kind, k)}, {rl.elem(j.dev)}, {rl.bits})"
        return Expr(dev,
                    f"std::stoi(s.cw(first_{kind.name}(prm) + {lit(k).orc})->results[{j.orc}].f[0])")

    def ret(self, value=True):
        self._emit(RetPV("THREW" if value == "threw" else "TRUE" if value else "FALSE"))

    def arg(self, i: int) -> Expr:
        """The predicate's integer argument i (dsl_predicate arg0 / arg1; the oracle CLI name's
        i-th ':' part)."""
        assert i in (0, 1)
        return Expr(f"(int)pr.arg{i}", f"a{i}_")

    def any_msg(self, msg: RecordType, cond: Callable) -> Expr:
        """Whether network() -- the state's messages, the successor's new ones and the dropped
        ones (SearchState.network(), SearchState.java:153-157; StatePredicate.
        containsMessageMatching, T/StatePredicate.java:146-149) -- holds a `msg` for which
        cond(m) is true; m.<field>, m.sender and m.to are the message's."""
        m = _MsgView(self.p, msg)
        c = lit(cond(m))
        dev = (f"view_any_record<Self>(v, [&](Rec r) {{ return rec_type(r) == {msg.index} && ({c.dev}); }})")
        orc = f"any_net_(s, [&](const Envelope& e) {{ return e.m.type == \"{msg.name}\" && ({c.orc}); }})"
        return Expr(dev, orc)


class _MsgView:
    """A network message inside q.any_msg: its fields, sender and receiver."""

    def __init__(self, proto: Protocol, msg: RecordType):
        object.__setattr__(self, "_p", proto)
        object.__setattr__(self, "_m", msg)

    @property
    def sender(self) -> Expr:
        return Expr("rec_from(r)", "e.from")

    @property
    def to(self) -> Expr:
        return Expr("rec_to(r)", "e.to")

    def __getattr__(self, name):
        m = self._m
        for i, (n, b) in enumerate(m.fields):
            if n == name:
                off = sum(bb for _, bb in m.fields[:i])
                return Expr(f"(int)((r >> {off}) & {(1 << b) - 1}u)", f"std::stoi(e.m.f[{i}])")
        raise KeyError(f"{m.name} has no field {name}")


def record_pred(proto: Protocol, fn: Callable, cached: Optional[list] = None) -> List[Stmt]:
    """The predicate's statements; `cached` receives the (kind, constant instance) pairs whose
    words the device form reads from a register copy."""
    q = PredHandler(proto)
    fn(q)
    if cached is not None:
        cached.extend(q.cached)
    return q.stmts


def record(proto: Protocol, kind: NodeKind, fn: Callable, event=None, is_timer=False, cmd=None) -> List[Stmt]:
    h = Handler(proto, kind, event, is_timer, cmd)
    if cmd is not None:
        fn(h, cmd)
    else:
        fn(h)
    return h.stmts
