"""Protocol descriptors: how a reference protocol configuration maps onto the engine.

Each descriptor fixes the node address table (node index -> reference address string), the
``dsl_protocol_desc`` parameters, and renders decoded events in the reference's
``MessageEnvelope`` / ``TimerEnvelope`` toString shape, e.g.
``Message(client1 -> pingserver, PingRequest(ping-1))`` (framework/tst/dslabs/framework/testing/
MessageEnvelope.java), so traces can be compared with (and replayed on) the oracle.
"""
from __future__ import annotations

from typing import List, Sequence

from . import _lib
from .search import SearchState

DSL_PROTO_PINGPONG = 1
DSL_PROTO_SIPAXOS = 2
DSL_PROTO_SYNTHETIC = 3
DSL_PROTO_AMOKV = 4
DSL_PROTO_MULTIPAXOS = 5
DSL_PROTO_PB = 6
DSL_PROTO_MINITEST = 7


class Protocol:
    proto_id = 0
    addresses: List[str] = []

    def params(self) -> Sequence[int]:
        raise NotImplementedError

    def desc(self) -> _lib.dsl_protocol_desc:
        d = _lib.dsl_protocol_desc()
        d.protocol = self.proto_id
        ps = list(self.params())
        d.n_params = len(ps)
        for i, v in enumerate(ps):
            d.params[i] = int(v)
        return d

    def address_index(self, address) -> int:
        if isinstance(address, int):
            return address
        try:
            return self.addresses.index(address)
        except ValueError:
            raise ValueError(f"unknown address {address!r}") from None

    def render_event(self, e) -> str:
        raise NotImplementedError

    def initial_state(self) -> SearchState:
        return SearchState(self)


class PingPong(Protocol):
    """lab0 PingPong: 1 server ("pingserver"), ``clients`` ClientWorkers with
    ``repeatedPings(pings)`` (labs/lab0-pingpong/tst/dslabs/pingpong/PingTest.java:44-51)."""

    proto_id = DSL_PROTO_PINGPONG

    def __init__(self, clients: int = 1, pings: int = 10, check_value: bool = True, reset_timer: bool = True):
        self.clients = clients
        self.pings = pings
        self.check_value = check_value
        self.reset_timer = reset_timer
        self.addresses = ["pingserver"] + [f"client{i}" for i in range(1, clients + 1)]

    def params(self):
        return [self.clients, self.pings, int(self.check_value), int(self.reset_timer)]

    def render_event(self, e) -> str:
        v = e.fields[0]
        if e.is_timer:
            return f"Timer(-> {self.addresses[e.to]}, PingTimer(ping-{v}))"
        name = "PingRequest" if e.type == 0 else "PongReply"
        return f"Message({self.addresses[e.from_]} -> {self.addresses[e.to]}, {name}(ping-{v}))"


def pingpong_state(clients: int = 1, pings: int = 10, **kw) -> SearchState:
    """initSearchState.addServer(sa); addClientWorker(client(i), repeatedPings(pings)) for i."""
    return PingPong(clients, pings, **kw).initial_state()


class SIPaxos(Protocol):
    """Single-instance Paxos Made Simple (SingleInstancePaxos.java:50-127): proposers
    "proposer1..P" with initial values, acceptors "acceptor1..A"."""

    proto_id = DSL_PROTO_SIPAXOS
    PREDICATES = {"Agreement": 100, "Integrity": 101, "Termination": 102}

    def __init__(self, proposers: int = 2, acceptors: int = 3, values=("a", "b"), incorrect: bool = False):
        assert len(values) == proposers
        self.proposers = proposers
        self.acceptors = acceptors
        self.values = list(values)
        self.incorrect = incorrect
        self.addresses = [f"proposer{i}" for i in range(1, proposers + 1)] + \
                         [f"acceptor{i}" for i in range(1, acceptors + 1)]

    def params(self):
        return [self.proposers, self.acceptors, int(self.incorrect)]

    def predicate(self, name):
        from .search import StatePredicate
        return StatePredicate(name, self.PREDICATES[name])

    def render_event(self, e) -> str:
        if e.is_timer:
            return f"Timer(-> {self.addresses[e.to]}, Propose())"
        n, an, av = e.fields[0], e.fields[1], e.fields[2]
        if e.type == 0:
            body = f"Prepare({n})"
        elif e.type == 1:
            body = f"PrepareAck({n}, null, )" if an == 0 else f"PrepareAck({n}, {an}, {self.values[av - 1]})"
        elif e.type == 2:
            body = f"Accept({n}, {self.values[av - 1]})"
        else:
            body = f"AcceptAck({n})"
        return f"Message({self.addresses[e.from_]} -> {self.addresses[e.to]}, {body})"


class MultiPaxos(Protocol):
    """lab3 Multi-Paxos (builder-authored): servers "server1..n", clients
    "client1..c"; each client runs a KVStoreWorkload of Put / Append / Get commands on the key
    "foo" (KVStoreWorkload.java:40-66, :184-188). Values are token sequences (a workload's
    tokens, <= 4 per value); result codes: 7 PutOk, 6 KeyNotFound, else a value."""

    proto_id = DSL_PROTO_MULTIPAXOS
    PREDICATES = {"LOGS_CONSISTENT_ALL_SLOTS": (400, "Non-empty log slots consistent"),
                  "LOGS_CONSISTENT": (401, "Active log slots consistent"),
                  "APPENDS_LINEARIZABLE": (300, "Sequence of appends to the same key is linearizable")}
    OPS = {"PUT": 1, "APPEND": 2, "GET": 3}
    PUT_OK, KEY_NOT_FOUND = 7, 6
    STATUS = {"EMPTY": 0, "ACCEPTED": 1, "CHOSEN": 2, "CLEARED": 3}  # PaxosLogSlotStatus
    WORKLOADS = {  # same names as the oracle's --workload: (commands, expected results, value tokens)
        "append-xy": ([["APPEND:foo:X"], ["APPEND:foo:Y"]], [[], []], ["X", "Y", "Z"]),
        "append-xy-expect": ([["APPEND:foo:X"], ["APPEND:foo:Y"]], [["X"], ["XY"]], ["X", "Y", "Z"]),
        "append-x": ([["APPEND:foo:X"]], [["X"]], ["X", "Y", "Z"]),
        "append-xz": ([["APPEND:foo:X", "APPEND:foo:Z"], ["APPEND:foo:Y"]], [[], []], ["X", "Y", "Z"]),
        # KVStoreWorkload.putAppendGetWorkload (PaxosTest.test27)
        "put-append-get": ([["PUT:foo:bar", "APPEND:foo:baz", "GET:foo"]], [["Ok", "barbaz", "barbaz"]],
                           ["bar", "baz"]),
    }

    def __init__(self, servers: int = 3, clients: int = 2, workload: str = "append-xy"):
        cmds, exp, tokens = self.WORKLOADS[workload]
        self.workload = workload
        self.servers = servers
        self.clients = clients
        self.tokens = tokens
        self.cmds = [[self._parse_cmd(c) for c in cl] for cl in cmds[:clients]]
        self.expected = exp[:clients]
        self.addresses = [f"server{i}" for i in range(1, servers + 1)] + [f"client{i}" for i in range(1, clients + 1)]

    @staticmethod
    def _parse_cmd(t: str):
        parts = t.split(":")
        return (parts[0], parts[2] if len(parts) > 2 else None)

    def encode_value(self, s: str) -> int:
        toks, i = [], 0
        while i < len(s):
            for k, tok in enumerate(self.tokens):
                if s.startswith(tok, i):
                    toks.append(k + 1)
                    i += len(tok)
                    break
            else:
                raise ValueError(f"value {s!r} is not a sequence of the workload's tokens")
        r = len(toks)
        for i, t in enumerate(toks):
            r |= t << (3 + 2 * i)
        return r

    def encode_result(self, op: str, s: str) -> int:
        if op == "PUT":
            return self.PUT_OK
        if op == "GET" and s == "KeyNotFound":
            return self.KEY_NOT_FOUND
        return self.encode_value(s)

    def decode_result(self, r: int) -> str:
        if r == self.PUT_OK:
            return "Ok"
        if r == self.KEY_NOT_FOUND:
            return "KeyNotFound"
        return "".join(self.tokens[((r >> (3 + 2 * i)) & 3) - 1] for i in range(r & 7))

    def params(self):
        ps = [self.servers, self.clients]
        for c in range(2):
            cl = self.cmds[c] if c < self.clients else []
            exp = self.expected[c] if c < self.clients else []
            ops = [self.OPS[op] for op, _ in cl] + [0] * (3 - len(cl))
            vals = [0 if v is None else self.tokens.index(v) + 1 for _, v in cl] + [0] * (3 - len(cl))
            e = [self.encode_result(cl[k][0], x) for k, x in enumerate(exp)] + [-1] * (3 - len(exp))
            ps += [len(cl)] + ops + vals + e
        return ps

    def kv_code(self, cmd: str) -> int:
        """A KV command as hasCommand's code: a workload command ("APPEND:foo:X", "PUT:foo:bar",
        "GET:foo"), the oracle's form ("X", "=bar", "?"), or None = null."""
        if cmd is None:
            return 0
        if ":" not in cmd:
            cmd = "GET:foo" if cmd == "?" else f"PUT:foo:{cmd[1:]}" if cmd.startswith("=") else f"APPEND:foo:{cmd}"
        op, v = self._parse_cmd(cmd)
        return (self.OPS[op] << 2) | (0 if v is None else self.tokens.index(v) + 1)

    def predicate(self, name):
        """LOGS_CONSISTENT_ALL_SLOTS, LOGS_CONSISTENT, APPENDS_LINEARIZABLE; slotValid:i;
        hasStatus:serverK:i:STATUS; hasCommand:serverK:i:CMD (CMD a workload command, or null)
        (PaxosTest.java:113-346)."""
        from .search import StatePredicate
        if name in self.PREDICATES:
            pid, full = self.PREDICATES[name]
            return StatePredicate(full, pid)
        parts = name.split(":")
        if parts[0] == "slotValid":
            return StatePredicate(f"Logs consistent for slot {parts[1]}", 402, int(parts[1]))
        if parts[0] == "hasStatus":
            a, i, st = parts[1], int(parts[2]), parts[3]
            return StatePredicate(f"{a} has status {st} in slot {i}", 403, a, (i << 4) | self.STATUS[st],
                                  address_args=(0,))
        if parts[0] == "hasCommand":
            a, i = parts[1], int(parts[2])
            c = ":".join(parts[3:])
            code = self.kv_code(None if c == "null" else c)
            return StatePredicate(f"{a} has command {c} in slot {i}", 404, a, (i << 8) | code, address_args=(0,))
        raise KeyError(name)

    # ---- rendering in the oracle's toString form ------------------------------------------------
    def _cmd(self, cmd: int) -> str:
        if cmd == 0:
            return "noop"
        c = 1 if cmd >= 4 else 0
        q = cmd - 3 * c
        op, v = self.cmds[c][q - 1]
        body = {"PUT": f"={v}", "GET": "?"}.get(op, v)
        return f"{self.servers + c}#{q}:{body}"

    @staticmethod
    def _ballot(cb: int) -> str:
        return f"({cb >> 2},{cb & 3})"

    @staticmethod
    def _mballot(m: int) -> int:
        return ((m & 0xF) << 2) | ((m >> 4) & 3)

    def _entry(self, e: int) -> str:
        st, b, cmd = e & 3, (e >> 2) & 0x3F, (e >> 8) & 7
        if st == 0:
            return "E"
        if st == 2:
            return "C:" + self._cmd(cmd)
        return "A" + self._ballot(b) + ":" + self._cmd(cmd)

    def render_event(self, e) -> str:
        a = self.addresses
        if e.is_timer:
            if e.type == 8:
                return f"Timer(-> {a[e.to]}, TickTimer())"
            return f"Timer(-> {a[e.to]}, ClientTimer({e.fields[0]}))"
        m = e.fields[0]
        t = e.type
        if t == 0:
            body = f"PaxosRequest({self._cmd(m & 7)})"
        elif t == 1:
            body = f"PaxosReply({m & 3}, {self.decode_result((m >> 2) & 0xFFF)})"
        elif t == 2:
            body = f"P1a({self._ballot(self._mballot(m))})"
        elif t == 3:
            log = ";".join(self._entry((m >> (6 + 11 * i)) & 0x7FF) for i in range(4))
            body = f"P1b({self._ballot(self._mballot(m))}, {log})"
        elif t == 4:
            body = f"P2a({self._ballot(self._mballot(m))}, {(m >> 6) & 7}, {self._cmd((m >> 9) & 7)})"
        elif t == 5:
            body = f"P2b({self._ballot(self._mballot(m))}, {(m >> 6) & 7})"
        elif t == 6:
            body = f"Decision({m & 7}, {self._cmd((m >> 3) & 7)})"
        else:
            body = f"Heartbeat({self._ballot(self._mballot(m))})"
        return f"Message({a[e.from_]} -> {a[e.to]}, {body})"


class Synthetic(Protocol):
    """The table-driven synthetic protocol of BASELINE config C3 (builder-defined):
    nodes "node1..N", each with a value v in [0, K), a poke counter and four always-deliverable
    timers SynthTimer(0..3); transitions come from a seeded splitmix64 table. 64-byte packed
    state, ~20-25 enabled events per state: a dedup / all-to-all stress test."""

    proto_id = DSL_PROTO_SYNTHETIC
    SEED = 0x5EEDD51AB5

    def __init__(self, nodes: int = 5, values: int = 64, poke_mod: int = 7, seed: int = SEED):
        self.nodes = nodes
        self.values = values
        self.poke_mod = poke_mod
        self.seed = seed
        self.addresses = [f"node{i}" for i in range(1, nodes + 1)]

    def params(self):
        return [self.nodes, self.values, self.poke_mod, self.seed]

    def predicate(self, name):
        from .search import StatePredicate
        if name == "NOT_ALL_MAX":
            return StatePredicate("NOT_ALL_MAX", 200)
        if name.startswith("COUNTER_LT:"):
            _, node, bound = name.split(":")
            return StatePredicate(name, 201, int(node), int(bound))
        raise KeyError(name)

    def render_event(self, e) -> str:
        if e.is_timer:
            return f"Timer(-> {self.addresses[e.to]}, SynthTimer({e.fields[0]}))"
        return f"Message({self.addresses[e.from_]} -> {self.addresses[e.to]}, Poke())"


class AmoKV(Protocol):
    """lab1 at-most-once client/server KV store (builder-authored): "server"
    (SimpleServer over AMOApplication(KVStore)) and ClientWorkers "client1..c" (SimpleClient).
    Workloads are the KVStoreWorkload ones the lab1 search tests use
    (labs/lab1-clientserver/tst/dslabs/kvstore/KVStoreWorkload.java, ClientServerPart2Test.java)."""

    proto_id = DSL_PROTO_AMOKV
    PREDICATES = {"APPENDS_LINEARIZABLE": (300, "Sequence of appends to the same key is linearizable")}
    # same names and templates as oracle/proto_amokv.hpp (commands, results, numTimes)
    WORKLOADS = {
        "diffkey3": (["APPEND:KEY-%a:0", "APPEND:KEY-%a:1", "APPEND:KEY-%a:2"], ["0", "01", "012"], 1),
        "diffkey2": (["APPEND:KEY-%a:0", "APPEND:KEY-%a:1"], ["0", "01"], 1),
        "samekey3": (["APPEND:foo:%i"], [], 3),
        "samekey2": (["APPEND:foo:%i"], [], 2),
        "appendappendget": (["APPEND:foo:bar", "APPEND:foo:bar", "GET:foo"], ["bar", "barbar", "barbar"], 1),
        "putappendget": (["PUT:foo:bar", "APPEND:foo:baz", "GET:foo"], ["Ok", "barbaz", "barbaz"], 1),
        "getput": (["GET:foo", "PUT:foo:bar", "GET:foo"], ["KeyNotFound", "Ok", "bar"], 1),
    }
    OPS = {"GET": 0, "PUT": 1, "APPEND": 2}
    RTYPES = ["AppendResult", "GetResult", "KeyNotFound", "PutOk"]

    def __init__(self, clients: int = 2, workload: str = "diffkey3"):
        cmds, results, times = self.WORKLOADS[workload]
        self.clients = clients
        self.workload = workload
        self.addresses = ["server"] + [f"client{i}" for i in range(1, clients + 1)]
        self.keys, self.syms = [], []
        self.cmds = []  # per client: [(op, key, value)]
        self.expected = []  # per client: [result string or None]
        n = len(cmds) * times
        self.ncmds = n
        for c in range(1, clients + 1):
            cl, ex = [], []
            for i in range(n):
                t = cmds[i % len(cmds)].replace("%a", f"client{c}").replace("%i", str(i + 1))
                sp = t.split(":", 2)
                op = sp[0]
                key = sp[1] if op != "GET" or len(sp) == 2 else sp[1] + sp[2]
                val = sp[2] if op != "GET" else None
                if key not in self.keys:
                    self.keys.append(key)
                if val is not None and val not in self.syms:
                    self.syms.append(val)
                cl.append((op, key, val))
                ex.append(results[i % len(cmds)].replace("%a", f"client{c}").replace("%i", str(i + 1))
                          if results else None)
            self.cmds.append(cl)
            self.expected.append(ex)
        assert len(self.keys) <= 3 and len(self.syms) <= 4 and n <= 3 and clients <= 3
        assert len({len(s) for s in self.syms}) <= 1, "value tokens must have equal length"

    def _value_bits(self, s: str) -> int:
        toks, w = [], len(self.syms[0]) if self.syms else 1
        for k in range(0, len(s), w):
            toks.append(self.syms.index(s[k:k + w]))
        v = len(toks)
        for j, t in enumerate(toks):
            v |= t << (4 + 2 * j)
        return v

    def _result_bits(self, op: str, r: str) -> int:
        if op == "APPEND":
            return 0 | (self._value_bits(r) << 2)
        if op == "GET":
            return 2 if r == "KeyNotFound" else 1 | (self._value_bits(r) << 2)
        return 3  # PutOk

    def params(self):
        ps = [self.clients, self.ncmds]
        for c in range(3):
            for k in range(3):
                if c < self.clients and k < self.ncmds:
                    op, key, val = self.cmds[c][k]
                    exp = self.expected[c][k]
                    ps += [self.OPS[op], self.keys.index(key), self.syms.index(val) if val is not None else 0,
                           self._result_bits(op, exp) if exp is not None else -1]
                else:
                    ps += [0, 0, 0, -1]
        return ps

    def predicate(self, name):
        from .search import StatePredicate
        pid, full = self.PREDICATES[name]
        return StatePredicate(full, pid)

    def _value_str(self, v: int) -> str:
        return "".join(self.syms[(v >> (4 + 2 * j)) & 3] for j in range(v & 15))

    def _result_str(self, r: int) -> str:
        t, v = r & 3, r >> 2
        if t == 0:
            return f"AppendResult({self._value_str(v)})"
        if t == 1:
            return f"GetResult({self._value_str(v)})"
        return "KeyNotFound()" if t == 2 else "PutOk()"

    def _cmd_str(self, c: int, seq: int) -> str:
        op, key, val = self.cmds[c - 1][seq - 1]
        return {"GET": f"Get({key})", "PUT": f"Put({key}, {val})", "APPEND": f"Append({key}, {val})"}[op]

    def render_event(self, e) -> str:
        a = self.addresses
        if e.is_timer:
            return f"Timer(-> {a[e.to]}, ClientTimer({e.fields[0]}))"
        seq = e.fields[0]
        if e.type == 0:
            return f"Message({a[e.from_]} -> {a[e.to]}, Request({self._cmd_str(e.from_, seq)}, {seq}))"
        return f"Message({a[e.from_]} -> {a[e.to]}, Reply({self._result_str(e.fields[1])}, {seq}))"


class PB(Protocol):
    """lab2 primary-backup with a ViewServer (builder-authored): "viewserver",
    PBServers "server1..S", ClientWorkers "client1..c" around PBClients; KVStore workloads as in
    lab1 (PrimaryBackupTest uses putGetWorkload, PrimaryBackupTest.java:680-711)."""

    proto_id = DSL_PROTO_PB
    WORKLOADS = dict(AmoKV.WORKLOADS, putget=(["PUT:foo:bar", "GET:foo"], ["Ok", "bar"], 1))
    RTYPES = AmoKV.RTYPES

    def __init__(self, servers: int = 2, clients: int = 1, workload: str = "putget"):
        self.servers = servers
        self.clients = clients
        self.workload = workload
        self.addresses = ["viewserver"] + [f"server{i}" for i in range(1, servers + 1)] + \
                         [f"client{i}" for i in range(1, clients + 1)]
        # reuse the KV workload expansion of AmoKV (commands per client, keys, value tokens)
        kv = AmoKV.__new__(AmoKV)
        saved = AmoKV.WORKLOADS
        AmoKV.WORKLOADS = self.WORKLOADS
        try:
            AmoKV.__init__(kv, clients, workload)
        finally:
            AmoKV.WORKLOADS = saved
        self.kv = kv
        assert len(kv.keys) <= 2 and servers <= 3 and clients <= 2 and kv.ncmds <= 3

    def _value_bits(self, s: str) -> int:
        w = len(self.kv.syms[0]) if self.kv.syms else 1
        toks = [self.kv.syms.index(s[k:k + w]) for k in range(0, len(s), w)]
        assert len(toks) <= 3
        v = len(toks)
        for j, t in enumerate(toks):
            v |= t << (2 + 2 * j)
        return v

    def _result_bits(self, op: str, r: str) -> int:
        if op == "APPEND":
            return 0 | (self._value_bits(r) << 2)
        if op == "GET":
            return 2 if r == "KeyNotFound" else 1 | (self._value_bits(r) << 2)
        return 3

    def params(self):
        kv = self.kv
        ps = [self.servers, self.clients, kv.ncmds]
        for c in range(2):
            for k in range(3):
                if c < self.clients and k < kv.ncmds:
                    op, key, val = kv.cmds[c][k]
                    exp = kv.expected[c][k]
                    ps += [AmoKV.OPS[op], kv.keys.index(key), kv.syms.index(val) if val is not None else 0,
                           self._result_bits(op, exp) if exp is not None else -1]
                else:
                    ps += [0, 0, 0, -1]
        return ps

    @staticmethod
    def _view_bits(n: int, p: int, b: int) -> int:
        return n | (max(p, 0) << 4) | (max(b, 0) << 6)

    def predicate(self, name):
        """hasViewReply:N (viewNum >= N), hasViewReply:N:P:B (exactly View(N, P, B); -1 = null,
        PrimaryBackupTest.java:104-117) and viewRepliesSent:N:P:B:addr+addr+... (initView's goal,
        :136-156); P and B are server indices (1 = server1)."""
        from .search import StatePredicate
        if name.startswith("hasViewReply:"):
            parts = [int(x) for x in name.split(":")[1:]]
            if len(parts) == 1:
                return StatePredicate(f"ViewReply with viewNum: {parts[0]}", 500, parts[0])
            n, p, b = parts
            return StatePredicate(f"ViewReply with View({n}, {p}, {b})", 501, self._view_bits(n, p, b))
        if name.startswith("viewRepliesSent:"):
            _, n, p, b, to = name.split(":")
            mask = 0
            for a in to.split("+"):
                mask |= 1 << self.address_index(a)
            return StatePredicate(f"ViewReply for View({n}, {p}, {b}) sent to {to}, primary ack sent", 502,
                                  self._view_bits(int(n), int(p), int(b)), mask)
        raise KeyError(name)

    def initView(self, viewNum: int, primary: str, backup=None, *clients, start=None, device: int = -1,
                 max_time_secs: int = 30):
        """PrimaryBackupTest.initView (PrimaryBackupTest.java:124-187): a BFS (network off except the
        ViewServer's links and primary <-> backup) for a state where View(viewNum, primary, backup)
        has ViewReplies sent to the primary, the backup and `clients` and the primary's ack Ping is
        in the network, without any later view; then those ViewReplies and the ack are delivered in
        turn (stepMessage). Returns the prepared start state."""
        from . import _lib
        from .search import Search, SearchSettings
        pi = self.address_index(primary)
        bi = self.address_index(backup) if backup is not None else -1
        to_init = [primary] + ([backup] if backup is not None else []) + list(clients)
        n1 = viewNum + 1
        s = SearchSettings().maxTimeSecs(max_time_secs)
        s.addPrune(self.predicate(f"hasViewReply:{n1}"))
        s.addPrune(self.predicate(f"hasViewReply:{viewNum}").and_(
            self.predicate(f"hasViewReply:{viewNum}:{pi}:{bi}").negate()))
        s.networkActive(False).nodeActive("viewserver", True)
        if backup is not None:
            s.linkActive(primary, backup, True).linkActive(backup, primary, True)
        s.addGoal(self.predicate(f"viewRepliesSent:{viewNum}:{pi}:{bi}:{'+'.join(to_init)}").and_(
            self.predicate(f"hasViewReply:{n1}").negate()))
        r = Search.bfs(start if start is not None else self.initial_state(), s, device)
        goal = r.goalMatchingState()
        if goal is None:
            raise RuntimeError(f"initView: no state with View({viewNum}, {primary}, {backup}) started: "
                               f"{r.endCondition().name}")
        view = self._view_bits(viewNum, pi, bi)
        evs = []
        for a in to_init:  # the ViewReplies, then the primary's ack
            e = _lib.dsl_event()
            e.from_, e.to, e.type, e.n_fields = 0, self.address_index(a), 2, 1
            e.fields[0] = view
            evs.append(e)
        e = _lib.dsl_event()
        e.from_, e.to, e.type, e.n_fields = pi, 0, 0, 1
        e.fields[0] = viewNum
        evs.append(e)
        rr = Search.replay(goal, SearchSettings(), evs, minimize=False, device=device)
        st = rr.lastState()
        if st is None or st.depth() != goal.depth() + len(evs):
            raise RuntimeError("initView: a prepared message could not be delivered")
        return st

    # ---- rendering in the oracle's toString form ------------------------------------------------
    def _value_str(self, v: int) -> str:
        return "".join(self.kv.syms[(v >> (2 + 2 * j)) & 3] for j in range(v & 3))

    def _result_str(self, r: int) -> str:
        t, v = r & 3, r >> 2
        if t == 0:
            return f"AppendResult({self._value_str(v)})"
        if t == 1:
            return f"GetResult({self._value_str(v)})"
        return "KeyNotFound()" if t == 2 else "PutOk()"

    @staticmethod
    def _view_str(v: int) -> str:
        p, b = (v >> 4) & 3, (v >> 6) & 3
        return f"View({v & 15}, {p if p else -1}, {b if b else -1})"

    def _app_str(self, app: int) -> str:
        w1, w2 = app & 0xFFFFFFF, app >> 28
        s = ""
        for k, key in enumerate(self.kv.keys):
            v = (w1 >> (8 * k)) & 0xFF
            if v & 3:
                s += f"{key}={self._value_str(v)};"
        s += "|"
        for c, amo in enumerate([(w1 >> 16) & 0xFFF, w2 & 0xFFF]):
            if amo & 3:
                s += f"{1 + self.servers + c}:{amo & 3}:{self._result_str(amo >> 2)};"
        return s

    def render_event(self, e) -> str:
        a = self.addresses
        if e.is_timer:
            if e.type == 9:
                return f"Timer(-> {a[e.to]}, PingCheckTimer())"
            if e.type == 10:
                return f"Timer(-> {a[e.to]}, PingTimer())"
            return f"Timer(-> {a[e.to]}, ClientTimer({e.fields[0]}))"
        m, t = e.fields[0], e.type
        if t == 0:
            body = f"Ping({m & 15})"
        elif t == 1:
            body = "GetView()"
        elif t == 2:
            body = f"ViewReply({self._view_str(m & 0xFF)})"
        elif t == 3:
            body = f"Request({m & 3})"
        elif t == 4:
            body = f"Reply({self._result_str((m >> 2) & 0x3FF)}, {m & 3})"
        elif t == 5:
            body = f"StateTransfer({self._view_str(m & 0xFF)}, {self._app_str((m >> 8) & ((1 << 40) - 1))})"
        elif t == 6:
            body = f"StateTransferAck({m & 15})"
        else:
            name = "Forward" if t == 7 else "ForwardAck"
            body = f"{name}({m & 15}, {(m >> 4) & 7}, {(m >> 7) & 3})"
        return f"Message({a[e.from_]} -> {a[e.to]}, {body})"


class MiniTest(Protocol):
    """The two-node fixture of the reference's trace-minimizer tests
    (framework/tst-self/dslabs/framework/testing/search/SearchAndTraceMinimizerTest.java:430-471):
    servers "a" and "b", messages Foo and Bar; predicates ``foo``, ``fooException`` and
    ``alwaysException`` (:104-126, :255-260)."""

    proto_id = DSL_PROTO_MINITEST

    def __init__(self):
        self.addresses = ["a", "b"]

    def params(self):
        return []

    def predicate(self, name):
        from .search import StatePredicate
        ids = {"foo": 700, "fooException": 701, "alwaysException": 702}
        if name not in ids:
            raise KeyError(name)
        return StatePredicate(name, ids[name])

    def render_event(self, e) -> str:
        body = "Foo()" if e.type == 0 else "Bar()"
        return f"Message({self.addresses[e.from_]} -> {self.addresses[e.to]}, {body})"

    def event(self, frm: str, to: str, name: str):
        """A dsl_event for Message(frm -> to, name()) (MessageEnvelope of the reference test)."""
        e = _lib.dsl_event()
        e.from_ = self.address_index(frm)
        e.to = self.address_index(to)
        e.type = {"Foo": 0, "Bar": 1}[name]
        return e


class IRProtocol(Protocol):
    """A protocol generated from the protocol IR (dslabs_amd/ir/specs/<spec>.py; device form
    csrc/protocols/gen/, oracle form oracle/gen/). Parameters by the spec's names; events render
    as the oracle's object form does (integer fields)."""

    def __init__(self, spec: str, **params):
        import importlib
        self.spec = importlib.import_module(f"dslabs_amd.ir.specs.{spec}").P
        self.proto_id = self.spec.proto_id
        known = {p.name for p in self.spec.params}
        bad = set(params) - known
        if bad:
            raise ValueError(f"unknown parameters {sorted(bad)} for {spec}")
        self.values = {p.name: int(params.get(p.name, p.default)) for p in self.spec.params}
        self.addresses = self.spec.address_names(self.values)

    def params(self):
        return [self.values[p.name] for p in self.spec.params]

    def render_event(self, e) -> str:
        a = self.addresses
        fields = ", ".join(str(e.fields[i]) for i in range(e.n_fields))
        if e.is_timer:
            return f"Timer(-> {a[e.to]}, {self.spec.timers[e.type - len(self.spec.messages)].name}({fields}))"
        return f"Message({a[e.from_]} -> {a[e.to]}, {self.spec.messages[e.type].name}({fields}))"


class PingPongIR(IRProtocol):
    """lab0 PingPong generated from the protocol IR (dslabs_amd/ir/specs/pingpong.py)."""

    def __init__(self, clients: int = 1, pings: int = 10, check_value: bool = True, reset_timer: bool = True):
        super().__init__("pingpong", clients=clients, pings=pings, check_value=int(check_value),
                         reset_timer=int(reset_timer))


class AmoKVIR(IRProtocol):
    """lab1 AMO KV generated from the protocol IR (dslabs_amd/ir/specs/amokv.py), with AmoKV's
    workloads (the same command tables and result encodings)."""

    def __init__(self, clients: int = 2, workload: str = "diffkey3"):
        kv = AmoKV(clients, workload)
        tables = {n: [[0] * 3 for _ in range(3)] for n in ("op", "key", "sym")}
        tables["expected"] = [[-1] * 3 for _ in range(3)]
        ps = kv.params()[2:]
        for c in range(3):
            for k in range(3):
                op, key, sym, exp = ps[4 * (3 * c + k): 4 * (3 * c + k) + 4]
                tables["op"][c][k], tables["key"][c][k], tables["sym"][c][k] = op, key, sym
                tables["expected"][c][k] = exp
        super().__init__("amokv", clients=clients, ncmds=kv.ncmds)
        self.kv = kv
        self._tables = tables

    def params(self):
        ps = super().params()
        for n in ("op", "key", "sym", "expected"):
            for row in self._tables[n]:
                ps += row
        return ps

    def oracle_args(self):
        return ["--proto", "amokv_ir", "--clients", str(self.values["clients"]), "--ir-params",
                ",".join(str(x) for x in self.params())]


class PBIR(IRProtocol):
    """lab2 primary-backup + ViewServer (BASELINE C4) generated from the protocol IR
    (dslabs_amd/ir/specs/pb.py), with PB's workloads (the same command tables and result encodings)
    and predicates (hasViewReply(n), hasViewReply(n, p, b), initView's viewRepliesSent: network
    predicates in the IR; the ClientWorker family)."""

    IR_NAMES = {500: "hasViewReply", 501: "hasViewReplyExact", 502: "viewRepliesSent"}

    def __init__(self, servers: int = 2, clients: int = 1, workload: str = "putget"):
        pb = PB(servers, clients, workload)
        ps = pb.params()
        super().__init__("pb", servers=servers, clients=clients, ncmds=ps[2])
        self.pb = pb
        self._tables = {n: [[0] * 3 for _ in range(2)] for n in ("op", "key", "sym")}
        self._tables["expected"] = [[-1] * 3 for _ in range(2)]
        for c in range(2):
            for k in range(3):
                op, key, sym, exp = ps[3 + 4 * (3 * c + k): 3 + 4 * (3 * c + k) + 4]
                self._tables["op"][c][k], self._tables["key"][c][k], self._tables["sym"][c][k] = op, key, sym
                self._tables["expected"][c][k] = exp

    def params(self):
        ps = super().params()
        for n in ("op", "key", "sym", "expected"):
            for row in self._tables[n]:
                ps += row
        return ps

    def predicate(self, name):
        return self.pb.predicate(name)

    def oracle_args(self):
        return ["--proto", "pb_ir", "--ir-params", ",".join(str(x) for x in self.params())]

    def ir_oracle_name(self, name: str) -> str:
        """A PB predicate name (PB.predicate's forms) as the IR oracle's NAME:arg0[:arg1]."""
        sp = self.pb.predicate(name)
        ir = self.IR_NAMES[sp.pred_id]
        return f"{ir}:{sp.arg0}" + (f":{sp.arg1}" if sp.pred_id == 502 else "")


class MultiPaxosIR(IRProtocol):
    """lab3 Multi-Paxos (BASELINE C5) generated from the protocol IR (dslabs_amd/ir/specs/multipaxos.py),
    with MultiPaxos's workloads (the same command tables and result encodings) and predicates
    (LOGS_CONSISTENT_ALL_SLOTS, LOGS_CONSISTENT, APPENDS_LINEARIZABLE and the ClientWorker family)."""

    def __init__(self, servers: int = 3, clients: int = 2, workload: str = "append-xy"):
        mp = MultiPaxos(servers, clients, workload)
        ps = mp.params()[2:]  # per client: ncmds, ops[3], vals[3], expected[3]
        self._tables = {"ncmd": [[ps[10 * c]] for c in range(2)],
                        "op": [ps[10 * c + 1: 10 * c + 4] for c in range(2)],
                        "val": [ps[10 * c + 4: 10 * c + 7] for c in range(2)],
                        "expected": [ps[10 * c + 7: 10 * c + 10] for c in range(2)]}
        super().__init__("multipaxos", servers=servers, clients=clients)
        self.mp = mp
        self.workload = workload

    def params(self):
        ps = super().params()
        for n in ("ncmd", "op", "val", "expected"):
            for row in self._tables[n]:
                ps += row
        return ps

    def predicate(self, name):
        return self.mp.predicate(name)

    def oracle_args(self):
        return ["--proto", "multipaxos_ir", "--ir-params", ",".join(str(x) for x in self.params())]

    IR_NAMES = {402: "slotValid", 403: "hasStatus", 404: "hasCommand"}

    def ir_oracle_name(self, name: str) -> str:
        """A lab3 argument predicate (MultiPaxos.predicate's slotValid:i / hasStatus:serverK:i:S /
        hasCommand:serverK:i:C) as the IR oracle's NAME:arg0[:arg1] (the server as its node index)."""
        sp = self.mp.predicate(name)
        if sp.pred_id == 402:
            return f"slotValid:{sp.arg0}"
        a0 = int(name.split(":")[1][len("server"):]) - 1
        return f"{self.IR_NAMES[sp.pred_id]}:{a0}:{sp.arg1}"
