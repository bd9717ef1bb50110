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
