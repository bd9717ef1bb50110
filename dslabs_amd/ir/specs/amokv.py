"""lab1 at-most-once KV store in the protocol IR (the same protocol as csrc/protocols/amokv.hpp,
restated): SimpleServer over AMOApplication(KVStore) (lab1 README; KVStore.java:
59-78 as lab1 specifies it) and SimpleClient inside ClientWorker with a per-client command table
(KVStoreWorkload.java:40-66, :76-133). A Request carries its sequence number; its command is the
sender's workload command of that number. KV values are token sequences len:4 | tokens 2 bits
each from bit 4 (at most 9); a result is type:2 | value << 2 (0 AppendResult, 1 GetResult,
2 KeyNotFound, 3 PutOk), never 0 once set."""
from ... import _lib
from ..core import Protocol

P = Protocol("amokv_ir", _lib.DSL_PROTO_AMOKV_IR, "AmoKVIR", doc=__doc__)
P.param("clients", 2, 1, 3)
P.param("ncmds", 3, 1, 3)
OP_GET, OP_PUT, OP_APPEND = 0, 1, 2
P.param_table("op", 3, 3, 0, 2)
P.param_table("key", 3, 3, 0, 2)
P.param_table("sym", 3, 3, 0, 3)
P.param_table("expected", 3, 3, -1, (1 << 24) - 1, default=-1)
P.workload_size = "ncmds"
P.net_cap = 24
P.max_sends = 1

Request = P.message("Request", seq=2)
Reply = P.message("Reply", seq=2, result=24)
ClientTimer = P.timer("ClientTimer", (100, 100), seq=2)

server = P.node("server", count=1, max_count=1, single_name="server", arrays={"kv": (22, 3), "amo": (26, 3)})
client = P.client_worker("client", count="clients", max_count=3, result_field="result", results_cap=3, timer_cap=4,
                         seq=2, result=24)


def _expected(c, k):
    from ..core import Expr
    return Expr(f"sel_param(p.expected, {c.dev}, {k.dev} - 1)", f"prm.expected[{c.orc}][{k.orc} - 1]")


P.expected_result = _expected


@server.on(Request)
def _request(h):  # SimpleServer.handleRequest over AMOApplication(KVStore)
    c = h.let("c", h.sender - 1)
    seq = h.let("seq", h.msg.seq)
    with h.if_((c < 0) | (c >= h.param("clients")) | (seq < 1) | (seq > h.param("ncmds"))):
        h.throw("request from an unknown client or command")
    amo = h.let("amo", h.at("amo", c))
    last = h.let("last", amo.band(3))
    with h.if_(seq < last):
        h.ret()  # a superseded command: no reply
    r = h.var("r", amo.shr(2))  # seq == last: the cached result
    with h.if_(seq > last):  # AMOApplication: execute once, cache the result
        k = h.let("k", seq - 1)
        op = h.let("op", h.ptab("op", c, k))
        key = h.let("key", h.ptab("key", c, k))
        sym = h.let("sym", h.ptab("sym", c, k))
        v = h.let("v", h.at("kv", key))
        with h.if_(op == OP_GET):
            with h.if_(v.band(15) != 0):
                h.assign("r", v.shl(2).bor(1))  # GetResult(value)
            with h.else_():
                h.assign("r", 2)  # KeyNotFound
        with h.if_(op == OP_PUT):
            h.set_at("kv", key, sym.shl(4).bor(1))
            h.assign("r", 3)  # PutOk
        with h.if_(op == OP_APPEND):
            n = h.let("n", v.band(15))
            with h.if_(n >= 9):
                h.overflow("value longer than 9 tokens")
            v2 = h.let("v2", (v - n).bor(n + 1).bor(sym.shl((n * 2) + 4)))
            h.set_at("kv", key, v2)
            h.assign("r", v2.shl(2))  # AppendResult(new value)
        h.set_at("amo", c, seq.bor(r.shl(2)))
    h.send(Reply, to=h.sender, seq=seq, result=r)


@client.send_command
def _send_command(h, cmd):  # SimpleClient.sendCommand: seq = cmd, Request to the server, ClientTimer
    h.set("seq", cmd)
    h.set("result", 0)
    h.send(Request, to=h.node(server, 1), seq=cmd)
    h.set_timer(ClientTimer, seq=cmd)


@client.on(Reply)
def _reply(h):  # SimpleClient.handleReply
    with h.if_((h.f.result == 0) & (h.msg.seq == h.f.seq)):
        h.set("result", h.msg.result)


@client.on_timer(ClientTimer)
def _timer(h):  # SimpleClient.onClientTimer: re-send and re-set while the command is pending
    with h.if_((h.f.result == 0) & (h.timer.seq == h.f.seq)):
        h.send(Request, to=h.node(server, 1), seq=h.timer.seq)
        h.set_timer(ClientTimer, seq=h.timer.seq)
