"""lab3 Multi-Paxos in the protocol IR -- BASELINE config C5's protocol, the same one as
csrc/protocols/multipaxos.hpp and oracle/proto_multipaxos.hpp, restated once here
and generated into both forms. It follows labs/lab3-paxos/README.md:25-106 (PMMC roles in one
server, stable leader + heartbeat-check timer, clients broadcasting requests, AMO KV store) and
exposes what PaxosTest's predicates read (PaxosTest.java:113-346).

Servers "server1.." (node 0 .. servers-1), clients "client1.." after them. Ballot = (round,
leader) compared as round << 2 | leader; (0, server1) is active at start. A log entry is 11 bits:
status:2 | ballot:6 | cmd:3 (EMPTY 0, ACCEPTED 1, CHOSEN 2; a chosen entry keeps ballot 0).
Command id 1 + 3 c + (q - 1) is client c's q-th command (0 = no-op); its KV op (1 Put, 2 Append,
3 Get) and value token come from the workload tables. The key's value is len:3 | tokens 2 bits
each; a result is 7 PutOk, 6 KeyNotFound or a value. The application state is a function of the
executed log prefix, so it is recomputed, not stored. Server Tick timers (100 ms) are re-set on
every fire; a client's ClientTimer(seq) (100 ms) re-sends while its command is pending."""
import itertools

from ... import _lib
from ..core import Expr, Protocol, lit, select

P = Protocol("multipaxos_ir", _lib.DSL_PROTO_MULTIPAXOS_IR, "MultiPaxosIR", doc=__doc__)
P.param("servers", 3, 1, 3)
P.param("clients", 2, 1, 2)
P.param_table("ncmd", 2, 1, 0, 3)
P.param_table("op", 2, 3, 0, 3)       # 1 Put, 2 Append, 3 Get
P.param_table("val", 2, 3, 0, 3)      # value token 1..3 (0 for a Get)
P.param_table("expected", 2, 3, -1, 4095, default=-1)
P.workload_size = lambda h, c: h.ptab("ncmd", c, 0)
P.expected_result = lambda c, k: Expr(f"sel_param(p.expected, {c.dev}, {k.dev} - 1)",
                                      f"prm.expected[{c.orc}][{k.orc} - 1]")
P.net_cap = 64
P.max_sends = 12  # P1b completing phase 1: a P2a to both others for each of 4 slots + 4 replies
P.sends_distinct = True  # distinct destinations or slots per send (protocheck: dup_sends == 0)
EMPTY, ACCEPTED, CHOSEN = 0, 1, 2
PUT, APPEND, GET = 1, 2, 3
PUT_OK, KEY_NOT_FOUND = 7, 6
SLOTS, MAX_ROUND = 4, 15

# message types in the hand-written protocol's order (its handler classes)
Request = P.message("Request", cmd=3)
Reply = P.message("Reply", seq=2, result=12)
P1a = P.message("P1a", round=4, leader=2)
P1b = P.message("P1b", round=4, leader=2, l1=11, l2=11, l3=11, l4=11)
P2a = P.message("P2a", round=4, leader=2, slot=3, cmd=3)
P2b = P.message("P2b", round=4, leader=2, slot=3)
Decision = P.message("Decision", slot=3, cmd=3)
Heartbeat = P.message("Heartbeat", round=4, leader=2)
Tick = P.timer("Tick", (100, 100))
ClientTimer = P.timer("ClientTimer", (100, 100), seq=2)

server = P.node("server", count="servers", max_count=3,
                arrays={"log": (11, SLOTS), "p1blog": (11, SLOTS), "votes": (3, SLOTS)},
                round=4, leader=2, active=1, electing=1, heard=1, missed=2, p1bvotes=3, slotout=3, slotin=3)
server.timer_cap = 2  # [Tick], plus the re-set one until the fired entry is removed
client = P.client_worker("client", count="clients", max_count=2, result_field="result", results_cap=3, timer_cap=3,
                         seq=2, pending=1, result=12)

_uid = itertools.count()


def _n(base):  # a fresh local name (helpers are inlined several times into one handler)
    return f"{base}{next(_uid)}"


# ---- expressions ------------------------------------------------------------------------------------
def st(e):
    return lit(e).band(3)


def eb(e):
    return lit(e).shr(2).band(63)


def ec(e):
    return lit(e).shr(8).band(7)


def mk(status, b, cmd):
    return lit(status).bor(lit(b).shl(2)).bor(lit(cmd).shl(8))


def ballot(h):
    return h.f.round.shl(2).bor(h.f.leader)


def mballot(h):
    return h.msg.round.shl(2).bor(h.msg.leader)


def popc3(v):
    v = lit(v)
    return v.band(1) + v.shr(1).band(1) + v.shr(2).band(1)


def majority(h, votes):
    return popc3(votes) * 2 > h.count(server)


def cmd_client(cmd):
    return select(lit(cmd) >= 4, 1, 0)


def cmd_seq(cmd):
    return lit(cmd) - cmd_client(cmd) * 3


def me(h):
    return h.index(server)


# ---- helpers (inlined statements) -----------------------------------------------------------------
def bcast(h, msg, **vals):
    for j in range(3):
        with h.if_((lit(j) < h.count(server)) & (lit(j) != me(h))):
            h.send(msg, to=h.node(server, j + 1), **vals)


def kv_apply(h, cmd, kv):
    """KVStore.execute of command `cmd` on the key's value (local `kv`): the result (a local)."""
    c = h.let(_n("c"), cmd_client(cmd))
    op = h.let(_n("op"), h.ptab("op", c, cmd_seq(cmd) - 1))
    v = h.let(_n("v"), h.ptab("val", c, cmd_seq(cmd) - 1))
    x = h.var(_n("x"), 0)
    with h.if_(op == PUT):
        h.assign(kv.dev[2:], lit(1).bor(v.shl(3)))
        h.assign(x.dev[2:], PUT_OK)
    with h.if_(op == APPEND):
        n = h.let(_n("len"), kv.band(7))
        h.assign(kv.dev[2:], (n + 1).bor(kv.band(-8)).bor(v.shl(lit(3) + n * 2)))
        h.assign(x.dev[2:], kv)
    with h.if_(op == GET):
        h.assign(x.dev[2:], select(kv.band(7) != 0, kv, KEY_NOT_FOUND))
    return x


def execute(h):
    """Executes the chosen slots from slotOut on, in order; an active leader replies."""
    so0 = h.let(_n("so0"), h.f.slotout)
    act = h.let(_n("act"), h.f.active)
    kv, ls0, ls1 = h.var(_n("kv"), 0), h.var(_n("ls0"), 0), h.var(_n("ls1"), 0)
    so, run = h.var(_n("so"), so0), h.var(_n("run"), 1)
    for slot in range(1, SLOTS + 1):
        e = h.let(_n("e"), h.at("log", slot - 1))
        cmd = h.let(_n("cmd"), ec(e))
        c, q = h.let(_n("c"), cmd_client(cmd)), h.let(_n("q"), cmd_seq(cmd))
        before = h.let(_n("before"), lit(slot) < so0)
        now = h.let(_n("now"), (~before) & (run != 0) & (st(e) == CHOSEN))
        h.assign(run.dev[2:], select((run != 0) & (before | now), 1, 0))
        with h.if_((before | now) & (cmd != 0) & (select(c, ls1, ls0) < q)):
            x = kv_apply(h, cmd, kv)
            with h.if_(c != 0):
                h.assign(ls1.dev[2:], q)
            with h.else_():
                h.assign(ls0.dev[2:], q)
            with h.if_(now & (act != 0)):
                h.send(Reply, to=h.node(client, c + 1), seq=q, result=x)
        with h.if_(now):
            h.assign(so.dev[2:], slot + 1)
    h.set("slotout", so)


def adopt(h, b):
    """A higher ballot steps this server down."""
    with h.if_(b > ballot(h)):
        h.set("round", b.shr(2))
        h.set("leader", b.band(3))
        h.set("active", 0)
        h.set("electing", 0)
        h.set("p1bvotes", 0)
        for j in range(SLOTS):
            h.set_at("votes", j, 0)
            h.set_at("p1blog", j, 0)


def choose(h, slot):
    """Marks the slot chosen and broadcasts the Decision (the handler's tail executes it)."""
    cmd = h.let(_n("ccmd"), ec(h.at("log", lit(slot) - 1)))
    h.set_at("log", lit(slot) - 1, mk(CHOSEN, 0, cmd))
    h.set_at("votes", lit(slot) - 1, 0)
    bcast(h, Decision, slot=slot, cmd=cmd)


def propose(h, slot, cmd):
    h.set_at("log", lit(slot) - 1, mk(ACCEPTED, ballot(h), cmd))
    h.set_at("votes", lit(slot) - 1, lit(1).shl(me(h)))
    bcast(h, P2a, round=h.f.round, leader=h.f.leader, slot=slot, cmd=cmd)
    with h.if_(majority(h, lit(1).shl(me(h)))):  # a one-server group
        choose(h, slot)


def merge(h, slot, e):
    """Phase-1 merge of one log entry: chosen wins, else the highest accepted ballot."""
    e = h.let(_n("me"), e)
    m = h.let(_n("mm"), h.at("p1blog", slot - 1))
    with h.if_(st(e) == CHOSEN):
        h.set_at("p1blog", slot - 1, mk(CHOSEN, 0, ec(e)))
    with h.else_():
        with h.if_((st(e) == ACCEPTED) & (st(m) != CHOSEN) & ((st(m) == EMPTY) | (eb(m) < eb(e)))):
            h.set_at("p1blog", slot - 1, e)


def become_leader(h):
    """Phase 1 complete: re-propose the merged log (chosen entries adopted, holes become no-ops);
    slotIn after the last used slot."""
    h.set("active", 1)
    h.set("electing", 0)
    h.set("p1bvotes", 0)
    merged = [h.let(_n("mg"), h.at("p1blog", j)) for j in range(SLOTS)]
    last = h.var(_n("last"), 0)
    for i in range(1, SLOTS + 1):
        with h.if_((st(merged[i - 1]) != EMPTY) | (st(h.at("log", i - 1)) != EMPTY)):
            h.assign(last.dev[2:], i)
    for j in range(SLOTS):
        h.set_at("p1blog", j, 0)
    for i in range(1, SLOTS + 1):
        m = merged[i - 1]
        with h.if_((lit(i) <= last) & (st(h.at("log", i - 1)) != CHOSEN)):
            with h.if_(st(m) == CHOSEN):
                h.set_at("log", i - 1, mk(CHOSEN, 0, ec(m)))
                h.set_at("votes", i - 1, 0)
            with h.else_():
                propose(h, i, select(st(m) == ACCEPTED, ec(m), 0))
    h.set("slotin", last + 1)


def executed(h, c0, q0):
    """The executed prefix (slots < slotOut): client c0's last executed sequence number and the
    result command (c0, q0) had (the AMO cache's entry)."""
    upto = h.let(_n("upto"), h.f.slotout)
    kv, ls0, ls1, r = h.var(_n("kv"), 0), h.var(_n("ls0"), 0), h.var(_n("ls1"), 0), h.var(_n("r"), 0)
    for slot in range(1, SLOTS + 1):
        cmd = h.let(_n("cmd"), ec(h.at("log", slot - 1)))
        c, q = h.let(_n("c"), cmd_client(cmd)), h.let(_n("q"), cmd_seq(cmd))
        with h.if_((lit(slot) < upto) & (cmd != 0) & (select(c, ls1, ls0) < q)):
            x = kv_apply(h, cmd, kv)
            with h.if_(c != 0):
                h.assign(ls1.dev[2:], q)
            with h.else_():
                h.assign(ls0.dev[2:], q)
            with h.if_((c == c0) & (q == q0)):
                h.assign(r.dev[2:], x)
    return r, select(c0, ls1, ls0)


# ---- servers ----------------------------------------------------------------------------------------
@server.init
def _server_init(h):
    h.set("slotout", 1)
    h.set("slotin", 1)
    with h.if_(me(h) == 0):
        h.set("active", 1)  # server1 leads ballot (0, server1)
    h.set_timer(Tick)


@server.on(Request)
def _request(h):
    cmd = h.let("cmd", h.msg.cmd)
    c, q = h.let("c", cmd_client(cmd)), h.let("q", cmd_seq(cmd))
    r, ls = executed(h, c, q)
    ls = h.let("ls", ls)
    with h.if_(ls >= q):  # AMO: already executed; an active leader replies from the cache
        with h.if_((h.f.active != 0) & (ls == q)):
            h.send(Reply, to=h.node(client, c + 1), seq=q, result=r)
        h.ret()
    slot, inlog = h.var("slot", h.f.slotin), h.var("inlog", 0)
    for k in range(1, SLOTS + 1):
        e = h.let(_n("e"), h.at("log", k - 1))
        with h.if_((st(e) != EMPTY) & (lit(k + 1) > slot)):
            h.assign("slot", k + 1)
        with h.if_((st(e) != EMPTY) & (ec(e) == cmd)):
            h.assign("inlog", 1)
    with h.if_((h.f.active == 0) | (slot > SLOTS) | (inlog != 0)):
        h.ret()
    h.set("slotin", slot + 1)
    propose(h, slot, cmd)
    with h.if_(majority(h, lit(1).shl(me(h)))):
        h.flag("exec")


@server.on(P2a)
def _p2a(h):
    b = h.let("b", mballot(h))
    with h.if_(b < ballot(h)):
        h.ret()
    adopt(h, b)
    h.set("heard", 1)
    slot = h.let("slot", h.msg.slot)
    with h.if_(st(h.at("log", slot - 1)) != CHOSEN):
        h.set_at("log", slot - 1, mk(ACCEPTED, b, h.msg.cmd))
    h.send(P2b, to=h.sender, round=h.msg.round, leader=h.msg.leader, slot=slot)


@server.on(P2b)
def _p2b(h):
    b, slot = h.let("b", mballot(h)), h.let("slot", h.msg.slot)
    with h.if_((h.f.active == 0) | (b != ballot(h)) | (st(h.at("log", slot - 1)) != ACCEPTED)):
        h.ret()
    v = h.let("v", h.at("votes", slot - 1).bor(lit(1).shl(h.sender - h.node(server, 1))))
    h.set_at("votes", slot - 1, v)
    with h.if_(~majority(h, v)):
        h.ret()
    choose(h, slot)
    h.flag("exec")


@server.on(Decision)
def _decision(h):
    slot = h.let("slot", h.msg.slot)
    with h.if_(st(h.at("log", slot - 1)) == CHOSEN):
        h.ret()
    h.set_at("log", slot - 1, mk(CHOSEN, 0, h.msg.cmd))
    h.set_at("votes", slot - 1, 0)
    h.flag("exec")


@server.on(Heartbeat)
def _heartbeat(h):
    b = h.let("b", mballot(h))
    with h.if_(b < ballot(h)):
        h.ret()
    adopt(h, b)
    h.set("heard", 1)


@server.on(P1a)
def _p1a(h):
    b = h.let("b", mballot(h))
    with h.if_(b < ballot(h)):
        h.ret()
    adopt(h, b)
    h.set("heard", 1)
    h.send(P1b, to=h.sender, round=h.msg.round, leader=h.msg.leader, l1=h.at("log", 0), l2=h.at("log", 1),
           l3=h.at("log", 2), l4=h.at("log", 3))


@server.on(P1b)
def _p1b(h):
    b = h.let("b", mballot(h))
    with h.if_((h.f.electing == 0) | (b != ballot(h))):
        h.ret()
    v = h.let("v", h.f.p1bvotes.bor(lit(1).shl(h.sender - h.node(server, 1))))
    h.set("p1bvotes", v)
    for k, f in enumerate(("l1", "l2", "l3", "l4")):
        merge(h, k + 1, getattr(h.msg, f))
    with h.if_(~majority(h, v)):
        h.ret()
    h.flag("lead")


@server.tail
def _server_tail(h):  # on_message's common tail: a completed phase 1, then execute (one copy each)
    with h.if_(h.flagged("lead")):
        become_leader(h)
    execute(h)


@server.on_timer(Tick)
def _tick(h):
    with h.if_(h.f.active != 0):
        bcast(h, Heartbeat, round=h.f.round, leader=h.f.leader)
    with h.else_():
        with h.if_(h.f.heard != 0):
            h.set("heard", 0)
            h.set("missed", 0)
        with h.else_():
            mis = h.let("mis", select(h.f.missed + 1 > 2, 2, h.f.missed + 1))
            h.set("missed", mis)
            with h.if_((mis >= 2) & (h.f.round < MAX_ROUND)):  # two ticks without the leader: phase 1
                h.set("missed", 0)
                h.set("heard", 0)
                h.set("round", h.f.round + 1)
                h.set("leader", me(h))
                h.set("electing", 1)
                h.set("active", 0)
                for j in range(SLOTS):
                    h.set_at("votes", j, 0)
                    h.set_at("p1blog", j, 0)
                h.set("p1bvotes", lit(1).shl(me(h)))
                for k in range(1, SLOTS + 1):
                    merge(h, k, h.at("log", k - 1))
                bcast(h, P1a, round=h.f.round, leader=h.f.leader)
                with h.if_(majority(h, lit(1).shl(me(h)))):  # a one-server group leads at once
                    become_leader(h)
                    execute(h)
    h.set_timer(Tick)


# no-op filters (the hand-written surely_noop, read off the handlers above)
@server.noop(Request)
def _n_request(h):
    return h.f.active == 0  # not the active leader: neither replies nor proposes


@server.noop(P2a)
def _n_p2a(h):
    return mballot(h) < ballot(h)


@server.noop(P1a)
def _n_p1a(h):
    return mballot(h) < ballot(h)


@server.noop(Heartbeat)
def _n_heartbeat(h):
    return (mballot(h) < ballot(h)) | ((mballot(h) == ballot(h)) & (h.f.heard != 0))


@server.noop(P2b)
def _n_p2b(h):
    v = h.at("votes", h.msg.slot - 1)
    counted = v.shr(h.sender - h.node(server, 1)).band(1) != 0
    return (h.f.active == 0) | (mballot(h) != ballot(h)) | (st(h.at("log", h.msg.slot - 1)) != ACCEPTED) | \
        (counted & ~majority(h, v))


@server.noop(Decision)
def _n_decision(h):
    return st(h.at("log", h.msg.slot - 1)) == CHOSEN


@server.noop(P1b)
def _n_p1b(h):
    return (h.f.electing == 0) | (mballot(h) != ballot(h))


# ---- clients (PaxosClient inside a ClientWorker) ----------------------------------------------------
def _broadcast_request(h, q):
    cid = h.let(_n("cid"), h.index(client) * 3 + q)  # 1 + 3 c + (q - 1)
    for j in range(3):
        with h.if_(lit(j) < h.count(server)):
            h.send(Request, to=h.node(server, j + 1), cmd=cid)


@client.send_command
def _send_command(h, cmd):
    h.set("seq", cmd)
    h.set("pending", 1)
    h.set("result", 0)
    _broadcast_request(h, cmd)
    h.set_timer(ClientTimer, seq=cmd)


@client.on(Reply)
def _reply(h):
    with h.if_((h.f.pending != 0) & (h.msg.seq == h.f.seq)):
        h.set("result", h.msg.result)
        h.set("pending", 0)


@client.on_timer(ClientTimer)
def _client_timer(h):
    with h.if_((h.f.pending != 0) & (h.timer.seq == h.f.seq)):
        _broadcast_request(h, h.timer.seq)
        h.set_timer(ClientTimer, seq=h.timer.seq)


@client.noop(Reply)
def _n_reply(h):  # a Reply the client does not take, with the ClientWorker loop idle
    takes = (h.f.pending != 0) & (h.msg.seq == h.f.seq)
    harvest = (h.length("_results") < h.wsize()) & (h.f.result != 0)
    return (~takes) & (~harvest)


# ---- predicates (PaxosTest.java:113-346; KVStoreWorkload.java:282-340) ------------------------------
def _kv_cmd(q, cmd):
    """PaxosServer.command(i) as a KV command code (op << 2 | value token; 0 = null)."""
    c = cmd_client(cmd)
    return select(lit(cmd) != 0, q.ptab("op", c, cmd_seq(cmd) - 1).shl(2).bor(q.ptab("val", c, cmd_seq(cmd) - 1)), 0)


@P.predicate("Non-empty log slots consistent", ids=[400, 401],
             names=["LOGS_CONSISTENT_ALL_SLOTS", "LOGS_CONSISTENT"], reads={"server": ["log"]})
def _logs_consistent(q):
    """slotValid (PaxosTest.java:215-279) for every slot: with no garbage collection LOGS_CONSISTENT
    and LOGS_CONSISTENT_ALL_SLOTS coincide, and slots past the last non-empty one are valid."""
    for slot in range(1, SLOTS + 1):
        is_chosen, conflict = q.var(_n("isch"), 0), q.var(_n("confl"), 0)
        chosen, count = q.var(_n("chosen"), 0), q.var(_n("count"), 0)
        for s in range(3):
            with q.if_(lit(s) < q.count(server)):
                e = q.let(_n("e"), q.at_node(server, s, "log", slot - 1))
                with q.if_(st(e) == CHOSEN):
                    x = q.let(_n("x"), _kv_cmd(q, ec(e)))
                    with q.if_((is_chosen != 0) & (x != chosen)):
                        q.assign(conflict.dev[2:], 1)
                    q.assign(chosen.dev[2:], x)
                    q.assign(is_chosen.dev[2:], 1)
        for s in range(3):
            with q.if_(lit(s) < q.count(server)):
                e = q.let(_n("e"), q.at_node(server, s, "log", slot - 1))
                with q.if_((st(e) != EMPTY) & ((st(e) != ACCEPTED) | (_kv_cmd(q, ec(e)) == chosen))):
                    q.assign(count.dev[2:], count + 1)
        with q.if_((is_chosen != 0) & ((conflict != 0) | (count * 2 <= q.count(server)))):
            q.ret(False)
    q.ret(True)


@P.predicate("Logs consistent for slot", ids=[402], names=["slotValid"], reads={"server": ["log"]}, nargs=1)
def _slot_valid(q):
    """PaxosTest.slotValid(st, i) (PaxosTest.java:215-279): no garbage collection, so a slot below
    1 is invalid (not CLEARED below firstNonCleared) and one past the log is EMPTY everywhere."""
    i = q.let("i", q.arg(0))
    with q.if_(i < 1):
        q.ret(False)
    with q.if_(i > SLOTS):
        q.ret(True)
    is_chosen, conflict = q.var("isch", 0), q.var("confl", 0)
    chosen, count = q.var("chosen", 0), q.var("count", 0)
    for s in range(3):
        with q.if_(lit(s) < q.count(server)):
            e = q.let(_n("e"), q.at_node(server, s, "log", i - 1))
            with q.if_(st(e) == CHOSEN):
                x = q.let(_n("x"), _kv_cmd(q, ec(e)))
                with q.if_((is_chosen != 0) & (x != chosen)):
                    q.assign("confl", 1)
                q.assign("chosen", x)
                q.assign("isch", 1)
    for s in range(3):
        with q.if_(lit(s) < q.count(server)):
            e = q.let(_n("e"), q.at_node(server, s, "log", i - 1))
            with q.if_((st(e) != EMPTY) & ((st(e) != ACCEPTED) | (_kv_cmd(q, ec(e)) == chosen))):
                q.assign("count", count + 1)
    with q.if_((is_chosen != 0) & ((conflict != 0) | (count * 2 <= q.count(server)))):
        q.ret(False)
    q.ret(True)


def _server_entry(q, code_shift):
    """The log entry of server arg0 (a node address; a non-server throws: the reference's
    (PaxosServer) st.server(a) cast) in slot arg1 >> code_shift (EMPTY outside the log)."""
    k = q.let(_n("k"), q.arg(0) - q.node(server, 1))
    with q.if_((k < 0) | (k >= q.count(server))):
        q.ret("threw")
    slot = q.let(_n("slot"), q.arg(1).shr(code_shift))
    e = q.var(_n("se"), 0)
    with q.if_((slot >= 1) & (slot <= SLOTS)):
        q.assign(e.dev[2:], q.at_node(server, k, "log", slot - 1))
    return e


@P.predicate("Server has status in slot", ids=[403], names=["hasStatus"], reads={"server": ["log"]}, nargs=2)
def _has_status(q):
    """PaxosTest.hasStatus(a, i, s) (PaxosTest.java:113-117): arg1 = i << 4 | status."""
    e = _server_entry(q, 4)
    with q.if_(st(e) == q.arg(1).band(15)):
        q.ret(True)
    q.ret(False)


@P.predicate("Server has command in slot", ids=[404], names=["hasCommand"], reads={"server": ["log"]}, nargs=2)
def _has_command(q):
    """PaxosTest.hasCommand(a, i, c) (PaxosTest.java:119-123): arg1 = i << 8 | KV command code
    (op << 2 | value token; 0 = null: an empty slot or a no-op)."""
    e = _server_entry(q, 8)
    c = q.let("cc", select(st(e) == EMPTY, 0, _kv_cmd(q, ec(e))))
    with q.if_(c == q.arg(1).band(255)):
        q.ret(True)
    q.ret(False)


@P.predicate("Sequence of appends to the same key is linearizable", ids=[300],
             names=["APPENDS_LINEARIZABLE"], reads={"client": ["_results"]})
def _appends_linearizable(q):
    """Clients in address order, their (command, result) pairs in order: a non-Append command
    throws; every result ends with its own value; no two results have equal length and each is a
    prefix of every longer one (pairwise: the sorted chain of the reference)."""
    items = []
    for c in range(2):
        for k in range(3):
            pres = q.let(_n("pres"), (lit(c) < q.count(client)) & (lit(k) < q.results_len(client, c)))
            with q.if_(pres & (q.ptab("op", c, k) != APPEND)):
                q.ret("threw")  # "Client workers have non-Append Commands"
            r = q.let(_n("res"), select(pres, q.result(client, c, k), 0))
            n = q.let(_n("rlen"), r.band(7))
            with q.if_(pres & ((n == 0) | (n > 4) | (r.shr(lit(1) + n * 2).band(3) != q.ptab("val", c, k)))):
                q.ret(False)
            items.append((pres, r, n))
    for (pa, ra, na), (pb, rb, nb) in itertools.combinations(items, 2):
        with q.if_(pa & pb):
            with q.if_(na == nb):
                q.ret(False)
            lo = select(na < nb, na, nb)
            mask = lit(1).shl(lo * 2) - 1
            with q.if_(ra.shr(3).band(mask) != rb.shr(3).band(mask)):
                q.ret(False)
    q.ret(True)
