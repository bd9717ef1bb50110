"""lab2 primary-backup with a ViewServer in the protocol IR -- BASELINE config C4's protocol, the
same one as csrc/protocols/pb.hpp and oracle/proto_pb.hpp, restated once here and
generated into both forms. It follows labs/lab2-primarybackup/README.md:154-330.

Nodes: "viewserver" (node 0), "server1..S" (nodes 1..S: a server's id in a view is its node index,
0 = null), "client1..c" after them (ClientWorkers around PBClients). ViewServer: the first pinging
server is primary of view 1; a server is dead when it did not ping between the last two
PingCheckTimers; a view changes only after its primary acknowledged it (Ping(current viewNum)); a
check replaces a dead primary by a live backup (stuck otherwise), drops a dead backup and fills a
missing backup from the lowest live idle server; a ping also fills a missing backup. PBServer: pings
every 25 ms with its latest view number (the last started one while it is the primary of a view whose
backup has not acknowledged the state transfer); a new view with it as primary and a backup sends
StateTransfer (the application: two key values, two AMO entries); the backup installs it once and
acknowledges; the primary serves requests once started, forwarding each to its backup and executing
it when the backup has. PBClient: lab1's client plus a cached view. KV values are len:2 | tokens 2 bits
each (at most 3); a result is type:2 | value << 2 (0 AppendResult, 1 GetResult, 2 KeyNotFound,
3 PutOk); an AMO entry is seq:2 | result:10.

Unlike the hand-written form, which keeps the ViewServer's highest ViewReply number as a field for
hasViewReply(n), the predicates here read the network (q.any_msg), as PrimaryBackupTest's do
(PrimaryBackupTest.java:104-156); the two forms have equal per-depth counts (the field is a
function of the network)."""
from ... import _lib
from ..core import Expr, Protocol, lit

P = Protocol("pb_ir", _lib.DSL_PROTO_PB_IR, "PBIR", doc=__doc__)
P.param("servers", 2, 1, 3)
P.param("clients", 1, 1, 2)
P.param("ncmds", 2, 1, 3)
P.param_table("op", 2, 3, 0, 2)       # 0 Get, 1 Put, 2 Append
P.param_table("key", 2, 3, 0, 1)
P.param_table("sym", 2, 3, 0, 3)
P.param_table("expected", 2, 3, -1, 1023, default=-1)
P.workload_size = "ncmds"
P.expected_result = lambda c, k: Expr(f"sel_param(p.expected, {c.dev}, {k.dev} - 1)",
                                      f"prm.expected[{c.orc}][{k.orc} - 1]")
P.net_cap = 64
P.max_sends = 3
OP_GET, OP_PUT, OP_APPEND = 0, 1, 2
R_APPEND, R_GET, R_NOTFOUND, R_PUTOK = 0, 1, 2, 3
MAX_VIEW = 15

# message types in the hand-written protocol's order (its handler classes)
Ping = P.message("Ping", num=4)
GetView = P.message("GetView")
ViewReply = P.message("ViewReply", num=4, p=2, b=2)
Request = P.message("Request", seq=2)
Reply = P.message("Reply", seq=2, result=10)
StateTransfer = P.message("StateTransfer", num=4, p=2, b=2, kv0=8, kv1=8, amo0=12, amo1=12)
StateTransferAck = P.message("StateTransferAck", num=4)
Forward = P.message("Forward", num=4, client=3, seq=2)
ForwardAck = P.message("ForwardAck", num=4, client=3, seq=2)
PingCheckTimer = P.timer("PingCheckTimer", (100, 100))
PingTimer = P.timer("PingTimer", (25, 25))
ClientTimer = P.timer("ClientTimer", (100, 100), seq=2)

vs = P.node("viewserver", count=1, max_count=1, single_name="viewserver",
            vnum=4, vp=2, vb=2, acked=1, recent=3, alive=3)
vs.timer_cap = 2  # [PingCheckTimer], plus the re-set one until the fired entry is removed
server = P.node("server", count="servers", max_count=3, arrays={"kv": (8, 2), "amo": (12, 2)},
                vnum=4, vp=2, vb=2, started=1, last=4)
server.timer_cap = 2
client = P.client_worker("client", count="clients", max_count=2, result_field="result", results_cap=3, timer_cap=4,
                         cvnum=4, cprim=2, seq=2, result=10)


def view_bits(num, p, b):
    return lit(num).bor(lit(p).shl(4)).bor(lit(b).shl(6))


# ---- ViewServer ------------------------------------------------------------------------------------
def _idle(h, alive, p, b, name):
    """The lowest live server other than p and b (0: none)."""
    h.var(name, 0)
    for s in (3, 2, 1):  # the last assignment is the lowest
        with h.if_((lit(s) <= h.param("servers")) & (alive.shr(s - 1).band(1) == 1) & (lit(s) != p) & (lit(s) != b)):
            h.assign(name, s)
    return Expr("l_" + name, "l_" + name)


def _new_view(h, p, b):
    with h.if_(h.f.vnum + 1 > MAX_VIEW):
        h.overflow("view number past 15")
    h.set("vnum", h.f.vnum + 1)
    h.set("vp", p)
    h.set("vb", b)
    h.set("acked", 0)


@vs.init
def _vs_init(h):
    h.set_timer(PingCheckTimer)


@vs.on(Ping)
def _vs_ping(h):
    frm = h.let("frm", h.sender)
    with h.if_((frm < 1) | (frm > h.param("servers"))):
        h.throw("Ping from a node that is not a server")
    h.set("recent", h.f.recent.bor(lit(1).shl(frm - 1)))
    with h.if_(h.f.vnum == 0):  # any server may be the first primary
        h.set("vnum", 1)
        h.set("vp", frm)
        h.set("vb", 0)
        h.set("acked", 0)
    with h.if_((frm == h.f.vp) & (h.msg.num == h.f.vnum)):
        h.set("acked", 1)
    with h.if_((h.f.acked == 1) & (h.f.vb == 0)):
        live = h.let("live", h.f.recent.bor(h.f.alive))
        s = _idle(h, live, h.f.vp, 0, "pidle")
        with h.if_(s != 0):
            _new_view(h, h.f.vp, s)
    h.send(ViewReply, to=frm, num=h.f.vnum, p=h.f.vp, b=h.f.vb)


@vs.on(GetView)
def _vs_getview(h):
    h.send(ViewReply, to=h.sender, num=h.f.vnum, p=h.f.vp, b=h.f.vb)


@vs.on_timer(PingCheckTimer)
def _vs_check(h):
    alive = h.let("alv", h.f.recent)
    h.set("alive", alive)
    h.set("recent", 0)
    with h.if_((h.f.acked == 1) & (h.f.vnum != 0)):
        pp = h.let("pp", h.f.vp)
        bb = h.let("bb", h.f.vb)
        p_alive = h.let("palive", alive.shr(pp - 1).band(1))
        b_alive = h.let("balive", (bb != 0) & (alive.shr(bb - 1).band(1) == 1))
        with h.if_(p_alive == 0):
            with h.if_(b_alive):
                s1 = _idle(h, alive, bb, 0, "cidle1")
                _new_view(h, bb, s1)
        with h.if_((p_alive == 1) & (bb != 0) & ~b_alive):
            s2 = _idle(h, alive, pp, 0, "cidle2")
            _new_view(h, pp, s2)
        with h.if_((p_alive == 1) & (bb == 0)):
            s3 = _idle(h, alive, pp, 0, "cidle3")
            with h.if_(s3 != 0):
                _new_view(h, pp, s3)
    h.set_timer(PingCheckTimer)


# ---- PBServer ----------------------------------------------------------------------------------------
def _execute(h, c, seq, r):
    """AMOApplication(KVStore).execute of client c's command seq into local r: the result, or -1
    for a superseded command."""
    amo = h.let("amo", h.at("amo", c))
    last = h.let("lastseq", amo.band(3))
    h.assign(r, -1)
    with h.if_(seq == last):
        h.assign(r, amo.shr(2))
    with h.if_(seq > last):
        k = h.let("k", seq - 1)
        op = h.let("op", h.ptab("op", c, k))
        key = h.let("key", h.ptab("key", c, k))
        sym = h.let("sym", h.ptab("sym", c, k))
        v = h.let("v", h.at("kv", key))
        with h.if_(op == OP_GET):
            with h.if_(v.band(3) != 0):
                h.assign(r, v.shl(2).bor(R_GET))
            with h.else_():
                h.assign(r, R_NOTFOUND)
        with h.if_(op == OP_PUT):
            h.set_at("kv", key, sym.shl(2).bor(1))
            h.assign(r, R_PUTOK)
        with h.if_(op == OP_APPEND):
            n = h.let("n", v.band(3))
            with h.if_(n >= 3):
                h.overflow("value longer than 3 tokens")
            v2 = h.let("v2", (v - n).bor(n + 1).bor(sym.shl((n * 2) + 2)))
            h.set_at("kv", key, v2)
            h.assign(r, v2.shl(2))  # AppendResult (type 0)
        h.set_at("amo", c, seq.bor(Expr("l_" + r, "l_" + r).shl(2)))


@server.init
def _server_init(h):
    h.send(Ping, to=h.node(vs, 1), num=0)
    h.set_timer(PingTimer)


@server.on(ViewReply)
def _server_viewreply(h):
    with h.if_(h.msg.num <= h.f.vnum):
        h.ret()
    h.set("vnum", h.msg.num)
    h.set("vp", h.msg.p)
    h.set("vb", h.msg.b)
    h.set("started", 0)
    with h.if_(h.msg.p == h.self):
        with h.if_(h.msg.b == 0):
            h.set("started", 1)
            h.set("last", h.msg.num)
        with h.else_():
            h.send(StateTransfer, to=h.msg.b, num=h.msg.num, p=h.msg.p, b=h.msg.b, kv0=h.at("kv", 0),
                   kv1=h.at("kv", 1), amo0=h.at("amo", 0), amo1=h.at("amo", 1))


@server.on(StateTransfer)
def _server_st(h):
    with h.if_((h.msg.num < h.f.vnum) | (h.msg.b != h.self) | (h.msg.p != h.sender)):
        h.ret()
    # a backup installs a view's state once: a redelivered transfer must not undo what was forwarded since
    with h.if_((h.msg.num == h.f.vnum) & (h.f.started == 1)):
        h.ret()
    h.set("vnum", h.msg.num)
    h.set("vp", h.msg.p)
    h.set("vb", h.msg.b)
    h.set("started", 1)
    h.set_at("kv", 0, h.msg.kv0)
    h.set_at("kv", 1, h.msg.kv1)
    h.set_at("amo", 0, h.msg.amo0)
    h.set_at("amo", 1, h.msg.amo1)
    h.send(StateTransferAck, to=h.sender, num=h.msg.num)


@server.on(StateTransferAck)
def _server_stack(h):
    with h.if_((h.f.vp == h.self) & (h.f.started == 0) & (h.msg.num == h.f.vnum)):
        h.set("started", 1)
        h.set("last", h.f.vnum)


@server.on(Request)
def _server_request(h):
    seq = h.let("seq", h.msg.seq)
    c = h.let("c", h.sender - h.node(client, 1))
    with h.if_((c < 0) | (c >= h.param("clients")) | (seq < 1) | (seq > h.param("ncmds"))):
        h.throw("request from an unknown client or command")
    with h.if_((h.f.vp != h.self) | (h.f.started == 0)):
        h.ret()
    with h.if_(h.f.vb == 0):
        r = h.var("r", -1)
        _execute(h, c, seq, "r")
        with h.if_(r >= 0):
            h.send(Reply, to=h.sender, seq=seq, result=r)
    with h.else_():
        h.send(Forward, to=h.f.vb, num=h.f.vnum, client=h.sender, seq=seq)


def _forward_checks(h):
    seq = h.let("seq", h.msg.seq)
    ca = h.let("ca", h.msg.client)
    c = h.let("c", ca - h.node(client, 1))
    with h.if_((c < 0) | (c >= h.param("clients")) | (seq < 1) | (seq > h.param("ncmds"))):
        h.throw("forward of an unknown client or command")
    return seq, ca, c


@server.on(Forward)
def _server_forward(h):
    seq, ca, c = _forward_checks(h)
    with h.if_((h.f.vnum != h.msg.num) | (h.f.vb != h.self) | (h.f.vp != h.sender)):
        h.ret()
    r = h.var("r", -1)
    _execute(h, c, seq, "r")
    h.send(ForwardAck, to=h.sender, num=h.msg.num, client=ca, seq=seq)


@server.on(ForwardAck)
def _server_forwardack(h):
    seq, ca, c = _forward_checks(h)
    with h.if_((h.f.vp != h.self) | (h.f.started == 0) | (h.f.vnum != h.msg.num)):
        h.ret()
    r = h.var("r", -1)
    _execute(h, c, seq, "r")
    with h.if_(r >= 0):
        h.send(Reply, to=ca, seq=seq, result=r)


@server.on_timer(PingTimer)
def _server_ping(h):  # the latest view, unless primary of a view not yet started
    n = h.let("n", h.f.vnum)
    with h.if_((h.f.vp == h.self) & (h.f.started == 0)):
        h.send(Ping, to=h.node(vs, 1), num=h.f.last)
    with h.else_():
        h.send(Ping, to=h.node(vs, 1), num=n)
    h.set_timer(PingTimer)


# ---- PBClient (inside a ClientWorker) ------------------------------------------------------------------
def _send_pending(h, seq):
    with h.if_(h.f.cprim != 0):
        h.send(Request, to=h.f.cprim, seq=seq)
    with h.else_():
        h.send(GetView, to=h.node(vs, 1))


@client.send_command
def _send_command(h, cmd):  # PBClient.sendCommand: seq = cmd, the request (or GetView), ClientTimer
    h.set("seq", cmd)
    h.set("result", 0)
    _send_pending(h, cmd)
    h.set_timer(ClientTimer, seq=cmd)


@client.on(ViewReply)
def _client_viewreply(h):
    with h.if_(h.msg.num > h.f.cvnum):
        h.set("cvnum", h.msg.num)
        h.set("cprim", h.msg.p)
        with h.if_((h.f.seq > 0) & (h.f.result == 0)):
            _send_pending(h, h.f.seq)


@client.on(Reply)
def _client_reply(h):
    with h.if_((h.f.seq > 0) & (h.f.result == 0) & (h.msg.seq == h.f.seq)):
        h.set("result", h.msg.result)


@client.on_timer(ClientTimer)
def _client_timer(h):  # re-ask the ViewServer and re-send while the command is pending
    with h.if_((h.f.seq > 0) & (h.f.result == 0) & (h.timer.seq == h.f.seq)):
        h.send(GetView, to=h.node(vs, 1))
        with h.if_(h.f.cprim != 0):
            h.send(Request, to=h.f.cprim, seq=h.timer.seq)
        h.set_timer(ClientTimer, seq=h.timer.seq)


# ---- predicates (PrimaryBackupTest.java:104-156): network predicates ----------------------------------
@P.predicate("ViewReply with viewNum", [500], ["hasViewReply"], {}, nargs=1, network=True)
def _has_view_reply(q):  # hasViewReply(n): a ViewReply with viewNum >= n
    with q.if_(q.any_msg(ViewReply, lambda m: m.num >= q.arg(0))):
        q.ret(True)
    q.ret(False)


@P.predicate("ViewReply with View", [501], ["hasViewReplyExact"], {}, nargs=1, network=True)
def _has_view_reply_exact(q):  # hasViewReply(n, p, b): a ViewReply with exactly that view (num | p << 4 | b << 6)
    with q.if_(q.any_msg(ViewReply, lambda m: view_bits(m.num, m.p, m.b) == q.arg(0))):
        q.ret(True)
    q.ret(False)


@P.predicate("ViewReply for View sent to nodes, primary ack sent", [502], ["viewRepliesSent"], {}, nargs=2,
             network=True)
def _view_replies_sent(q):  # initView's goal: the view's replies to every node of mask arg1, the primary's ack
    view = q.let("view", q.arg(0))
    prim = q.let("prim", view.shr(4).band(3))
    num = q.let("num", view.band(15))
    with q.if_(~q.any_msg(Ping, lambda m: (m.sender == prim) & (m.to == 0) & (m.num == num))):
        q.ret(False)
    for j in range(1 + 3 + 2):  # every node index of the largest run (viewserver, 3 servers, 2 clients)
        with q.if_((q.arg(1).shr(j).band(1) == 1) &
                   ~q.any_msg(ViewReply, lambda m, j=j: (m.to == j) & (view_bits(m.num, m.p, m.b) == view))):
            q.ret(False)
    q.ret(True)
