"""lab0 PingPong in the protocol IR (the same protocol as csrc/protocols/pingpong.hpp, restated):
labs/lab0-pingpong/src/dslabs/pingpong/PingServer.java:29-32 (handlePingRequest),
PingClient.java:41-87 (sendCommand / handlePongReply / onPingTimer), Timers.java:7-11
(PingTimer, RETRY_MILLIS = 10 ms), inside ClientWorker with PingTest's repeatedPings workload
(tst/dslabs/pingpong/PingTest.java:44-51): command k is Ping(k), its expected result Pong(k). The
README mutants are parameters (README.md:299-306 no timer re-set, :342-347 no value check)."""
from ... import _lib
from ..core import Protocol

P = Protocol("pingpong_ir", _lib.DSL_PROTO_PINGPONG_IR, "PingPongIR", doc=__doc__)
P.param("clients", 1, 1, 4)
P.param("pings", 10, 1, 15)
P.param("check_value", 1, 0, 1)
P.param("reset_timer", 1, 0, 1)
P.workload_size = "pings"
P.expected_result = lambda c, k: k
P.net_cap = 120
P.max_sends = 2

PingRequest = P.message("PingRequest", value=4)
PongReply = P.message("PongReply", value=4)
PingTimer = P.timer("PingTimer", (10, 10), value=4)

server = P.node("pingserver", count=1, max_count=1, single_name="pingserver")
client = P.client_worker("client", count="clients", max_count=4, result_field="pong", results_cap=15, timer_cap=15,
                         ping=4, pong=4)


@server.on(PingRequest)
def _handle_ping(h):  # PingServer.handlePingRequest: Pong(value) back to the sender
    h.send(PongReply, to=h.sender, value=h.msg.value)


@client.send_command
def _send_command(h, cmd):  # PingClient.sendCommand
    h.set("ping", cmd)
    h.set("pong", 0)
    h.send(PingRequest, to=h.node(server, 1), value=cmd)
    h.set_timer(PingTimer, value=cmd)


@client.on(PongReply)
def _handle_pong(h):  # PingClient.handlePongReply
    with h.if_((h.param("check_value") == 0) | (h.f.ping == h.msg.value)):
        h.set("pong", h.msg.value)


@client.on_timer(PingTimer)
def _on_ping_timer(h):  # PingClient.onPingTimer
    with h.if_((h.f.ping == h.timer.value) & (h.f.pong == 0)):
        h.send(PingRequest, to=h.node(server, 1), value=h.timer.value)
        with h.if_(h.param("reset_timer") != 0):
            h.set_timer(PingTimer, value=h.timer.value)
