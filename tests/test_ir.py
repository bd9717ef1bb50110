"""The protocol IR (dslabs_amd/ir): PingPong generated from dslabs_amd/ir/specs/pingpong.py into the
device form (csrc/protocols/gen/pingpong_ir.hpp) and the oracle's object form
(oracle/gen/proto_pingpong_ir.hpp) reproduces the hand-written protocol's golden vectors -- the
reference-pinned lab0 numbers (README 120 states / depth 29, 84 at the goal level, the mutant's
depth-3 violation) included -- on the oracle, on the host-compiled device form (exact-equality
host BFS, tests/hostcheck) and on the multithreaded CPU baseline over the same device code."""
import json
import os
import subprocess
import sys

import pytest

import argmap
import oracle_util
from test_hostcheck import _X, protocheck, run  # noqa: F401  (fixture)
from tools import cpu_baseline

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LAB0 = json.load(open(os.path.join(HERE, "golden", "lab0.json")))
KV = json.load(open(os.path.join(HERE, "golden", "amokv.json")))
# AMO-KV fixtures whose predicates the IR covers (RESULTS_OK / CLIENTS_DONE; not APPENDS_LINEARIZABLE)
KV_NAMES = sorted(n for n in KV if "APPENDS_LINEARIZABLE" not in KV[n]["args"])
# the engine finishes a terminal's level (--finish-level fixtures) or exhausts the space
NAMES = sorted(n for n in LAB0 if "--finish-level" in LAB0[n]["args"] or LAB0[n]["end"] == "SPACE_EXHAUSTED")


def _ir_args(args):
    return ["pingpong_ir" if a == "pingpong" else a for a in args]


def test_generated_files_are_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_ir.py"), "--check"], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout


@pytest.mark.parametrize("name", sorted(LAB0))
def test_ir_oracle_matches_handwritten(name):
    case = LAB0[name]
    r = oracle_util.run("bfs", _ir_args(case["args"]), timeout=300)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]
    assert r["states"] == case["states"]


@pytest.mark.parametrize("name", NAMES)
def test_ir_device_form_on_cpu(name):
    """The generated device handlers in the multithreaded CPU BFS (tools/cpu_bfs.cpp)."""
    case = LAB0[name]
    args = _ir_args(case["args"])
    proto = argmap.protocol(args)
    r = cpu_baseline.run(proto, argmap.settings(args, proto, table_log2=20), threads=2)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]


@pytest.mark.parametrize("ps,oracle_args", [
    ([8, 1, 10, 1, 1, "--", 1, "/", "/", 2, -1],
     ["--proto", "pingpong", "--clients", "1", "--pings", "10", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE"]),
    ([8, 2, 4, 1, 0, "--", 1, "/", "/", 2, -1],
     ["--proto", "pingpong", "--clients", "2", "--pings", "4", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE",
      "--mutant-no-reset"]),
])
def test_ir_device_form_host_bfs(protocheck, ps, oracle_args):  # noqa: F811
    """Exact-equality host BFS over the generated handlers, with the incremental fingerprint,
    row emission and judge cross-checks of tests/hostcheck."""
    got = run(protocheck, ps)
    want = oracle_util.run("bfs", oracle_args)
    assert got["per_depth"] == want["per_depth"]
    assert got["fp_mismatch"] == 0 and got["emit_mismatch"] == 0 and got["judge_mismatch"] == 0


def _kv_ir(args):
    from dslabs_amd.protocols import AmoKVIR
    c, wl = int(args[args.index("--clients") + 1]), args[args.index("--workload") + 1]
    rest, i = [], 0
    while i < len(args):
        if args[i] in ("--proto", "--clients", "--workload"):
            i += 2
            continue
        rest.append(args[i])
        i += 1
    return AmoKVIR(c, wl), rest


@pytest.mark.parametrize("name", KV_NAMES)
def test_ir_amokv_oracle_matches_golden(name):
    case = KV[name]
    proto, rest = _kv_ir(case["args"])
    r = oracle_util.run("bfs", proto.oracle_args() + rest, timeout=600)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]


@pytest.mark.parametrize("name", KV_NAMES)
def test_ir_amokv_device_form_on_cpu(name):
    case = KV[name]
    if "--finish-level" not in case["args"] and case["end"] != "SPACE_EXHAUSTED":
        pytest.skip("the oracle stopped mid-level (no --finish-level)")
    proto, rest = _kv_ir(case["args"])
    r = cpu_baseline.run(proto, argmap.settings(rest, proto, table_log2=22), threads=2)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]


# ---- lab3 Multi-Paxos (BASELINE C5's protocol) from the IR: dslabs_amd/ir/specs/multipaxos.py ------------------
MP = json.load(open(os.path.join(HERE, "golden", "multipaxos.json")))
# the IR oracle runs the whole C5 d12 space in minutes: it gets d8, the CPU BFS below d12
MP_ORACLE = sorted(n for n in MP if n != "mp_c5_d12")


def _mp_ir(args):
    """The IR protocol for a multipaxos fixture's --servers / --clients / --workload, and the rest of
    its arguments (predicates, settings)."""
    from dslabs_amd.protocols import MultiPaxosIR
    opt = lambda n, d: args[args.index(n) + 1] if n in args else d  # noqa: E731
    proto = MultiPaxosIR(int(opt("--servers", 3)), int(opt("--clients", 2)), opt("--workload", "append-xy"))
    rest, i = [], 0
    while i < len(args):
        if args[i] in ("--proto", "--servers", "--clients", "--workload"):
            i += 2
            continue
        rest.append(args[i])
        i += 1
    return proto, rest


@pytest.mark.parametrize("name", MP_ORACLE)
def test_ir_multipaxos_oracle_matches_golden(name):
    """The IR's oracle form against the hand-written protocol's golden vectors (both oracle forms
    are independent restatements; the fixtures came from oracle/proto_multipaxos.hpp)."""
    case = MP[name]
    proto, rest = _mp_ir(case["args"])
    r = oracle_util.run("bfs", proto.oracle_args() + rest, timeout=600)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]  # with --finish-level: the terminal's depth is the last one


@pytest.mark.parametrize("name", sorted(MP))
def test_ir_multipaxos_device_form_on_cpu(name):
    """The generated device handlers, predicates and no-op filter in the multithreaded CPU BFS --
    BASELINE C5 at its full depth 12 included."""
    case = MP[name]
    proto, rest = _mp_ir(case["args"])
    r = cpu_baseline.run(proto, argmap.settings(rest, proto, table_log2=22), threads=4)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]


@pytest.mark.parametrize("servers,clients,workload,tail", [
    (3, 2, "append-xy", ["--", 1, 400, 300, "/", "/", 9]),
    (3, 2, "append-xz", ["--", 1, 401, 300, "/", "/", 7]),
    (2, 1, "append-x", ["--", 1, 400, 300, "/", "/", 2, 11]),
    (1, 1, "put-append-get", ["--", 1, "/", "/", 2, -1]),
])
def test_ir_multipaxos_device_form_host_bfs(protocheck, servers, clients, workload, tail):  # noqa: F811
    """Exact-equality host BFS over the generated Multi-Paxos: per-depth counts equal the
    hand-written protocol's on the oracle, and the incremental fingerprint, row emission,
    incremental judge (the predicates' declared read sets) and the generated no-op filter are
    cross-checked on every successor."""
    from dslabs_amd.protocols import MultiPaxos, MultiPaxosIR
    got = run(protocheck, [10] + MultiPaxosIR(servers, clients, workload).params() + tail)
    want = run(protocheck, [5] + MultiPaxos(servers, clients, workload).params() + tail)
    assert got["per_depth"] == want["per_depth"]
    assert got["end"] == want["end"]
    assert got["fp_mismatch"] == 0 and got["emit_mismatch"] == 0 and got["judge_mismatch"] == 0
    assert got["skip_mismatch"] == 0 and got["skipped"] > 0  # the generated no-op filter is sound and used
    assert got["dup_sends"] == 0  # the spec's sends_distinct (the Sender skips its duplicate check)


# ---- lab2 primary-backup + ViewServer (BASELINE C4's protocol) from the IR: dslabs_amd/ir/specs/pb.py ---------
PBG = json.load(open(os.path.join(HERE, "golden", "pb.json")))
_PB_LEAF = r"(hasViewReply|viewRepliesSent)(:[^,()]+)"


def _pb_ir(args):
    """The IR protocol for a pb.json fixture's --servers / --clients / --workload, and the rest of its
    arguments (predicates, settings, network shape)."""
    from dslabs_amd.protocols import PBIR
    opt = lambda n, d: args[args.index(n) + 1] if n in args else d  # noqa: E731
    proto = PBIR(int(opt("--servers", 2)), int(opt("--clients", 1)), opt("--workload", "putget"))
    rest, i = [], 0
    while i < len(args):
        if args[i] in ("--proto", "--servers", "--clients", "--workload"):
            i += 2
            continue
        rest.append(args[i])
        i += 1
    return proto, rest


def _pb_oracle_args(proto, rest):
    """The fixture's arguments for the IR oracle: PB's predicate leaves (hasViewReply:n[:p:b],
    viewRepliesSent:...) spelled as the spec's network predicates (PBIR.ir_oracle_name)."""
    import re
    out = []
    for k, a in enumerate(rest):
        if k and rest[k - 1] in ("--inv", "--goal", "--prune"):
            a = re.sub(_PB_LEAF, lambda m: proto.ir_oracle_name(m.group(0)), a)
        out.append(a)
    return proto.oracle_args() + out


@pytest.mark.parametrize("name", sorted(PBG))
def test_ir_pb_oracle_matches_golden(name):
    """The IR's oracle form (argument and network predicates included) against the hand-written
    protocol's golden vectors -- initView's network-off search with its viewRepliesSent goal among them."""
    case = PBG[name]
    proto, rest = _pb_ir(case["args"])
    r = oracle_util.run("bfs", _pb_oracle_args(proto, rest), timeout=600)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]
    assert r["states"] == case["states"]


@pytest.mark.parametrize("name", sorted(PBG))
def test_ir_pb_device_form_on_cpu(name):
    """The generated PB device handlers and predicates in the multithreaded CPU BFS."""
    case = PBG[name]
    proto, rest = _pb_ir(case["args"])
    r = cpu_baseline.run(proto, argmap.settings(rest, proto, table_log2=22), threads=4)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]


@pytest.mark.parametrize("servers,clients,workload,tail", [
    (2, 1, "putget", ["--", 1, "/", "/", 2, "500:4", 13]),
    (3, 1, "putget", ["--", 1, "/", "/", 2, "500:3", 10]),
    (2, 2, "appendappendget", ["--", 1, "/", "/", 2, "500:3", 9]),
])
def test_ir_pb_device_form_host_bfs(protocheck, servers, clients, workload, tail):  # noqa: F811
    """Exact-equality host BFS over the generated PB against the hand-written PB (tests/hostcheck,
    protocol 6) on the same predicates: per-depth counts, and the incremental fingerprint, row
    emission and incremental judge of the generated form on every successor."""
    from dslabs_amd.protocols import PB, PBIR
    got = run(protocheck, [11] + PBIR(servers, clients, workload).params() + tail)
    want = run(protocheck, [6] + PB(servers, clients, workload).params() + tail)
    assert got["per_depth"] == want["per_depth"]
    assert got["end"] == want["end"]
    assert got["fp_mismatch"] == 0 and got["emit_mismatch"] == 0 and got["judge_mismatch"] == 0


# ---- lab3 argument predicates on the IR Multi-Paxos: slotValid(i), hasStatus(a, i, s), hasCommand(a, i, c) ---------
_MP_LEAF = r"(slotValid|hasStatus|hasCommand)(:[^,()]+)"


def _mp_oracle_args(proto, rest):
    """The arguments for the IR oracle: PaxosTest's predicate leaves as the spec's NAME:arg0[:arg1]."""
    import re
    out = []
    for k, a in enumerate(rest):
        if k and rest[k - 1] in ("--inv", "--goal", "--prune"):
            a = re.sub(_MP_LEAF, lambda m: proto.ir_oracle_name(m.group(0)), a)
        out.append(a)
    return proto.oracle_args() + out


def _lab3_cases():
    from test_gpu_multipaxos import LIVE
    return LIVE


@pytest.mark.parametrize("name", sorted(_lab3_cases()))
def test_ir_multipaxos_lab3_predicates(name):
    """PaxosTest's predicate flows (the hand-written protocol's lab3 cases, PaxosTest.java:113-346,
    test27 included): the IR oracle and the generated device form in the CPU BFS against the
    hand-written protocol on the oracle, per depth."""
    args = _lab3_cases()[name] + ["--finish-level"]
    if "--max-depth" in args:  # the CPU suite stops at depth 8 (the GPU test runs the fixture's depth)
        i = args.index("--max-depth") + 1
        args = args[:i] + [str(min(8, int(args[i])))] + args[i + 1:]
    want = oracle_util.run("bfs", args, timeout=300)
    proto, rest = _mp_ir(args)
    got = oracle_util.run("bfs", _mp_oracle_args(proto, rest), timeout=300)
    assert got["end"] == want["end"] and got["per_depth"] == want["per_depth"]
    r = cpu_baseline.run(proto, argmap.settings(rest, proto, table_log2=20), threads=4)
    assert r["end"] == want["end"] and r["per_depth"] == want["per_depth"]


@pytest.mark.parametrize("tail", [
    ["--", 1, 401, "/", f"403:1:{(1 << 4) | 2}", "/", 10],
    ["--", f"403:0:{(1 << 4) | 2},not,404:0:{(1 << 8) | _X},or", "402:1", "/", "/", 10],
    ["--", 400, "/", f"403:0:{(2 << 4) | 2},403:1:{(2 << 4) | 1},-403:2:{(2 << 4) | 0},or,and", "/", 9],
    ["--", "402:1,402:2,and", "402:0,not", "/", "/", 8],
])
def test_ir_multipaxos_lab3_predicates_host_bfs(protocheck, tail):  # noqa: F811
    """Exact host BFS: the generated argument predicates against the hand-written ones
    (tests/hostcheck, protocols 10 and 5), with the incremental judge cross-checked on every
    successor (their declared read set: the servers' logs)."""
    from dslabs_amd.protocols import MultiPaxos, MultiPaxosIR
    got = run(protocheck, [10] + MultiPaxosIR(3, 2, "append-xy").params() + tail)
    want = run(protocheck, [5] + MultiPaxos(3, 2, "append-xy").params() + tail)
    assert got["per_depth"] == want["per_depth"] and got["end"] == want["end"]
    assert got["terminals_at_depth"] == want["terminals_at_depth"]
    assert got["fp_mismatch"] == 0 and got["emit_mismatch"] == 0 and got["judge_mismatch"] == 0
