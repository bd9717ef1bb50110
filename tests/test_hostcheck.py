"""Protocol ENCODINGS (packed-state transition functions, host-compiled) vs the oracle.

This checks the device protocols' semantics on CPU; the kernels themselves are checked by the
-m gpu tests. tests/hostcheck/protocheck.cpp is a test tool, never part of the product."""
import json
import os
import subprocess

import pytest

import oracle_util
from dslabs_amd.protocols import MultiPaxos

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mp(servers, clients, workload):
    """protocheck's protocol arguments for Multi-Paxos: the id, then the engine's parameters."""
    return [5] + MultiPaxos(servers, clients, workload).params()


_MP3 = ["--inv", "RESULTS_OK", "--inv", "LOGS_CONSISTENT_ALL_SLOTS", "--inv", "APPENDS_LINEARIZABLE"]
_PAG = mp(1, 1, "put-append-get")
_X = MultiPaxos(3, 2, "append-xy").kv_code("APPEND:foo:X")
SRC = os.path.join(ROOT, "tests", "hostcheck", "protocheck.cpp")
BIN = os.path.join(ROOT, "tests", "hostcheck", "_build", "protocheck")


@pytest.fixture(scope="module")
def protocheck():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    deps = [SRC] + [os.path.join(dp, f) for dp, _, fs in os.walk(os.path.join(ROOT, "dslabs_amd", "csrc"))
                    for f in fs]
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(os.path.getmtime(d) for d in deps):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-Wno-unused-result", "-o", BIN, SRC],
                       check=True)
    return BIN


def run(bin_, args):
    out = subprocess.run([bin_] + [str(a) for a in args], check=True, capture_output=True, text=True, timeout=600)
    return json.loads(out.stdout)


# (protocheck args, oracle args)
CASES = {
    "pp_1c10p": ([1, 1, 10, 1, 1, "--", 1, "/", "/", 2, -1],
                 ["--proto", "pingpong", "--clients", "1", "--pings", "10", "--inv", "RESULTS_OK", "--prune",
                  "CLIENTS_DONE"]),
    "pp_3c3p": ([1, 3, 3, 1, 1, "--", 1, "/", "/", 2, -1],
                ["--proto", "pingpong", "--clients", "3", "--pings", "3", "--inv", "RESULTS_OK", "--prune",
                 "CLIENTS_DONE"]),
    "pp_mutant_noreset": ([1, 2, 3, 1, 0, "--", 1, "/", "/", 2, -1],
                          ["--proto", "pingpong", "--clients", "2", "--pings", "3", "--inv", "RESULTS_OK",
                           "--prune", "CLIENTS_DONE", "--mutant-no-reset"]),
    "pp_mutant_nocheck": ([1, 1, 10, 0, 1, "--", 1, "/", 2, "/", -1],
                          ["--proto", "pingpong", "--clients", "1", "--pings", "10", "--inv", "RESULTS_OK",
                           "--goal", "CLIENTS_DONE", "--mutant-no-check", "--finish-level"]),
    "sip_2p3a_d7": ([2, 2, 3, 0, "--", 101, 100, "/", "/", 7],
                    ["--proto", "sipaxos", "--proposers", "2", "--acceptors", "3", "--values", "a,b", "--inv",
                     "Integrity", "--inv", "Agreement", "--max-depth", "7"]),
    "sip_3p3a_d6": ([2, 3, 3, 0, "--", 101, 100, "/", "/", 6],
                    ["--proto", "sipaxos", "--proposers", "3", "--acceptors", "3", "--values", "a,b,c", "--inv",
                     "Integrity", "--inv", "Agreement", "--max-depth", "6"]),
    "sip_incorrect_2p3a_d9": ([2, 2, 3, 1, "--", 101, 100, "/", "/", 9],
                              ["--proto", "sipaxos", "--proposers", "2", "--acceptors", "3", "--values", "a,b",
                               "--inv", "Integrity", "--inv", "Agreement", "--incorrect", "--max-depth", "9"]),
    "sip_2p5a_d6": ([2, 2, 5, 0, "--", 101, 100, "/", "/", 6],
                    ["--proto", "sipaxos", "--proposers", "2", "--acceptors", "5", "--values", "a,b", "--inv",
                     "Integrity", "--inv", "Agreement", "--max-depth", "6"]),
    "mp_c5_d10": (mp(3, 2, "append-xy") + ["--", 1, 400, 300, "/", "/", 10],
                  ["--proto", "multipaxos", "--workload", "append-xy"] + _MP3 + ["--max-depth", "10"]),
    "mp_xz_d8": (mp(3, 2, "append-xz") + ["--", 1, 400, 300, "/", "/", 8],
                 ["--proto", "multipaxos", "--workload", "append-xz"] + _MP3 + ["--max-depth", "8"]),
    "mp_2s1c_d11": (mp(2, 1, "append-x") + ["--", 1, 400, 300, "/", "/", 2, 11],
                    ["--proto", "multipaxos", "--servers", "2", "--clients", "1", "--workload", "append-x"] + _MP3 +
                    ["--prune", "CLIENTS_DONE", "--max-depth", "11"]),
    # PaxosTest.test27 (PaxosTest.java:1214-1228): singleton Paxos, putAppendGetWorkload, goal
    # CLIENTS_DONE at depth exactly 6; then exhaustive with CLIENTS_DONE pruned
    "mp_test27_goal": (_PAG + ["--", 1, "/", 2, "/", 6],
                       ["--proto", "multipaxos", "--servers", "1", "--clients", "1", "--workload", "put-append-get",
                        "--inv", "RESULTS_OK", "--goal", "CLIENTS_DONE", "--max-depth", "6", "--finish-level"]),
    "mp_test27_exhaustive": (_PAG + ["--", 1, "/", "/", 2, -1],
                             ["--proto", "multipaxos", "--servers", "1", "--clients", "1", "--workload",
                              "put-append-get", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE"]),
    # lab3 predicates (PaxosTest.java:113-346) and StatePredicate combinators (:397-431)
    "mp_goal_has_status": (mp(3, 2, "append-xy") + ["--", 1, 401, "/", f"403:1:{(1 << 4) | 2}", "/", 10],
                           ["--proto", "multipaxos", "--workload", "append-xy", "--inv", "RESULTS_OK", "--inv",
                            "LOGS_CONSISTENT", "--goal", "hasStatus:server2:1:CHOSEN", "--max-depth", "10",
                            "--finish-level"]),
    "mp_inv_implies": (mp(3, 2, "append-xy") + ["--", f"403:0:{(1 << 4) | 2},not,404:0:{(1 << 8) | _X},or", "402:1",
                                                "/", "/", 10],
                       ["--proto", "multipaxos", "--workload", "append-xy", "--inv",
                        "implies(hasStatus:server1:1:CHOSEN,hasCommand:server1:1:X)", "--inv", "slotValid:1",
                        "--max-depth", "10", "--finish-level"]),
    "mp_goal_and_or": (mp(3, 2, "append-xy") + ["--", 400, "/",
                                                f"403:0:{(2 << 4) | 2},403:1:{(2 << 4) | 1},-403:2:{(2 << 4) | 0},or,and",
                                                "/", 9],
                       ["--proto", "multipaxos", "--workload", "append-xy", "--inv", "LOGS_CONSISTENT_ALL_SLOTS",
                        "--goal", "and(hasStatus:server1:2:CHOSEN,or(hasStatus:server2:2:ACCEPTED,"
                        "!hasStatus:server3:2:EMPTY))", "--max-depth", "9", "--finish-level"]),
    # synthetic C3: nodes K P seed -- invariant NOT_ALL_MAX (200)
    "synth_c3_d6": ([3, 5, 64, 7, 0x5EEDD51AB5, "--", 200, "/", "/", 6],
                    ["--proto", "synthetic", "--inv", "NOT_ALL_MAX", "--max-depth", "6"]),
    "synth_2n_k4": ([3, 2, 4, 2, 0x5EEDD51AB5, "--", "/", "/", -1],
                    ["--proto", "synthetic", "--nodes", "2", "--values", "4", "--poke-mod", "2"]),
    # lab1 AMO KV (C2): params from dslabs_amd.protocols.AmoKV(clients, workload).params()
    "kv_test09": ([4, 2, 3, 2, 0, 0, 4, 2, 0, 1, 264, 2, 0, 2, 2316, 2, 1, 0, 4, 2, 1, 1, 264, 2, 1, 2, 2316, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, -1, "--", 1, "/", "/", 2, -1],
                  ["--proto", "amokv", "--clients", "2", "--workload", "diffkey3", "--inv", "RESULTS_OK", "--prune",
                   "CLIENTS_DONE"]),
    "kv_test10": ([4, 2, 3, 2, 0, 0, -1, 2, 0, 1, -1, 2, 0, 2, -1, 2, 0, 0, -1, 2, 0, 1, -1, 2, 0, 2, -1, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, -1, "--", 300, "/", "/", 2, -1],
                  ["--proto", "amokv", "--clients", "2", "--workload", "samekey3", "--inv", "APPENDS_LINEARIZABLE",
                   "--prune", "CLIENTS_DONE"]),
    "kv_putappendget": ([4, 1, 3, 1, 0, 0, 3, 2, 0, 1, 264, 0, 0, 0, 265, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, -1, "--", 1, "/", "/", 2, -1],
                        ["--proto", "amokv", "--clients", "1", "--workload", "putappendget", "--inv", "RESULTS_OK",
                         "--prune", "CLIENTS_DONE"]),
    # the minimizer fixture of SearchAndTraceMinimizerTest (no parameters)
    "mini_inv_foo": ([7, "--", 700, "/", "/", -1], ["--proto", "minitest", "--inv", "foo", "--finish-level"]),
    "mini_goal_notfoo": ([7, "--", "/", -700, "/", -1], ["--proto", "minitest", "--goal", "!foo", "--finish-level"]),
    # lab2 PB + ViewServer (C4): params from dslabs_amd.protocols.PB(servers, clients, workload)
    "pb_2s1c_d14": ([6, 2, 1, 2, 1, 0, 0, 3, 0, 0, 0, 5, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, -1, "--", 1, "/", "/", 2, "500:4", 14],
                    ["--proto", "pb", "--servers", "2", "--clients", "1", "--workload", "putget", "--inv", "RESULTS_OK",
                     "--prune", "CLIENTS_DONE", "--prune", "hasViewReply:4", "--max-depth", "14"]),
    "pb_3s1c_d10": ([6, 3, 1, 2, 1, 0, 0, 3, 0, 0, 0, 5, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, -1, 0, 0, 0, -1, "--", 1, "/", "/", 2, "500:3", 10],
                    ["--proto", "pb", "--servers", "3", "--clients", "1", "--workload", "putget", "--inv", "RESULTS_OK",
                     "--prune", "CLIENTS_DONE", "--prune", "hasViewReply:3", "--max-depth", "10"]),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_encoding_matches_oracle(protocheck, name):
    pargs, oargs = CASES[name]
    got = run(protocheck, pargs)
    want = oracle_util.run("bfs", oargs, timeout=600)
    assert got["end"] == want["end"]
    assert got["per_depth"] == want["per_depth"]
    assert got["fp_mismatch"] == 0 and got["emit_mismatch"] == 0 and got["judge_mismatch"] == 0
    assert got["dup_sends"] == 0
    assert got["skip_mismatch"] == 0  # every event k_level skips (NoopFilter) is a true no-op


@pytest.mark.parametrize("form", ["vstest", "vstest_ir"])
def test_device_viewserver_passes_reference_unit_tests(protocheck, form):
    """The device ViewServer handler (PB node 0) against ViewServerTest test01-test12: the
    hand-written one (csrc/protocols/pb.hpp) and the one generated from dslabs_amd/ir/specs/pb.py."""
    out = subprocess.run([protocheck, form], check=True, capture_output=True, text=True, timeout=60)
    res = json.loads(out.stdout)["results"]
    assert len(res) == 12 and all(r["ok"] for r in res), res
