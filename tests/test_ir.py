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
from test_hostcheck import protocheck, run  # noqa: F401  (fixture)
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
