"""Regenerates tests/golden/*.json from the CPU oracle (oracle/_build/dslabs_oracle).

Every fixture records the oracle arguments, the oracle's output, and -- where the reference
itself states a number -- the pinned reference fact with its source (paths relative to
/root/reference). tests/test_oracle_golden.py checks oracle == fixture == pinned facts.
Usage: python tests/golden/make_golden.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle_util  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

PP = ["--proto", "pingpong"]
LAB0 = {
    # labs/lab0-pingpong/tst/dslabs/pingpong/PingTest.java:128-140 (test04 phase 2)
    "lab0_1c10p_exhaustive": dict(
        args=PP + ["--clients", "1", "--pings", "10", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE"],
        pinned={"states": 120, "max_depth": 29, "end": "SPACE_EXHAUSTED",
                "source": "labs/lab0-pingpong/README.md:282-285 (Explored: 120, Depth: 29)"}),
    # test04 phase 1: goal CLIENTS_DONE (finish-level = level-synchronous terminal rule)
    "lab0_1c10p_goal": dict(
        args=PP + ["--clients", "1", "--pings", "10", "--inv", "RESULTS_OK", "--goal", "CLIENTS_DONE",
                   "--finish-level"],
        pinned={"terminal_depth": 20, "states": 84, "end": "GOAL_FOUND",
                "source": "labs/lab0-pingpong/README.md:276-279 (Explored: 84, Depth: 20 -- the "
                          "multithreaded JVM had completed the goal level)"}),
    "lab0_1c2p_goal": dict(
        args=PP + ["--clients", "1", "--pings", "2", "--inv", "RESULTS_OK", "--goal", "CLIENTS_DONE"],
        pinned={"states": 6, "terminal_depth": 4, "end": "GOAL_FOUND",
                "source": "labs/lab0-pingpong/img/state-graph.png, README.md:509-597 (6 states, goal depth 4)"}),
    "lab0_1c2p_goal_level": dict(
        args=PP + ["--clients", "1", "--pings", "2", "--inv", "RESULTS_OK", "--goal", "CLIENTS_DONE",
                   "--finish-level"], pinned={"terminal_depth": 4, "end": "GOAL_FOUND", "source": "as above"}),
    "lab0_1c2p_exhaustive": dict(
        args=PP + ["--clients", "1", "--pings", "2", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE"],
        pinned={"states": 8, "max_depth": 5, "source": "SURVEY.md §8c derived vector (independent restatement)"}),
    "lab0_2c10p_exhaustive": dict(
        args=PP + ["--clients", "2", "--pings", "10", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE"],
        pinned={"states": 14640, "max_depth": 59,
                "per_depth": [1, 2, 3, 6, 9, 12, 18, 24, 30, 40, 50, 60, 75, 90, 105, 126, 147, 168, 196, 224, 252,
                              286, 318, 348, 383, 414, 441, 472, 497, 516, 538, 552, 560, 570, 572, 568, 565, 554,
                              537, 520, 495, 464, 433, 396, 356, 318, 277, 236, 199, 162, 128, 100, 75, 54, 39, 26,
                              16, 10, 5, 2],
                "source": "SURVEY.md §8c derived vector (independent restatement), BASELINE.md C1"}),
    # README "When Things Go Wrong": pong-value check removed (README.md:342-347)
    "lab0_mutant_nocheck": dict(
        args=PP + ["--clients", "1", "--pings", "10", "--inv", "RESULTS_OK", "--goal", "CLIENTS_DONE",
                   "--mutant-no-check", "--finish-level"],
        pinned={"terminal_depth": 3, "end": "INVARIANT_VIOLATED",
                "trace": ["Message(client1 -> pingserver, PingRequest(ping-1))",
                          "Message(pingserver -> client1, PongReply(ping-1))",
                          "Message(pingserver -> client1, PongReply(ping-1))"],
                "detail": "client1 got Pong(ping-1), expected Pong(ping-2)",
                "source": "labs/lab0-pingpong/README.md:366-423 (3-event trace; 'client1 got "
                          "PingApplication.Pong(value=ping-1), expected PingApplication.Pong(value=ping-2)')"}),
    # 1 client, 3 pings, partitioned (no messages): only timers fire; exhausted immediately
    "lab0_1c3p_partition": dict(
        args=PP + ["--clients", "1", "--pings", "3", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE",
                   "--partition", "pingserver|client1"], pinned={}),
    "lab0_2c4p_maxdepth7": dict(
        args=PP + ["--clients", "2", "--pings", "4", "--inv", "RESULTS_OK", "--max-depth", "7"], pinned={}),
    "lab0_2c3p_notimers": dict(
        args=PP + ["--clients", "2", "--pings", "3", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE",
                   "--no-timers", "client2"], pinned={}),
    "lab0_3c3p_exhaustive": dict(
        args=PP + ["--clients", "3", "--pings", "3", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE"], pinned={}),
    "lab0_mutant_noreset": dict(
        args=PP + ["--clients", "2", "--pings", "3", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE",
                   "--mutant-no-reset"], pinned={}),
}


def gen(cases, fname):
    out = {}
    for name, c in cases.items():
        r = oracle_util.run("bfs", c["args"], timeout=c.get("timeout", 600))
        if r.get("terminals"):
            t = r["terminals"]
            r["terminal_depth"] = t[0]["depth"]
        out[name] = {"args": c["args"], "pinned": c["pinned"], "end": r["end"], "states": r["states"],
                     "max_depth": r["max_depth"], "per_depth": r["per_depth"],
                     "terminal_depth": r.get("terminal_depth", -1),
                     "terminal_kinds": sorted({t["kind"] for t in r.get("terminals", [])}),
                     "terminals": r.get("terminals", [])[:8]}
        print(name, r["end"], r["states"], r["max_depth"])
    with open(os.path.join(HERE, fname), "w") as f:
        json.dump(out, f, indent=1)


def gen_lab0_sip():
    gen(LAB0, "lab0.json")
    SIP = {
        "sipaxos_2p3a_d9": dict(
            args=["--proto", "sipaxos", "--proposers", "2", "--acceptors", "3", "--values", "a,b", "--inv",
                  "Integrity", "--inv", "Agreement", "--max-depth", "9"],
            pinned={"per_depth": [1, 2, 9, 34, 112, 360, 1143, 3556, 10884, 32981],
                    "source": "SURVEY.md §8c derived vector (independent restatement)"}),
        "sipaxos_2p3a_d6": dict(
            args=["--proto", "sipaxos", "--proposers", "2", "--acceptors", "3", "--values", "a,b", "--inv",
                  "Integrity", "--inv", "Agreement", "--max-depth", "6"], pinned={}),
        # IncorrectSingleInstancePaxos (BadProposer, :53-63): no Agreement violation through depth 11
        # (the first one is at depth 14, found on the GPU; tests/test_gpu_sipaxos.py replays it here)
        "sipaxos_incorrect_2p3a": dict(
            args=["--proto", "sipaxos", "--proposers", "2", "--acceptors", "3", "--values", "a,b", "--inv",
                  "Integrity", "--inv", "Agreement", "--incorrect", "--max-depth", "11", "--finish-level"],
            pinned={}),
        "sipaxos_3p3a_d6": dict(
            args=["--proto", "sipaxos", "--proposers", "3", "--acceptors", "3", "--values", "a,b,c", "--inv",
                  "Integrity", "--inv", "Agreement", "--max-depth", "6"], pinned={}),
    }
    gen(SIP, "sipaxos.json")
    tq = oracle_util.run("timerqueue", [])
    with open(os.path.join(HERE, "timerqueue.json"), "w") as f:
        json.dump({"source": "framework/tst-self/dslabs/framework/testing/search/TimerQueueTest.java:153-175",
                   "columns": ["min1", "max1", "min2", "max2", "te1_deliverable", "te2_in_deliverable",
                               "te2_isDeliverable"], "cases": tq["cases"]}, f)


MP = ["--proto", "multipaxos"]
INV3 = ["--inv", "RESULTS_OK", "--inv", "LOGS_CONSISTENT_ALL_SLOTS", "--inv", "APPENDS_LINEARIZABLE"]
MULTIPAXOS = {
    # BASELINE C5: 3 servers, 2 clients (append(foo,X) / append(foo,Y)), maxDepth 12, timers on
    "mp_c5_d12": dict(args=MP + ["--workload", "append-xy"] + INV3 + ["--max-depth", "12"], pinned={}),
    "mp_c5_d8": dict(args=MP + ["--workload", "append-xy"] + INV3 + ["--max-depth", "8"], pinned={}),
    "mp_c5_notimers_d10": dict(args=MP + ["--workload", "append-xy"] + INV3 + ["--max-depth", "10", "--no-timers",
                                                                                "server1", "--no-timers", "server2",
                                                                                "--no-timers", "server3",
                                                                                "--no-timers", "client1",
                                                                                "--no-timers", "client2"], pinned={}),
    # PaxosTest.test22 phase 1: partition(server1, server2, client1), goal !NONE_DECIDED
    "mp_test22_phase1": dict(args=MP + ["--workload", "append-xy-expect", "--inv", "RESULTS_OK", "--inv",
                                        "LOGS_CONSISTENT_ALL_SLOTS", "--goal", "!NONE_DECIDED", "--partition",
                                        "server1,server2,client1", "--finish-level"], pinned={}),
    # full network with expected results X / XY: client2 can be ordered first -> violation
    "mp_expect_violation": dict(args=MP + ["--workload", "append-xy-expect", "--inv", "RESULTS_OK", "--inv",
                                           "LOGS_CONSISTENT_ALL_SLOTS", "--goal", "CLIENTS_DONE", "--finish-level"],
                                pinned={}),
    # PaxosTest.test27 (:1214-1228): singleton group, putAppendGetWorkload, CLIENTS_DONE at depth 6
    "mp_test27": dict(args=MP + ["--servers", "1", "--clients", "1", "--workload", "put-append-get", "--inv",
                                 "RESULTS_OK", "--goal", "CLIENTS_DONE", "--finish-level"],
                      pinned={"terminal_depth": 6, "end": "GOAL_FOUND",
                              "source": "labs/lab3-paxos/tst/dslabs/paxos/PaxosTest.java:1214-1228 "
                                        "(assertGoalFound, goal depth 6)"}),
    # singleton group, one command: CLIENTS_DONE after 2 steps
    "mp_singleton": dict(args=MP + ["--servers", "1", "--clients", "1", "--workload", "append-x"] + INV3 +
                         ["--goal", "CLIENTS_DONE", "--finish-level"],
                         pinned={}),
    "mp_2s1c_prune": dict(args=MP + ["--servers", "2", "--clients", "1", "--workload", "append-x"] + INV3 +
                          ["--prune", "CLIENTS_DONE", "--max-depth", "11"], pinned={}),
    "mp_xz_d8": dict(args=MP + ["--workload", "append-xz"] + INV3 + ["--max-depth", "8"], pinned={}),
}

SY = ["--proto", "synthetic"]
SYNTHETIC = {
    # BASELINE C3 (builder-defined): 5 nodes, K = 64, pokes at v % 7 == 0, seed
    # 0x5EEDD51AB5; the bench runs the same configuration to maxDepth 10 (~8e8 states).
    "synth_c3_d5": dict(args=SY + ["--inv", "NOT_ALL_MAX", "--max-depth", "5"], pinned={}),
    "synth_3n_k8_d9": dict(args=SY + ["--nodes", "3", "--values", "8", "--poke-mod", "3", "--inv", "NOT_ALL_MAX",
                                      "--max-depth", "9", "--finish-level"], pinned={}),
    # a reachable value bound: the first violation depth and its trace
    "synth_counter_violation": dict(args=SY + ["--nodes", "4", "--values", "32", "--inv", "COUNTER_LT:2:30",
                                               "--finish-level"], pinned={}),
    # goal + prune combination
    "synth_goal_prune": dict(args=SY + ["--nodes", "3", "--values", "64", "--goal", "!COUNTER_LT:0:63", "--prune",
                                        "!COUNTER_LT:1:40", "--finish-level"], pinned={}),
    # the whole reachable space of a small configuration (no depth bound)
    "synth_2n_k4_exhaustive": dict(args=SY + ["--nodes", "2", "--values", "4", "--poke-mod", "2"], pinned={}),
}

KV = ["--proto", "amokv"]
AMOKV = {
    # ClientServerPart2Test.test09 (:221-238): 2 clients, appendDifferentKeyWorkload(3), RESULTS_OK
    "kv_test09_exhaustive": dict(args=KV + ["--clients", "2", "--workload", "diffkey3", "--inv", "RESULTS_OK",
                                            "--prune", "CLIENTS_DONE"], pinned={}),
    "kv_test09_goal": dict(args=KV + ["--clients", "2", "--workload", "diffkey3", "--inv", "RESULTS_OK", "--goal",
                                      "CLIENTS_DONE", "--finish-level"], pinned={}),
    # ClientServerPart2Test.test10 (:243-263): 2 clients, APPEND:foo:%i x 3, APPENDS_LINEARIZABLE
    "kv_test10_exhaustive": dict(args=KV + ["--clients", "2", "--workload", "samekey3", "--inv",
                                            "APPENDS_LINEARIZABLE", "--prune", "CLIENTS_DONE"], pinned={}),
    "kv_3c_diffkey3": dict(args=KV + ["--clients", "3", "--workload", "diffkey3", "--inv", "RESULTS_OK", "--prune",
                                      "CLIENTS_DONE"], pinned={}),
    # BASELINE C2 at 3 clients: 1,225,876 states (the oracle takes ~6 min; checked on the GPU only)
    "kv_3c_samekey3": dict(args=KV + ["--clients", "3", "--workload", "samekey3", "--inv", "APPENDS_LINEARIZABLE",
                                      "--prune", "CLIENTS_DONE"], pinned={}),
    # test08-style workloads with two clients on one key: RESULTS_OK is violated
    "kv_appendappendget_2c": dict(args=KV + ["--clients", "2", "--workload", "appendappendget", "--inv",
                                             "RESULTS_OK", "--prune", "CLIENTS_DONE", "--finish-level"], pinned={}),
    "kv_putappendget_1c": dict(args=KV + ["--clients", "1", "--workload", "putappendget", "--inv", "RESULTS_OK",
                                          "--prune", "CLIENTS_DONE"], pinned={}),
    "kv_getput_2c": dict(args=KV + ["--clients", "2", "--workload", "getput", "--inv", "RESULTS_OK", "--prune",
                                    "CLIENTS_DONE", "--finish-level"], pinned={}),
    # APPENDS_LINEARIZABLE over a workload with a GET: the predicate throws (invariant violated)
    "kv_linearizable_throws": dict(args=KV + ["--clients", "1", "--workload", "appendappendget", "--inv",
                                              "APPENDS_LINEARIZABLE", "--prune", "CLIENTS_DONE", "--finish-level"],
                                   pinned={}),
    "kv_test10_partition": dict(args=KV + ["--clients", "2", "--workload", "samekey2", "--inv",
                                           "APPENDS_LINEARIZABLE", "--prune", "CLIENTS_DONE", "--partition",
                                           "server,client1|client2"], pinned={}),
}

PBA = ["--proto", "pb"]
PBQ = ["--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE", "--prune", "hasViewReply:4"]
PBF = {
    # BASELINE C4 (PrimaryBackupTest.test17-style, :680-711): 2 servers + ViewServer, 1 client
    # putGetWorkload, prunes CLIENTS_DONE and hasViewReply(INITIAL_VIEWNUM + 3), from the start state
    "pb_2s1c_d15": dict(args=PBA + ["--servers", "2", "--clients", "1", "--workload", "putget"] + PBQ +
                        ["--max-depth", "15"], pinned={}),
    "pb_2s1c_goal": dict(args=PBA + ["--servers", "2", "--clients", "1", "--workload", "putget", "--inv",
                                     "RESULTS_OK", "--goal", "CLIENTS_DONE", "--prune", "hasViewReply:4",
                                     "--finish-level"], pinned={}),
    # test17's third server, inactive (nodeActive(server(3), false))
    "pb_3s1c_inactive_d12": dict(args=PBA + ["--servers", "3", "--clients", "1", "--workload", "putget"] + PBQ +
                                 ["--inactive", "server3", "--max-depth", "12"], pinned={}),
    "pb_2s2c_d11": dict(args=PBA + ["--servers", "2", "--clients", "2", "--workload", "putget"] + PBQ +
                        ["--max-depth", "11"], pinned={}),
    # a view change is reachable: ViewReply for view 3
    "pb_view3_goal": dict(args=PBA + ["--servers", "2", "--clients", "1", "--workload", "putget", "--goal",
                                      "hasViewReply:3", "--finish-level"], pinned={}),
    # PrimaryBackupTest.initView(server1, server2, client1) (:124-187): the search for View(2, 1, 2)
    # started, network off except the ViewServer and server1 <-> server2 (network predicates)
    "pb_initview_search": dict(args=PBA + ["--servers", "2", "--clients", "1", "--workload", "putget", "--prune",
                                           "hasViewReply:3", "--prune", "and(hasViewReply:2,!hasViewReply:2:1:2)",
                                           "--network-off", "--active", "viewserver", "--link", "server1,server2",
                                           "--link", "server2,server1", "--goal",
                                           "and(viewRepliesSent:2:1:2:server1+server2+client1,!hasViewReply:3)",
                                           "--finish-level"], pinned={}),
    # two clients appending to one key with expected results: RESULTS_OK is violated
    "pb_2c_results_violation": dict(args=PBA + ["--servers", "2", "--clients", "2", "--workload",
                                                "appendappendget", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE",
                                                "--prune", "hasViewReply:3", "--finish-level"], pinned={}),
}

# Deep fixtures (tests/golden/deep.json): the oracle needs tens of minutes and tens of GB each, so
# they are generated only on request (python tests/golden/make_golden.py deep) and checked on the
# GPU only (tests/test_gpu_deep.py); oracle_elapsed_s records what each took.
DEEP = {
    # BASELINE C5 to maxDepth 14: 8,808,218 states (36 min, ~24 GB on the oracle)
    "mp_c5_d14": dict(args=MP + ["--workload", "append-xy"] + INV3 + ["--max-depth", "14"], pinned={},
                      timeout=7200),
    # IncorrectSingleInstancePaxos through depth 14, where the GPU finds the first Agreement
    # violation (T/visualization/examples/paxosmadesimple/IncorrectSingleInstancePaxos.java:42-64)
    "sipaxos_incorrect_d14": dict(args=["--proto", "sipaxos", "--proposers", "2", "--acceptors", "3", "--values",
                                        "a,b", "--inv", "Integrity", "--inv", "Agreement", "--incorrect",
                                        "--max-depth", "14", "--finish-level"], pinned={}, timeout=7200),
    # BASELINE C3 through depth 7
    "synth_c3_d7": dict(args=SY + ["--inv", "NOT_ALL_MAX", "--max-depth", "7"], pinned={}, timeout=7200),
    # ... and through depth 8: 30,341,487 states (19 min on the oracle), the deepest C3 pin
    "synth_c3_d8": dict(args=SY + ["--inv", "NOT_ALL_MAX", "--max-depth", "8"], pinned={}, timeout=7200),
}


def gen_deep(names=None):
    """Regenerates the named deep cases (all by default), keeping the others of deep.json."""
    path = os.path.join(HERE, "deep.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name, c in DEEP.items():
        if names and name not in names:
            continue
        r = oracle_util.run("bfs", c["args"], timeout=c["timeout"])
        t = r.get("terminals", [])
        out[name] = {"args": c["args"], "pinned": c["pinned"], "end": r["end"], "states": r["states"],
                     "max_depth": r["max_depth"], "per_depth": r["per_depth"],
                     "terminal_depth": t[0]["depth"] if t else -1,
                     "terminal_kinds": sorted({x["kind"] for x in t}), "terminals": t[:8],
                     "oracle_elapsed_s": r["elapsed_s"]}
        print(name, r["end"], r["states"], r["max_depth"])
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


# Deep vectors of the multithreaded host BFS (tools/cpu_bfs.cpp): another engine than the kernels
# (a host visited set and host frontiers) over the same packed transition functions, for depths the
# oracle cannot reach in this container. The whole C3 bench configuration (BASELINE C3, maxDepth 10,
# 780,909,037 states: a 2^31-slot host table of 16 GiB plus the depth-9 frontier) runs on the build
# container's 8 cores in minutes; its depth-0..8 prefix is the oracle's synth_c3_d8.
# python tests/golden/make_golden.py deep-cpu
DEEP_CPU = {
    "synth_c3_d10_cpu_bfs": dict(workload="synthetic", depth=10, table_log2=31),
}


def gen_deep_cpu(names=None):
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    import bench
    from tools import cpu_baseline
    path = os.path.join(HERE, "deep.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name, c in DEEP_CPU.items():
        if names and name not in names:
            continue
        proto, s, _ = bench.build_search(c["workload"], c["depth"])
        t0 = time.time()
        r = cpu_baseline.run(proto, s, table_log2=c["table_log2"], timeout=6 * 3600)
        out[name] = {"source": "tools/cpu_bfs.cpp via tools/cpu_baseline.run (bench.build_search(%r, %d))"
                               % (c["workload"], c["depth"]),
                     "end": r["end"], "states": r["states"], "max_depth": len(r["per_depth"]) - 1,
                     "per_depth": r["per_depth"], "threads": r["threads"], "table_log2": c["table_log2"],
                     "elapsed_s": round(time.time() - t0, 1)}
        print(name, r["end"], r["states"], out[name]["elapsed_s"])
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    which = set(sys.argv[1:]) or {"lab0", "sipaxos", "multipaxos", "synthetic", "amokv", "pb"}
    if "lab0" in which or "sipaxos" in which:
        gen_lab0_sip()
    if "multipaxos" in which:
        gen(MULTIPAXOS, "multipaxos.json")
    if "synthetic" in which:
        gen(SYNTHETIC, "synthetic.json")
    if "amokv" in which:
        gen(AMOKV, "amokv.json")
    if "pb" in which:
        gen(PBF, "pb.json")
        vs = oracle_util.run("vstest", [])
        with open(os.path.join(HERE, "viewserver.json"), "w") as f:
            json.dump({"source": "labs/lab2-primarybackup/tst/dslabs/primarybackup/ViewServerTest.java:156-303",
                       "results": vs["results"]}, f, indent=1)
    if "deep" in which:
        gen_deep()
    if "deep-cpu" in which:
        gen_deep_cpu()
    deep = {w[len("deep:"):] for w in which if w.startswith("deep:")}  # e.g. deep:synth_c3_d7
    if deep:
        gen_deep(deep)
