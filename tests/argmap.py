"""Maps oracle CLI arguments (tests/golden/*.json "args") onto the engine's Python API, so each
committed oracle fixture is replayed on the GPU with the same meaning."""
from dslabs_amd import CLIENTS_DONE, NONE_DECIDED, RESULTS_OK, SearchSettings, clientDone
from dslabs_amd.protocols import PB, PBIR, AmoKV, AmoKVIR, MiniTest, MultiPaxos, MultiPaxosIR, PingPong, PingPongIR, SIPaxos, Synthetic


def _opt(args, name, default=None):
    return args[args.index(name) + 1] if name in args else default


def protocol(args):
    p = _opt(args, "--proto", "pingpong")
    if p == "pingpong":
        return PingPong(int(_opt(args, "--clients", 1)), int(_opt(args, "--pings", 10)),
                        check_value="--mutant-no-check" not in args, reset_timer="--mutant-no-reset" not in args)
    if p == "amokv_ir":  # tests give --clients / --workload (the oracle takes AmoKVIR.oracle_args())
        return AmoKVIR(int(_opt(args, "--clients", 2)), _opt(args, "--workload", "diffkey3"))
    if p == "pingpong_ir":
        return PingPongIR(int(_opt(args, "--clients", 1)), int(_opt(args, "--pings", 10)),
                          check_value="--mutant-no-check" not in args, reset_timer="--mutant-no-reset" not in args)
    if p == "sipaxos":
        vals = _opt(args, "--values", "a,b").split(",")
        return SIPaxos(int(_opt(args, "--proposers", 2)), int(_opt(args, "--acceptors", 3)), vals,
                       incorrect="--incorrect" in args)
    if p == "multipaxos_ir":  # tests give --servers / --clients / --workload (the oracle takes MultiPaxosIR.oracle_args())
        return MultiPaxosIR(int(_opt(args, "--servers", 3)), int(_opt(args, "--clients", 2)),
                            _opt(args, "--workload", "append-xy"))
    if p == "multipaxos":
        return MultiPaxos(int(_opt(args, "--servers", 3)), int(_opt(args, "--clients", 2)),
                          _opt(args, "--workload", "append-xy"))
    if p == "pb_ir":  # tests give --servers / --clients / --workload (the oracle takes PBIR.oracle_args())
        return PBIR(int(_opt(args, "--servers", 2)), int(_opt(args, "--clients", 1)), _opt(args, "--workload", "putget"))
    if p == "pb":
        return PB(int(_opt(args, "--servers", 2)), int(_opt(args, "--clients", 1)), _opt(args, "--workload", "putget"))
    if p == "amokv":
        return AmoKV(int(_opt(args, "--clients", 2)), _opt(args, "--workload", "diffkey3"))
    if p == "synthetic":
        return Synthetic(int(_opt(args, "--nodes", 5)), int(_opt(args, "--values", 64)), int(_opt(args, "--poke-mod", 7)),
                         int(_opt(args, "--seed", str(Synthetic.SEED)), 0))
    if p == "minitest":
        return MiniTest()
    raise ValueError(p)


def predicate(proto, name):
    """An oracle predicate argument: NAME, !P, and(P,Q), or(P,Q), implies(P,Q) (nested)."""
    if name.startswith("!"):
        return predicate(proto, name[1:]).negate()
    for op in ("and(", "or(", "implies("):
        if name.startswith(op) and name.endswith(")"):
            inner, depth = name[len(op):-1], 0
            for k, ch in enumerate(inner):
                depth += ch == "("
                depth -= ch == ")"
                if ch == "," and depth == 0:
                    a, b = predicate(proto, inner[:k]), predicate(proto, inner[k + 1:])
                    return a.and_(b) if op == "and(" else a.or_(b) if op == "or(" else a.implies(b)
            raise ValueError(name)
    neg = False
    std = {"RESULTS_OK": RESULTS_OK, "CLIENTS_DONE": CLIENTS_DONE, "NONE_DECIDED": NONE_DECIDED}
    if name in std:
        p = std[name]
    elif name.startswith("clientDone:"):
        p = clientDone(name.split(":", 1)[1])
    else:
        p = proto.predicate(name)
    return p.negate() if neg else p


def settings(args, proto, table_log2=24):
    s = SearchSettings()
    s.table_log2_slots = table_log2
    i = 0
    while i < len(args):
        a = args[i]
        v = args[i + 1] if i + 1 < len(args) else None
        if a == "--inv":
            s.addInvariant(predicate(proto, v))
        elif a == "--goal":
            s.addGoal(predicate(proto, v))
        elif a == "--prune":
            s.addPrune(predicate(proto, v))
        elif a == "--max-depth":
            s.maxDepth(int(v))
        elif a == "--no-timers":
            s.deliverTimers(v, False)
        elif a == "--inactive":
            s.nodeActive(v, False)
        elif a == "--network-off":
            s.networkActive(False)
        elif a == "--active":
            s.nodeActive(v, True)
        elif a == "--link":
            s.linkActive(*v.split(","), True)
        elif a == "--partition":
            s.partition(*[g.split(",") for g in v.split("|")])
        i += 1
    return s
