"""The Java integration layer (java/src) cannot be compiled here (no JDK), so its
native-memory contract is checked statically: every struct size and field offset the Panama FFM
binding (java/src/.../gpu/Dsl.java) hard-codes equals the C header's (through the ctypes mirror,
itself checked against the header by test_capi.py); every downcall's descriptor matches the
ctypes prototype of the same symbol; the ABI version, protocol, end-condition and predicate ids
the Java side uses equal the header's enums; and the lab3 registry (MultiPaxosCodec) uses the
device layout's constants (multipaxos.hpp) and, by its token rule, builds the parameter vectors
dslabs_amd/protocols.py builds."""
import ctypes
import os
import re

from dslabs_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "src", "dslabs", "framework", "testing", "search")
DSL = open(os.path.join(JAVA, "gpu", "Dsl.java")).read()
HEADER = open(os.path.join(ROOT, "include", "dslabs_hip.h")).read()


def consts(text=DSL):
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"\b([A-Z][A-Z0-9_]+) = (-?\d+)", text)}


FIELDS = {
    "dsl_protocol_desc": {"PROTOCOL_DESC": None, "DESC_PROTOCOL": "protocol", "DESC_N_PARAMS": "n_params",
                          "DESC_PARAMS": "params"},
    "dsl_predicate": {"PREDICATE": None, "PRED_ID": "pred_id", "PRED_NEGATE": "negate", "PRED_ARG0": "arg0",
                      "PRED_ARG1": "arg1"},
    "dsl_settings": {"SETTINGS": None, "MAX_DEPTH": "max_depth", "MAX_TIME_MS": "max_time_ms",
                     "NETWORK_ACTIVE": "network_active", "DELIVER_TIMERS": "deliver_timers",
                     "LINK_ACTIVE": "link_active", "SENDER_ACTIVE": "sender_active",
                     "RECEIVER_ACTIVE": "receiver_active", "TIMERS_ACTIVE": "timers_active",
                     "N_INVARIANTS": "n_invariants", "N_GOALS": "n_goals", "N_PRUNES": "n_prunes",
                     "INVARIANTS": "invariants", "GOALS": "goals", "PRUNES": "prunes",
                     "TABLE_LOG2": "table_log2_slots", "N_POOL": "n_pool", "MAX_FRONTIER": "max_frontier_states",
                     "MEMORY_BUDGET": "memory_budget_bytes", "POOL": "pool", "DO_CHECKS": "do_checks",
                     "CHECK_SAMPLE": "check_sample"},
    "dsl_engine_config": {"ENGINE_CONFIG": None, "CFG_DEVICE": "device", "CFG_RANK": "rank",
                          "CFG_WORLD": "world_size", "CFG_VSHARDS": "virtual_shards", "CFG_COMM_ID": "comm_id",
                          "CFG_REPLICATE_BELOW": "replicate_below", "CFG_FLAGS": "flags"},
    "dsl_event": {"EVENT": None, "EV_IS_TIMER": "is_timer", "EV_FROM": "from_", "EV_TO": "to", "EV_TYPE": "type",
                  "EV_N_FIELDS": "n_fields", "EV_TIMER_MIN": "timer_min", "EV_TIMER_MAX": "timer_max",
                  "EV_FIELDS": "fields"},
    "dsl_result": {"RESULT": None, "RES_END": "end_condition", "RES_TERMINAL_DEPTH": "terminal_depth",
                   "RES_PRED_INDEX": "predicate_index", "RES_MAX_DEPTH": "max_depth", "RES_STATES": "states",
                   "RES_N_LEVELS": "n_levels", "RES_TRACE_LEN": "trace_len", "RES_PER_DEPTH": "per_depth",
                   "RES_TRACE": "trace", "RES_TERMINAL_STATE": "terminal_state", "RES_STATE_BYTES": "state_bytes",
                   "RES_INITIAL_DEPTH": "initial_depth", "RES_ELAPSED": "elapsed_s", "RES_CHECKS_RUN": "checks_run",
                   "RES_NOT_DETERMINISTIC": "not_deterministic", "RES_NOT_IDEMPOTENT": "not_idempotent",
                   "RES_FIRST_NOT_DETERMINISTIC": "first_not_deterministic",
                   "RES_FIRST_NOT_IDEMPOTENT": "first_not_idempotent"},
}


def test_java_struct_offsets_match_the_c_abi():
    c = consts()
    checked = 0
    for struct, fields in FIELDS.items():
        S = getattr(_lib, struct)
        for jname, field in fields.items():
            if field is None:
                assert c["SIZE_" + jname] == ctypes.sizeof(S), (struct, jname)
            else:
                assert c["OFF_" + jname] == getattr(S, field).offset, (struct, jname)
            checked += 1
    assert checked == 67


def test_java_end_conditions_and_predicate_ids_match_the_header():
    c = consts()
    for n in ("EXCEPTION_THROWN", "INVARIANT_VIOLATED", "GOAL_FOUND", "SPACE_EXHAUSTED", "TIME_EXHAUSTED"):
        v = int(re.search(r"DSL_%s = (\d+)" % n, HEADER).group(1))
        assert c["END_" + n] == v
    ids = {n: int(v) for n, v in re.findall(r"DSL_PRED_([A-Z_]+) = (\d+)", HEADER)}
    reg = open(os.path.join(JAVA, "gpu", "GpuProtocols.java")).read()
    assert '"Clients got expected results", %d' % ids["RESULTS_OK"] in reg
    assert '"All clients\' workloads finished", %d' % ids["CLIENTS_DONE"] in reg
    assert '"No results returned", %d' % ids["NONE_DECIDED"] in reg
    for name, key in (("Agreement", "SIP_AGREEMENT"), ("Integrity", "SIP_INTEGRITY"), ("Termination", "SIP_TERMINATION")):
        assert 'case "%s" -> new GpuPredicates.Leaf(%d, 0, 0);' % (name, ids[key]) in reg
    preds = open(os.path.join(JAVA, "gpu", "GpuPredicates.java")).read()
    assert "AND = %d, OR = %d, IMPLIES = %d" % (ids["AND"], ids["OR"], ids["IMPLIES"]) in preds


def test_java_abi_version_and_protocol_ids_match_the_header():
    c = consts()
    assert c["ABI_VERSION"] == int(re.search(r"#define DSL_ABI_VERSION (\d+)", HEADER).group(1)) == _lib.DSL_ABI_VERSION
    assert c["MAX_EVENT_FIELDS"] == int(re.search(r"#define DSL_MAX_EVENT_FIELDS (\d+)", HEADER).group(1))
    assert c["MAX_POOL"] == int(re.search(r"#define DSL_MAX_POOL (\d+)", HEADER).group(1))
    for j, h in (("PINGPONG", "PINGPONG"), ("SIPAXOS", "SIPAXOS"), ("MULTIPAXOS", "MULTIPAXOS"), ("AMOKV", "AMOKV"),
                 ("PB", "PB")):
        assert c["PROTO_" + j] == int(re.search(r"DSL_PROTO_%s = (\d+)" % h, HEADER).group(1))
    assert "dsl_abi_version" in DSL and "abi != ABI_VERSION" in DSL


# Panama ValueLayouts of Dsl.java's descriptors -> the ctypes kinds they must stand for
def _kind(ct):
    if ct is None:
        return "void"
    if ct in (ctypes.c_int, ctypes.c_int32):
        return "I"
    if ct in (ctypes.c_size_t, ctypes.c_int64, ctypes.c_uint64):
        return "J"
    return "A"  # pointers, c_void_p, c_char_p


def test_java_downcalls_match_the_c_prototypes():
    lib = _lib.load()
    names = {"I": "I", "A": "A", "ValueLayout.JAVA_LONG": "J", "ValueLayout.JAVA_INT": "I"}
    found = 0
    for m in re.finditer(r'fn\("(dsl_\w+)", FunctionDescriptor\.(of|ofVoid)\(([^)]*)\)\)', DSL):
        sym, kind, args = m.group(1), m.group(2), [a.strip() for a in m.group(3).split(",") if a.strip()]
        java = [names[a] for a in args]
        ret = "void" if kind == "ofVoid" else java.pop(0)
        f = getattr(lib, sym)
        assert sym in HEADER, sym
        assert ret == ("void" if f.restype is None else _kind(f.restype)), sym
        assert java == [_kind(a) for a in (f.argtypes or [])], sym
        found += 1
    assert found == 13  # create / set_settings / set_initial / run / result_free / destroy / last_error /
    #                      device_count / abi_version / replay / set_dropped / drop_pending_messages /
    #                      undrop_messages


MPC = open(os.path.join(JAVA, "gpu", "MultiPaxosCodec.java")).read()
MPH = open(os.path.join(ROOT, "dslabs_amd", "csrc", "protocols", "multipaxos.hpp")).read()


def test_java_multipaxos_codec_constants_match_the_device_layout():
    from dslabs_amd.protocols import MultiPaxos
    c = consts(MPC)
    assert (c["MAX_SERVERS"], c["MAX_CLIENTS"], c["MAX_CMDS"], c["SLOTS"], c["MAX_TOKENS"]) == tuple(
        int(re.search(r"\b%s = (\d+)" % k, MPH).group(1)) for k in ("kMaxServers", "kMaxClients", "kMaxCmds", "kSlots",
                                                                  "kMaxTokens"))
    enum = re.search(r"enum \{ M_REQUEST = 0, ([^}]*)\}", MPH).group(1)
    names = ["M_REQUEST"] + [e.split("=")[0].strip() for e in enum.split(",")]
    for i, n in enumerate(names[:8]):
        assert c[n] == i, n
    assert c["T_TICK"] == int(re.search(r"T_TICK = (\d+)", MPH).group(1))
    assert c["T_CLIENT"] == int(re.search(r"T_CLIENT = (\d+)", MPH).group(1))
    for op, v in MultiPaxos.OPS.items():
        assert c["OP_" + op] == v == int(re.search(r"OP_%s = (\d+)" % op, MPH).group(1))
    assert c["RESULT_PUT_OK"] == MultiPaxos.PUT_OK == int(re.search(r"kPutOk = (\d+)", MPH).group(1))
    assert c["RESULT_KEY_NOT_FOUND"] == MultiPaxos.KEY_NOT_FOUND == int(re.search(r"kKeyNotFound = (\d+)", MPH).group(1))
    # the record payload formulas the codec documents are the device header's
    assert "ballot_field(int b) { return (uint64_t)(b >> 2) | ((uint64_t)(b & 3) << 4); }" in MPH
    assert '"round")).longValue() | ((Number) field(ballot, "leader")).longValue() << 4' in MPC
    assert "mk_entry(int status, int ballot, int cmd)" in MPH and "status | ballotOrder(" in MPC
    assert "bits |= e << (11 * k)" in MPC and "((lg >> (16 * k)) & 0x7ffull) << (11 * k)" in MPH
    # PaxosLogSlotStatus ordinals (the codec writes Enum.ordinal()) are the device's status codes
    assert list(MultiPaxos.STATUS.values()) == [0, 1, 2, 3]
    # the lab3 solution's bounds and timer lengths are the device's
    srv = open(os.path.join(ROOT, "java", "src", "dslabs", "paxos", "PaxosServer.java")).read()
    tim = open(os.path.join(ROOT, "java", "src", "dslabs", "paxos", "Timers.java")).read()
    assert "SLOTS = 4, MAX_ROUND = 15" in srv and "kSlots = 4" in MPH and "kMaxRound = 15" in MPH
    assert "TICK_MILLIS = 100" in tim and "CLIENT_RETRY_MILLIS = 100" in tim and "kTick = 100, kClientRetry = 100" in MPH


def _java_rule_params(servers, clients, workload):
    """MultiPaxosCodec.params() as a rule: tokens = the sorted distinct Put / Append values; a
    value is len | token ids; results PutOk 7 / KeyNotFound 6 / a value; -1 = no expected result."""
    from dslabs_amd.protocols import MultiPaxos
    cmds, exp, _ = MultiPaxos.WORKLOADS[workload]
    cmds, exp = cmds[:clients], exp[:clients]
    toks = sorted({c.split(":")[2] for cl in cmds for c in cl if not c.startswith("GET")})
    w = len(toks[0])

    def value(s):
        r = len(s) // w
        for i in range(len(s) // w):
            r |= (toks.index(s[i * w:(i + 1) * w]) + 1) << (3 + 2 * i)
        return r

    ps = [servers, clients]
    for c in range(2):
        cl = cmds[c] if c < clients else []
        ex = exp[c] if c < clients else []
        ops = [MultiPaxos.OPS[x.split(":")[0]] for x in cl]
        vals = [0 if x.startswith("GET") else toks.index(x.split(":")[2]) + 1 for x in cl]
        res = []
        for k, r in enumerate(ex):
            op = cl[k].split(":")[0]
            res.append(7 if op == "PUT" else 6 if r == "KeyNotFound" else value(r))
        ps += [len(cl)] + ops + [0] * (3 - len(cl)) + vals + [0] * (3 - len(cl)) + res + [-1] * (3 - len(res))
    return ps, toks


def _decoded(ps, toks):
    """A parameter vector with token ids replaced by the strings they stand for."""
    out = list(ps[:2])
    for c in range(2):
        b = 2 + 10 * c
        out += ps[b:b + 4] + [toks[v - 1] if v else None for v in ps[b + 4:b + 7]]
        for r in ps[b + 7:b + 10]:
            out.append(r if r in (-1, 6, 7) else "".join(toks[((r >> (3 + 2 * i)) & 3) - 1] for i in range(r & 7)))
    return out


def test_java_multipaxos_params_equal_protocols_py():
    from dslabs_amd.protocols import MultiPaxos
    for wl in MultiPaxos.WORKLOADS:
        for servers, clients in ((3, 2), (3, 1), (1, 1), (2, 2)):
            if clients > len(MultiPaxos.WORKLOADS[wl][0]):
                continue
            mp = MultiPaxos(servers, clients, wl)
            ps, toks = _java_rule_params(servers, clients, wl)
            if toks == mp.tokens[:len(toks)]:  # the same token numbering: the same vector
                assert ps == mp.params(), (wl, servers, clients)
            # a workload using a subset of protocols.py's tokens numbers them densely: the same
            # commands and results under another (isomorphic) numbering
            assert _decoded(ps, toks) == _decoded(mp.params(), mp.tokens), (wl, servers, clients)
    assert "TreeSet<String> t = new TreeSet<>()" in open(os.path.join(JAVA, "gpu", "GpuProtocols.java")).read()


def test_java_multipaxos_predicate_leaves():
    from dslabs_amd.protocols import MultiPaxos
    reg = open(os.path.join(JAVA, "gpu", "GpuProtocols.java")).read()
    ids = {n: int(v) for n, v in re.findall(r"DSL_PRED_([A-Z_]+) = (\d+)", HEADER)}
    mp = MultiPaxos(3, 2, "append-xy")
    for key, (pid, full) in MultiPaxos.PREDICATES.items():
        assert '"%s"' % full in reg, full
        assert "Leaf(%d, 0, 0)" % pid in reg
    assert ids["LOGS_CONSISTENT"] == 400 and ids["LOGS_CONSISTENT_ACTIVE"] == 401
    assert "Leaf(402," in reg and ids["SLOT_VALID"] == 402
    assert "Leaf(403," in reg and ids["HAS_STATUS"] == 403
    assert "Leaf(404," in reg and ids["HAS_COMMAND"] == 404
    # the names protocols.py gives the parametrized predicates are the ones the Java patterns parse
    pats = {k: re.search(r'%s = Pattern.compile\("([^"]*)"\)' % k, reg).group(1).replace("\\\\", "\\")
            for k in ("HAS_STATUS", "HAS_COMMAND", "SLOT_VALID")}
    assert re.fullmatch(pats["HAS_STATUS"], mp.predicate("hasStatus:server2:3:CHOSEN").name)
    assert re.fullmatch(pats["SLOT_VALID"], mp.predicate("slotValid:2").name)
    hc = re.fullmatch(pats["HAS_COMMAND"], "server1 has command KVStore.Append(key=foo, value=X) in slot 1")
    assert hc and hc.group(2) == "KVStore.Append(key=foo, value=X)"
    kv = re.search(r'KV = Pattern.compile\("([^"]*)"\)', MPC).group(1).replace("\\\\", "\\")
    m = re.fullmatch(kv, "KVStore.Append(key=foo, value=X)")
    assert m and m.groups() == ("Append", "foo", "X")
    assert (MultiPaxos.OPS["APPEND"] << 2 | 1) == mp.kv_code("APPEND:foo:X")


AKC = open(os.path.join(JAVA, "gpu", "AmoKVCodec.java")).read()
AKH = open(os.path.join(ROOT, "dslabs_amd", "csrc", "protocols", "amokv.hpp")).read()
PBC = open(os.path.join(JAVA, "gpu", "PBCodec.java")).read()
PBH = open(os.path.join(ROOT, "dslabs_amd", "csrc", "protocols", "pb.hpp")).read()


def _hpp(text, name):
    return int(re.search(r"\b%s = (\d+)" % name, text).group(1))


def test_java_amokv_codec_matches_the_device_layout_and_protocols_py():
    """lab1 (C2): AmoKVCodec's bounds, op / result / message codes, value and result bit layouts are
    amokv.hpp's and protocols.py AmoKV's; its parameter rule (keys and value tokens numbered by first
    use, client-major) builds AmoKV.params() for every workload."""
    from dslabs_amd.protocols import AmoKV
    c = consts(AKC)
    assert (c["MAX_CLIENTS"], c["MAX_CMDS"], c["MAX_KEYS"], c["MAX_LEN"]) == tuple(
        _hpp(AKH, k) for k in ("kMaxClients", "kMaxCmds", "kMaxKeys", "kMaxLen"))
    for op, v in AmoKV.OPS.items():
        assert c["OP_" + op] == v == _hpp(AKH, "OP_" + op)
    for i, n in enumerate(AmoKV.RTYPES):
        key = {"AppendResult": "R_APPEND", "GetResult": "R_GET", "KeyNotFound": "R_NOTFOUND", "PutOk": "R_PUTOK"}[n]
        assert c[key] == i == _hpp(AKH, key)
    for n in ("M_REQUEST", "M_REPLY", "T_CLIENT"):
        assert c[n] == _hpp(AKH, n)
    assert c["RETRY_MILLIS"] == _hpp(AKH, "kRetry")
    assert "r |= (long) t << (4 + 2 * i)" in AKC and "v |= t << (4 + 2 * j)" in open(
        os.path.join(ROOT, "dslabs_amd", "protocols.py")).read()
    assert "R_APPEND | v << 2" in AKC and "R_GET | v << 2" in AKC
    assert "int b = 2 + 4 * (c * MAX_CMDS + k);" in AKC and "const int b = 2 + 4 * (c * kMaxCmds + k);" in AKH
    # the Java rule (first-use numbering of keys and tokens, client-major) restated: AmoKV.params()
    for wl in AmoKV.WORKLOADS:
        for clients in (1, 2, 3):
            kv = AmoKV(clients, wl)
            keys, syms = [], []
            for cl in kv.cmds:
                for op, key, val in cl:
                    keys += [key] if key not in keys else []
                    syms += [val] if val is not None and val not in syms else []
            assert keys == kv.keys and syms == kv.syms, wl
    # Java timers / messages carry the device's fields
    tim = open(os.path.join(ROOT, "java", "src", "dslabs", "clientserver", "Timers.java")).read()
    assert "CLIENT_RETRY_MILLIS = 100" in tim and "private final int sequenceNum;" in tim
    assert 'Dsl.Event.message(from, to, M_REQUEST, seq, 0)' in AKC and 'e->n_fields = 2;' in AKH


def test_java_pb_codec_matches_the_device_layout_and_protocols_py():
    """lab2 (C4): PBCodec's bounds, message / timer codes, view, value, result and state-transfer
    bit layouts are pb.hpp's; timer periods are the device's; the predicate patterns parse the
    reference's predicate names (PrimaryBackupTest.java:104-156)."""
    from dslabs_amd.protocols import PB
    c = consts(PBC)
    assert (c["MAX_SERVERS"], c["MAX_CLIENTS"], c["MAX_CMDS"], c["MAX_KEYS"]) == tuple(
        _hpp(PBH, k) for k in ("kMaxServers", "kMaxClients", "kMaxCmds", "kMaxKeys"))
    enum = re.search(r"enum \{ M_PING = 0, ([^}]*)\}", PBH).group(1)
    names = ["M_PING"] + [e.split("=")[0].strip() for e in enum.split(",")]
    for i, n in enumerate(names[:9]):
        assert c[n] == i, n
    for n in ("T_PINGCHECK", "T_PING", "T_CLIENT"):
        assert c[n] == _hpp(PBH, n)
    for op, v in (("GET", 0), ("PUT", 1), ("APPEND", 2)):
        assert c["OP_" + op] == v == _hpp(PBH, "OP_" + op)
    assert "n | p << 4 | b << 6" in PBC and "return n | (p << 4) | (b << 6); }" in PBH
    assert PB._view_bits(3, 1, 2) == 3 | 1 << 4 | 2 << 6
    assert "r |= (long) t << (2 + 2 * i)" in PBC and "v |= t << (2 + 2 * j)" in open(
        os.path.join(ROOT, "dslabs_amd", "protocols.py")).read()
    assert "bits |= v << (8 * k)" in PBC and "const int vb = 32 + 8 * key;" in PBH  # keys in w1
    assert "(seq | r << 2) << (16 + 12 * c)" in PBC and "put(w, 48, 12, na); else put(w, 64, 12, na)" in PBH
    assert "v | app << 8" in PBC and "(uint64_t)v | (app << 8)" in PBH
    assert "| (long) ca << 4" in PBC and "((uint64_t)from << 4) | ((uint64_t)seq << 7)" in PBH
    assert "int b = 3 + 4 * (c * MAX_CMDS + k);" in PBC and "const int b = 3 + 4 * (c * kMaxCmds + k);" in PBH
    tim = open(os.path.join(ROOT, "java", "src", "dslabs", "primarybackup", "Timers.java")).read()
    assert "PING_CHECK_MILLIS = 100" in tim and "PING_MILLIS = 25" in tim and "CLIENT_RETRY_MILLIS = 100" in tim
    assert "e->timer_min = e->timer_max = 25;" in PBH
    reg = open(os.path.join(JAVA, "gpu", "GpuProtocols.java")).read()
    view = re.search(r'String VIEW = "([^"]*)";', reg).group(1).replace("\\\\", "\\")
    pats = {k: re.search(r'%s =\s*Pattern.compile\(([^;]*)\);' % k, reg).group(1) for k in
            ("HAS_VIEW_REPLY", "HAS_VIEW_REPLY_EXACT", "VIEW_REPLIES_SENT")}
    java = {k: "".join(view if part.strip() == "VIEW" else part.strip().strip('"') for part in v.split("+"))
            .replace("\\\\", "\\") for k, v in pats.items()}
    assert re.fullmatch(java["HAS_VIEW_REPLY"], "ViewReply with viewNum: 4")
    m = re.fullmatch(java["HAS_VIEW_REPLY_EXACT"], "ViewReply with View(viewNum=2, primary=server1, backup=null)")
    assert m and m.groups() == ("2", "server1", "null")
    m = re.fullmatch(java["VIEW_REPLIES_SENT"], "ViewReply for View(viewNum=2, primary=server1, backup=server2) "
                     "sent to nodes [server1, server2, client1], primary ack sent")
    assert m and m.groups() == ("2", "server1", "server2", "server1, server2, client1")
    ids = {n: int(v) for n, v in re.findall(r"DSL_PRED_([A-Z_]+) = (\d+)", HEADER)}
    assert "Leaf(500," in reg and ids["PB_HAS_VIEW_REPLY"] == 500
    assert "Leaf(501," in reg and ids["PB_VIEW_REPLY_EXACT"] == 501
    assert "Leaf(502," in reg and ids["PB_VIEW_REPLIES_SENT"] == 502


def test_java_dropped_network_uses_the_engine():
    """A dropped-network start state is packed on the engine (drop, then undrop from / to), not sent
    to the JVM search as round 3's GpuBFS did."""
    bfs = open(os.path.join(JAVA, "GpuBFS.java")).read()
    assert "hasDroppedNetwork" not in bfs
    assert "eng.setDropped(eng.dropPending(packed, undrop.from(), undrop.to()))" in bfs
    assert 'getDeclaredField("droppedNetwork")' in bfs and 'getDeclaredField("network")' in bfs


def test_java_pb_codec_bounds_every_packed_field():
    """every PB message encoder refuses (null: JVM fallback) a value wider than its device
    field -- viewNum 4 bits, sequenceNum 2 bits (pb.hpp: m & 15, (m >> 7) & 3) -- instead of
    spilling into the client-address bits."""
    src = open(os.path.join(JAVA, "gpu", "PBCodec.java")).read()
    assert src.count("bounded(") >= 5  # the helper + Ping, Request, Reply, StateTransferAck
    assert "v < 0 || v > 15 || seq < 0 || seq > 3" in src  # Forward / ForwardAck
    assert "n > 15" in src  # ViewReply / StateTransfer views
    assert "r < 0 || seq < 0 || seq > 3) return -1;" in src  # the lastResults of a StateTransfer's app


def test_java_kvstore_types_are_the_reference_lombok_declarations():
    """the KV command and result types are the reference stub's own Lombok @Data
    classes (labs/lab1-clientserver/src/dslabs/kvstore/KVStore.java:15-58, fluent accessors from
    the repository's lombok.config), not records with hand-written strings, so their toString is
    Lombok's "KVStore.Append(key=foo, value=X)" -- the form PaxosTest's hasCommand names carry
    (PaxosTest.java:119-121) and MultiPaxosCodec parses."""
    src = open(os.path.join(ROOT, "java", "src", "dslabs", "kvstore", "KVStore.java")).read()
    want = {"Get": ["key"], "Put": ["key, value"], "Append": ["key, value"], "GetResult": ["value"],
            "KeyNotFound": [], "PutOk": [], "AppendResult": ["value"]}
    for cls, fields in want.items():
        m = re.search(r"@Data\s+public static final class %s implements (\w+) \{(.*?)\n  \}" % cls, src, re.S)
        assert m, cls
        body = m.group(2)
        for f in fields:
            assert "@NonNull private final String %s;" % f in body, (cls, f)
        assert "toString" not in body
    assert "record " not in src and "toString()" not in src.split("public class KVStore")[1]
    codec = open(os.path.join(JAVA, "gpu", "MultiPaxosCodec.java")).read()
    pat = re.search(r'Pattern KV = Pattern\.compile\("(.*)"\);', codec).group(1).replace("\\\\", "\\")
    for s, g in (("KVStore.Append(key=foo, value=X)", ("Append", "foo", "X")), ("KVStore.Get(key=foo)", ("Get", "foo", None)),
                 ("KVStore.Put(key=foo, value=XY)", ("Put", "foo", "XY"))):
        assert re.fullmatch(pat, s).groups() == g, s
    # the Paxos / PB message and timer classes are Lombok @Data too (no hand-written strings)
    seen = 0
    for d in ("paxos", "primarybackup", "clientserver"):
        for f in os.listdir(os.path.join(ROOT, "java", "src", "dslabs", d)):
            text = open(os.path.join(ROOT, "java", "src", "dslabs", d, f)).read()
            assert not re.search(r"\nrecord \w+\(.*\) implements (?:Message|Timer)", text), f
            for m in re.finditer(r"\n((?:public )?(?:final )?class (\w+) implements (?:Message|Timer)\b)", text):
                assert "@Data\n" + m.group(1) in text, (f, m.group(2))
                seen += 1
            assert "String toString()" not in text, f
    assert seen >= 12, seen


def test_java_error_checks_keep_the_jvm_search():
    """GlobalSettings.doErrorChecks / doAllChecks (Search.java:201-220) report every
    offending event with its starting Java SearchState through CheckLogger, which the device cannot
    supply; so a checked run keeps the JVM search (before any engine is created), and the encoder
    never turns the device's sampled checks on (their counts would be dropped)."""
    bfs = open(os.path.join(JAVA, "GpuBFS.java")).read()
    i = bfs.index("public static SearchResults bfs(")
    body = bfs[i:bfs.index("new Dsl.Engine(", i)]
    assert "if (GlobalSettings.doErrorChecks()) return Search.bfs(init, settings);" in body
    enc = open(os.path.join(JAVA, "gpu", "GpuPredicates.java")).read()
    assert "m.set(ValueLayout.JAVA_INT, Dsl.OFF_DO_CHECKS, Dsl.CHECKS_NONE);" in enc
    assert "doAllChecks()" not in enc and "doErrorChecks()" not in enc
