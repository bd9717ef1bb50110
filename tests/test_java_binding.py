"""The Java integration layer (java/src) cannot be compiled here (no JDK), so its
native-memory contract is checked statically: every struct size and field offset the Panama FFM
binding (java/src/.../gpu/Dsl.java) hard-codes equals the C header's (through the ctypes mirror,
itself checked against the header by test_capi.py), and the end-condition and predicate ids the
Java registry uses equal the header's enums."""
import ctypes
import os
import re

from dslabs_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "src", "dslabs", "framework", "testing", "search")
DSL = open(os.path.join(JAVA, "gpu", "Dsl.java")).read()
HEADER = open(os.path.join(ROOT, "include", "dslabs_hip.h")).read()


def consts():
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"\b((?:OFF|SIZE|END)_[A-Z0-9_]+) = (-?\d+)", DSL)}


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
                     "MEMORY_BUDGET": "memory_budget_bytes", "POOL": "pool"},
    "dsl_engine_config": {"ENGINE_CONFIG": None, "CFG_DEVICE": "device", "CFG_RANK": "rank",
                          "CFG_WORLD": "world_size", "CFG_VSHARDS": "virtual_shards", "CFG_COMM_ID": "comm_id",
                          "CFG_REPLICATE_BELOW": "replicate_below"},
    "dsl_event": {"EVENT": None, "EV_IS_TIMER": "is_timer", "EV_FROM": "from_", "EV_TO": "to", "EV_TYPE": "type",
                  "EV_N_FIELDS": "n_fields", "EV_TIMER_MIN": "timer_min", "EV_TIMER_MAX": "timer_max",
                  "EV_FIELDS": "fields"},
    "dsl_result": {"RESULT": None, "RES_END": "end_condition", "RES_TERMINAL_DEPTH": "terminal_depth",
                   "RES_PRED_INDEX": "predicate_index", "RES_MAX_DEPTH": "max_depth", "RES_STATES": "states",
                   "RES_N_LEVELS": "n_levels", "RES_TRACE_LEN": "trace_len", "RES_PER_DEPTH": "per_depth",
                   "RES_TRACE": "trace", "RES_TERMINAL_STATE": "terminal_state", "RES_STATE_BYTES": "state_bytes",
                   "RES_INITIAL_DEPTH": "initial_depth", "RES_ELAPSED": "elapsed_s"},
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
    assert checked == 59


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
