"""C ABI: the library builds for gfx950, loads, and exports every symbol include/dslabs_hip.h
declares. No compute calls (there is no GPU in the CPU job)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    with open(os.path.join(ROOT, "include", "dslabs_hip.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(dsl_[a-z_]+)\s*\(", src)))


def test_header_and_binding_agree():
    from dslabs_amd import _lib
    assert sorted(_lib.EXPORTED) == _declared()


def _lib_version():
    from dslabs_amd import _lib
    return _lib.DSL_ABI_VERSION


def test_abi_version_matches_the_header():
    with open(os.path.join(ROOT, "include", "dslabs_hip.h")) as f:
        v = int(re.search(r"#define DSL_ABI_VERSION (\d+)", f.read()).group(1))
    assert v == _lib_version()


def test_library_exports_all_symbols(lib):
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.dsl_abi_version() == _lib_version()


def test_struct_layouts(lib):
    from dslabs_amd import _lib
    # sizes must match the C structs (checked against offsets hard-coded from the header)
    assert ctypes.sizeof(_lib.dsl_predicate) == 24
    assert ctypes.sizeof(_lib.dsl_event) == 32 + 8 * 8
    assert ctypes.sizeof(_lib.dsl_protocol_desc) == 8 + 8 * 64


def test_state_bytes_without_device(lib):
    from dslabs_amd.protocols import PingPong
    # 5 nodes x 5 words + count + 120 32-bit records, padded to 16 bytes
    assert lib.dsl_state_bytes(ctypes.byref(PingPong(1, 10).desc())) == 592


def test_create_fails_loudly_without_device(lib):
    import pytest
    from dslabs_amd import _lib
    if lib.dsl_device_count() > 0:
        pytest.skip("a GPU is visible")
    from dslabs_amd.protocols import pingpong_state
    from dslabs_amd import Search
    with pytest.raises(_lib.EngineError) as ei:
        Search.bfs(pingpong_state(1, 2))
    assert "DSL_ERR_NO_DEVICE" in str(ei.value)


def test_ctypes_structs_match_the_c_header(tmp_path):
    """sizeof / offsetof of every ABI struct, compiled from include/dslabs_hip.h with gcc, against
    the ctypes mirrors in dslabs_amd/_lib.py."""
    import subprocess
    from dslabs_amd import _lib
    structs = {"dsl_protocol_desc": ["protocol", "params"], "dsl_engine_config": ["comm_id", "replicate_below", "flags"],
               "dsl_host_comm": ["allgather_u64", "alltoallv", "flags"],
               "dsl_settings": ["table_log2_slots", "max_frontier_states"], "dsl_event": ["fields"],
               "dsl_result": ["per_depth", "trace", "terminal_state"], "dsl_stats": ["table_slots", "probes", "host_syncs", "rccl_version", "cost_x_us", "shard_work_min"],
               "dsl_dfs_config": ["max_probes", "max_trace", "no_minimize"], "dsl_predicate": ["arg1"]}
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "dslabs_hip.h"', "int main(void) {"]
    for st, fields in structs.items():
        src.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for f in fields:
            src.append(f'printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    src.append("return 0; }")
    c = tmp_path / "abi.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "abi"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(c)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                       text=True).stdout.splitlines())
    from dslabs_amd import distributed
    for st, fields in structs.items():
        cls = getattr(_lib, st, None) or getattr(distributed, st)
        assert ctypes.sizeof(cls) == int(got[st]), st
        for f in fields:
            assert getattr(cls, f).offset == int(got[f"{st}.{f}"]), (st, f)


def test_drop_and_undrop_pending_messages_without_device(lib):
    """SearchState.dropPendingMessages / undropMessages* (SearchState.java:538-561) on packed
    states (host functions of the library): dropping empties the network into the dropped set,
    undropping everything restores the state exactly, undropMessagesFrom restores a subset."""
    from dslabs_amd.protocols import MultiPaxos, PingPong
    for proto in (PingPong(2, 3), MultiPaxos(3, 2, "append-xy")):
        st = proto.initial_state()
        init = st._packed_now()
        st.dropPendingMessages()
        assert st.droppedMessages() == sorted(set(st.droppedMessages()))
        st.undropMessages()
        assert st.packed == init  # sends of init() are the whole network; all come back
        st.dropPendingMessages()
        n_all = len(st.droppedMessages())
        st.undropMessagesFrom(proto.addresses[0])
        st2 = proto.initial_state()
        st2.dropPendingMessages()
        assert len(st2.droppedMessages()) == n_all
        st2.dropPendingMessages()  # dropping twice keeps the set
        assert len(st2.droppedMessages()) == n_all
