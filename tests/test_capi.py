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


def test_library_exports_all_symbols(lib):
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.dsl_abi_version() == 1


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
