"""bench.py's roofline objects on CPU: the random-access ceiling picked from the committed
calibration (profiles/r04_random_access_calibration.jsonl) and the probe mode by table size."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402


def test_random_access_roofline_modes():
    c3 = bench.random_access_roofline(1 << 35, 2.0e10, 5.0e9)  # the C3 bench's 32 GiB table
    assert c3["probe_mode"].startswith("load") and c3["calibrated_table_bytes"] == 1 << 35
    assert abs(c3["time_share"] - (2.0e10 / c3["load_ceiling_per_s"] + 5.0e9 / c3["cas_ceiling_per_s"])) < 1e-3
    c5 = bench.random_access_roofline(1 << 25, 4.0e9, 1.3e9)  # C5 d12's 32 MiB table: one CAS per probe
    assert c5["probe_mode"] == "CAS" and c5["calibrated_table_bytes"] == 1 << 25
    assert abs(c5["time_share"] - 4.0e9 / c5["cas_ceiling_per_s"]) < 1e-3
    assert 0 < c5["time_share"] < c3["time_share"] < 1.5
