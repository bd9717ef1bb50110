"""Runs the CPU oracle (oracle/_build/dslabs_oracle). Test infrastructure only."""
from __future__ import annotations

import json
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle", "_build", "dslabs_oracle")


def ensure_built() -> str:
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return ORACLE


def run(mode: str, args, timeout: float = 120) -> dict:
    ensure_built()
    out = subprocess.run([ORACLE, mode] + list(args), check=True, capture_output=True, text=True,
                         timeout=timeout)
    return json.loads(out.stdout)


def replay(args, events, timeout: float = 60) -> dict:
    with tempfile.NamedTemporaryFile("w", suffix=".trace", delete=False) as f:
        f.write("\n".join(events) + "\n")
        path = f.name
    try:
        return run("replay", list(args) + ["--trace-file", path], timeout=timeout)
    finally:
        os.unlink(path)


def replay_search(args, events, minimize: bool, timeout: float = 60) -> dict:
    """TraceReplaySearch on the oracle (checkState per step, TraceMinimizer when `minimize`;
    with "--human-readable" in args the reported state's trace is SearchState.humanReadableTrace)."""
    with tempfile.NamedTemporaryFile("w", suffix=".trace", delete=False) as f:
        f.write("\n".join(events) + "\n")
        path = f.name
    try:
        return run("replaysearch", list(args) + ["--trace-file", path] + (["--minimize"] if minimize else []),
                   timeout=timeout)
    finally:
        os.unlink(path)
