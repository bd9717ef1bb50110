"""Register / LDS / scratch budget of the built kernels, read from the code object's metadata (the
authoritative numbers: rocprofv3's VGPR_Count column reports 64 for k_level<MultiPaxos>, whose code
object says .vgpr_count 128 and .agpr_count 0 -- 4 waves per SIMD of the 512-entry register file).

  python3 tools/kernel_meta.py [lib.so] [name-regex]   ->  one JSON line per matching kernel
"""
from __future__ import annotations

import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
FIELDS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
          ".private_segment_fixed_size", ".group_segment_fixed_size", ".max_flat_workgroup_size")


def code_object(lib: str, tmp: str) -> str:
    """The gfx950 code object of a HIP fat binary (llvm-objdump --offloading writes it beside lib)."""
    src = os.path.join(tmp, os.path.basename(lib))
    shutil.copy(lib, src)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", src], check=True, cwd=tmp,
                   capture_output=True)
    for f in os.listdir(tmp):
        if "gfx950" in f:
            return os.path.join(tmp, f)
    raise SystemExit("no gfx950 code object in " + lib)


def kernels(co: str) -> list[dict]:
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                           capture_output=True, text=True).stdout
    out, cur = [], {}
    for line in notes.splitlines():
        s = line.strip().lstrip("- ").strip()
        for f in FIELDS + (".name",):
            if s.startswith(f + ":"):
                v = s.split(":", 1)[1].strip()
                if f == ".name":
                    cur["name"] = v
                else:
                    cur[f[1:]] = int(v)
        if s.startswith(".wavefront_size:") and "name" in cur:  # the last field of a kernel's map
            out.append(cur)
            cur = {}
    return out


def main() -> None:
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "dslabs_amd", "libdslabs_hip.so")
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_level")
    with tempfile.TemporaryDirectory() as tmp:
        for k in kernels(code_object(lib, tmp)):
            if pat.search(k["name"]):
                dem = subprocess.run(["c++filt", k["name"]], capture_output=True, text=True).stdout.strip()
                k["kernel"] = dem.split("(")[0]
                k["waves_per_simd"] = min(8, 512 // max(1, k.get("vgpr_count", 0) + k.get("agpr_count", 0)))
                print(json.dumps(k))


if __name__ == "__main__":
    main()
