"""Generates the device and oracle forms of every IR protocol spec (dslabs_amd/ir/specs/*.py):
dslabs_amd/csrc/protocols/gen/<name>.hpp and oracle/gen/proto_<name>.hpp.
usage: python tools/gen_ir.py [--check]   (--check: exit 1 if a generated file is stale)"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dslabs_amd.ir import gen_device, gen_oracle  # noqa: E402

SPECS = ["pingpong", "amokv", "multipaxos", "pb"]


def outputs():
    for name in SPECS:
        mod = importlib.import_module(f"dslabs_amd.ir.specs.{name}")
        src = f"dslabs_amd/ir/specs/{name}.py"
        yield os.path.join(ROOT, "dslabs_amd", "csrc", "protocols", "gen", f"{mod.P.name}.hpp"), \
            gen_device.generate(mod.P, src)
        mod = importlib.reload(mod)  # fresh declarations (layout() appends internal fields)
        yield os.path.join(ROOT, "oracle", "gen", f"proto_{mod.P.name}.hpp"), gen_oracle.generate(mod.P, src)


def main():
    check = "--check" in sys.argv
    stale = []
    for path, text in outputs():
        old = open(path).read() if os.path.exists(path) else None
        if old != text:
            stale.append(path)
            if not check:
                os.makedirs(os.path.dirname(path), exist_ok=True)
                with open(path, "w") as f:
                    f.write(text)
    for p in stale:
        print(("stale: " if check else "wrote: ") + os.path.relpath(p, ROOT))
    return 1 if (check and stale) else 0


if __name__ == "__main__":
    sys.exit(main())
