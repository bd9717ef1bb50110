"""Summarizes a tools/gpu_prof.sh run (rocprofv3 kernel trace + separate PMC passes) for the
dominant kernel k_level: per-launch duration, FETCH_SIZE / WRITE_SIZE (KB in rocprofv3), HBM
traffic per launch with the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE reports half the
bytes of 16-byte-per-lane reads: x2), and the SQ counters. Writes one JSON object.

    python tools/pmc_summary.py gpurun_out/prof_TAG [k_levelINS_10MultiPaxosELb0E] > profiles/rNN_pmc_WORKLOAD_dDEPTH.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = "k_level"


def per_dispatch(path):
    by = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        by[d][r["Counter_Name"]] = float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    return by


def code_object_meta(pattern):
    """.vgpr_count / .agpr_count / spills / scratch / LDS of the kernel whose mangled name matches
    `pattern` (e.g. k_levelINS_10MultiPaxosELb0E) in the in-tree library's code object
    (tools/kernel_meta.py; None when the library or the LLVM tools are missing)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "dslabs_amd", "libdslabs_hip%s.so" % (
        "_" + os.environ["DSL_LIB_VARIANT"] if os.environ.get("DSL_LIB_VARIANT") else ""))
    try:
        out = subprocess.run([sys.executable, os.path.join(root, "tools", "kernel_meta.py"), lib, pattern],
                             capture_output=True, text=True, timeout=120).stdout
    except Exception:
        return None
    for line in out.splitlines():
        k = json.loads(line)
        return {x: k[x] for x in ("kernel", "vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count",
                                  "private_segment_fixed_size", "group_segment_fixed_size", "waves_per_simd")}
    return None


def main(d):
    out = {"kernel": KERNEL, "source": os.path.basename(d.rstrip("/"))}
    kt = os.path.join(d, "kt", "run_kernel_trace.csv")
    if os.path.exists(kt):
        rows = [r for r in csv.DictReader(open(kt)) if KERNEL in r["Kernel_Name"]]
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
        out["launches_traced"] = len(durs)
        out["avg_launch_ms"] = sum(durs) / max(1, len(durs))
        # rocprofv3's columns (on gfx950 its VGPR_Count reads 64 for a 128-VGPR k_level); the
        # code object's own metadata (tools/kernel_meta.py) is authoritative, added when the
        # library is at hand
        out["vgpr_rocprof"] = rows[0].get("VGPR_Count") if rows else None
        out["scratch_bytes_per_lane"] = rows[0].get("Scratch_Size") if rows else None
        if rows and len(sys.argv) > 2:  # the instantiation (rocprofv3 -T truncates the name to k_level)
            out["code_object"] = code_object_meta(sys.argv[2])
    tot = defaultdict(float)
    n = 0
    for f in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
        disp = per_dispatch(f)
        n = max(n, len(disp))
        for v in disp.values():
            for k, x in v.items():
                tot[k] += x
    if n:
        out["pmc_launches"] = n
        out["counters_total"] = {k: v for k, v in sorted(tot.items())}
        fetch = tot.get("FETCH_SIZE", 0.0) * 1024
        write = tot.get("WRITE_SIZE", 0.0) * 1024
        out["fetch_bytes_raw_per_launch"] = fetch / n
        out["write_bytes_per_launch"] = write / n
        # gfx950: FETCH_SIZE counts half the bytes of 16-B/lane reads (the staging and bucket loads)
        out["hbm_bytes_per_launch"] = (2 * fetch + write) / n
        # the PMC passes run one search (bench.py --steps 1 --warmup 0): totals are per step, and
        # bench.py divides them by its own launches per step (queued levels that stopped early are
        # dispatched but do no work)
        out["hbm_bytes_per_step"] = 2 * fetch + write
        # raw per-search counters: bench.py applies the calibrated correction
        # (profiles/r01_hbm_calibration.json: FETCH_SIZE is exact for the random 64-B bucket lines
        # and half of the 16-B/lane streaming staging reads; WRITE_SIZE is exact)
        out["fetch_bytes_per_step"] = fetch
        out["write_bytes_per_step"] = write
        # visited-set atomics (north_star: atomic throughput of the probe/insert): every atomic
        # request at the L2 per search, over the search's k_level time (launches in one search x
        # the traced average launch)
        if "TCC_ATOMIC_sum" in tot:
            out["atomics_per_step"] = tot["TCC_ATOMIC_sum"]
            out["atomics_to_dram_per_step"] = tot.get("TCC_EA0_WRREQ_ATOMIC_DRAM_sum")
            if out.get("avg_launch_ms"):
                out["atomics_per_s"] = tot["TCC_ATOMIC_sum"] / (out["avg_launch_ms"] * n / 1e3)
        if tot.get("TCC_EA0_RDREQ_sum"):
            # memory-side reads that went to DRAM (the rest were served by the Infinity Cache)
            out["dram_read_frac"] = tot.get("TCC_EA0_RDREQ_DRAM_sum", 0) / tot["TCC_EA0_RDREQ_sum"]
            if tot.get("TCC_EA0_WRREQ_sum"):
                out["dram_write_frac"] = tot.get("TCC_EA0_WRREQ_DRAM_sum", 0) / tot["TCC_EA0_WRREQ_sum"]
        if tot.get("TCC_HIT_sum") is not None and tot.get("TCC_MISS_sum") is not None:
            out["l2_hit_rate"] = tot["TCC_HIT_sum"] / max(1.0, tot["TCC_HIT_sum"] + tot["TCC_MISS_sum"])
        if "SQ_WAVE_CYCLES" in tot and tot.get("SQ_WAVE_CYCLES"):
            out["wait_frac"] = tot.get("SQ_WAIT_ANY", 0) / tot["SQ_WAVE_CYCLES"] if "SQ_WAIT_ANY" in tot else None
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
