"""Ratios of rocprofv3 FETCH_SIZE / WRITE_SIZE to the known bytes of tools/hbm_calib.hip's kernels.
usage: python tools/hbm_calib.py OUTDIR   (OUTDIR/fetch, OUTDIR/write from tools/gpu_calib.sh)"""
import csv
import glob
import json
import sys

BYTES = 2 << 30


def dispatches(d, counter):
    rows = {}
    for f in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = int(r["Dispatch_Id"])
            rows.setdefault(k, [r["Kernel_Name"], 0.0])[1] += float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def main(d):
    fetch = dispatches(d + "/fetch", "FETCH_SIZE")
    write = dispatches(d + "/write", "WRITE_SIZE")
    out = []
    for (name, fkb), (_, wkb) in zip(fetch, write):
        short = name.split("(")[0].replace("void ", "")
        out.append({"kernel": short, "fetch_over_bytes": round(fkb * 1024 / BYTES, 3),
                    "write_over_bytes": round(wkb * 1024 / BYTES, 3)})
    json.dump({"buffer_bytes": BYTES, "dispatches": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
