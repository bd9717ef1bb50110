"""LDS counters of k_level from one rocprofv3 --pmc pass (tools/gpu_variants.sh): extra bank-conflict
cycles per LDS instruction, and the wave wait fraction. usage: python3 tools/pmc_lds.py DIR LABEL"""
import csv
import glob
import os
import sys
from collections import defaultdict

tot = defaultdict(float)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_level" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
lds, conf = tot.get("SQ_INSTS_LDS", 0), tot.get("SQ_LDS_BANK_CONFLICT", 0)
wc, wa = tot.get("SQ_WAVE_CYCLES", 0), tot.get("SQ_WAIT_ANY", 0)
print(f"{sys.argv[2] if len(sys.argv) > 2 else ''}: SQ_INSTS_LDS {lds:.4g} SQ_LDS_BANK_CONFLICT {conf:.4g} "
      f"conflict/inst {conf / lds if lds else 0:.3f} wait/wave {wa / wc if wc else 0:.3f}")
