"""Per-level k_level durations (us) of the last BFS in a rocprofv3 --kernel-trace CSV: the
k_level dispatches after the last k_setup (k_seed before round 2's setup kernel). usage: python3 tools/level_times.py run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last_seed = max(i for i, r in enumerate(rows) if ("k_seed" in r["Kernel_Name"] or "k_setup" in r["Kernel_Name"]))
lv = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[last_seed:]
      if "k_level" in r["Kernel_Name"]]
t0 = int(rows[last_seed]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in rows[last_seed:])
print(" ".join(f"{x:.1f}" for x in lv), f"| sum {sum(lv):.1f} us, seed..end {(t1 - t0) / 1e3:.1f} us")
