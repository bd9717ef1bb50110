"""Where a search's wall time goes beyond its kernels (rocprofv3 kernel trace of bench.py): per
search, the device-idle gaps between k_setup and the first level, between levels, and from the last
level to the next search's k_setup. usage: python3 tools/search_gaps.py run_kernel_trace.csv"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ev = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
setups = [i for i, e in enumerate(ev) if "k_setup" in e[0]]
searches = []
for a, b in zip(setups, setups[1:] + [len(ev)]):
    seg = ev[a:b]
    busy = sum(e[2] - e[1] for e in seg)
    span = (ev[b][1] if b < len(ev) else seg[-1][2]) - seg[0][1]
    lv = [e for e in seg if "k_level" in e[0] and "record" not in e[0]]
    first_gap = lv[0][1] - seg[0][2] if lv else 0
    tail = (ev[b][1] - lv[-1][2]) if lv and b < len(ev) else 0
    searches.append((span, busy, first_gap, tail, len(seg)))
last = searches[-12:-1] if len(searches) > 12 else searches[:-1]
f = lambda i: statistics.median(x[i] for x in last) / 1e3
print(f"searches {len(searches)}; median of the last {len(last)} (us): setup->setup {f(0):.1f}, "
      f"kernel busy {f(1):.1f}, k_setup end -> first level {f(2):.1f}, last level end -> next k_setup {f(3):.1f}, "
      f"dispatches {statistics.median(x[4] for x in last)}")
for name in sorted({e[0][:50] for s in [ev[setups[-2]:setups[-1]]] for e in s}):
    pass
seg = ev[setups[-2]:setups[-1]]
t0 = seg[0][1]
print("last full search:", " ".join(f"{e[0].split('(')[0].split('<')[0][-22:]}@{(e[1] - t0) / 1e3:.1f}+{(e[2] - e[1]) / 1e3:.1f}" for e in seg))
