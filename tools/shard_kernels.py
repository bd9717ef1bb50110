"""Per-kernel GPU time of the last search in a rocprofv3 kernel trace of tools/shard_scale.py (the
dispatches after the last W k_setup launches). usage: python3 tools/shard_kernels.py trace.csv W"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
W = int(sys.argv[2])
setups = [i for i, r in enumerate(rows) if "k_setup" in r["Kernel_Name"]]
last = rows[setups[-W]:]
agg = collections.defaultdict(lambda: [0, 0.0])
names = ("k_level_record", "k_level", "k_probe_slab", "k_new_list", "k_materialize", "k_copy_segments",
         "k_route_headers", "k_unspill", "k_setup", "k_respill", "k_probe_remote")
for r in last:
    n = next((k for k in names if k in r["Kernel_Name"]), r["Kernel_Name"][:40])
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
t0, t1 = int(last[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in last)
tot = sum(v[1] for v in agg.values())
print(f"# W={W}: last search, {len(last)} dispatches, kernel time {tot:.1f} us, first start -> last end {(t1 - t0) / 1e3:.1f} us")
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:34s} {v[0]:5d} launches {v[1]:10.1f} us")

# per level: the dispatches from one level's first k_level to the next level's (sharded levels run
# k_level on every shard, then the exchange kernels); the sum per kernel / W is one GPU's share
levels, cur, prev_level = [], None, False
for r in last:
    is_level = "k_level" in r["Kernel_Name"] and "record" not in r["Kernel_Name"]
    if is_level and not prev_level:
        cur = collections.defaultdict(float)
        levels.append(cur)
    prev_level = is_level
    if cur is None:
        continue
    n = next((k for k in names if k in r["Kernel_Name"]), "other")
    cur[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("# per level (us, summed over the W shards): " + ", ".join(names[:6]))
for i, lv in enumerate(levels):
    print(f"level {i + 1}: " + " ".join(f"{lv.get(k, 0):.0f}" for k in names[:6]) + f" | total {sum(lv.values()):.0f}")
