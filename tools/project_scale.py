"""Projects the 1/2/4/8-GPU time of one search from virtual-shard measurements (one GPU): the
kernel trace of a W-shard run gives each sharded level's kernel time summed over the shards
(one GPU's share = the sum / W, the shards' work being balanced), its DSL_LEVEL_TRACE lines give
the slab (records per sub-slab, cs) of every sharded level, and the unsharded (W = 1) trace gives
the replicated levels. xGMI is not measured here: a level's two exchange rounds are priced at
BW GB/s per link (every pair of GPUs has its own link, so a GPU's W - 1 regions move in parallel)
plus a fixed per-round latency, and the level's one host round trip at SYNC us.

usage: python3 tools/project_scale.py TRACE_W1.csv ERR_W1 TRACE_W.csv ERR_W W [BW_GBs] [ROUND_US] [SYNC_US]"""
import collections
import csv
import re
import sys


def level_kernels(path, shards):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    setups = [i for i, r in enumerate(rows) if "k_setup" in r["Kernel_Name"]]
    last = rows[setups[-shards]:]
    levels, cur, prev = [], None, False
    for r in last:
        is_level = "k_level" in r["Kernel_Name"] and "record" not in r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if shards == 1 and is_level and dur < 8.0:
            continue  # a queued level after the queue's stop rule (returns at once)
        if is_level and (not prev or shards == 1):  # one GPU: the device queue runs levels back to back
            cur = collections.defaultdict(float)
            levels.append(cur)
        prev = is_level
        if cur is not None and "k_copy_segments" not in r["Kernel_Name"]:
            name = "k_level" if is_level else r["Kernel_Name"].split("(")[0].split("<")[0][-24:]
            cur[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return levels


def shard_lines(path):
    out = {}
    for line in open(path):
        m = re.match(r"\[shard\] depth (\d+) cs (\d+) last (\d)", line)
        if m:
            out[int(m.group(1))] = (int(m.group(2)), int(m.group(3)))  # the last search's wins
    return out


def main():
    t1, e1, tw, ew, W = sys.argv[1:6]
    W = int(W)
    bw = float(sys.argv[6]) if len(sys.argv) > 6 else 50.0
    round_us = float(sys.argv[7]) if len(sys.argv) > 7 else 10.0
    sync_us = float(sys.argv[8]) if len(sys.argv) > 8 else 25.0
    single = level_kernels(t1, 1)
    multi = level_kernels(tw, W)
    slabs = shard_lines(ew)
    t_single = sum(sum(l.values()) for l in single)
    t_multi = 0.0
    rep_t, sh_t = [], []
    print(f"# W={W}: per level, one GPU's time (us): kernels (sum over shards / W), exchange at {bw} GB/s per link "
          f"+ {round_us} us per round, {sync_us} us host round trip; replicated levels as on one GPU")
    for i, lv in enumerate(multi):
        depth = i + 1
        k = sum(lv.values())
        if depth in slabs:
            cs, last = slabs[depth]
            region = (22 + 32 * cs) * 12  # bytes of one (source, owner) region: 12-byte packed records (round 6)
            comm = region / (bw * 1e3) + round_us + (0 if last else (16 + 32 * cs) / (bw * 1e3) + round_us)  # round B: a byte per record
            t = k / W + comm + sync_us
            print(f"level {depth}: sharded, kernels {k / W:.1f} + exchange {comm:.1f} + sync {sync_us} = {t:.1f} "
                  f"(one GPU: {sum(single[i].values()):.1f})")
            sh_t.append(t)
        else:
            t = sum(single[i].values())
            print(f"level {depth}: replicated {t:.1f}")
            sh_t.append(None)
        rep_t.append(sum(single[i].values()))
        t_multi += t
    print(f"kernels of one search on one GPU {t_single:.1f} us; projected at W={W}: {t_multi:.1f} us "
          f"-> {t_single / t_multi:.2f}x (per-search host time excluded from both)")
    # the cost rule's plan: replicated up to some level, sharded from there on (a sharded level's
    # tables no longer hold every state), the switch where it pays most
    best, best_s = sum(rep_t), len(rep_t)
    for sw in range(len(rep_t)):
        if any(x is None for x in sh_t[sw:]):
            continue
        t = sum(rep_t[:sw]) + sum(sh_t[sw:])
        if t < best:
            best, best_s = t, sw
    plan = "replicated throughout" if best_s == len(rep_t) else f"sharded from level {best_s + 1}"
    print(f"best plan ({plan}): {best:.1f} us -> {t_single / best:.2f}x")


if __name__ == "__main__":
    main()
