# SQ instruction counters of k_level (one search, d12) for the product library and the variants
# in $DSL_VARIANTS; one rocprofv3 --pmc pass per counter group.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_r02
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for V in base $DSL_VARIANTS; do
  LV=$V; [ "$V" = base ] && LV=""
  for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"; do
    N=$(echo $P | cut -d' ' -f1)
    DSL_LIB_VARIANT=$LV timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'k_level' -f csv -T -d $OUT/${V}_$N -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS} > $OUT/${V}_$N.json 2> $OUT/${V}_$N.err
  done
done
python3 - <<'PY'
import csv, glob, os, collections
out = "gpurun_out/pmc_r02"
res = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + "/*/run_counter_collection.csv"):
    v = os.path.basename(os.path.dirname(f)).split("_SQ")[0]
    for r in csv.DictReader(open(f)):
        res[v][r["Counter_Name"]] += float(r["Counter_Value"])
for v, d in sorted(res.items()):
    print(v, " ".join("%s=%.4g" % (k.replace("SQ_", ""), x) for k, x in sorted(d.items())))
PY
