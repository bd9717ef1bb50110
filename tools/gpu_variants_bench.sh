# Bench line of each library variant (DSL_LIB_VARIANT), $VN rounds: VARIANTS="w4 w6" plus the
# product library (""), BENCH_ARGS passed to bench.py --no-cpu-baseline.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04_${TAG:-var}
mkdir -p $OUT
for i in $(seq 1 ${VN:-2}); do
  for v in product $VARIANTS; do
    vv=$v; [ "$v" = product ] && vv=""
    DSL_LIB_VARIANT=$vv timeout -k 10 150 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$v.$i.json 2>> $OUT/err.log
    python3 -c "import json; a=json.load(open('$OUT/$v.$i.json')); r=a['roofline']; print('%-8s %.4g states/s %.3f ms k=%.4f slots=%s' % ('$v', a['value'], a['ms_per_step'], r['avg_launch_ms'], r.get('level_slots')))"
  done
done
