# A/B of library variants (DSL_LIB_VARIANT): VARIANTS="pad0 pad1" beside the product library (NOPRODUCT=1: without it),
# $VN alternating rounds of bench.py --no-cpu-baseline $BENCH_ARGS; then, with PMC=1, one
# LDS-counter pass per variant (SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT, SQ_WAVE_CYCLES, SQ_WAIT_ANY).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-var}
mkdir -p $OUT
LIST="product $VARIANTS"; [ -n "$NOPRODUCT" ] && LIST="$VARIANTS"
for i in $(seq 1 ${VN:-2}); do
  for v in $LIST; do
    vv=$v; [ "$v" = product ] && vv=""
    DSL_LIB_VARIANT=$vv timeout -k 10 200 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$v.$i.json 2>> $OUT/err.log
    python3 -c "import json; a=json.load(open('$OUT/$v.$i.json')); r=a['roofline']; print('%-8s %.4g states/s %.3f ms k=%.4f slots=%s' % ('$v', a['value'], a['ms_per_step'], r['avg_launch_ms'], r.get('level_slots')))"
  done
done
if [ -n "$PMC" ]; then
  for v in product $VARIANTS; do
    vv=$v; [ "$v" = product ] && vv=""
    DSL_LIB_VARIANT=$vv timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-include-regex 'k_level' -f csv -T -d $OUT/pmc_$v -o run -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} --steps 1 --warmup 0 > $OUT/pmc_$v.json 2> $OUT/pmc_$v.err
    python3 tools/pmc_lds.py $OUT/pmc_$v $v
  done
fi
echo variants done
