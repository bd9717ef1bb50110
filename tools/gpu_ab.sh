# A/B of an environment switch on the default bench line: bench.py alternately without and with
# $AB_ENV (e.g. AB_ENV=DSL_QSPAN_FIXED=1), $AB_N rounds each, --no-cpu-baseline.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04_${TAG:-ab}
mkdir -p $OUT
for i in $(seq 1 ${AB_N:-3}); do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/a$i.json 2>> $OUT/err.log
  timeout -k 10 120 env $AB_ENV python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/b$i.json 2>> $OUT/err.log
  python3 -c "import json,sys; a=json.load(open('$OUT/a$i.json')); b=json.load(open('$OUT/b$i.json')); print('A %.4g %.3f ms k=%.4f | B %.4g %.3f ms k=%.4f' % (a['value'], a['ms_per_step'], a['roofline']['avg_launch_ms'], b['value'], b['ms_per_step'], b['roofline']['avg_launch_ms']))"
done
