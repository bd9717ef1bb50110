# GPU run of the product library: the GPU suite and smoke (TESTS selects tests, default all;
# NOTESTS=1 skips them), then the default bench line unless NOBENCH=1. Output: gpurun_out/$TAG.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
if [ -z "$NOTESTS" ]; then
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
fi
if [ -z "$NOBENCH" ]; then
timeout -k 10 300 python3 bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
cut -c1-300 $OUT/bench.json
fi
echo suite done
