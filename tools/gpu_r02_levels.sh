# Per-level k_level durations of the C5 bench search (kernel trace, one dispatch per row) and the
# engine's level trace (queued and unqueued). usage: bash tools/gpu_r02_levels.sh TAG [bench args]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/levels_$TAG
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/kt -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > $OUT/kt_bench.json 2> $OUT/kt.err
DSL_LEVEL_TRACE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > $OUT/lt.json 2> $OUT/lt.err
DSL_LEVEL_TRACE=1 DSL_NO_QUEUE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > $OUT/ltnq.json 2> $OUT/ltnq.err
echo done $TAG
