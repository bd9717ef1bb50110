# Per-level k_level durations of the C5 d12 search for each library variant in $DSL_VARIANTS
# ("default" = the product library). usage: DSL_VARIANTS="a b" bash tools/gpu_level_times.sh TAG [bench args]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/vlev_$TAG
mkdir -p $OUT
for r in 1 2; do
for V in $DSL_VARIANTS; do
  LV=$V; [ "$V" = default ] && LV=
  DSL_LIB_VARIANT=$LV timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $OUT/kt_${V}_$r -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > $OUT/b_${V}_$r.json 2> $OUT/e_${V}_$r.err
  echo "$V/$r: $(python3 tools/level_times.py $OUT/kt_${V}_$r/run_kernel_trace.csv)" | tee -a $OUT/summary.txt
done
done
echo done $TAG
