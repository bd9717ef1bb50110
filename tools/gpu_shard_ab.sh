# A/B of the sharded path's kernels on virtual shards: kernel traces of tools/shard_scale.py for
# library variants (VARIANTS, beside the product library) and k_materialize grid caps (MATB), then
# tools/shard_kernels.py per-level summaries. Output: gpurun_out/$TAG/.
# usage: TAG=x VARIANTS="routeblock" MATB="256 8192" MATP="4 8" WL="multipaxos 12" W=8 bash tools/gpu_shard_ab.sh
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-shard_ab}
mkdir -p $OUT
W=${W:-8}
WL=${WL:-multipaxos 12}
if [ "${WL%% *}" = "multipaxos" ]; then ARGS="--workload $WL"; REP=10000; else ARGS="$WL"; REP=100000; fi
run() {  # name, env...
  local name=$1; shift
  mkdir -p $OUT/$name
  env "$@" DSL_LEVEL_TRACE=1 DSL_SCALE_REPLICATE_BELOW=$REP timeout -k 10 300 rocprofv3 --kernel-trace -f csv -T -d $OUT/$name/kt -o run -- python3 tools/shard_scale.py $ARGS $W > $OUT/$name/out.jsonl 2> $OUT/$name/err.txt
  python3 tools/shard_kernels.py $OUT/$name/kt/run_kernel_trace.csv $W > $OUT/$name/kernels.txt
  echo "== $name"; tail -6 $OUT/$name/kernels.txt
}
for v in product $VARIANTS; do
  vv=$v; [ "$v" = product ] && vv=""
  run $v DSL_LIB_VARIANT=$vv
done
for m in $MATB; do
  run matb$m DSL_MAT_BLOCKS=$m
done
for m in $MATP; do  # states per wave, grid 4096 workgroups
  run matp$m DSL_MAT_PER=$m DSL_MAT_BLOCKS=4096
done
echo shard ab done
