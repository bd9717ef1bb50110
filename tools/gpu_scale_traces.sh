# Kernel traces (rocprofv3) + level traces of tools/shard_scale.py for 1/2/4/8 virtual shards:
# C5 d12 (levels of >= 10,000 frontier states sharded) and C3 d9 (>= 100,000), for
# tools/project_scale.py. Output: gpurun_out/$TAG/{c5,c3}_w$W/.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-scale}
mkdir -p $OUT
for W in 1 2 4 8; do
  mkdir -p $OUT/c5_w$W $OUT/c3_w$W
  DSL_LEVEL_TRACE=1 DSL_SCALE_REPLICATE_BELOW=10000 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -T -d $OUT/c5_w$W/kt -o run -- python3 tools/shard_scale.py --workload multipaxos 12 $W > $OUT/c5_w$W/out.jsonl 2> $OUT/c5_w$W/err.txt
  DSL_LEVEL_TRACE=1 DSL_SCALE_REPLICATE_BELOW=100000 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -T -d $OUT/c3_w$W/kt -o run -- python3 tools/shard_scale.py 9 $W > $OUT/c3_w$W/out.jsonl 2> $OUT/c3_w$W/err.txt
  echo "W=$W done"
done
