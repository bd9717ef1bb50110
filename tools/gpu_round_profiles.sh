# The round's measurement set on the product library: the default bench line (C5 d12, with its CPU
# baseline), the C3 d10 line, rocprofv3 kernel traces + PMC passes of both (tools/gpu_pmc.sh) and
# the C5 per-level k_level durations (tools/gpu_level_times.sh). usage: bash tools/gpu_round_profiles.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 bench.py > $OUT/bench_c5.json 2> $OUT/bench_c5.err
cut -c1-160 $OUT/bench_c5.json
timeout -k 10 300 python3 bench.py --workload synthetic > $OUT/bench_c3.json 2> $OUT/bench_c3.err
cut -c1-160 $OUT/bench_c3.json
bash tools/gpu_pmc.sh ${TAG}_c5
bash tools/gpu_pmc.sh ${TAG}_c3 --workload synthetic
DSL_VARIANTS=default bash tools/gpu_level_times.sh $TAG
echo profiles done
