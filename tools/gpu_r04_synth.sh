# Round-4 C3 measurement: the synthetic d10 bench line (CPU baseline included), then kernel trace +
# stats and the PMC passes of the same workload (tools/gpu_r02_prof.sh).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04_synth
mkdir -p $OUT
timeout -k 10 400 python3 bench.py --workload synthetic --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
cut -c1-400 $OUT/bench.json
bash tools/gpu_r02_prof.sh r04_synth_d10 --workload synthetic --steps 3 --warmup 1
echo done
