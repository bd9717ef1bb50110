# Round-4 closing run (product library): the GPU suite and smoke, the default bench line (C5 d12,
# CPU baseline included), then kernel trace + stats and the PMC passes of the same workload
# (tools/gpu_r02_prof.sh).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-final} NOBENCH=1 bash tools/gpu_r04.sh
OUT=gpurun_out/r04_${TAG:-final}
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
cut -c1-300 $OUT/bench.json
bash tools/gpu_r02_prof.sh r04_${TAG:-final}_c5_d12
echo done
