set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DSL_VARIANTS="x2hseq" bash tools/gpu_r02_x2.sh
DSL_LIB_VARIANT=phases timeout -k 10 200 python3 bench.py --no-cpu-baseline --depth 12 --steps 1 --warmup 1 > gpurun_out/ph12.json 2> gpurun_out/ph12.err
grep -A1 "depth 1[12] " gpurun_out/ph12.err | tail -n 4
