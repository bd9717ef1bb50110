set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 > gpurun_out/b12.json
timeout -k 10 300 python3 bench.py --no-cpu-baseline --depth 14 --steps 3 > gpurun_out/b14.json
DSL_LIB_VARIANT=phases timeout -k 10 200 python3 bench.py --no-cpu-baseline --depth 12 --steps 1 --warmup 1 > gpurun_out/ph12.json 2> gpurun_out/ph12.err
DSL_LIB_VARIANT=phases timeout -k 10 200 python3 bench.py --no-cpu-baseline --depth 14 --steps 1 --warmup 0 > gpurun_out/ph14.json 2> gpurun_out/ph14.err
DSL_LEVEL_TRACE=1 DSL_NO_QUEUE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --depth 12 --steps 1 --warmup 1 > gpurun_out/lt12.json 2> gpurun_out/lt12.err
echo ok
