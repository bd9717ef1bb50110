# Queued small levels vs. one launch per level (DSL_NO_QUEUE), d12/d14, plus a kernel trace.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/q12.json
DSL_NO_QUEUE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/nq12.json
python3 -c "
import json
for f in ['q12','nq12']:
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
DSL_LEVEL_TRACE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/lt12.json 2> gpurun_out/lt12.err
timeout -k 10 200 python3 bench.py --no-cpu-baseline --depth 14 > gpurun_out/q14.json
python3 -c "
import json
d=json.load(open('gpurun_out/q14.json')); print('q14', d['value'], d['ms_per_step'])"
mkdir -p gpurun_out/kt12
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/kt12 -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/kt12.json 2> gpurun_out/kt12.err
