# Quick perf check: GPU tests (subset or all) then d12/d14 bench (+ phases of d14 if built).
# usage: bash tools/gpu_perf.sh [pytest -k expr]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
fi
tail -1 gpurun_out/gpu_tests.log
for i in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > gpurun_out/p12.json
timeout -k 10 300 python3 bench.py --no-cpu-baseline --depth 14 > gpurun_out/p14.json
python3 -c "
import json
for f in ['p12','p14']:
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
if [ -f dslabs_amd/libdslabs_hip_phases.so ]; then
DSL_LIB_VARIANT=phases timeout -k 10 200 python3 bench.py --no-cpu-baseline --depth 14 --steps 1 --warmup 0 > gpurun_out/ph.json 2> gpurun_out/ph.err
grep phases gpurun_out/ph.err | tail -3
fi
