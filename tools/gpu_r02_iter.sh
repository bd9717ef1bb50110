# Round-2 iteration: GPU tests, then d12/d14 bench of the product library and of the variants in
# $DSL_VARIANTS, then the phase breakdown of the instrumented build. usage: bash tools/gpu_r02_iter.sh [pytest -k expr]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K=${1:-}
if [ -n "$K" ]; then KA="-k $K"; else KA=""; fi
if [ -z "$NOTESTS" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $KA > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/gpu_tests.log
fi
for V in "" $DSL_VARIANTS; do
  DSL_LIB_VARIANT=$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 > gpurun_out/b12_$V.json
  DSL_LIB_VARIANT=$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --depth 14 --steps 3 > gpurun_out/b14_$V.json
  python3 -c "
import json
for f in ['b12_$V','b14_$V']:
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
done
if [ -f dslabs_amd/libdslabs_hip_phases.so ]; then
DSL_LIB_VARIANT=phases timeout -k 10 200 python3 bench.py --no-cpu-baseline --depth 12 --steps 1 --warmup 1 > gpurun_out/ph12.json 2> gpurun_out/ph12.err
grep phases gpurun_out/ph12.err | tail -n 4
fi
