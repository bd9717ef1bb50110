# Bench only (+ phase breakdown of the instrumented build if present). usage: bash tools/gpu_bench.sh [extra bench args]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/bench_d12.json
timeout -k 10 300 python3 bench.py --no-cpu-baseline --depth 14 "$@" > gpurun_out/bench_d14.json
python3 -c "
import json
for f in ['bench_d12','bench_d14']:
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])
"
if [ -f dslabs_amd/libdslabs_hip_phases.so ]; then
DSL_LIB_VARIANT=phases timeout -k 10 200 python3 bench.py --no-cpu-baseline --depth 14 --steps 1 --warmup 0 > gpurun_out/ph.json 2> gpurun_out/ph.err
grep phases gpurun_out/ph.err | tail -3
fi
for V in $DSL_VARIANTS; do
  DSL_LIB_VARIANT=$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --depth 14 > gpurun_out/bench_d14_$V.json
  echo "$V: $(python3 -c "import json; d=json.load(open('gpurun_out/bench_d14_$V.json')); print(d['value'], d['roofline']['avg_launch_ms'])")"
done
