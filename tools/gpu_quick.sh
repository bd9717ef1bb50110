# GPU parity tests + bench (d12 default, then d14). usage: bash tools/gpu_quick.sh [pytest -k expr]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K=${1:-}
if [ -n "$K" ]; then KA="-k $K"; else KA=""; fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $KA > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_d12.json
timeout -k 10 300 python3 bench.py --no-cpu-baseline --depth 14 > gpurun_out/bench_d14.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d gpurun_out/kt14 -o run -- python3 bench.py --no-cpu-baseline --depth 14 --steps 1 > /dev/null 2> gpurun_out/kt14.err
python3 -c "
import json
for f in ['bench_d12','bench_d14']:
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])
"
cut -d, -f1-4 gpurun_out/kt14/run_kernel_stats.csv
